"""C5 (50k blended triangles, 1080p): (triangle, wave-block) units of the ordered raster's blend loop for
64x4, 32x8 and 16x16 wave blocks, and the fragment count (exact span rule).  CPU only, ~5 min."""
import sys, numpy as np
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import scenes
W,H=1920,1080
xy,z,c=scenes.triangle_soup(50000,W,H,256.0,seed=1234,alpha=(0.2,0.8))
sx=xy[:,0::2]; sy=xy[:,1::2]
# per triangle: rows ceil(ymin)..ceil(ymax)-1, span per row via crossings
tot={}
frag=0
shapes=[(64,4),(32,8),(16,16)]
units={s:0 for s in shapes}
for t in range(len(xy)):
    X=sx[t]; Y=sy[t]
    y0=max(int(np.ceil(Y.min())),0); y1=min(int(np.ceil(Y.max())),H)
    if y1<=y0: continue
    y=np.arange(y0,y1,dtype=np.float64)
    cr=np.full((len(y),3),np.nan)
    for k in range(3):
        i,j=k,(k+1)%3
        st=(Y[i]>y)!=(Y[j]>y)
        with np.errstate(all="ignore"):
            xc=(X[j]-X[i])*(y-Y[i])/(Y[j]-Y[i])+X[i]
        cr[st,k]=xc[st]
    with np.errstate(all="ignore"):
        lo=np.clip(np.ceil(np.nanmin(cr,1)),0,W); hi=np.clip(np.ceil(np.nanmax(cr,1)),0,W)
    ok=~np.isnan(lo)&~np.isnan(hi)&(hi>lo)
    y=y[ok].astype(int); lo=lo[ok].astype(int); hi=hi[ok].astype(int)
    frag+=int((hi-lo).sum())
    for (bw,bh) in shapes:
        s=set()
        for yy,a,b in zip(y,lo,hi):
            for bx in range(a//bw,(b-1)//bw+1):
                s.add((yy//bh,bx))
        units[(bw,bh)]+=len(s)
print("fragments",frag)
for k,v in units.items(): print(k, v, "px/unit %.1f"%(frag/v))
