import ctypes, time, numpy as np, sys
sys.path.insert(0, '.')
from libnativecpurenderer_amd import _lib
g = _lib.load()
def vp(a): return a.ctypes.data_as(ctypes.c_void_p)
for frames, s in ((20000, 1), (20000, 16), (int(44100*114), 4410)):
    d = np.random.default_rng(1).uniform(-.5, .5, size=2*frames)
    a = g.CreateAudioClipFromBuffer(44100, 2, frames, vp(d))
    out = np.empty(1); g.GetAudioClipBuffer(a, vp(np.empty(2*frames)))
    t0 = time.perf_counter(); g.OverlayAudioClip(a, a, s, False); g.GetAudioClipBuffer(a, vp(np.empty(2*frames))); t1 = time.perf_counter()
    print(frames, s, "%.3f ms" % ((t1-t0)*1e3), "per chain step %.3f us" % ((t1-t0)*1e6/ (frames/s)))
    g.DestroyAudioClip(a)
