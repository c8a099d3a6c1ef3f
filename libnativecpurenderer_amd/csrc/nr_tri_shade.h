// nr_tri_shade.h — per-pixel pieces of the order-free raster (nr_tri_free.hip,
// k_vis): the depth of one fragment as a packed visibility key, and the
// deferred shading of a pixel from its winning triangle (record ->
// barycentrics -> colour -> ApplyPixel, cpp:515-549 -> framebuffer, depth and
// frame output).
#pragma once

#include "nr_tri.h"

// Index checks of the shading passes (a build with -DNR_SHADE_CHECK=1 only:
// tools/exp/check.so, loaded with NR_LIB=...): a failed check prints the
// pixel and the indices instead of reading out of range silently.
#ifndef NR_SHADE_CHECK
#define NR_SHADE_CHECK 0
#endif
#if NR_SHADE_CHECK
#define NR_DEV_CHECK(cond, ...)                       \
    do {                                              \
        if (!(cond)) printf("NR_SHADE_CHECK " __VA_ARGS__); \
    } while (0)
#else
#define NR_DEV_CHECK(cond, ...) \
    do {                        \
    } while (0)
#endif

namespace nrtri {

// Doubles of a shading record (build_record): Gouraud sx0 sy0 e1x e1y e2x e2y
// inv | c0 rgb | (c1-c0) rgb | (c2-c0) rgb; flat rgb.
template <bool GOURAUD>
struct RecLen {
    static constexpr int REC = GOURAUD ? 16 : 3;
};

// Depth of a shaded pixel (winner kv; (u32)kv == 0: no fragment won it):
// the winner's depth, or a pending depth clear.
template <int ZMODE>
__device__ __forceinline__ void store_depth(const FrameParams& fp, i64 p, u64 kv) {
    if (ZMODE == 1 && (u32)kv) out_store<u32>(fp.depth + p, (u32)(kv >> 32));
    else if (ZMODE != 0 && fp.pendDepth) out_store<u32>(fp.depth + p, fp.pendDepthValue);
}

// Framebuffer (+ frame output, nr_tri.h store_frame_out) value of pixel p =
// (px, py), written once.
__device__ __forceinline__ void store_colour(const FrameParams& fp, i64 p, i64 px, i64 py, f64 cr, f64 cg, f64 cb,
                                             f64 ca) {
    const int ipp = fp.ipp;
    f64* dst = fp.fb + p * ipp;
    out_store<f64>(dst, cr); out_store<f64>(dst + 1, cg); out_store<f64>(dst + 2, cb);
    if (ipp == 4) out_store<f64>(dst + 3, ca);
    store_frame_out(fp, p, px, py, cr, cg, cb, ca);
}

// ApplyPixel (cpp:529-547) of the winner's colour.  ca == 1 except for
// non-finite barycentrics; the destination is read only then.
__device__ __forceinline__ void apply_winner(const FrameParams& fp, i64 p, f64& cr, f64& cg, f64& cb, f64& ca) {
    cr *= fp.ct[0]; cg *= fp.ct[1]; cb *= fp.ct[2]; ca *= fp.ct[3];
    if (ca != 1) {
        const f64* dst = fp.fb + p * fp.ipp;
        f64 R, G, B;
        if (fp.pendColor) {
            R = G = B = fp.pendColorValue;
        } else {
            R = dst[0]; G = dst[1]; B = dst[2];
        }
        cr = R * (1 - ca) + cr * ca;
        cg = G * (1 - ca) + cg * ca;
        cb = B * (1 - ca) + cb * ca;
    }
}

// Pending clears of a pixel no fragment won.
template <int ZMODE>
__device__ __forceinline__ void store_clear(const FrameParams& fp, i64 p, i64 px, i64 py) {
    if (fp.pendColor) {
        const f64 v = fp.pendColorValue;
        store_colour(fp, p, px, py, v, v, v, v);
    }
    store_depth<ZMODE>(fp, p, 0);
}

// A winner's source data for its shading record: vertices and the rgb of
// each vertex (alpha is not needed, see ShadeStage), loaded as 16 + 8 bytes
// per vertex colour.
template <bool GOURAUD>
struct RecordSrc {
    f64 p[GOURAUD ? 6 : 1];
    f64 c[GOURAUD ? 9 : 3];
};

template <bool GOURAUD>
__device__ __forceinline__ void load_record_src(const FrameParams& fp, i64 t, RecordSrc<GOURAUD>& s) {
    if constexpr (GOURAUD) load_tri_xy(fp.src.xy, t, s.p);
    const int nv = GOURAUD ? 3 : 1, stride = GOURAUD ? 12 : 4;
#pragma unroll
    for (int v = 0; v < nv; ++v) {
        const f64* q = fp.src.rgba + t * stride + 4 * v;
        const double2 rg = *reinterpret_cast<const double2*>(q);
        s.c[3 * v] = rg.x; s.c[3 * v + 1] = rg.y; s.c[3 * v + 2] = q[2];
    }
}

// Shading record from its source (the expressions of the per-pixel path, once).
template <bool GOURAUD>
__device__ __forceinline__ void build_record(const FrameParams& fp, const RecordSrc<GOURAUD>& s, f64* r) {
    if constexpr (GOURAUD) {
        f64 sx[3], sy[3];
#pragma unroll
        for (int v = 0; v < 3; ++v) nr_xform(fp.m, s.p[2 * v], s.p[2 * v + 1], sx[v], sy[v]);
        const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
        r[0] = sx[0]; r[1] = sy[0]; r[2] = e1x; r[3] = e1y; r[4] = e2x; r[5] = e2y;
        r[6] = 1.0 / (e1x * e2y - e2x * e1y);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            r[7 + k] = s.c[k];
            r[10 + k] = s.c[3 + k] - s.c[k];
            r[13 + k] = s.c[6 + k] - s.c[k];
        }
    } else {
        r[0] = s.c[0]; r[1] = s.c[1]; r[2] = s.c[2];
    }
}

// Shading record of triangle t.
template <bool GOURAUD>
__device__ __forceinline__ void make_record(const FrameParams& fp, i64 t, f64* r) {
    RecordSrc<GOURAUD> s;
    load_record_src<GOURAUD>(fp, t, s);
    build_record<GOURAUD>(fp, s, r);
}

// Colour of pixel (px, py) from a record.
template <bool GOURAUD>
__device__ __forceinline__ void record_colour(const f64* r, i64 px, i64 py, f64& cr, f64& cg, f64& cb, f64& ca) {
    if (GOURAUD) {
        const f64 dx = (f64)px - r[0], dy = (f64)py - r[1];
        const f64 w1 = (dx * r[5] - r[4] * dy) * r[6];
        const f64 w2 = (r[2] * dy - dx * r[3]) * r[6];
        cr = r[7] + r[10] * w1 + r[13] * w2;
        cg = r[8] + r[11] * w1 + r[14] * w2;
        cb = r[9] + r[12] * w1 + r[15] * w2;
        ca = 1.0 + 0.0 * w1 + 0.0 * w2;   // c[3] + (c[7]-c[3])*w1 + (c[11]-c[3])*w2 with unit alphas
    } else {
        cr = r[0]; cg = r[1]; cb = r[2]; ca = 1.0;
    }
}

// Depth (quantised) of one covered fragment at pixel x = X of a row dy below
// vertex 0 (expressions as the oracle): the per-pixel step of every
// order-free raster.
__device__ __forceinline__ u32 frag_depth(f64 X, f64 dy, f64 sx0, f64 e1x, f64 e1y, f64 e2x, f64 e2y, f64 inv, f64 zz0,
                                          f64 dz1, f64 dz2) {
    const f64 dx = X - sx0;
    const f64 w1 = (dx * e2y - e2x * dy) * inv;
    const f64 w2 = (e1x * dy - dx * e1y) * inv;
    const f64 zz = zz0 + dz1 * w1 + dz2 * w2;
    return nr_quantize_depth_hw(zz);
}
// ... into the tile's LDS keys (k_vis).
template <int ZMODE>
__device__ __forceinline__ void frag_key(u64* key, const u32* zin, int p, f64 X, f64 dy, f64 sx0, f64 e1x, f64 e1y,
                                         f64 e2x, f64 e2y, f64 inv, f64 zz0, f64 dz1, f64 dz2, u64 id1) {
    const u32 zq = frag_depth(X, dy, sx0, e1x, e1y, e2x, e2y, inv, zz0, dz1, dz2);
    if (ZMODE == 1) atomicMin(&key[p], ((u64)zq << 32) | id1);
    else if (zq < zin[p]) atomicMax(&key[p], id1);
}

}  // namespace nrtri
