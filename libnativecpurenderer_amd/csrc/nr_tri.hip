// nr_tri.hip — the triangle / depth / Gouraud path (the north-star hot path).
//
// Semantics (no reference implementation exists; defined
// in the reference's idiom, DESIGN.md §3, restated in oracle/oracle.c):
//   vertices -> context transform (cpp:446-453) -> screen space;
//   coverage = even-odd pointInPolygon (cpp:822-845) at integer pixels;
//   w1,w2 barycentric in f64, attr = a0 + (a1-a0)*w1 + (a2-a0)*w2;
//   depth u32 LESS, written only when test+write are on;
//   blend = ApplyPixel (cpp:515-549) in submission order.
//
// Pipeline (one DrawTriangles call = one batch, all async on the stream):
//   1 k_tri_count   per triangle: screen bbox -> number of 64x32 tiles touched
//   2 scan          exclusive sum of the counts (hipcub)
//   3 k_tri_emit    (tile, triangle) pairs, written in triangle order
//   4 sort          stable radix sort by tile -> per-tile lists stay in
//                   submission order (painter's order is preserved)
//   5 k_tile_ranges start/end of each tile's list
//   6 k_tile_raster one 512-thread workgroup per 64x32 tile: the tile's colour
//                   and Z live in registers (8 waves x 4 rows x 64 lanes) for
//                   the whole list; per 64-triangle chunk the setup and the
//                   exact per-row coverage spans are staged in LDS, then each
//                   wave walks the chunk in order and blends its covered lanes.
//                   The framebuffer tile is read at most once and written once;
//                   a pending uniform clear is applied on chip (never read).
//
// Per-row spans are bit-identical to the per-pixel even-odd test: for a row y
// the crossing x of an edge depends only on y, the two straddling edges give
// crossings ca, cb and (x < ca) != (x < cb)  <=>  ceil(min) <= x < ceil(max).
#include "nr_common.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

namespace {

constexpr int TW = 64;           // tile width  = one wave's lanes
constexpr int TH = 32;           // tile height = 8 waves x 4 rows
constexpr int RPW = 4;           // rows per wave
constexpr int NWAVE = TH / RPW;  // 8
constexpr int WG = NWAVE * 64;   // 512 threads
constexpr int CH = 64;           // triangles staged per chunk

struct TriSrc {
    const f64* xy;
    const f64* z;
    const f64* rgba;
    int gouraud;
    i64 n;
};

struct BinParams {
    TriSrc src;
    f64 m[6];
    i64 W, H;
    int tiles_x;
};

__device__ __forceinline__ f64 clampd(f64 v, f64 lo, f64 hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Screen-space vertices of triangle t (cpp:446-453 applied to each vertex).
__device__ __forceinline__ void tri_screen(const TriSrc& s, const f64* m, i64 t, f64 (&sx)[3], f64 (&sy)[3]) {
    const f64* p = s.xy + t * 6;
#pragma unroll
    for (int v = 0; v < 3; ++v) nr_xform(m, p[2 * v], p[2 * v + 1], sx[v], sy[v]);
}

// Tile rectangle touched by a triangle; false if it produces no fragment.
// Rows: a row y has a straddling edge iff ymin <= y < ymax (exact), so
// [ceil(ymin), ceil(ymax)).  Columns: crossings lie in [xmin, xmax] up to
// rounding, so [floor(xmin)-2, ceil(xmax)+2]; for |coord| > 1e7 the full width.
__device__ __forceinline__ bool tri_tiles(const f64 (&sx)[3], const f64 (&sy)[3], i64 W, i64 H, int& tx0, int& tx1,
                                          int& ty0, int& ty1) {
    bool finite = true, huge = false;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        finite = finite && isfinite(sx[v]) && isfinite(sy[v]);
        huge = huge || fabs(sx[v]) > 1e7 || fabs(sy[v]) > 1e7;
    }
    if (!finite) return false;
    f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
    f64 den = e1x * e2y - e2x * e1y;
    if (den == 0) return false;
    f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
    i64 r0 = (i64)clampd(ceil(ymn), 0.0, (f64)H);
    i64 r1 = (i64)clampd(ceil(ymx), 0.0, (f64)H);
    if (r0 >= r1) return false;
    i64 c0 = 0, c1 = W - 1;
    if (!huge) {
        f64 xmn = fmin(fmin(sx[0], sx[1]), sx[2]), xmx = fmax(fmax(sx[0], sx[1]), sx[2]);
        c0 = (i64)clampd(floor(xmn) - 2, 0.0, (f64)(W - 1));
        c1 = (i64)clampd(ceil(xmx) + 2, -1.0, (f64)(W - 1));
        if (ceil(xmx) + 2 < 0 || floor(xmn) - 2 > (f64)(W - 1)) return false;
    }
    if (c0 > c1) return false;
    tx0 = (int)(c0 / TW); tx1 = (int)(c1 / TW);
    ty0 = (int)(r0 / TH); ty1 = (int)((r1 - 1) / TH);
    return true;
}

// Per-triangle tile count.  With `nonopaque` set, also flags any vertex
// alpha != 1 (device-pointer batches whose opacity the host cannot know).
__global__ __launch_bounds__(256) void k_tri_count(const BinParams bp, unsigned long long* __restrict__ cnt,
                                                   u32* __restrict__ nonopaque) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    bool bad = false;
    if (t < bp.src.n) {
        f64 sx[3], sy[3];
        tri_screen(bp.src, bp.m, t, sx, sy);
        int tx0, tx1, ty0, ty1;
        unsigned long long c = 0;
        if (tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1))
            c = (unsigned long long)(tx1 - tx0 + 1) * (ty1 - ty0 + 1);
        cnt[t] = c;
        if (nonopaque) {
            if (bp.src.gouraud) {
                const f64* a = bp.src.rgba + t * 12;
                bad = a[3] != 1 || a[7] != 1 || a[11] != 1;
            } else {
                bad = bp.src.rgba[t * 4 + 3] != 1;
            }
        }
    }
    if (nonopaque) {
        const unsigned long long m = __ballot(bad);
        if (m && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1)) atomicOr(nonopaque, 1u);
    }
}

__global__ __launch_bounds__(256) void k_tri_emit(const BinParams bp, const unsigned long long* __restrict__ off,
                                                  u32* __restrict__ keys, u32* __restrict__ vals) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= bp.src.n) return;
    f64 sx[3], sy[3];
    tri_screen(bp.src, bp.m, t, sx, sy);
    int tx0, tx1, ty0, ty1;
    if (!tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) return;
    unsigned long long o = off[t];
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            keys[o] = (u32)(ty * bp.tiles_x + tx);
            vals[o] = (u32)t;
            ++o;
        }
}

__global__ __launch_bounds__(256) void k_tile_ranges(const u32* __restrict__ keys, u32 P, u32* __restrict__ start,
                                                     u32* __restrict__ end) {
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const u32 k = keys[i];
    if (i == 0 || keys[i - 1] != k) start[k] = i;
    if (i == P - 1 || keys[i + 1] != k) end[k] = i + 1;
}

struct RasterParams {
    TriSrc src;
    f64 m[6];
    f64 ct[4];
    f64* fb;
    u32* depth;
    i64 W, H;
    int ipp;
    int tiles_x;
    int depthTest, depthWrite;
    int pendColor;
    f64 pendColorValue;
    int pendDepth;
    u32 pendDepthValue;
    const u32* list;
    const u32* tstart;
    const u32* tend;
    unsigned long long* fragCounter;   // non-null: count covered fragments
};

// LDS staging slots of a chunk (SoA, CH entries each)
enum {
    S_X0 = 0, S_Y0, S_X1, S_Y1, S_X2, S_Y2,   // screen-space vertices
    S_E1X, S_E1Y, S_E2X, S_E2Y, S_INV,         // barycentric setup
    S_Z0, S_DZ1, S_DZ2,                        // depth: z0, z1-z0, z2-z0
    S_C0,                                      // colour c0[4] (flat: the colour)
    S_D1 = S_C0 + 4,                           // c1-c0 [4] (Gouraud)
    S_D2 = S_D1 + 4,                           // c2-c0 [4] (Gouraud)
    S_NSLOT = S_D2 + 4
};

template <bool GOURAUD, bool DEPTH, bool COUNT>
__global__ __launch_bounds__(WG) void k_tile_raster(const RasterParams rp) {
    const int tile = blockIdx.x;
    const int tx = tile % rp.tiles_x, ty = tile / rp.tiles_x;
    const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const u32 ls = rp.tstart[tile], le = rp.tend[tile];
    if (ls == le && !rp.pendColor && !(DEPTH && rp.pendDepth)) return;

    __shared__ f64 S[S_NSLOT][CH];
    __shared__ iu8 XS[CH][TH], XE[CH][TH];
    __shared__ iu8 NE[CH][NWAVE];
    __shared__ iu8 VALID[CH];
    __shared__ unsigned long long fragSum;
    if (COUNT && tid == 0) fragSum = 0;

    // ---- the tile's pixel state, resident in registers for the whole list
    const i64 px = x0 + lane;
    const int ipp = rp.ipp;
    f64 cr[RPW], cg[RPW], cb[RPW], ca[RPW];
    u32 cz[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const i64 py = y0 + wave * RPW + r;
        cr[r] = cg[r] = cb[r] = ca[r] = 0;
        cz[r] = 0xFFFFFFFFu;
        if (px < rp.W && py < rp.H) {
            if (rp.pendColor) {
                cr[r] = cg[r] = cb[r] = ca[r] = rp.pendColorValue;
            } else {
                const f64* p = rp.fb + (py * rp.W + px) * ipp;
                cr[r] = p[0]; cg[r] = p[1]; cb[r] = p[2];
                if (ipp == 4) ca[r] = p[3];
            }
            if (DEPTH) cz[r] = rp.pendDepth ? rp.pendDepthValue : rp.depth[py * rp.W + px];
        }
    }
    const f64 ct0 = rp.ct[0], ct1 = rp.ct[1], ct2 = rp.ct[2], ct3 = rp.ct[3];
    const i64 wlim = rp.W - x0 < TW ? rp.W - x0 : TW;   // valid lanes of this tile
    unsigned long long myFrags = 0;

    for (u32 base = ls; base < le; base += CH) {
        const int cnt = (le - base) < (u32)CH ? (int)(le - base) : CH;
        // ---- (a) triangle setup, one thread per triangle
        if (tid < cnt) {
            const i64 t = rp.list[base + tid];
            f64 sx[3], sy[3];
            tri_screen(rp.src, rp.m, t, sx, sy);
            bool ok = isfinite(sx[0]) && isfinite(sy[0]) && isfinite(sx[1]) && isfinite(sy[1]) &&
                      isfinite(sx[2]) && isfinite(sy[2]);
            const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
            const f64 den = e1x * e2y - e2x * e1y;
            ok = ok && den != 0;
            VALID[tid] = ok;
            S[S_X0][tid] = sx[0]; S[S_Y0][tid] = sy[0];
            S[S_X1][tid] = sx[1]; S[S_Y1][tid] = sy[1];
            S[S_X2][tid] = sx[2]; S[S_Y2][tid] = sy[2];
            S[S_E1X][tid] = e1x; S[S_E1Y][tid] = e1y; S[S_E2X][tid] = e2x; S[S_E2Y][tid] = e2y;
            S[S_INV][tid] = 1.0 / den;
            if (DEPTH) {
                f64 z0 = 0, z1 = 0, z2 = 0;
                if (rp.src.z) { z0 = rp.src.z[t * 3]; z1 = rp.src.z[t * 3 + 1]; z2 = rp.src.z[t * 3 + 2]; }
                S[S_Z0][tid] = z0; S[S_DZ1][tid] = z1 - z0; S[S_DZ2][tid] = z2 - z0;
            }
            if (GOURAUD) {
                const f64* c = rp.src.rgba + t * 12;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    S[S_C0 + k][tid] = c[k];
                    S[S_D1 + k][tid] = c[4 + k] - c[k];
                    S[S_D2 + k][tid] = c[8 + k] - c[k];
                }
            } else {
                const f64* c = rp.src.rgba + t * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) S[S_C0 + k][tid] = c[k];
            }
        }
        __syncthreads();
        // ---- (b) exact coverage spans: thread = (triangle k, wave-row group rg)
        {
            const int k = tid >> 3, rg = tid & 7;
            if (k < cnt) {
                bool any = false;
                const bool ok = VALID[k];
                const f64 sx[3] = {S[S_X0][k], S[S_X1][k], S[S_X2][k]};
                const f64 sy[3] = {S[S_Y0][k], S[S_Y1][k], S[S_Y2][k]};
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    const int row = rg * RPW + r;
                    const i64 gy = y0 + row;
                    int xs = 0, xe = 0;
                    if (ok && gy < rp.H) {
                        const f64 y = (f64)gy;
                        f64 c[2] = {0, 0};
                        int nc = 0;
                        // edges in pointInPolygon's order: (i=0,j=2) (i=1,j=0) (i=2,j=1)
#pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            const int j = (i + 2) % 3;
                            if ((sy[i] > y) != (sy[j] > y)) {
                                const f64 cc = (sx[j] - sx[i]) * (y - sy[i]) / (sy[j] - sy[i]) + sx[i];
                                if (nc == 0) c[0] = cc; else c[1] = cc;
                                ++nc;
                            }
                        }
                        if (nc == 2) {
                            const f64 lo = fmin(c[0], c[1]), hi = fmax(c[0], c[1]);
                            xs = (int)clampd(ceil(lo) - (f64)x0, 0.0, (f64)wlim);
                            xe = (int)clampd(ceil(hi) - (f64)x0, 0.0, (f64)wlim);
                            if (xe < xs) xe = xs;
                        }
                    }
                    XS[k][row] = (iu8)xs;
                    XE[k][row] = (iu8)xe;
                    any = any || xs < xe;
                    if (COUNT) myFrags += (unsigned long long)(xe - xs);
                }
                NE[k][rg] = any;
            }
        }
        __syncthreads();
        // ---- (c) in-order raster of the chunk; each wave owns 4 rows
        for (int k = 0; k < cnt; ++k) {
            if (!NE[k][wave]) continue;
            const f64 sx0 = S[S_X0][k], sy0 = S[S_Y0][k];
            const f64 e1x = S[S_E1X][k], e1y = S[S_E1Y][k], e2x = S[S_E2X][k], e2y = S[S_E2Y][k];
            const f64 inv = S[S_INV][k];
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int row = wave * RPW + r;
                const int xs = XS[k][row], xe = XE[k][row];
                if (lane < xs || lane >= xe) continue;
                f64 w1 = 0, w2 = 0;
                if (DEPTH || GOURAUD) {
                    const f64 dx = (f64)(x0 + lane) - sx0, dy = (f64)(y0 + row) - sy0;
                    w1 = (dx * e2y - e2x * dy) * inv;
                    w2 = (e1x * dy - dx * e1y) * inv;
                }
                u32 zq = 0;
                if (DEPTH) {
                    const f64 zz = S[S_Z0][k] + S[S_DZ1][k] * w1 + S[S_DZ2][k] * w2;
                    zq = nr_quantize_depth(zz);
                    if (!(zq < cz[r])) continue;
                }
                f64 R, G, B, A;
                if (GOURAUD) {
                    R = S[S_C0 + 0][k] + S[S_D1 + 0][k] * w1 + S[S_D2 + 0][k] * w2;
                    G = S[S_C0 + 1][k] + S[S_D1 + 1][k] * w1 + S[S_D2 + 1][k] * w2;
                    B = S[S_C0 + 2][k] + S[S_D1 + 2][k] * w1 + S[S_D2 + 2][k] * w2;
                    A = S[S_C0 + 3][k] + S[S_D1 + 3][k] * w1 + S[S_D2 + 3][k] * w2;
                } else {
                    R = S[S_C0 + 0][k]; G = S[S_C0 + 1][k]; B = S[S_C0 + 2][k]; A = S[S_C0 + 3][k];
                }
                // ApplyPixel (cpp:529-547) on the register-resident pixel
                R *= ct0; G *= ct1; B *= ct2; A *= ct3;
                if (A != 1) {
                    R = cr[r] * (1 - A) + R * A;
                    G = cg[r] * (1 - A) + G * A;
                    B = cb[r] * (1 - A) + B * A;
                }
                cr[r] = R; cg[r] = G; cb[r] = B; ca[r] = A;
                if (DEPTH && rp.depthWrite) cz[r] = zq;
            }
        }
        __syncthreads();
    }

    // ---- write the tile back once
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const i64 py = y0 + wave * RPW + r;
        if (px < rp.W && py < rp.H) {
            f64* p = rp.fb + (py * rp.W + px) * ipp;
            p[0] = cr[r]; p[1] = cg[r]; p[2] = cb[r];
            if (ipp == 4) p[3] = ca[r];
            if (DEPTH && (rp.depthWrite || rp.pendDepth)) rp.depth[py * rp.W + px] = cz[r];
        }
    }
    if (COUNT) {
        atomicAdd(&fragSum, myFrags);
        __syncthreads();
        if (tid == 0) atomicAdd(rp.fragCounter, fragSum);
    }
}

// ---------------------------------------------------------------------------
// Order-free raster for opaque batches (every fragment overwrites: alpha == 1
// after the colour transform).  Sequential semantics then reduce per pixel to
//   Z LESS + write : winner = min over (zq, tri) with zq < z_init -> key min
//   Z LESS, no write: winner = last tri with zq < z_init           -> id max
//   no Z test       : winner = last covering tri                    -> id max
// so fragments are processed in any order with 64-bit LDS atomics on a packed
// key ((zq << 32) | tri+1), then one resolve per pixel shades only the winner
// (deferred shading).  Bit-identical to the ordered path by construction.
// Fragment-parallel: per 256-triangle chunk the exact row spans are counted,
// prefix-summed, and every thread takes fragments (binary search -> tri, row
// walk -> x), so tiny triangles keep all 64 lanes busy.
// ---------------------------------------------------------------------------
constexpr int FCH = 256;
enum { F_X0 = 0, F_Y0, F_X1, F_Y1, F_X2, F_Y2, F_E1X, F_E1Y, F_E2X, F_E2Y, F_INV, F_Z0, F_DZ1, F_DZ2, F_NSLOT };

template <int ZMODE, bool GOURAUD, bool COUNT>   // ZMODE 0: no test, 1: LESS+write, 2: LESS no write
__global__ __launch_bounds__(WG) void k_tile_raster_free(const RasterParams rp) {
    constexpr bool DEPTH = ZMODE != 0;
    const int tile = blockIdx.x;
    const int tx = tile % rp.tiles_x, ty = tile / rp.tiles_x;
    const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
    const int tid = threadIdx.x;
    const u32 ls = rp.tstart[tile], le = rp.tend[tile];
    if (ls == le && !rp.pendColor && !(DEPTH && rp.pendDepth)) return;

    __shared__ u64 key[TH * TW];
    __shared__ u32 zin[ZMODE == 2 ? TH * TW : 1];
    __shared__ f64 S[F_NSLOT][FCH];
    __shared__ u32 TIDX[FCH];
    __shared__ iu8 XS[FCH][TH], XE[FCH][TH];
    __shared__ u32 OFF[FCH + 1];
    __shared__ iu8 RR0[FCH];

    const int wlim = (int)(rp.W - x0 < TW ? rp.W - x0 : TW);
    const int hlim = (int)(rp.H - y0 < TH ? rp.H - y0 : TH);
    for (int p = tid; p < TH * TW; p += WG) {
        const int lx = p & (TW - 1), ly = p / TW;
        u32 z0 = 0xFFFFFFFFu;
        if (DEPTH && lx < wlim && ly < hlim)
            z0 = rp.pendDepth ? rp.pendDepthValue : rp.depth[(y0 + ly) * rp.W + x0 + lx];
        key[p] = ZMODE == 1 ? ((u64)z0 << 32) : 0ull;
        if (ZMODE == 2) zin[p] = z0;
    }
    u64 fragTotal = 0;

    for (u32 base = ls; base < le; base += FCH) {
        const int cnt = (le - base) < (u32)FCH ? (int)(le - base) : FCH;
        __syncthreads();
        // ---- (a) setup + exact spans, one thread per triangle
        if (tid < cnt) {
            const u32 t = rp.list[base + tid];
            f64 sx[3], sy[3];
            tri_screen(rp.src, rp.m, t, sx, sy);
            bool ok = isfinite(sx[0]) && isfinite(sy[0]) && isfinite(sx[1]) && isfinite(sy[1]) &&
                      isfinite(sx[2]) && isfinite(sy[2]);
            const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
            const f64 den = e1x * e2y - e2x * e1y;
            ok = ok && den != 0;
            S[F_X0][tid] = sx[0]; S[F_Y0][tid] = sy[0];
            S[F_E1X][tid] = e1x; S[F_E1Y][tid] = e1y; S[F_E2X][tid] = e2x; S[F_E2Y][tid] = e2y;
            S[F_INV][tid] = 1.0 / den;
            if (DEPTH) {
                f64 z0 = 0, z1 = 0, z2 = 0;
                if (rp.src.z) { z0 = rp.src.z[(i64)t * 3]; z1 = rp.src.z[(i64)t * 3 + 1]; z2 = rp.src.z[(i64)t * 3 + 2]; }
                S[F_Z0][tid] = z0; S[F_DZ1][tid] = z1 - z0; S[F_DZ2][tid] = z2 - z0;
            }
            TIDX[tid] = t;
            int r0 = 0;
            u32 nf = 0;
            if (ok) {
                // rows with a straddling edge: ymin <= y < ymax (exact)
                const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
                r0 = (int)clampd(ceil(ymn) - (f64)y0, 0.0, (f64)hlim);
                const int r1 = (int)clampd(ceil(ymx) - (f64)y0, 0.0, (f64)hlim);
                for (int r = r0; r < r1; ++r) {
                    const f64 y = (f64)(y0 + r);
                    f64 c[2] = {0, 0};
                    int nc = 0;
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        const int j = (i + 2) % 3;
                        if ((sy[i] > y) != (sy[j] > y)) {
                            const f64 cc = (sx[j] - sx[i]) * (y - sy[i]) / (sy[j] - sy[i]) + sx[i];
                            if (nc == 0) c[0] = cc; else c[1] = cc;
                            ++nc;
                        }
                    }
                    int xs = 0, xe = 0;
                    if (nc == 2) {
                        const f64 lo = fmin(c[0], c[1]), hi = fmax(c[0], c[1]);
                        xs = (int)clampd(ceil(lo) - (f64)x0, 0.0, (f64)wlim);
                        xe = (int)clampd(ceil(hi) - (f64)x0, 0.0, (f64)wlim);
                        if (xe < xs) xe = xs;
                    }
                    XS[tid][r] = (iu8)xs;
                    XE[tid][r] = (iu8)xe;
                    nf += (u32)(xe - xs);
                }
            }
            RR0[tid] = (iu8)r0;
            OFF[tid] = nf;
        }
        __syncthreads();
        // ---- (b) exclusive scan of the fragment counts (wave 0)
        if (tid < 64) {
            u32 v[FCH / 64];
            u32 sum = 0;
#pragma unroll
            for (int i = 0; i < FCH / 64; ++i) {
                const int idx = tid * (FCH / 64) + i;
                v[i] = idx < cnt ? OFF[idx] : 0u;
                sum += v[i];
            }
            u32 incl = sum;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const u32 o = __shfl_up(incl, d, 64);
                if (tid >= d) incl += o;
            }
            u32 ex = incl - sum;
#pragma unroll
            for (int i = 0; i < FCH / 64; ++i) {
                OFF[tid * (FCH / 64) + i] = ex;
                ex += v[i];
            }
            if (tid == 63) OFF[FCH] = incl;
        }
        __syncthreads();
        // ---- (c) fragment-parallel visibility
        const u32 F = OFF[cnt];
        if (COUNT) fragTotal += F;
        for (u32 f = tid; f < F; f += WG) {
            int lo = 0, hi = cnt;            // OFF[lo] <= f < OFF[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (OFF[mid] <= f) lo = mid; else hi = mid;
            }
            const int k = lo;
            u32 l = f - OFF[k];
            int r = RR0[k];
            for (;;) {
                const u32 len = (u32)(XE[k][r] - XS[k][r]);
                if (l < len) break;
                l -= len;
                ++r;
            }
            const int lx = XS[k][r] + (int)l;
            const int p = r * TW + lx;
            const u64 id1 = (u64)TIDX[k] + 1;
            if (ZMODE == 0) {
                atomicMax(&key[p], id1);
            } else {
                const f64 dx = (f64)(x0 + lx) - S[F_X0][k], dy = (f64)(y0 + r) - S[F_Y0][k];
                const f64 w1 = (dx * S[F_E2Y][k] - S[F_E2X][k] * dy) * S[F_INV][k];
                const f64 w2 = (S[F_E1X][k] * dy - dx * S[F_E1Y][k]) * S[F_INV][k];
                const f64 zz = S[F_Z0][k] + S[F_DZ1][k] * w1 + S[F_DZ2][k] * w2;
                const u32 zq = nr_quantize_depth(zz);
                if (ZMODE == 1) atomicMin(&key[p], ((u64)zq << 32) | id1);
                else if (zq < zin[p]) atomicMax(&key[p], id1);
            }
        }
    }
    __syncthreads();

    // ---- resolve: one pass over the tile, shading only the winners
    const int ipp = rp.ipp;
    const f64 ct0 = rp.ct[0], ct1 = rp.ct[1], ct2 = rp.ct[2], ct3 = rp.ct[3];
    for (int p = tid; p < TH * TW; p += WG) {
        const int lx = p & (TW - 1), ly = p / TW;
        if (lx >= wlim || ly >= hlim) continue;
        const i64 px = x0 + lx, py = y0 + ly;
        f64* dst = rp.fb + (py * rp.W + px) * ipp;
        f64 R, G, B, A = 0;
        if (rp.pendColor) {
            R = G = B = A = rp.pendColorValue;
        } else {
            R = dst[0]; G = dst[1]; B = dst[2];
            if (ipp == 4) A = dst[3];
        }
        const u64 kv = key[p];
        const u32 id1 = (u32)kv;
        if (id1) {
            const i64 t = (i64)id1 - 1;
            f64 sx[3], sy[3];
            tri_screen(rp.src, rp.m, t, sx, sy);
            const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
            const f64 inv = 1.0 / (e1x * e2y - e2x * e1y);
            f64 cr, cg, cb, ca;
            if (GOURAUD) {
                const f64 dx = (f64)px - sx[0], dy = (f64)py - sy[0];
                const f64 w1 = (dx * e2y - e2x * dy) * inv;
                const f64 w2 = (e1x * dy - dx * e1y) * inv;
                const f64* c = rp.src.rgba + t * 12;
                cr = c[0] + (c[4] - c[0]) * w1 + (c[8] - c[0]) * w2;
                cg = c[1] + (c[5] - c[1]) * w1 + (c[9] - c[1]) * w2;
                cb = c[2] + (c[6] - c[2]) * w1 + (c[10] - c[2]) * w2;
                ca = c[3] + (c[7] - c[3]) * w1 + (c[11] - c[3]) * w2;
            } else {
                const f64* c = rp.src.rgba + t * 4;
                cr = c[0]; cg = c[1]; cb = c[2]; ca = c[3];
            }
            // ApplyPixel (cpp:529-547); A == 1 for every batch routed here
            cr *= ct0; cg *= ct1; cb *= ct2; ca *= ct3;
            if (ca != 1) {
                cr = R * (1 - ca) + cr * ca;
                cg = G * (1 - ca) + cg * ca;
                cb = B * (1 - ca) + cb * ca;
            }
            R = cr; G = cg; B = cb; A = ca;
        }
        dst[0] = R; dst[1] = G; dst[2] = B;
        if (ipp == 4) dst[3] = A;
        if (ZMODE == 1) rp.depth[py * rp.W + px] = (u32)(kv >> 32);
        else if (ZMODE == 2 && rp.pendDepth) rp.depth[py * rp.W + px] = zin[p];
    }
    if (COUNT && tid == 0) atomicAdd(rp.fragCounter, fragTotal);
}

template <int Z, bool G, bool C>
void launch_free(const RasterParams& rp, int ntiles, hipStream_t s) {
    hipLaunchKernelGGL((k_tile_raster_free<Z, G, C>), dim3(ntiles), dim3(WG), 0, s, rp);
}

template <bool C>
void launch_free_c(const RasterParams& rp, int zmode, bool g, int ntiles, hipStream_t s) {
    if (zmode == 1) { if (g) launch_free<1, true, C>(rp, ntiles, s); else launch_free<1, false, C>(rp, ntiles, s); }
    else if (zmode == 2) { if (g) launch_free<2, true, C>(rp, ntiles, s); else launch_free<2, false, C>(rp, ntiles, s); }
    else { if (g) launch_free<0, true, C>(rp, ntiles, s); else launch_free<0, false, C>(rp, ntiles, s); }
}

template <bool G, bool D, bool C>
void launch_raster(const RasterParams& rp, int ntiles, hipStream_t s) {
    hipLaunchKernelGGL((k_tile_raster<G, D, C>), dim3(ntiles), dim3(WG), 0, s, rp);
}

template <bool C>
void launch_raster_c(const RasterParams& rp, bool g, bool d, int ntiles, hipStream_t s) {
    if (g && d) launch_raster<true, true, C>(rp, ntiles, s);
    else if (g) launch_raster<true, false, C>(rp, ntiles, s);
    else if (d) launch_raster<false, true, C>(rp, ntiles, s);
    else launch_raster<false, false, C>(rp, ntiles, s);
}

// Grows a set of same-capacity device arrays to hold `need` elements each.
template <typename T, size_t K>
static bool grow_set(T* (&ptrs)[K], size_t* cap, size_t need) {
    if (*cap >= need && ptrs[0]) return true;
    size_t n = std::max(need, *cap * 3 / 2);
    for (size_t k = 0; k < K; ++k) {
        if (ptrs[k]) NR_CHECK(hipFree(ptrs[k]));
        ptrs[k] = nullptr;
    }
    for (size_t k = 0; k < K; ++k)
        if (hipMalloc((void**)&ptrs[k], n * sizeof(T)) != hipSuccess) {
            nr_set_error_msg("triangle scratch: hipMalloc failed");
            *cap = 0;
            return false;
        }
    *cap = n;
    return true;
}

static bool grow_temp(TriScratch& sc, size_t need) {
    if (need <= sc.temp_bytes && sc.temp) return true;
    if (sc.temp) NR_CHECK(hipFree(sc.temp));
    if (hipMalloc(&sc.temp, need) != hipSuccess) {
        nr_set_error_msg("triangle scratch: hipMalloc failed");
        sc.temp = nullptr; sc.temp_bytes = 0;
        return false;
    }
    sc.temp_bytes = need;
    return true;
}

// Opacity of a batch: every vertex alpha == 1 (then, with colourTransform[3]
// == 1, every fragment overwrites and the order-free raster applies).
enum Opacity { OPQ_UNKNOWN = 0, OPQ_OPAQUE, OPQ_BLENDED };

static Opacity host_opacity(const f64* rgba, i64 n, bool gouraud) {
    const i64 stride = gouraud ? 12 : 4;
    for (i64 t = 0; t < n; ++t)
        for (int v = 0; v < (gouraud ? 3 : 1); ++v)
            if (rgba[t * stride + v * 4 + 3] != 1) return OPQ_BLENDED;
    return OPQ_OPAQUE;
}

// Bins + rasterises one batch (all triangles of one draw call).
static void draw_batch(RenderContext* ctx, const TriSrc& src, Opacity opq) {
    if (src.n <= 0 || ctx->width <= 0 || ctx->height <= 0) return;
    hipStream_t s = ctx->stream;
    TriScratch& sc = ctx->tri;
    const int tiles_x = (int)((ctx->width + TW - 1) / TW);
    const int tiles_y = (int)((ctx->height + TH - 1) / TH);
    const int ntiles = tiles_x * tiles_y;
    const bool depth = ctx->depthTest;
    if (depth) nr_ensure_depth(ctx);

    BinParams bp;
    bp.src = src;
    for (int k = 0; k < 6; ++k) bp.m[k] = ctx->m[k];
    bp.W = ctx->width; bp.H = ctx->height; bp.tiles_x = tiles_x;

    u64* tri_bufs[2] = {sc.cnt, sc.off};
    if (!grow_set(tri_bufs, &sc.tri_cap, (size_t)src.n)) return;
    sc.cnt = tri_bufs[0]; sc.off = tri_bufs[1];
    u32* tile_bufs[2] = {sc.tile_start, sc.tile_end};
    if (!grow_set(tile_bufs, &sc.tile_cap, (size_t)ntiles)) return;
    sc.tile_start = tile_bufs[0]; sc.tile_end = tile_bufs[1];
    if (!sc.h_total) NR_CHECK(hipHostMalloc((void**)&sc.h_total, 4 * sizeof(u64)));
    if (!sc.d_flag) NR_CHECK(hipMalloc(&sc.d_flag, sizeof(u32)));
    u32* nonopaque = nullptr;
    if (opq == OPQ_UNKNOWN && ctx->ct[3] == 1) {
        NR_CHECK(hipMemsetAsync(sc.d_flag, 0, sizeof(u32), s));
        nonopaque = sc.d_flag;
    }

    const int g1 = (int)((src.n + 255) / 256);
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_TRI_COUNT, &e0, &e1);
    hipLaunchKernelGGL(k_tri_count, dim3(g1), dim3(256), 0, s, bp, sc.cnt, nonopaque);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TRI_COUNT, e0, e1);

    size_t need = 0;
    NR_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, sc.cnt, sc.off, (int)src.n, s));
    if (!grow_temp(sc, need)) return;
    nr_timing_begin(ctx, NRK_TRI_SCAN, &e0, &e1);
    NR_CHECK(hipcub::DeviceScan::ExclusiveSum(sc.temp, need, sc.cnt, sc.off, (int)src.n, s));
    nr_timing_end(ctx, NRK_TRI_SCAN, e0, e1);

    // total pair count: the one host sync of the pipeline (sizes the sort)
    NR_CHECK(hipMemcpyAsync(&sc.h_total[0], sc.off + (src.n - 1), sizeof(u64), hipMemcpyDeviceToHost, s));
    NR_CHECK(hipMemcpyAsync(&sc.h_total[1], sc.cnt + (src.n - 1), sizeof(u64), hipMemcpyDeviceToHost, s));
    if (nonopaque) {
        sc.h_total[3] = 0;
        NR_CHECK(hipMemcpyAsync(&sc.h_total[3], nonopaque, sizeof(u32), hipMemcpyDeviceToHost, s));
    }
    NR_CHECK(hipStreamSynchronize(s));
    const u64 P = sc.h_total[0] + sc.h_total[1];
    if (nonopaque) opq = (sc.h_total[3] & 0xFFFFFFFFull) ? OPQ_BLENDED : OPQ_OPAQUE;

    if (P > (1ull << 31) && src.n > 1) {
        // too many pairs for one pass: split the batch; submission order kept
        TriSrc a = src, b = src;
        a.n = src.n / 2;
        b.n = src.n - a.n;
        b.xy = src.xy + a.n * 6;
        b.z = src.z ? src.z + a.n * 3 : nullptr;
        b.rgba = src.rgba + a.n * (src.gouraud ? 12 : 4);
        draw_batch(ctx, a, opq);
        draw_batch(ctx, b, opq);
        return;
    }

    NR_CHECK(hipMemsetAsync(sc.tile_start, 0, (size_t)ntiles * sizeof(u32), s));
    NR_CHECK(hipMemsetAsync(sc.tile_end, 0, (size_t)ntiles * sizeof(u32), s));

    const u32* list = sc.tile_start;   // never dereferenced when every list is empty
    if (P > 0) {
        u32* pair_bufs[4] = {sc.keys[0], sc.keys[1], sc.vals[0], sc.vals[1]};
        if (!grow_set(pair_bufs, &sc.pair_cap, (size_t)P)) return;
        sc.keys[0] = pair_bufs[0]; sc.keys[1] = pair_bufs[1]; sc.vals[0] = pair_bufs[2]; sc.vals[1] = pair_bufs[3];

        nr_timing_begin(ctx, NRK_TRI_EMIT, &e0, &e1);
        hipLaunchKernelGGL(k_tri_emit, dim3(g1), dim3(256), 0, s, bp, sc.off, sc.keys[0], sc.vals[0]);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_TRI_EMIT, e0, e1);

        int bits = 1;
        while ((1 << bits) < ntiles) ++bits;
        size_t sneed = 0;
        NR_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sneed, sc.keys[0], sc.keys[1], sc.vals[0], sc.vals[1],
                                                    (int)P, 0, bits, s));
        if (!grow_temp(sc, sneed)) return;
        nr_timing_begin(ctx, NRK_TRI_SORT, &e0, &e1);
        NR_CHECK(hipcub::DeviceRadixSort::SortPairs(sc.temp, sneed, sc.keys[0], sc.keys[1], sc.vals[0], sc.vals[1],
                                                    (int)P, 0, bits, s));
        nr_timing_end(ctx, NRK_TRI_SORT, e0, e1);

        nr_timing_begin(ctx, NRK_TILE_RANGES, &e0, &e1);
        hipLaunchKernelGGL(k_tile_ranges, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, sc.keys[1], (u32)P,
                           sc.tile_start, sc.tile_end);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_TILE_RANGES, e0, e1);
        list = sc.vals[1];
    }

    RasterParams rp;
    rp.src = src;
    for (int k = 0; k < 6; ++k) rp.m[k] = ctx->m[k];
    for (int k = 0; k < 4; ++k) rp.ct[k] = ctx->ct[k];
    rp.fb = ctx->buffer;
    rp.depth = ctx->depth;
    rp.W = ctx->width; rp.H = ctx->height;
    rp.ipp = ctx->enableAlpha ? 4 : 3;
    rp.tiles_x = tiles_x;
    rp.depthTest = depth;
    rp.depthWrite = ctx->depthWrite;
    rp.pendColor = ctx->pendColor;
    rp.pendColorValue = ctx->pendColorValue;
    rp.pendDepth = depth && ctx->pendDepth;
    rp.pendDepthValue = ctx->pendDepthValue;
    rp.list = list;
    rp.tstart = sc.tile_start;
    rp.tend = sc.tile_end;
    rp.fragCounter = nullptr;
    if (ctx->countFragments) {
        if (!sc.d_frag) NR_CHECK(hipMalloc(&sc.d_frag, sizeof(u64)));
        NR_CHECK(hipMemsetAsync(sc.d_frag, 0, sizeof(u64), s));
        rp.fragCounter = sc.d_frag;
    }

    // every fragment overwrites -> order-free visibility + deferred shading
    const bool orderFree = opq == OPQ_OPAQUE && ctx->ct[3] == 1 && ctx->forceOrdered == 0;
    const int zmode = depth ? (ctx->depthWrite ? 1 : 2) : 0;
    ctx->lastPath = orderFree ? 1 : 2;
    nr_timing_begin(ctx, NRK_TILE_RASTER, &e0, &e1);
    if (orderFree) {
        if (rp.fragCounter) launch_free_c<true>(rp, zmode, src.gouraud != 0, ntiles, s);
        else launch_free_c<false>(rp, zmode, src.gouraud != 0, ntiles, s);
    } else {
        if (rp.fragCounter) launch_raster_c<true>(rp, src.gouraud != 0, depth, ntiles, s);
        else launch_raster_c<false>(rp, src.gouraud != 0, depth, ntiles, s);
    }
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TILE_RASTER, e0, e1);

    if (rp.fragCounter) {
        NR_CHECK(hipMemcpyAsync(&sc.h_total[2], sc.d_frag, sizeof(u64), hipMemcpyDeviceToHost, s));
        NR_CHECK(hipStreamSynchronize(s));
        ctx->fragTotal += sc.h_total[2];
    }

    // the raster consumed the pending clears
    ctx->pendColor = false;
    if (depth) ctx->pendDepth = false;
}

}  // namespace

extern "C" {

// New (no reference counterpart): depth-test LESS on/off, depth write on/off.
void SetDepthState(RenderContext* ctx, bool test, bool write) {
    ctx->depthTest = test;
    ctx->depthWrite = write;
}

// New: clear the u32 depth buffer (deferred; consumed on chip by the raster).
void ClearDepth(RenderContext* ctx, u32 value) {
    ctx->pendDepth = true;
    ctx->pendDepthValue = value;
}

// New: copy the W*H u32 depth buffer to the host.
void GetDepthBuffer(RenderContext* ctx, u32* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_ensure_depth(ctx);
    nr_materialize_depth(ctx);
    NR_CHECK(hipMemcpyAsync(out, ctx->depth, (size_t)(ctx->width * ctx->height) * sizeof(u32), hipMemcpyDeviceToHost,
                            ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
}

// New: triangles from device-resident arrays (xy n*6, z n*3 or NULL,
// rgba n*4 flat / n*12 Gouraud), in the context's transform.
void DrawTrianglesDevice(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (n <= 0) return;
    if (!ctx->depthTest) nr_materialize_depth(ctx);
    TriSrc src{xy, z, rgba, gouraud ? 1 : 0, n};
    draw_batch(ctx, src, OPQ_UNKNOWN);
}

static void draw_known(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud,
                       Opacity opq) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (n <= 0) return;
    if (!ctx->depthTest) nr_materialize_depth(ctx);
    TriSrc src{xy, z, rgba, gouraud ? 1 : 0, n};
    draw_batch(ctx, src, opq);
}

// New: triangles from host arrays (copied to HBM first).
void DrawTriangles(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (n <= 0) return;
    const size_t ncol = gouraud ? 12 : 4;
    const size_t need = (size_t)n * (6 + 3 + ncol);
    f64* stage_buf[1] = {ctx->tri.stage};
    if (!grow_set(stage_buf, &ctx->tri.stage_cap, need)) return;
    ctx->tri.stage = stage_buf[0];
    f64* dxy = ctx->tri.stage;
    f64* dz = dxy + (size_t)n * 6;
    f64* dc = dz + (size_t)n * 3;
    NR_CHECK(hipMemcpyAsync(dxy, xy, (size_t)n * 6 * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    if (z) NR_CHECK(hipMemcpyAsync(dz, z, (size_t)n * 3 * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipMemcpyAsync(dc, rgba, (size_t)n * ncol * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));   // caller may reuse its arrays on return
    draw_known(ctx, dxy, z ? dz : nullptr, dc, n, gouraud, host_opacity(rgba, n, gouraud));
}

// New: a device-resident triangle soup (the H2D point; drawn many times).
TriangleBuffer* CreateTriangleBuffer(i64 n, const f64* xy, const f64* z, const f64* rgba, bool gouraud) {
    TriangleBuffer* tb = new TriangleBuffer();
    tb->n = n;
    tb->gouraud = gouraud;
    tb->opaque = n > 0 && host_opacity(rgba, n, gouraud) == OPQ_OPAQUE;
    NR_CHECK(hipGetDevice(&tb->device));
    hipStream_t s = nr_stream_for(tb->device);
    const size_t ncol = gouraud ? 12 : 4;
    if (n > 0) {
        NR_CHECK(hipMalloc(&tb->xy, (size_t)n * 6 * sizeof(f64)));
        NR_CHECK(hipMalloc(&tb->rgba, (size_t)n * ncol * sizeof(f64)));
        NR_CHECK(hipMemcpyAsync(tb->xy, xy, (size_t)n * 6 * sizeof(f64), hipMemcpyHostToDevice, s));
        NR_CHECK(hipMemcpyAsync(tb->rgba, rgba, (size_t)n * ncol * sizeof(f64), hipMemcpyHostToDevice, s));
        if (z) {
            NR_CHECK(hipMalloc(&tb->z, (size_t)n * 3 * sizeof(f64)));
            NR_CHECK(hipMemcpyAsync(tb->z, z, (size_t)n * 3 * sizeof(f64), hipMemcpyHostToDevice, s));
        }
        NR_CHECK(hipStreamSynchronize(s));
    }
    return tb;
}

void DestroyTriangleBuffer(TriangleBuffer* tb) {
    if (!tb) return;
    NR_CHECK(hipSetDevice(tb->device));
    NR_CHECK(hipStreamSynchronize(nr_stream_for(tb->device)));
    if (tb->xy) NR_CHECK(hipFree(tb->xy));
    if (tb->z) NR_CHECK(hipFree(tb->z));
    if (tb->rgba) NR_CHECK(hipFree(tb->rgba));
    delete tb;
}

i64 GetTriangleBufferCount(TriangleBuffer* tb) { return tb->n; }

// New: count covered on-screen pixel x triangle pairs (the "shaded+Z-tested
// fragments" work count of the Mpixels/s metric).  Counting uses a separate
// kernel variant and syncs per draw: enable it outside timed regions.
void SetFragmentCounting(RenderContext* ctx, bool on) {
    ctx->countFragments = on;
    ctx->fragTotal = 0;
}
i64 GetFragmentCount(RenderContext* ctx) { return (i64)ctx->fragTotal; }

void DrawTriangleBuffer(RenderContext* ctx, TriangleBuffer* tb) {
    draw_known(ctx, tb->xy, tb->z, tb->rgba, tb->n, tb->gouraud, tb->opaque ? OPQ_OPAQUE : OPQ_BLENDED);
}

// New: which raster the last batch took (1 = order-free, 2 = ordered).
i64 GetLastRasterPath(RenderContext* ctx) { return ctx->lastPath; }

// New (testing / A-B measurement): force the ordered raster for every batch.
void SetForceOrderedRaster(RenderContext* ctx, bool on) { ctx->forceOrdered = on ? 1 : 0; }

}  // extern "C"
