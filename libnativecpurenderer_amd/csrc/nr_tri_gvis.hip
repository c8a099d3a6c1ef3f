// nr_tri_gvis.hip — whole-frame visibility buffer for opaque batches of small
// triangles (the C3 / 1M-triangle meshes): the order-free path without
// binning.
//
// An opaque batch under Z LESS + write reduces, per pixel, to the minimum of
// the packed key (zq << 32) | (tri + 1) over the pixel's fragments, started
// from (z_init << 32) (nr_tri_free.hip's header).  k_vis reduces the keys of
// one screen tile at a time in LDS, which needs the (tile, triangle) lists of
// a binning pass.  When the triangles are small (a few pixels each, as on a
// tessellated mesh), a thread per triangle walks its own rows and pixels
// with little divergence, so the reduction can instead go straight to a key
// buffer the size of the frame with global 64-bit atomic minimums
// (fire-and-forget: no value returned):
//
//   k_gvis_raster   thread = triangle: screen vertices, exact row spans (the
//                   f32 fast path of k_vis with its exact fallback), per
//                   covered pixel the fragment depth -> atomic min of its key
//   k_gvis_resolve  thread = 4 pixels of a row: winner -> shading record
//                   (reused while consecutive pixels share their winner) ->
//                   colour -> ApplyPixel -> framebuffer, depth and frame
//                   output written once (nr_tri_shade.h, as k_vis's shading);
//                   the keys of the pixels that had a winner are put back to
//                   the initial key the next batch will most likely need
//
// Two launches per batch, no lists, no capacity to validate, no host wait.
// Keys of pixels outside the owned tile rows of a sharded frame are never
// touched.  The key buffer's state (every owned key == init << 32 for one
// value `init`) is tracked on the host: a batch that starts from another
// state first runs k_gvis_init (keys from the pending depth clear, or from
// the depth buffer).
#include "nr_tri.h"
#include "nr_tri_shade.h"

#include <algorithm>
#include <cstdlib>

namespace nrtri {
namespace {

constexpr int GV_T = 256;    // raster: triangles per workgroup
constexpr int GV_Q = 4;      // resolve: pixels per thread
constexpr int GV_RT = 256;   // resolve: threads per workgroup (1024 pixels of one row)

// Pixel row of owned row ordinal `oy` (bands of TH rows; unsharded: oy).
__device__ __forceinline__ i64 owned_pixel_row(const BinParams& bp, int oy) {
    if (bp.period == 1) return oy;
    return (i64)owned_row_of(bp, oy / TH) * TH + (oy % TH);
}

// Every owned key = (pendDepth ? v : depth) << 32.
__global__ __launch_bounds__(GV_RT) void k_gvis_init(const BinParams bp, u64* __restrict__ gkey,
                                                     const u32* __restrict__ depth, int pend, u32 v) {
    const i64 y = owned_pixel_row(bp, (int)blockIdx.y);
    if (y >= bp.H) return;
    for (i64 x = (i64)blockIdx.x * GV_RT + threadIdx.x; x < bp.W; x += (i64)gridDim.x * GV_RT) {
        const i64 p = y * bp.W + x;
        gkey[p] = (u64)(pend ? v : depth[p]) << 32;
    }
}

#ifndef NR_GV_EXP
#define NR_GV_EXP 0   // A/B: 1 plain store instead of the atomic (timing only: wrong results), 2 load-then-atomic
#endif
__device__ __forceinline__ void gv_min(u64* a, u64 k) {
    if (NR_GV_EXP == 1) {
        *a = k;
    } else if (NR_GV_EXP == 2) {
        if (k < __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            __hip_atomic_fetch_min(a, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_fetch_min(a, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One thread per triangle.  Rows [ceil(ymin), ceil(ymax)) of the screen that
// the rank owns; per row the exact span [xs, xe) of the even-odd rule
// (relative to x0 = floor(xmin) - 2, clamped to the screen: a conservative
// left edge, as tri_tiles'), per pixel frag_depth -> atomic min.
template <bool COUNT>
__global__ __launch_bounds__(GV_T) void k_gvis_raster(const FrameParams fp, u64* __restrict__ gkey) {
    const i64 t = (i64)blockIdx.x * GV_T + threadIdx.x;
    unsigned long long frags = 0;
    if (t < fp.src.n) {
        f64 pxy[6];
        load_tri_xy(fp.src.xy, t, pxy);
        f64 zz0 = 0, dz1 = 0, dz2 = 0;
        if (fp.src.z) {
            const f64* qz = fp.src.z + t * 3;
            const f64 z0 = qz[0], z1 = qz[1], z2 = qz[2];
            zz0 = z0; dz1 = z1 - z0; dz2 = z2 - z0;
        }
        f64 sx[3], sy[3];
#pragma unroll
        for (int v = 0; v < 3; ++v) nr_xform(fp.m, pxy[2 * v], pxy[2 * v + 1], sx[v], sy[v]);
        const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
        const f64 den = e1x * e2y - e2x * e1y;
        bool live = tri_finite(sx, sy) && den != 0;
        const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
        const f64 xmn = fmin(fmin(sx[0], sx[1]), sx[2]), xmx = fmax(fmax(sx[0], sx[1]), sx[2]);
        const int r0 = live ? (int)clampd(ceil(ymn), 0.0, (f64)fp.H) : 0;
        const int r1 = live ? (int)clampd(ceil(ymx), 0.0, (f64)fp.H) : 0;
        const bool huge = fabs(xmn) > 1e7 || fabs(xmx) > 1e7 || fabs(ymn) > 1e7 || fabs(ymx) > 1e7;
        f64 x0 = 0;
        if (live && !huge) {
            if (ceil(xmx) + 2 < 0 || floor(xmn) - 2 > (f64)(fp.W - 1)) live = false;
            x0 = clampd(floor(xmn) - 2, 0.0, (f64)fp.W);
        }
        if (live && r0 < r1 && fp.period > 1) {   // a sharded frame: any owned tile row in [r0, r1)?
            bool any = false;
            for (int ty = r0 / TH; ty <= (r1 - 1) / TH && !any; ++ty) any = owned_row(ty, fp.period, fp.mask);
            live = any;
        }
        if (live && r0 < r1) {
            const f64 wlim = (f64)fp.W - x0;
            f64 sl[3];
            edge_slopes(sx, sy, sl);
            const f64 inv = 1.0 / den;
            const u64 id1 = (u64)t + 1;
            const Span32 S32 = span32_setup(sx, sy, sl, x0, (f64)r0);
            const i64 ix0 = (i64)x0;
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
            for (int r = r0; r < r1; ++r) {
                if (!owned_row(r / TH, fp.period, fp.mask)) continue;
                const f64 y = (f64)r;
                int xs, xe;
                if (!row_span32(S32, r - r0, y, (float)wlim, xs, xe)) row_span_in(sx, sy, y, x0, wlim, xs, xe);
                if (COUNT && xe > xs) frags += (unsigned long long)(xe - xs);
                const f64 dy = y - sy[0];
                u64* row = gkey + (i64)r * fp.W + ix0;
                f64 X = x0 + (f64)xs;
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
                for (int lx = xs; lx < xe; lx += 2, X += 2.0) {
                    const u32 za = frag_depth(X, dy, sx[0], e1x, e1y, e2x, e2y, inv, zz0, dz1, dz2);
                    gv_min(row + lx, ((u64)za << 32) | id1);
                    if (lx + 1 < xe) {
                        const u32 zb = frag_depth(X + 1.0, dy, sx[0], e1x, e1y, e2x, e2y, inv, zz0, dz1, dz2);
                        gv_min(row + lx + 1, ((u64)zb << 32) | id1);
                    }
                }
            }
        }
    }
    if (COUNT) {
        __shared__ unsigned long long sf;
        if (threadIdx.x == 0) sf = 0;
        __syncthreads();
        if (frags) atomicAdd(&sf, frags);
        __syncthreads();
        if (threadIdx.x == 0 && sf) atomicAdd(fp.fragCounter, sf);
    }
}

// One thread per GV_Q consecutive pixels of an owned row (grid.y = owned row
// ordinal).  Shading as k_vis's (shade_tile): store_depth, the winner's
// record -> record_colour -> apply_winner -> store_colour; a pixel no
// fragment won gets the pending clears.  `reset`: the keys of the pixels
// that had a winner go back to `next` (the other keys still hold it).
template <bool GOURAUD>
__global__ __launch_bounds__(GV_RT) void k_gvis_resolve(const FrameParams fp, const BinParams bp,
                                                        u64* __restrict__ gkey, int reset, u64 next) {
    const i64 y = owned_pixel_row(bp, (int)blockIdx.y);
    if (y >= fp.H) return;
    const i64 x = ((i64)blockIdx.x * GV_RT + threadIdx.x) * GV_Q;
    if (x >= fp.W) return;
    const i64 p0 = y * fp.W + x;
    const bool full = x + GV_Q <= fp.W;
    u64 kq[GV_Q];
    if (full && !(p0 & 1)) {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(gkey + p0);
        const ulonglong2 a = q[0], b = q[1];
        kq[0] = a.x; kq[1] = a.y; kq[2] = b.x; kq[3] = b.y;
    } else {
#pragma unroll
        for (int j = 0; j < GV_Q; ++j) kq[j] = x + j < fp.W ? gkey[p0 + j] : 0ull;
    }
    constexpr int REC = RecLen<GOURAUD>::REC;
    f64 rec[REC];
    u32 have = 0;   // winner whose record is in rec (0: none)
    u32 any = 0;
#pragma unroll
    for (int j = 0; j < GV_Q; ++j) {
        if (x + j >= fp.W) break;
        const i64 p = p0 + j, px = x + j;
        const u64 kv = kq[j];
        const u32 id = (u32)kv;
        any |= id;
        store_depth<1>(fp, p, kv);
        if (!id) {
            if (fp.pendColor) {
                const f64 v = fp.pendColorValue;
                store_colour(fp, p, px, y, v, v, v, v);
            }
            continue;
        }
        NR_DEV_CHECK(id <= (u32)fp.src.n, "gvis_resolve: pixel (%ld, %ld) winner %u of %ld triangles", (long)px,
                     (long)y, id, (long)fp.src.n);
        if (id != have) {
            make_record<GOURAUD>(fp, (i64)id - 1, rec);
            have = id;
        }
        f64 cr, cg, cb, ca;
        record_colour<GOURAUD>(rec, px, y, cr, cg, cb, ca);
        apply_winner(fp, p, cr, cg, cb, ca);
        store_colour(fp, p, px, y, cr, cg, cb, ca);
    }
    if (reset && any) {
        if (full && !(p0 & 1)) {
            ulonglong2* q = reinterpret_cast<ulonglong2*>(gkey + p0);
            q[0] = make_ulonglong2(next, next);
            q[1] = make_ulonglong2(next, next);
        } else {
#pragma unroll
            for (int j = 0; j < GV_Q; ++j)
                if (x + j < fp.W) gkey[p0 + j] = next;
        }
    }
}

// One thread per pixel of an owned row (consecutive lanes, consecutive
// pixels: the framebuffer rows are written as contiguous runs).
template <bool GOURAUD>
__global__ __launch_bounds__(GV_RT) void k_gvis_resolve1(const FrameParams fp, const BinParams bp,
                                                         u64* __restrict__ gkey, int reset, u64 next) {
    const i64 y = owned_pixel_row(bp, (int)blockIdx.y);
    if (y >= fp.H) return;
    const i64 x = (i64)blockIdx.x * GV_RT + threadIdx.x;
    if (x >= fp.W) return;
    const i64 p = y * fp.W + x;
    const u64 kv = gkey[p];
    const u32 id = (u32)kv;
    store_depth<1>(fp, p, kv);
    if (!id) {
        if (fp.pendColor) {
            const f64 v = fp.pendColorValue;
            store_colour(fp, p, x, y, v, v, v, v);
        }
        return;
    }
    NR_DEV_CHECK(id <= (u32)fp.src.n, "gvis_resolve: pixel (%ld, %ld) winner %u of %ld triangles", (long)x, (long)y, id,
                 (long)fp.src.n);
    f64 rec[RecLen<GOURAUD>::REC];
    make_record<GOURAUD>(fp, (i64)id - 1, rec);
    f64 cr, cg, cb, ca;
    record_colour<GOURAUD>(rec, x, y, cr, cg, cb, ca);
    apply_winner(fp, p, cr, cg, cb, ca);
    store_colour(fp, p, x, y, cr, cg, cb, ca);
    if (reset) gkey[p] = next;
}
#ifndef NR_GV_RES1
#define NR_GV_RES1 1
#endif

// NR_GVIS: -1 (unset) automatic, 0 never, 1 every eligible batch.
int gvis_env() {
    static const int v = [] {
        const char* e = getenv("NR_GVIS");
        return e ? atoi(e) : -1;
    }();
    return v;
}
// Automatic choice: batches of at least NR_GVIS_MIN_TRIS triangles whose mean
// screen area is at most NR_GVIS_AREA pixels.
f64 gvis_area() {
    static const f64 v = [] {
        const char* e = getenv("NR_GVIS_AREA");
        return e ? atof(e) : 48.0;
    }();
    return v;
}
i64 gvis_min_tris() {
    static const i64 v = [] {
        const char* e = getenv("NR_GVIS_MIN_TRIS");
        return e ? atol(e) : 65536;
    }();
    return v;
}

}  // namespace

bool gvis_wanted(const RenderContext* ctx, const TriSrc& src, f64 objMeanArea) {
    if (!(ctx->depthTest && ctx->depthWrite)) return false;   // LESS + write only (min of the packed keys)
    const int mode = ctx->tri.gvisMode ? ctx->tri.gvisMode : (gvis_env() < 0 ? 0 : (gvis_env() ? 1 : 2));
    if (mode == 1) return true;
    if (mode == 2) return false;
    // automatic: off -- measured slower than the tiled k_vis on every
    // configuration (the global 64-bit atomics run at ~36 G/s);
    // NR_GVIS_AUTO=1 turns the size rule below on
    static const bool autoOn = [] {
        const char* e = getenv("NR_GVIS_AUTO");
        return e && atoi(e) != 0;
    }();
    if (!autoOn) return false;
    if (src.n < gvis_min_tris() || !(objMeanArea >= 0)) return false;
    const f64 det = fabs(ctx->m[0] * ctx->m[3] - ctx->m[2] * ctx->m[1]);
    return objMeanArea * det <= gvis_area();
}

void draw_gvis(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp) {
    hipStream_t s = ctx->stream;
    TriScratch& sc = ctx->tri;
    const size_t npix = (size_t)(fp.W * fp.H);
    if (sc.gkey_cap < npix || !sc.gkey) {
        u64* kb[1] = {sc.gkey};
        if (!grow_set(kb, &sc.gkey_cap, std::max<size_t>(npix, 1))) return;
        sc.gkey = kb[0];
        sc.gkeyState = 0;
    }
    // the keys hold (gkeyInit << 32) for every owned pixel of this frame
    // geometry and ownership, or the batch initialises them first
    const u32 want = fp.pendDepth ? fp.pendDepthValue : 0u;
    const bool ready = sc.gkeyState == 1 && fp.pendDepth && sc.gkeyInit == want && sc.gkeyW == fp.W &&
                       sc.gkeyH == fp.H && sc.gkeyPeriod == fp.period && sc.gkeyMask == fp.mask;
    const unsigned orows = (unsigned)(bp.hrows * TH);
    hipEvent_t e0, e1;
    if (!ready) {
        nr_timing_begin(ctx, NRK_VIS_INIT, &e0, &e1);
        hipLaunchKernelGGL(k_gvis_init, dim3((unsigned)std::min<i64>((fp.W + GV_RT - 1) / GV_RT, 16), orows),
                           dim3(GV_RT), 0, s, bp, sc.gkey, (const u32*)fp.depth, fp.pendDepth, fp.pendDepthValue);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_VIS_INIT, e0, e1);
    }
    nr_timing_begin(ctx, NRK_GV_RASTER, &e0, &e1);
    const unsigned gr = (unsigned)((src.n + GV_T - 1) / GV_T);
    if (fp.fragCounter) hipLaunchKernelGGL(k_gvis_raster<true>, dim3(gr), dim3(GV_T), 0, s, fp, sc.gkey);
    else hipLaunchKernelGGL(k_gvis_raster<false>, dim3(gr), dim3(GV_T), 0, s, fp, sc.gkey);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_GV_RASTER, e0, e1);
    // a batch that started from a pending depth clear v puts its keys back to
    // v << 32 (the next frame's clear is most likely the same); otherwise the
    // keys are left as they are and the next batch initialises them
    const int reset = fp.pendDepth ? 1 : 0;
    const u64 next = (u64)want << 32;
    nr_timing_begin(ctx, NRK_GV_RESOLVE, &e0, &e1);
    if (NR_GV_RES1) {
        const dim3 rg((unsigned)((fp.W + GV_RT - 1) / GV_RT), orows);
        if (src.gouraud) hipLaunchKernelGGL(k_gvis_resolve1<true>, rg, dim3(GV_RT), 0, s, fp, bp, sc.gkey, reset, next);
        else hipLaunchKernelGGL(k_gvis_resolve1<false>, rg, dim3(GV_RT), 0, s, fp, bp, sc.gkey, reset, next);
    } else {
        const dim3 rg((unsigned)((fp.W + GV_RT * GV_Q - 1) / (GV_RT * GV_Q)), orows);
        if (src.gouraud) hipLaunchKernelGGL(k_gvis_resolve<true>, rg, dim3(GV_RT), 0, s, fp, bp, sc.gkey, reset, next);
        else hipLaunchKernelGGL(k_gvis_resolve<false>, rg, dim3(GV_RT), 0, s, fp, bp, sc.gkey, reset, next);
    }
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_GV_RESOLVE, e0, e1);
    sc.gkeyState = reset ? 1 : 0;
    sc.gkeyInit = want;
    sc.gkeyW = fp.W; sc.gkeyH = fp.H; sc.gkeyPeriod = fp.period; sc.gkeyMask = fp.mask;
}

}  // namespace nrtri
