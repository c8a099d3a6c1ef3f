// nr_tri_free.hip — visibility-buffer raster for opaque batches.
//
// When every fragment of a batch overwrites (every vertex alpha == 1 and
// colourTransform[3] == 1, so ApplyPixel's `a != 1` blend never runs) the
// sequential semantics reduce, per pixel, to an order-independent reduction:
//   Z LESS + write : winner = min over (zq, tri) with zq < z_init -> min of
//                    the packed key (zq << 32) | (tri + 1), init z_init << 32
//   Z LESS, no write: winner = last tri with zq < z_init            -> max id
//   no Z test       : winner = last covering tri                     -> max id
// Ties on zq resolve to the lower triangle index = the earlier submission,
// exactly as the sequential LESS test would.  So fragments are reduced in any
// order, with 64-bit LDS atomics, and only the winner is shaded (deferred).
//
//   1 k_free_count   tile histogram of (tile, triangle) pairs, aggregated in
//                    LDS per workgroup (one global atomic per touched tile)
//   2 k_free_plan    one workgroup: exclusive scans of the tile counts (list
//                    offsets) and of the slice counts (work items)
//   3 k_free_emit    per-tile lists (order inside a list is irrelevant here)
//   4 k_vis          one 256-thread workgroup per (tile, slice of <= 512
//                    triangles): exact row spans -> prefix sum -> fragment-
//                    parallel depth + LDS atomicMin on the tile's 2048 keys ->
//                    one coalesced store (or global atomicMin when a long list
//                    is split over several slices: the load-balancing step for
//                    mesh poles where thousands of tiny triangles meet)
//   5 k_resolve      one thread per pixel: winner -> barycentrics -> colour ->
//                    ApplyPixel -> framebuffer + depth written once; tiles
//                    with no triangle just receive a pending clear
#include "nr_tri.h"

namespace nrtri {
namespace {

constexpr int VWG = 256;     // k_vis workgroup
constexpr int FCH = 128;     // triangles staged per chunk in k_vis
constexpr u32 SLICE = 512;   // triangles per work item
constexpr int TPT = 4;       // triangles per thread in the binning kernels
constexpr int LDS_HIST_MAX = 16384;

template <bool LDSH>
__global__ __launch_bounds__(256) void k_free_count(const BinParams bp, u32* __restrict__ tile_cnt, int ntiles) {
    extern __shared__ u32 hist[];
    const int tid = threadIdx.x;
    if (LDSH) {
        for (int b = tid; b < ntiles; b += 256) hist[b] = 0;
        __syncthreads();
    }
    const i64 base = (i64)blockIdx.x * 256 * TPT;
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (t >= bp.src.n) break;
        f64 sx[3], sy[3];
        tri_screen(bp.src, bp.m, t, sx, sy);
        int tx0, tx1, ty0, ty1;
        if (!tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) continue;
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.nshards, bp.shard)) continue;
            for (int tx = tx0; tx <= tx1; ++tx) {
                const int bin = ty * bp.tiles_x + tx;
                if (LDSH) atomicAdd(&hist[bin], 1u);
                else atomicAdd(&tile_cnt[bin], 1u);
            }
        }
    }
    if (LDSH) {
        __syncthreads();
        for (int b = tid; b < ntiles; b += 256) {
            const u32 h = hist[b];
            if (h) atomicAdd(&tile_cnt[b], h);
        }
    }
}

// Single workgroup: off[i] = sum(cnt[<i]), soff[i] = sum(ceil(cnt[<i]/SLICE)),
// off[ntiles] = P, soff[ntiles] = number of work items; totals = {P, items,
// number of tiles split over more than one slice}.
// totals[3] = 1 when the pair list fits `cap`; every later kernel of the
// batch reads it and does nothing otherwise (the host then re-runs the batch
// with an exact allocation before anything else is enqueued, nr_settle).
// It also re-zeroes the tile counters for the next batch (after reading them)
// and the emit cursors, and mirrors the totals into pinned host memory, so a
// batch needs no memset and no copy command.
__global__ __launch_bounds__(1024) void k_free_plan(u32* __restrict__ cnt, int ntiles, u32* __restrict__ off,
                                                    u32* __restrict__ soff, u32* __restrict__ cur,
                                                    u32* __restrict__ totals, u32* __restrict__ host_totals, u32 cap) {
    __shared__ u32 sA[1024], sB[1024], sC[1024];
    const int tid = threadIdx.x;
    const int per = (ntiles + 1023) / 1024;
    const int b0 = tid * per, b1 = min(b0 + per, ntiles);
    u32 a = 0, b = 0, m = 0;
    for (int i = b0; i < b1; ++i) {
        const u32 c = cnt[i];
        a += c;
        b += (c + SLICE - 1) / SLICE;
        m += c > SLICE ? 1u : 0u;
    }
    sA[tid] = a; sB[tid] = b; sC[tid] = m;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const u32 va = tid >= d ? sA[tid - d] : 0u;
        const u32 vb = tid >= d ? sB[tid - d] : 0u;
        const u32 vc = tid >= d ? sC[tid - d] : 0u;
        __syncthreads();
        sA[tid] += va; sB[tid] += vb; sC[tid] += vc;
        __syncthreads();
    }
    u32 ea = sA[tid] - a, eb = sB[tid] - b;
    for (int i = b0; i < b1; ++i) {
        const u32 c = cnt[i];
        off[i] = ea;
        soff[i] = eb;
        ea += c;
        eb += (c + SLICE - 1) / SLICE;
        cnt[i] = 0;
        cur[i] = 0;
    }
    if (tid == 1023) {
        off[ntiles] = sA[1023];
        soff[ntiles] = sB[1023];
        const u32 t[4] = {sA[1023], sB[1023], sC[1023], sA[1023] <= cap ? 1u : 0u};
        for (int k = 0; k < 4; ++k) {
            totals[k] = t[k];
            __hip_atomic_store(&host_totals[k], t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <bool LDSH>
__global__ __launch_bounds__(256) void k_free_emit(const BinParams bp, const u32* __restrict__ off,
                                                   u32* __restrict__ cur, u32* __restrict__ list, int ntiles,
                                                   const u32* __restrict__ plan) {
    extern __shared__ u32 hist[];
    if (!plan[3]) return;
    const int tid = threadIdx.x;
    const i64 base = (i64)blockIdx.x * 256 * TPT;
    if (LDSH) {
        for (int b = tid; b < ntiles; b += 256) hist[b] = 0;
        __syncthreads();
        for (int k = 0; k < TPT; ++k) {
            const i64 t = base + k * 256 + tid;
            if (t >= bp.src.n) break;
            f64 sx[3], sy[3];
            tri_screen(bp.src, bp.m, t, sx, sy);
            int tx0, tx1, ty0, ty1;
            if (!tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) continue;
            for (int ty = ty0; ty <= ty1; ++ty)
                if (owned_row(ty, bp.nshards, bp.shard))
                    for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[ty * bp.tiles_x + tx], 1u);
        }
        __syncthreads();
        // reserve each touched tile's range once: hist[b] becomes the next slot
        for (int b = tid; b < ntiles; b += 256) {
            const u32 h = hist[b];
            if (h) hist[b] = off[b] + atomicAdd(&cur[b], h);
        }
        __syncthreads();
    }
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (t >= bp.src.n) break;
        f64 sx[3], sy[3];
        tri_screen(bp.src, bp.m, t, sx, sy);
        int tx0, tx1, ty0, ty1;
        if (!tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) continue;
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.nshards, bp.shard)) continue;
            for (int tx = tx0; tx <= tx1; ++tx) {
                const int bin = ty * bp.tiles_x + tx;
                const u32 slot = LDSH ? atomicAdd(&hist[bin], 1u) : off[bin] + atomicAdd(&cur[bin], 1u);
                list[slot] = (u32)t;
            }
        }
    }
}

// Neutral keys for tiles whose list is split over several slices (their
// slices merge with global atomics).
template <int ZMODE>
__global__ __launch_bounds__(256) void k_vis_init_multi(const FrameParams fp, const u32* __restrict__ off,
                                                        u64* __restrict__ vis, const u32* __restrict__ plan) {
    if (!plan[3]) return;
    const int tile = blockIdx.x;
    if (off[tile + 1] - off[tile] <= SLICE) return;
    const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
    const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
    for (int p = threadIdx.x; p < TW * TH; p += 256) {
        const i64 px = x0 + (p & (TW - 1)), py = y0 + p / TW;
        if (px < fp.W && py < fp.H) vis[py * fp.W + px] = ZMODE == 1 ? ~0ull : 0ull;
    }
}

enum { F_X0 = 0, F_Y0, F_X1, F_Y1, F_X2, F_Y2, F_INV, F_Z0, F_DZ1, F_DZ2, F_NSLOT };
constexpr int NW = VWG / 64;   // waves per k_vis workgroup

// Wave-synchronous ordering of this wave's own LDS traffic (a wave's LDS
// operations complete in order; this stops the compiler from reordering them).
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// One workgroup per work item (tile, slice of <= SLICE triangles).  The 4
// waves share only the tile's 2048 LDS keys; each wave independently walks
// 64-triangle chunks of the slice (chunk c goes to wave c % 4) with no
// workgroup barrier:
//   setup   one lane per triangle: screen vertices, 1/den, depths, the rows of
//           this tile it straddles (next chunk prefetched into registers)
//   scan    exclusive scan of the row counts with wave shuffles, then each
//           lane writes its triangle's lane index into a row->triangle map
//   rows    the chunk's (triangle, row) items over the 64 lanes: exact span
//           (row_span), then per pixel depth + LDS atomic on the packed key
template <int ZMODE, bool COUNT>   // ZMODE 0: no test, 1: LESS+write, 2: LESS no write
__global__ __launch_bounds__(VWG) void k_vis(const FrameParams fp, const u32* __restrict__ off,
                                             const u32* __restrict__ soff, const u32* __restrict__ list,
                                             u64* __restrict__ vis, const u32* __restrict__ plan) {
    constexpr bool DEPTH = ZMODE != 0;
    __shared__ u64 key[TH * TW];
    __shared__ u32 zin[ZMODE == 2 ? TH * TW : 1];
    __shared__ f64 S[NW][F_NSLOT][64];
    __shared__ iu8 MAP[NW][64 * TH];
    __shared__ iu8 RR0[NW][64];
    __shared__ unsigned short ROFF[NW][64];
    __shared__ u32 TT[NW][64];   // triangle id + 1 of each lane's triangle
    __shared__ int sTile;
    __shared__ unsigned long long sFrag;
    if (!plan[3]) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int ntiles = fp.tiles_x * fp.tiles_y;
    const u32 nitems = plan[1];
    unsigned long long myFrags = 0;
    if (COUNT && tid == 0) sFrag = 0;
    // grid-stride over the work items (the grid is sized from a capacity
    // bound, not from the item count, so no host sync is needed)
    for (u32 item = blockIdx.x; item < nitems; item += gridDim.x) {
        __syncthreads();
        if (tid == 0) {   // tile of this work item: last tile with soff[tile] <= item
            int lo = 0, hi = ntiles;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (soff[mid] <= item) lo = mid; else hi = mid;
            }
            sTile = lo;
        }
        __syncthreads();
        const int tile = sTile;
        const u32 t0 = off[tile], t1 = off[tile + 1];
        const u32 slice = item - soff[tile];
        const u32 ls = t0 + slice * SLICE;
        const u32 le = ls + SLICE < t1 ? ls + SLICE : t1;
        const bool multi = t1 - t0 > SLICE;
        const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
        const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
        const int wlim = (int)(fp.W - x0 < TW ? fp.W - x0 : TW);
        const int hlim = (int)(fp.H - y0 < TH ? fp.H - y0 : TH);

        for (int p = tid; p < TH * TW; p += VWG) {
            const int lx = p & (TW - 1), ly = p / TW;
            u32 z0 = 0xFFFFFFFFu;
            if (DEPTH && lx < wlim && ly < hlim)
                z0 = fp.pendDepth ? fp.pendDepthValue : fp.depth[(y0 + ly) * fp.W + x0 + lx];
            key[p] = ZMODE == 1 ? ((u64)z0 << 32) : 0ull;
            if (ZMODE == 2) zin[p] = z0;
        }
        __syncthreads();

        // this wave's chunks: c = wave, wave + NW, ...
        const u32 nch = (le - ls + 63) / 64;
        u32 pt = 0;
        f64 pxy[6], pz[3] = {0, 0, 0};
        auto prefetch = [&](u32 c) {
            const u32 b = ls + c * 64 + lane;
            if (c < nch && b < le) {
                pt = list[b];
                const f64* q = fp.src.xy + (i64)pt * 6;
#pragma unroll
                for (int v = 0; v < 6; ++v) pxy[v] = q[v];
                if (DEPTH && fp.src.z) {
                    const f64* qz = fp.src.z + (i64)pt * 3;
                    pz[0] = qz[0]; pz[1] = qz[1]; pz[2] = qz[2];
                }
            }
        };
        prefetch(wave);
        for (u32 c = wave; c < nch; c += NW) {
            const u32 base = ls + c * 64;
            const int cnt = (le - base) < 64u ? (int)(le - base) : 64;
            // ---- setup (lane = triangle)
            const u32 t = pt;
            int r0 = 0, nr = 0;
            if (lane < cnt) {
                f64 sx[3], sy[3];
#pragma unroll
                for (int v = 0; v < 3; ++v) nr_xform(fp.m, pxy[2 * v], pxy[2 * v + 1], sx[v], sy[v]);
                const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
                const f64 den = e1x * e2y - e2x * e1y;
                const bool ok = tri_finite(sx, sy) && den != 0;
                S[wave][F_X0][lane] = sx[0]; S[wave][F_Y0][lane] = sy[0];
                S[wave][F_X1][lane] = sx[1]; S[wave][F_Y1][lane] = sy[1];
                S[wave][F_X2][lane] = sx[2]; S[wave][F_Y2][lane] = sy[2];
                S[wave][F_INV][lane] = 1.0 / den;
                if (DEPTH) {
                    S[wave][F_Z0][lane] = pz[0]; S[wave][F_DZ1][lane] = pz[1] - pz[0];
                    S[wave][F_DZ2][lane] = pz[2] - pz[0];
                }
                if (ok) {
                    // rows with a straddling edge: ymin <= y < ymax (exact)
                    const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
                    r0 = (int)clampd(ceil(ymn) - (f64)y0, 0.0, (f64)hlim);
                    const int r1 = (int)clampd(ceil(ymx) - (f64)y0, 0.0, (f64)hlim);
                    nr = r1 > r0 ? r1 - r0 : 0;
                }
            }
            prefetch(c + NW);
            // ---- scan of the row counts, row -> triangle map
            int incl = nr;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int o = __shfl_up(incl, d, 64);
                if (lane >= d) incl += o;
            }
            const int ex = incl - nr;
            const int R = __shfl(incl, 63, 64);
            TT[wave][lane] = t + 1;
            RR0[wave][lane] = (iu8)r0;
            ROFF[wave][lane] = (unsigned short)ex;
            for (int j = 0; j < nr; ++j) MAP[wave][ex + j] = (iu8)lane;
            wave_lds_fence();
            // ---- (triangle, row) items over the lanes
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
            for (int it = lane; it < R; it += 64) {
                const int k = MAP[wave][it];
                const int r = RR0[wave][k] + (it - ROFF[wave][k]);
                const f64 sx[3] = {S[wave][F_X0][k], S[wave][F_X1][k], S[wave][F_X2][k]};
                const f64 sy[3] = {S[wave][F_Y0][k], S[wave][F_Y1][k], S[wave][F_Y2][k]};
                const f64 y = (f64)(y0 + r);
                int xs, xe;
                row_span(sx, sy, y, (f64)x0, (f64)wlim, xs, xe);
                if (COUNT) myFrags += (unsigned long long)(xe - xs);
                if (xs >= xe) continue;
                const u64 id1 = TT[wave][k];
                if (ZMODE == 0) {
#pragma clang loop vectorize(disable) interleave(disable)
                    for (int lx = xs; lx < xe; ++lx) atomicMax(&key[r * TW + lx], id1);
                    continue;
                }
                const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
                const f64 inv = S[wave][F_INV][k];
                const f64 zz0 = S[wave][F_Z0][k], dz1 = S[wave][F_DZ1][k], dz2 = S[wave][F_DZ2][k];
                const f64 dy = y - sy[0];   // (f64)j - pts[0][1], as the oracle
#pragma clang loop vectorize(disable) interleave(disable)
                for (int lx = xs; lx < xe; ++lx) {
                    const f64 dx = (f64)(x0 + lx) - sx[0];
                    const f64 w1 = (dx * e2y - e2x * dy) * inv;
                    const f64 w2 = (e1x * dy - dx * e1y) * inv;
                    const f64 zz = zz0 + dz1 * w1 + dz2 * w2;
                    const u32 zq = nr_quantize_depth(zz);
                    const int p = r * TW + lx;
                    if (ZMODE == 1) atomicMin(&key[p], ((u64)zq << 32) | id1);
                    else if (zq < zin[p]) atomicMax(&key[p], id1);
                }
            }
            wave_lds_fence();   // the next chunk overwrites this wave's staging
        }
        __syncthreads();
        for (int p = tid; p < TH * TW; p += VWG) {
            const int lx = p & (TW - 1), ly = p / TW;
            if (lx >= wlim || ly >= hlim) continue;
            u64* g = vis + (y0 + ly) * fp.W + x0 + lx;
            if (!multi) *g = key[p];
            else if (ZMODE == 1) atomicMin(g, key[p]);
            else atomicMax(g, key[p]);
        }
    }   // work items
    if (COUNT) {
        __syncthreads();
        atomicAdd(&sFrag, myFrags);
        __syncthreads();
        if (tid == 0) atomicAdd(fp.fragCounter, sFrag);
    }
}

// One thread per pixel (2-D grid: x blocks of 256, one row per blockIdx.y).
template <int ZMODE, bool GOURAUD>
__global__ __launch_bounds__(256) void k_resolve(const FrameParams fp, const u32* __restrict__ off,
                                                 const u64* __restrict__ vis, const u32* __restrict__ plan) {
    if (!plan[3]) return;
    const i64 px = (i64)blockIdx.x * 256 + threadIdx.x;
    // blockIdx.y enumerates the rows of the owned tile rows only
    const i64 py = ((i64)(blockIdx.y / TH) * fp.nshards + fp.shard) * TH + blockIdx.y % TH;
    if (px >= fp.W || py >= fp.H) return;
    const int tile = (int)(py / TH) * fp.tiles_x + (int)(px / TW);
    const i64 p = py * fp.W + px;
    const int ipp = fp.ipp;
    f64* dst = fp.fb + p * ipp;
    iu8* d8 = fp.frameU8 ? fp.frameU8 + p * ipp : nullptr;
    if (off[tile + 1] == off[tile]) {   // no triangle touches this tile
        if (fp.pendColor) {
            const f64 v = fp.pendColorValue;
            dst[0] = v; dst[1] = v; dst[2] = v;
            if (ipp == 4) dst[3] = v;
            if (d8) {
                const iu8 v8 = nr_to_u8(v);
                d8[0] = v8; d8[1] = v8; d8[2] = v8;
                if (ipp == 4) d8[3] = v8;
            }
        }
        if (ZMODE != 0 && fp.pendDepth) fp.depth[p] = fp.pendDepthValue;
        return;
    }
    const u64 kv = vis[p];
    const u32 id1 = (u32)kv;
    if (id1 == 0) {
        if (fp.pendColor) {
            const f64 v = fp.pendColorValue;
            dst[0] = v; dst[1] = v; dst[2] = v;
            if (ipp == 4) dst[3] = v;
            if (d8) {
                const iu8 v8 = nr_to_u8(v);
                d8[0] = v8; d8[1] = v8; d8[2] = v8;
                if (ipp == 4) d8[3] = v8;
            }
        }
        if (ZMODE != 0 && fp.pendDepth) fp.depth[p] = fp.pendDepthValue;
        return;
    }
    f64 R, G, B, A = 0;
    if (fp.pendColor) {
        R = G = B = A = fp.pendColorValue;
    } else {
        R = dst[0]; G = dst[1]; B = dst[2];
        if (ipp == 4) A = dst[3];
    }
    const i64 t = (i64)id1 - 1;
    f64 cr, cg, cb, ca;
    if (GOURAUD) {
        f64 sx[3], sy[3];
        tri_screen(fp.src, fp.m, t, sx, sy);
        const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
        const f64 inv = 1.0 / (e1x * e2y - e2x * e1y);
        const f64 dx = (f64)px - sx[0], dy = (f64)py - sy[0];
        const f64 w1 = (dx * e2y - e2x * dy) * inv;
        const f64 w2 = (e1x * dy - dx * e1y) * inv;
        const f64* c = fp.src.rgba + t * 12;
        cr = c[0] + (c[4] - c[0]) * w1 + (c[8] - c[0]) * w2;
        cg = c[1] + (c[5] - c[1]) * w1 + (c[9] - c[1]) * w2;
        cb = c[2] + (c[6] - c[2]) * w1 + (c[10] - c[2]) * w2;
        ca = c[3] + (c[7] - c[3]) * w1 + (c[11] - c[3]) * w2;
    } else {
        const f64* c = fp.src.rgba + t * 4;
        cr = c[0]; cg = c[1]; cb = c[2]; ca = c[3];
    }
    // ApplyPixel (cpp:529-547); ca * ct3 == 1 for every batch routed here
    cr *= fp.ct[0]; cg *= fp.ct[1]; cb *= fp.ct[2]; ca *= fp.ct[3];
    if (ca != 1) {
        cr = R * (1 - ca) + cr * ca;
        cg = G * (1 - ca) + cg * ca;
        cb = B * (1 - ca) + cb * ca;
    }
    dst[0] = cr; dst[1] = cg; dst[2] = cb;
    if (ipp == 4) dst[3] = ca;
    if (d8) {
        d8[0] = nr_to_u8(cr); d8[1] = nr_to_u8(cg); d8[2] = nr_to_u8(cb);
        if (ipp == 4) d8[3] = nr_to_u8(ca);
    }
    if (ZMODE == 1) fp.depth[p] = (u32)(kv >> 32);
    else if (ZMODE == 2 && fp.pendDepth) fp.depth[p] = fp.pendDepthValue;
}

template <int Z, bool C>
void launch_vis(const FrameParams& fp, const u32* off, const u32* soff, const u32* list, u64* vis, u32 grid,
                const u32* plan, hipStream_t s) {
    hipLaunchKernelGGL((k_vis<Z, C>), dim3(grid), dim3(VWG), 0, s, fp, off, soff, list, vis, plan);
}

template <int Z, bool G>
void launch_resolve(const FrameParams& fp, const u32* off, const u64* vis, const u32* plan, hipStream_t s) {
    const int owned = (fp.tiles_y - fp.shard + fp.nshards - 1) / fp.nshards;
    if (owned <= 0) return;
    dim3 grid((unsigned)((fp.W + 255) / 256), (unsigned)(owned * TH));
    hipLaunchKernelGGL((k_resolve<Z, G>), grid, dim3(256), 0, s, fp, off, vis, plan);
}

// Everything a batch needs to be re-run after an overflow (nr_settle).
struct PendingBatch {
    TriSrc src;
    FrameParams fp;
    BinParams bp;
};

// Enqueues one batch.  exact: read the pair/item totals back (host sync) and
// allocate exactly; otherwise size the list from `cap`, let the plan kernel
// check it on the device and validate later (nr_settle).
static bool free_enqueue(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp,
                         bool exact) {
    hipStream_t s = ctx->stream;
    TriScratch& sc = ctx->tri;
    const int ntiles = fp.tiles_x * fp.tiles_y;
    const int zmode = fp.depthTest ? (fp.depthWrite ? 1 : 2) : 0;
    const bool g = src.gouraud != 0;

    u32* tb[4] = {sc.fcnt, sc.foff, sc.fsoff, sc.fcur};
    const size_t oldcap = sc.ftile_cap;
    if (!grow_set(tb, &sc.ftile_cap, (size_t)ntiles + 1)) return false;
    sc.fcnt = tb[0]; sc.foff = tb[1]; sc.fsoff = tb[2]; sc.fcur = tb[3];
    if (sc.ftile_cap != oldcap) {   // counters start at zero; k_free_plan re-zeroes them after each use
        NR_CHECK(hipMemsetAsync(sc.fcnt, 0, sc.ftile_cap * sizeof(u32), s));
        NR_CHECK(hipMemsetAsync(sc.fcur, 0, sc.ftile_cap * sizeof(u32), s));
    }
    if (!sc.dplan) NR_CHECK(hipMalloc(&sc.dplan, 4 * sizeof(u32)));
    if (!sc.h_plan) {
        NR_CHECK(hipHostMalloc((void**)&sc.h_plan, 4 * sizeof(u32), hipHostMallocMapped | hipHostMallocCoherent));
        NR_CHECK(hipHostGetDevicePointer((void**)&sc.d_hplan, sc.h_plan, 0));
    }
    u64* vb[1] = {sc.vis};
    if (!grow_set(vb, &sc.vis_cap, (size_t)(ctx->width * ctx->height))) return false;
    sc.vis = vb[0];

    size_t cap = 0xFFFFFFFFull;
    if (!exact) {
        const u64 est = std::max<u64>(std::max<u64>(sc.lastPairs + sc.lastPairs / 4, (u64)src.n * 2), 1u << 20);
        cap = (size_t)std::min<u64>(sc.capOverride ? sc.capOverride : est, 0xFFFFFFF0ull);
        u32* lb[1] = {sc.flist};
        if (!grow_set(lb, &sc.flist_cap, cap)) return false;
        sc.flist = lb[0];
        if (!sc.capOverride) cap = std::min<size_t>(sc.flist_cap, 0xFFFFFFF0ull);
    }

    const bool ldsh = ntiles <= LDS_HIST_MAX;
    const size_t hbytes = ldsh ? (size_t)ntiles * sizeof(u32) : 0;
    const int gb = (int)((src.n + 256 * TPT - 1) / (256 * TPT));
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_TRI_COUNT, &e0, &e1);
    if (ldsh) hipLaunchKernelGGL(k_free_count<true>, dim3(gb), dim3(256), hbytes, s, bp, sc.fcnt, ntiles);
    else hipLaunchKernelGGL(k_free_count<false>, dim3(gb), dim3(256), 0, s, bp, sc.fcnt, ntiles);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TRI_COUNT, e0, e1);

    nr_timing_begin(ctx, NRK_TRI_SCAN, &e0, &e1);
    hipLaunchKernelGGL(k_free_plan, dim3(1), dim3(1024), 0, s, sc.fcnt, ntiles, sc.foff, sc.fsoff, sc.fcur, sc.dplan,
                       sc.d_hplan, (u32)cap);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TRI_SCAN, e0, e1);

    u32 grid;
    bool multi = true;
    if (exact) {
        NR_CHECK(hipStreamSynchronize(s));
        const u32 P = sc.h_plan[0];
        grid = sc.h_plan[1];
        multi = sc.h_plan[2] != 0;
        sc.lastPairs = P;
        u32* lb[1] = {sc.flist};
        if (!grow_set(lb, &sc.flist_cap, (size_t)std::max<u32>(P, 1))) return false;
        sc.flist = lb[0];
    } else {
        if (!sc.planEvent) NR_CHECK(hipEventCreateWithFlags(&sc.planEvent, hipEventDisableTiming));
        NR_CHECK(hipEventRecord(sc.planEvent, s));
        // a bound on the work items: every non-empty tile + one per full slice
        const u64 bound = (u64)ntiles + cap / SLICE + 1;
        grid = (u32)std::min<u64>(bound, 8192);
    }

    nr_timing_begin(ctx, NRK_TRI_EMIT, &e0, &e1);
    if (ldsh) hipLaunchKernelGGL(k_free_emit<true>, dim3(gb), dim3(256), hbytes, s, bp, sc.foff, sc.fcur, sc.flist, ntiles, sc.dplan);
    else hipLaunchKernelGGL(k_free_emit<false>, dim3(gb), dim3(256), 0, s, bp, sc.foff, sc.fcur, sc.flist, ntiles, sc.dplan);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TRI_EMIT, e0, e1);

    if (multi) {
        nr_timing_begin(ctx, NRK_VIS_INIT, &e0, &e1);
        if (zmode == 1) hipLaunchKernelGGL(k_vis_init_multi<1>, dim3(ntiles), dim3(256), 0, s, fp, sc.foff, sc.vis, sc.dplan);
        else hipLaunchKernelGGL(k_vis_init_multi<0>, dim3(ntiles), dim3(256), 0, s, fp, sc.foff, sc.vis, sc.dplan);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_VIS_INIT, e0, e1);
    }

    if (grid > 0) {
        nr_timing_begin(ctx, NRK_TILE_RASTER, &e0, &e1);
        const bool C = fp.fragCounter != nullptr;
        if (zmode == 1) { if (C) launch_vis<1, true>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); else launch_vis<1, false>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); }
        else if (zmode == 2) { if (C) launch_vis<2, true>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); else launch_vis<2, false>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); }
        else { if (C) launch_vis<0, true>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); else launch_vis<0, false>(fp, sc.foff, sc.fsoff, sc.flist, sc.vis, grid, sc.dplan, s); }
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_TILE_RASTER, e0, e1);
    }

    nr_timing_begin(ctx, NRK_RESOLVE, &e0, &e1);
    if (zmode == 1) { if (g) launch_resolve<1, true>(fp, sc.foff, sc.vis, sc.dplan, s); else launch_resolve<1, false>(fp, sc.foff, sc.vis, sc.dplan, s); }
    else if (zmode == 2) { if (g) launch_resolve<2, true>(fp, sc.foff, sc.vis, sc.dplan, s); else launch_resolve<2, false>(fp, sc.foff, sc.vis, sc.dplan, s); }
    else { if (g) launch_resolve<0, true>(fp, sc.foff, sc.vis, sc.dplan, s); else launch_resolve<0, false>(fp, sc.foff, sc.vis, sc.dplan, s); }
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_RESOLVE, e0, e1);
    return true;
}

}  // namespace

void draw_free(RenderContext* ctx, const TriSrc& src) {
    FrameParams fp = frame_params(ctx, src);
    if (ctx->frameOutput && fp.pendColor) {
        const size_t n = (size_t)(ctx->width * ctx->height * fp.ipp);
        if (n <= ctx->frameU8cap) fp.frameU8 = ctx->frameU8;
    }
    BinParams bp;
    bp.src = src;
    for (int k = 0; k < 6; ++k) bp.m[k] = ctx->m[k];
    bp.W = ctx->width; bp.H = ctx->height; bp.tiles_x = fp.tiles_x;
    bp.nshards = fp.nshards; bp.shard = fp.shard;
    // fragment counting reads a counter back anyway: run exact (synchronous)
    const bool exact = fp.fragCounter != nullptr;
    if (!free_enqueue(ctx, src, fp, bp, exact)) return;
    if (!exact) {
        PendingBatch* pb = new PendingBatch{src, fp, bp};
        ctx->pendingBatch = pb;
    }
    ctx->lastPath = 1;
    finish_batch(ctx, fp);
}

// Validates the last asynchronously sized batch of `ctx`: waits for its plan
// kernel (usually long finished), and if the pair list did not fit, re-runs
// the batch with an exact allocation.  Called at the start of every API
// entry point that enqueues work on, or reads, the context's buffers, so the
// re-run is ordered before anything that depends on the batch.
void settle(RenderContext* ctx) {
    PendingBatch* pb = reinterpret_cast<PendingBatch*>(ctx->pendingBatch);
    if (!pb) return;
    ctx->pendingBatch = nullptr;
    TriScratch& sc = ctx->tri;
    NR_CHECK(hipEventSynchronize(sc.planEvent));
    if (sc.h_plan[3]) {
        sc.lastPairs = sc.h_plan[0];
    } else {
        sc.lastPairs = sc.h_plan[0];
        free_enqueue(ctx, pb->src, pb->fp, pb->bp, true);   // context flags were applied at the first launch
    }
    delete pb;
}

}  // namespace nrtri
