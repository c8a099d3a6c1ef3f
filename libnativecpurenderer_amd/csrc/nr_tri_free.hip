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
//   4 k_vis          one 256-thread workgroup per (tile, slice of <= SLICE
//                    triangles; an empty tile is one item): each wave takes
//                    64-triangle chunks, lane = triangle -> exact row spans ->
//                    depth + LDS atomic on the tile's 2048 packed keys; then the same
//                    workgroup shades the tile (deferred: winner ->
//                    barycentrics -> colour -> ApplyPixel -> framebuffer,
//                    depth and u8 frame written once).  A tile whose list is
//                    split over several slices (the load-balancing step for
//                    dense tiles, e.g. mesh poles) merges its keys into `vis`
//                    with global atomics and the last slice to finish shades
//                    it and resets those keys.
#include "nr_tri.h"
#include "nr_tri_shade.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace nrtri {
namespace {

// Per-work-item clocks of k_vis (a build with -DNR_PROBE=1 only: tools/exp/probe.so,
// tools/exp/probe_items.py): item, {tile, list begin, end, slices}, start and end
// (s_memrealtime, 100 MHz), workgroup size.
#ifndef NR_PROBE
#define NR_PROBE 0
#endif
#if NR_PROBE
constexpr int PROBE_MAX = 65536;
__device__ unsigned long long nr_probe_buf[PROBE_MAX * 8];
__device__ unsigned int nr_probe_n;
__shared__ u64 pr_st[8];   // phase stamps of the current item (thread 0): 1 keys set, 2 raster, 3 merge, 4 hash, 5 records,
                           // 6 wave 0's first triangle data arrived, 7 wave 0's chunks done (before the barrier)
#define NR_PROBE_STAMP(k) do { if (threadIdx.x == 0) pr_st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ __forceinline__ void probe_item(u32 item, uint4 d, u64 t0, u64 t1, int nt) {
    const u32 k = atomicAdd(&nr_probe_n, 1u);
    if (k >= PROBE_MAX) return;
    unsigned long long* e = nr_probe_buf + (size_t)k * 8;
    e[0] = (u64)item | ((u64)nt << 32);
    e[1] = (u64)d.x | ((u64)d.w << 32);
    e[2] = (u64)d.y | ((u64)d.z << 32);
    auto rel = [&](int q) { return pr_st[q] >= t0 && pr_st[q] <= t1 ? (pr_st[q] - t0) & 0xFFFF : 0xFFFFull; };
    e[4] = rel(1) | (rel(2) << 16) | (rel(3) << 32) | (rel(4) << 48);
    e[5] = rel(5) | (rel(6) << 16) | (rel(7) << 32);
    __hip_atomic_store(&e[3], (t1 - t0) | (t0 << 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int q = 1; q < 8; ++q) pr_st[q] = 0;
}
#else
#define NR_PROBE_STAMP(k) do { } while (0)
#endif


constexpr int VWG = 256;  // k_vis workgroup
// k_vis occupancy: 4 waves per SIMD (<= 128 VGPRs, and LDS <= 40 KB per
// workgroup: 280 shading records over the keys + REC_EXTRA) measured 6-10 %
// faster on C3 than 3 (135 VGPRs, 53.5 KB); k_vis is latency-bound.
constexpr int VIS_WPE = 4;   // (5 waves: 96 VGPRs + 112 B spills, C3 +16 %, profiles/r05/ab_vis_occupancy.txt)
constexpr u32 SLICE = 1024;      // longest work item (triangles)
constexpr u32 SLICE_MIN = 64;    // shortest slice of a split tile
// Items the plan kernel aims for when it picks the slice length.  Round 4
// (warm binning, spill-free k_vis): 256, i.e. slices of 1024 for every batch of
// >= 2^17 owned pairs.  An 8-way C3 share (~150k pairs) used to get slices of
// 512: its split tiles' slot merges cost more than the longer slices (0.046 ->
// 0.041 ms per frame, C2 -1 %, C3 unchanged; profiles/r04/ab_slice_target.txt).
constexpr u32 SLICE_TARGET = 256;
constexpr int TPT = 4;   // triangles per thread in the binning kernels (2 / 8 measured slower, round 4)
constexpr int LDS_HIST_MAX = 16384;

// Tile rectangle of a triangle, packed for the emit pass (16 bits per bound;
// NO_RECT: the triangle produces no fragment).
constexpr u64 NO_RECT = ~0ull;
__device__ __forceinline__ u64 pack_rect(int tx0, int tx1, int ty0, int ty1) {
    return (u64)(u32)tx0 | ((u64)(u32)tx1 << 16) | ((u64)(u32)ty0 << 32) | ((u64)(u32)ty1 << 48);
}

// REC (ordered batches): also the triangle's setup record for the ordered
// raster (write_ordered_record), formed once here instead of in every tile.
template <bool LDSH, bool REC = false>
__global__ __launch_bounds__(256) void k_free_count(const BinParams bp, u32* __restrict__ tile_cnt, int ntiles,
                                                    u64* __restrict__ rects, f64* __restrict__ rec = nullptr) {
    extern __shared__ u32 hist[];
    const int tid = threadIdx.x;
    const i64 base = (i64)blockIdx.x * 256 * TPT;
    // every triangle's positions first (in flight during the histogram's
    // zeroing): one round of load latency, not TPT
    f64 pxy[TPT][6];
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (t < bp.src.n) load_tri_xy(bp.src.xy, t, pxy[k]);
    }
    // LDS histogram over the owned tile rows only (a sharded frame's share)
    const int hbins = bp.hrows * bp.tiles_x;
    if (LDSH) {
        for (int b = tid; b < hbins; b += 256) hist[b] = 0;
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (t >= bp.src.n) break;
        f64 sx[3], sy[3];
#pragma unroll
        for (int v = 0; v < 3; ++v) nr_xform(bp.m, pxy[k][2 * v], pxy[k][2 * v + 1], sx[v], sy[v]);
        int tx0, tx1, ty0, ty1;
        const bool hit = tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1);
        rects[t] = hit ? pack_rect(tx0, tx1, ty0, ty1) : NO_RECT;
        if (!hit) continue;
        if (REC) write_ordered_record(rec, t, sx, sy, bp.src.z);   // (hit: finite, den != 0)
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.period, bp.mask)) continue;
            const int hrow = (LDSH ? owned_ord(bp, ty) : ty) * bp.tiles_x;
            for (int tx = tx0; tx <= tx1; ++tx) {
                if (LDSH) atomicAdd(&hist[hrow + tx], 1u);
                else atomicAdd(&tile_cnt[hrow + tx], 1u);
            }
        }
    }
    if (LDSH) {
        __syncthreads();
        for (int b = tid; b < hbins; b += 256) {
            const u32 h = hist[b];
            if (h) {
                const int r = b / bp.tiles_x;
                atomicAdd(&tile_cnt[owned_row_of(bp, r) * bp.tiles_x + (b - r * bp.tiles_x)], h);
            }
        }
    }
}

// Single workgroup: off[i] = sum(cnt[<i]) (off[ntiles] = P) and the work
// items of k_vis, {tile, list begin, list end, slices of the tile}: an owned
// tile has max(1, ceil(cnt/SLICE)) of them (an empty tile is one item: k_vis
// writes its pending clear); totals = {P, items, number of split tiles}.
// totals[3] = 1 when the pair list fits `cap` and the items `icap`; every later kernel of the
// batch reads it and does nothing otherwise (the host then re-runs the batch
// with an exact allocation before anything else is enqueued, nr_settle).
// It also re-zeroes the tile counters for the next batch (after reading them)
// and the emit cursors, and mirrors the totals into pinned host memory, so a
// batch needs no memset and no copy command.
// Work items of an owned tile with c pairs: one item when c <= lim (an empty
// tile too: k_vis writes its pending clears); a dense tile (c > lim) is split
// into ni = ceil(c / dsl) slices of equal length.  lim and dsl come from the
// batch's slice length (plan kernels: split_limits).
__device__ __forceinline__ u32 tile_items(u32 c, bool owned, u32 lim, u32 dsl) {
    if (!owned) return 0u;
    return c > lim ? (c + dsl - 1) / dsl : 1u;
}
// Work item k of the ni items of a tile with c pairs from list offset ea:
// {tile, slice begin, slice end, w}, w = ni (items sharing the tile's merge,
// low 16 bits) | k << 16.  Slices are ceil(c / ni) long (the last one shorter,
// never empty: ceil(c / ni) <= dsl).
__device__ __forceinline__ uint4 tile_item(u32 tile, u32 ea, u32 c, u32 k, u32 ni) {
    if (ni == 1) return make_uint4(tile, ea, ea + c, 1u);
    const u32 q = (c + ni - 1) / ni;
    const u32 ls = ea + k * q;
    return make_uint4(tile, ls, min(ls + q, ea + c), ni | (k << 16));
}
// Split limits of a batch from its slice length: a tile of more than lim =
// min(slice, split_at) pairs is split into slices of about dsl = min(lim,
// dslice) (>= SLICE_MIN) pairs.  Splitting only the dense tiles, finer than the
// whole-tile limit, shortens the longest work items (k_vis's critical path)
// without splitting the many medium tiles.
__device__ __forceinline__ void split_limits(u32 slice, u32 split_at, u32 dslice, u32& lim, u32& dsl) {
    lim = min(slice, split_at);
    dsl = max((u32)SLICE_MIN, min(lim, dslice));
}

// Inclusive wave scan (64 lanes) with DPP row shifts and row broadcasts
// (VALU, a few cycles per step): Hillis-Steele inside each row of 16 lanes,
// then row 0's total into row 1 and row 2's into row 3 (row_bcast:15), then
// row 1's into rows 2 and 3 (row_bcast:31).  The __shfl_up form is a chain of
// six dependent LDS permutes (~100+ cycles each).
__device__ __forceinline__ u32 wave_scan(u32 v, int) {
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

constexpr int PLAN_T = 1024, PLAN_W = PLAN_T / 64;
constexpr u32 HEAVY_PAIRS = 256;   // a dense tile (for the k_vis workgroup-size choice)
// Size classes of a tile's work items: 0 empty; 1..PLAN_ONE one slice, by
// the count's bin (below); the PLAN_SPLIT highest for tiles split over
// several slices, by their slice count (>= 8, 4-7, 2-3).  Items are laid out
// largest class first: k_vis workgroups take items in index order, so the
// long ones start first and the short ones fill the tail (a longest-first
// schedule).  Results do not depend on the order (order-free raster).  The
// split classes come first, so split items take the indices [0, slices) --
// their key slots.  The densest tiles' slices first (round 4): their last
// slice merges the others' keys and shades the tile, the kernel's longest
// chain (a 16-slice 1080p tile started 62 us into a 98 us raster,
// tools/exp/probe_items.py).
// One-slice classes are PLAN_ONE equal bins of [1, lim] (octaves had left a
// C3 frame's items -- nearly all in [256, 1024] -- in two classes, in tile
// order within each): C3 -0.8 %, 1M tris at 1080p -1.3 %,
// C2 -2 % per frame (profiles/r03_c3/ab_class_lin.txt).
constexpr int PLAN_ONE = 10, PLAN_SPLIT = 3, PLAN_NB = 1 + PLAN_ONE + PLAN_SPLIT;
__device__ __forceinline__ int size_class(u32 c, u32 lim, u32 dsl) {
    if (c > lim) {
        const u32 ni = (c + dsl - 1) / dsl;
        return PLAN_NB - (ni >= 8 ? 1 : ni >= 4 ? 2 : 3);
    }
    if (c == 0) return 0;
    return 1 + min((int)((float)c * ((float)PLAN_ONE / (float)(lim + 1))), PLAN_ONE - 1);
}

// Tiles are taken PLAN_T at a time (thread = tile: coalesced), each round a
// workgroup scan carried over from the previous one.
__global__ __launch_bounds__(PLAN_T) void k_free_plan(u32* __restrict__ cnt, int ntiles, int tiles_x, int period,
                                                      u64 mask, u32* __restrict__ off, uint4* __restrict__ items,
                                                      u32* __restrict__ cur, u32* __restrict__ totals,
                                                      u64* __restrict__ host_totals, u32 cap, u32 icap, u32 seq,
                                                      u32 slice_target, u32 kcap, u32 split_at, u32 dslice) {
    __shared__ u32 sh[3][PLAN_W];
    __shared__ u32 bcnt[PLAN_NB], bcur[PLAN_NB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < PLAN_NB) bcnt[tid] = 0;
    // pass 0: the pair total sets the slice length, the smallest power of two
    // in [SLICE_MIN, SLICE] giving at most ~slice_target items of work
    // (short lists are sliced finer so that a sharded frame, whose dense tiles
    // are few, still fills the chip)
    u32 a = 0, hv = 0;
    for (int i = tid; i < ntiles; i += PLAN_T) {
        const u32 c = cnt[i];
        a += c;
        hv += c >= HEAVY_PAIRS ? 1u : 0u;
    }
    a = wave_scan(a, lane); hv = wave_scan(hv, lane);
    if (lane == 63) { sh[0][w] = a; sh[1][w] = hv; }
    __syncthreads();
    u32 ta = 0, th = 0;
#pragma unroll
    for (int k = 0; k < PLAN_W; ++k) { ta += sh[0][k]; th += sh[1][k]; }
    u32 slice = SLICE_MIN;
    while (slice < SLICE && (u64)slice * slice_target < ta) slice <<= 1;
    u32 lim, dsl;
    split_limits(slice, split_at, dslice, lim, dsl);
    __syncthreads();
    // pass 1: items (the capacity check needs the totals before any item is
    // written) and the number of items per size class
    u32 b = 0, m = 0;
    for (int i = tid; i < ntiles; i += PLAN_T) {
        const u32 c = cnt[i];
        const u32 ni = tile_items(c, owned_row(i / tiles_x, period, mask), lim, dsl);
        b += ni;
        m += ni > 1 ? ni : 0u;
        if (ni) atomicAdd(&bcnt[size_class(c, lim, dsl)], ni);
    }
    b = wave_scan(b, lane); m = wave_scan(m, lane);
    if (lane == 63) { sh[1][w] = b; sh[2][w] = m; }
    __syncthreads();
    u32 tb = 0, tm = 0;
#pragma unroll
    for (int k = 0; k < PLAN_W; ++k) { tb += sh[1][k]; tm += sh[2][k]; }
    const bool fits = ta <= cap && tb <= icap && tm <= kcap;
    if (tid == 0) {   // item ranges of the classes, largest class first
        u32 base = 0;
        for (int k = PLAN_NB - 1; k >= 0; --k) { bcur[k] = base; base += bcnt[k]; }
    }
    __syncthreads();
    // pass 2: offsets and items
    u32 carryA = 0;
    for (int r0 = 0; r0 < ntiles; r0 += PLAN_T) {
        const int i = r0 + tid;
        u32 c = 0, ni = 0;
        if (i < ntiles) {
            c = cnt[i];
            ni = tile_items(c, owned_row(i / tiles_x, period, mask), lim, dsl);
        }
        const u32 ia = wave_scan(c, lane);
        if (lane == 63) sh[0][w] = ia;
        __syncthreads();
        u32 ea = carryA + ia - c;
#pragma unroll
        for (int k = 0; k < PLAN_W; ++k) {
            if (k < w) ea += sh[0][k];
            carryA += sh[0][k];
        }
        __syncthreads();
        if (i < ntiles) {
            off[i] = ea;
            if (fits && ni) {
                const u32 eb = atomicAdd(&bcur[size_class(c, lim, dsl)], ni);
                for (u32 k = 0; k < ni; ++k) items[eb + k] = tile_item((u32)i, ea, c, k, ni);
            }
            cnt[i] = 0;
            cur[i] = 0;
        }
    }
    if (tid == 0) {
        off[ntiles] = ta;
        const u32 t[7] = {ta, tb, tm, fits ? 1u : 0u, seq, th, 0u};
        for (int k = 0; k < 4; ++k) totals[k] = t[k];
        // the host copy (nr_settle polls it): every word carries the batch's
        // sequence number in its high half and is stored on its own (8-byte
        // stores are single-copy atomic), so the host needs no ordering between
        // them and the kernel no release -- a system-scope release writes back
        // the whole L2 (buffer_wbl2), the dirty frame lines of the raster
        // running beside this kernel included (C3 -1.2 %, 8-way share -2 %,
        // profiles/r03_c3/ab_plan_release.txt)
        for (int k = 0; k < 7; ++k)
            __hip_atomic_store(&host_totals[k], ((u64)seq << 32) | t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The same plan with every tile count read once, into registers: thread t
// owns PR = 4 * ceil(ntiles / 4T) <= 16 consecutive tiles [t*PR, t*PR + PR), read and
// written as 16-byte vectors (the tile arrays are allocated to TILE_ARR entries,
// so the padding past ntiles -- never counted, so zero -- is in bounds), so
// the kernel makes one round of global loads instead of one per pass and per
// block of tiles.  Items are placed by size class without same-address LDS
// atomics (a wave's lanes mostly share a class, and such atomics serialise):
// per-lane class counts in registers, per-class wave scans, one LDS slot per
// (class, wave).  Launched with T = PLAN_T = 1024 threads whenever ntiles <=
// 16 * T (16384 tiles, an 8K frame; free_enqueue).
constexpr int PR_MAX = 16;
constexpr int TILE_ARR = 16 * 1024 + 4;   // minimum length of the per-tile arrays
template <int T, int PR>
__global__ __launch_bounds__(T) void k_free_plan_r(u32* __restrict__ cnt, int ntiles, int tiles_x, int period,
                                                   u64 mask, u32* __restrict__ off, uint4* __restrict__ items,
                                                   u32* __restrict__ cur, u32* __restrict__ totals,
                                                   u64* __restrict__ host_totals, u32 cap, u32 icap, u32 seq,
                                                   u32 slice_target, u32 kcap, u32 split_at, u32 dslice, u32 maxc) {
    constexpr int NWV = T / 64;
    __shared__ u32 sh[4][NWV];
    __shared__ u32 smax;   // longest tile list (ordered batches sort each list in LDS: <= maxc, 0 = no limit)
    __shared__ u32 csh[PLAN_NB][NWV];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (((ntiles + T - 1) / T) + 3) & ~3;
    const int i0 = tid * per;
    u32 c[PR];
#pragma unroll
    for (int q = 0; q < PR / 4; ++q) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (4 * q < per) v = reinterpret_cast<const uint4*>(cnt + i0)[q];
        c[4 * q] = v.x; c[4 * q + 1] = v.y; c[4 * q + 2] = v.z; c[4 * q + 3] = v.w;
    }
    u32 a = 0, hv = 0, mx = 0;
#pragma unroll
    for (int j = 0; j < PR; ++j) {
        a += c[j];
        hv += c[j] >= HEAVY_PAIRS ? 1u : 0u;
        mx = c[j] > mx ? c[j] : mx;
    }
    if (tid == 0) smax = 0;
    __syncthreads();
    if (maxc) atomicMax(&smax, mx);
    const u32 ia = wave_scan(a, lane), ih = wave_scan(hv, lane);
    if (lane == 63) { sh[0][w] = ia; sh[1][w] = ih; }
    __syncthreads();
    u32 ta = 0, th = 0, ea = ia - a;   // ea: list offset of this thread's first tile
#pragma unroll
    for (int k = 0; k < NWV; ++k) {
        if (k < w) ea += sh[0][k];
        ta += sh[0][k];
        th += sh[1][k];
    }
    u32 slice = SLICE_MIN;
    while (slice < SLICE && (u64)slice * slice_target < ta) slice <<= 1;
    u32 lim, dsl;
    split_limits(slice, split_at, dslice, lim, dsl);
    // items per tile, per-lane totals per size class (ownership: tile row of i0 + j)
    const int ty0 = i0 / tiles_x, tx0 = i0 - ty0 * tiles_x;
    u32 b = 0, m = 0, hc[PLAN_NB];
#pragma unroll
    for (int k = 0; k < PLAN_NB; ++k) hc[k] = 0;
    {
        int ty = ty0, tx = tx0;
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            const u32 ni = (j < per && i0 + j < ntiles) ? tile_items(c[j], owned_row(ty, period, mask), lim, dsl) : 0u;
            b += ni;
            m += ni > 1 ? ni : 0u;
            const int cls = size_class(c[j], lim, dsl);
#pragma unroll
            for (int k = 0; k < PLAN_NB; ++k) hc[k] += cls == k ? ni : 0u;
            if (++tx == tiles_x) { tx = 0; ++ty; }
        }
    }
    // per class: this lane's exclusive position among the wave's items
#pragma unroll
    for (int k = 0; k < PLAN_NB; ++k) {
        const u32 inc = wave_scan(hc[k], lane);
        if (lane == 63) csh[k][w] = inc;
        hc[k] = inc - hc[k];
    }
    const u32 ib = wave_scan(b, lane), im = wave_scan(m, lane);
    if (lane == 63) { sh[2][w] = ib; sh[3][w] = im; }
    __syncthreads();
    u32 tb = 0, tm = 0;
#pragma unroll
    for (int k = 0; k < NWV; ++k) { tb += sh[2][k]; tm += sh[3][k]; }
    const bool fits = ta <= cap && tb <= icap && tm <= kcap && (!maxc || smax <= maxc);
    // class ranges, largest class first, and each wave's base inside them:
    // thread k < PLAN_NB turns column k of csh into the wave bases of class k.
    // Every column is read (into registers) before any is rewritten: thread k
    // sums the columns of the classes above k while their threads rewrite them.
    u32 start = 0, col[NWV];
    if (tid < PLAN_NB) {
        for (int k = PLAN_NB - 1; k > tid; --k)
            for (int q = 0; q < NWV; ++q) start += csh[k][q];
#pragma unroll
        for (int q = 0; q < NWV; ++q) col[q] = csh[tid][q];
    }
    __syncthreads();
    if (tid < PLAN_NB) {
#pragma unroll
        for (int q = 0; q < NWV; ++q) {
            csh[tid][q] = start;
            start += col[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PLAN_NB; ++k) hc[k] += csh[k][w];
    {   // c[j] becomes tile j's list offset
        int ty = ty0, tx = tx0;
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            const u32 cj = c[j];
            c[j] = ea;
            const int i = i0 + j;
            const u32 ni = (j < per && i < ntiles) ? tile_items(cj, owned_row(ty, period, mask), lim, dsl) : 0u;
            const int cls = size_class(cj, lim, dsl);
            u32 eb = 0;
#pragma unroll
            for (int k = 0; k < PLAN_NB; ++k)
                if (cls == k) { eb = hc[k]; hc[k] += ni; }
            if (fits)
                for (u32 k = 0; k < ni; ++k) items[eb + k] = tile_item((u32)i, ea, cj, k, ni);
            ea += cj;
            if (++tx == tiles_x) { tx = 0; ++ty; }
        }
    }
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int q = 0; q < PR / 4; ++q) {
        if (4 * q < per) {
            reinterpret_cast<uint4*>(off + i0)[q] = make_uint4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
            reinterpret_cast<uint4*>(cnt + i0)[q] = z4;
            reinterpret_cast<uint4*>(cur + i0)[q] = z4;
        }
    }
    if (tid == 0) {
        off[ntiles] = ta;   // (the same value as the padding stores write there)
        const u32 t[7] = {ta, tb, tm, fits ? 1u : 0u, seq, th, smax};
        for (int k = 0; k < 4; ++k) totals[k] = t[k];
        for (int k = 0; k < 7; ++k)   // (host copy: see k_free_plan)
            __hip_atomic_store(&host_totals[k], ((u64)seq << 32) | t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool LDSH>
__global__ __launch_bounds__(256) void k_free_emit(const BinParams bp, const u32* __restrict__ off,
                                                   u32* __restrict__ cur, u32* __restrict__ list, int ntiles,
                                                   const u64* __restrict__ rects, const u32* __restrict__ plan) {
    extern __shared__ u32 hist[];
    if (!plan[3]) return;
    const int tid = threadIdx.x;
    const i64 base = (i64)blockIdx.x * 256 * TPT;
    u64 rk[TPT];   // every rectangle first: one round of load latency
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        rk[k] = t < bp.src.n ? rects[t] : NO_RECT;
    }
    const int hbins = bp.hrows * bp.tiles_x;   // (owned tile rows only, as k_free_count)
    if (LDSH) {
        for (int b = tid; b < hbins; b += 256) hist[b] = 0;
        __syncthreads();
        for (int k = 0; k < TPT; ++k) {
            const i64 t = base + k * 256 + tid;
            if (t >= bp.src.n) break;
            const u64 rc = rk[k];
            if (rc == NO_RECT) continue;
            const int tx0 = (int)(rc & 0xFFFF), tx1 = (int)((rc >> 16) & 0xFFFF);
            const int ty0 = (int)((rc >> 32) & 0xFFFF), ty1 = (int)(rc >> 48);
            for (int ty = ty0; ty <= ty1; ++ty)
                if (owned_row(ty, bp.period, bp.mask)) {
                    const int hrow = owned_ord(bp, ty) * bp.tiles_x;
                    for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[hrow + tx], 1u);
                }
        }
        __syncthreads();
        // reserve each touched tile's range once: hist[b] becomes the next slot
        for (int b = tid; b < hbins; b += 256) {
            const u32 h = hist[b];
            if (h) {
                const int r = b / bp.tiles_x;
                const int tile = owned_row_of(bp, r) * bp.tiles_x + (b - r * bp.tiles_x);
                hist[b] = off[tile] + atomicAdd(&cur[tile], h);
            }
        }
        __syncthreads();
    }
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (t >= bp.src.n) break;
        const u64 rc = rk[k];
        if (rc == NO_RECT) continue;
        const int tx0 = (int)(rc & 0xFFFF), tx1 = (int)((rc >> 16) & 0xFFFF);
        const int ty0 = (int)((rc >> 32) & 0xFFFF), ty1 = (int)(rc >> 48);
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.period, bp.mask)) continue;
            const int hrow = (LDSH ? owned_ord(bp, ty) : ty) * bp.tiles_x;
            for (int tx = tx0; tx <= tx1; ++tx) {
                const u32 slot = LDSH ? atomicAdd(&hist[hrow + tx], 1u)
                                      : off[hrow + tx] + atomicAdd(&cur[hrow + tx], 1u);
                list[slot] = (u32)t;
            }
        }
    }
}

// Warm binning: a TriangleBuffer drawn again under the binning key of its
// last validated binning, whose tile offsets and work items the context keeps
// (TriScratch::Schedule).  One pass over the triangles -- screen rectangle
// (as k_free_count), the workgroup's LDS histogram of its pairs over the owned
// tile rows, one range reservation per touched tile, the pairs (as
// k_free_emit) -- into the same [off[t], off[t + 1]) ranges: the count pass,
// the plan and the host's validation of the cold path are not needed,
// because the same buffer under the same key gives every tile exactly its
// former count.  LDSH: hist (next slot) and hlim (range end) per owned tile in
// LDS.
// The set's pair cursors are not reset between warm batches: the epoch-th
// warm batch of one schedule on this set finds cur[t] = epoch * count(t) and
// takes slots from there (cursor - epoch * count, count = off[t + 1] - off[t]).
// Checks: a tile found over its range stores the batch's tag in
// wstat[WS_TAG] (beside the cursors; its excess pairs are dropped), and k_vis
// checks every tile's cursor before it trusts the tile's list: after the e-th
// warm batch cur[t] must be (e + 1) * count(t), so an undercount or an
// overcount of that tile is seen there, and only that tile falls back
// (WarmCheck; round 6 -- until round 5 every binning workgroup added its pair
// total to one global sum word: ~4000 atomics on one address, 3.5 us of the
// 1080p frame, profiles/r05/ab_pair_sum.txt).  `inject` (tests only,
// SetWarmFaultInjection): 1 shifts the epoch (every touched tile out of its
// range), 3 drops workgroup 0's pairs (an undercount of its tiles).
// Can a cluster (user-space box {xmin, ymin, xmax, ymax}, TriangleBuffer::cbox)
// put a pair into an owned tile?  Its corners' screen positions bound every
// vertex's (the affine map's rounded products and sums are monotone in x and
// y), so a triangle's rows [ceil(ymin), ceil(ymax)) lie in the corners' row
// range (one row of margin each side); non-finite boxes are never culled.
// Columns follow tri_tiles: a triangle with a screen coordinate beyond 1e7
// is binned into every column of its rows, so a box with a corner beyond
// 1e7 (which may hold such a vertex) is never culled by x.
__device__ __forceinline__ bool cluster_may_touch(const BinParams& bp, const f64* box) {
    f64 y0 = INFINITY, y1 = -INFINITY, x0 = INFINITY, x1 = -INFINITY;
    bool huge = false;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        f64 sx, sy;
        nr_xform(bp.m, box[(c & 1) ? 2 : 0], box[(c & 2) ? 3 : 1], sx, sy);
        if (!isfinite(sx) || !isfinite(sy)) return true;
        huge = huge || fabs(sx) > 1e7 || fabs(sy) > 1e7;
        y0 = fmin(y0, sy); y1 = fmax(y1, sy); x0 = fmin(x0, sx); x1 = fmax(x1, sx);
    }
    if (!huge && (x1 < -4.0 || x0 > (f64)bp.W + 4.0)) return false;
    const f64 r0 = fmax(ceil(y0) - 1.0, 0.0), r1 = fmin(ceil(y1) + 1.0, (f64)bp.H);
    if (!(r0 < r1)) return false;
    if (bp.period == 1) return true;
    const int ty0 = (int)r0 / TH, ty1 = ((int)r1 - 1) / TH;
    for (int ty = ty0; ty <= ty1 && ty < ty0 + 64; ++ty)
        if (owned_row(ty, bp.period, bp.mask)) return true;
    return ty1 >= ty0 + 64;
}

// Loose ranges (a moving scene): a tile of c pairs under the schedule's
// transform gets room for loose_cap(c) under a transform that moves no vertex
// more than LOOSE_PX (a quarter more, and 64 pairs for the triangles that move
// in across its edges).  k_loose_off: one workgroup, off2 = exclusive scan of
// loose_cap(off[t + 1] - off[t]), once per schedule.
__host__ __device__ __forceinline__ u32 loose_cap(u32 c) { return c + c / 4 + 64; }
__global__ __launch_bounds__(1024) void k_loose_off(const u32* __restrict__ off, u32* __restrict__ off2, int ntiles) {
    __shared__ u32 wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (ntiles + 1023) / 1024;
    const int t0 = tid * per, t1 = min(ntiles, t0 + per);
    u32 s = 0;
    for (int t = t0; t < t1; ++t) s += loose_cap(off[t + 1] - off[t]);
    const u32 inc = wave_scan(s, lane);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    u32 run = inc - s;
    for (int k = 0; k < w; ++k) run += wsum[k];
    for (int t = t0; t < t1; ++t) {
        off2[t] = run;
        run += loose_cap(off[t + 1] - off[t]);
    }
    if (t0 < t1 && t1 == ntiles) off2[ntiles] = run;   // (the last non-empty chunk)
    if (ntiles == 0 && tid == 0) off2[0] = 0;
}

// the warm checks' words, right after a set's ntiles cursors: WS_TAG the tag of
// a batch with a tile over its range, WS_REP the tag of the last batch whose
// failure a k_vis workgroup reported (one report per batch)
enum { WS_REP = 0, WS_TAG = 1 };
template <bool LDSH>
__global__ __launch_bounds__(256) void k_bin_warm(const BinParams bp, const u32* __restrict__ off,
                                                  u32* __restrict__ cur, u32* __restrict__ list,
                                                  u32* __restrict__ wstat, u32 tag, u32 epoch,
                                                  const f64* __restrict__ cbox, const u32* __restrict__ blocks,
                                                  u32 inject, u32 loose) {
    extern __shared__ u32 hist[];
    const int tid = threadIdx.x;
    // (fault 1 under loose ranges: every touched tile's count runs far past its range)
    const u32 over = loose && inject == 1 ? 0x100000u : 0u;
    if (inject == 1 && !loose) epoch += 7;
    if (inject == 3 && blockIdx.x == 0) return;
    // (blocks: the schedule's active blocks, warm_blocks; the others hold no
    // cluster that reaches an owned tile)
    const i64 base = (i64)(blocks ? blocks[blockIdx.x] : blockIdx.x) * 256 * TPT;
    const int hbins = bp.hrows * bp.tiles_x;
    u32* hlim = hist + hbins;
    // this wave's cluster of each of its TPT triangle groups (NR_CLUSTER == 64:
    // one wave, so the test and the skip are wave-uniform)
    static_assert(NR_CLUSTER == 64, "a cluster is one wave's triangles");
    bool cl[TPT];
    bool anyc = false;
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 c = (base + k * 256) / NR_CLUSTER + __builtin_amdgcn_readfirstlane(tid >> 6);
        cl[k] = !cbox || c * NR_CLUSTER >= bp.src.n || cluster_may_touch(bp, cbox + c * 4);
        anyc = anyc || cl[k];
    }
    // a workgroup none of whose clusters reaches an owned tile has nothing to do
    // (most of them on a sharded frame's rank)
    if (cbox && !__syncthreads_or(anyc ? 1 : 0)) return;
    // (loading the positions before the cluster test -- one latency round
    // less, all bytes -- was not faster, round 4)
    f64 pxy[TPT][6];
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        if (cl[k] && t < bp.src.n) load_tri_xy(bp.src.xy, t, pxy[k]);
    }
    if (LDSH) for (int b = tid; b < hbins; b += 256) hist[b] = 0;
    if (LDSH) __syncthreads();   // (hist zeroed)
    u64 rk[TPT];
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        rk[k] = NO_RECT;
        if (t >= bp.src.n || !cl[k]) continue;
        f64 sx[3], sy[3];
#pragma unroll
        for (int v = 0; v < 3; ++v) nr_xform(bp.m, pxy[k][2 * v], pxy[k][2 * v + 1], sx[v], sy[v]);
        int tx0, tx1, ty0, ty1;
        if (!tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) continue;
        rk[k] = pack_rect(tx0, tx1, ty0, ty1);
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.period, bp.mask)) continue;
            if (!LDSH) continue;
            const int hrow = owned_ord(bp, ty) * bp.tiles_x;
            for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[hrow + tx], 1u);
        }
    }
    if (LDSH) {
        __syncthreads();
        for (int b = tid; b < hbins; b += 256) {   // reserve each touched tile's range once
            const u32 h = hist[b];
            if (h) {
                const int r = b / bp.tiles_x;
                const int tile = owned_row_of(bp, r) * bp.tiles_x + (b - r * bp.tiles_x);
                const u32 beg = off[tile], end = off[tile + 1];
                const u32 start = beg + atomicAdd(&cur[tile], h + over) - epoch * (end - beg);
                const bool bad = start < beg || start + h > end;
                hist[b] = bad ? end : start;   // (bad: every slot of this range fails slot < end)
                hlim[b] = end;
                // (loose ranges: an overflowing tile's cursor ends past its range, and k_vis
                // runs that tile over every triangle; the batch's other tiles are exact)
                if (bad && !loose) __hip_atomic_store(&wstat[WS_TAG], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (LDSH) __syncthreads();   // (LDS ranges reserved)
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
        const i64 t = base + k * 256 + tid;
        const u64 rc = rk[k];
        if (t >= bp.src.n || rc == NO_RECT) continue;
        const int tx0 = (int)(rc & 0xFFFF), tx1 = (int)((rc >> 16) & 0xFFFF);
        const int ty0 = (int)((rc >> 32) & 0xFFFF), ty1 = (int)(rc >> 48);
        for (int ty = ty0; ty <= ty1; ++ty) {
            if (!owned_row(ty, bp.period, bp.mask)) continue;
            const int hrow = (LDSH ? owned_ord(bp, ty) : ty) * bp.tiles_x;
            for (int tx = tx0; tx <= tx1; ++tx) {
                u32 slot, end;
                if (LDSH) {
                    slot = atomicAdd(&hist[hrow + tx], 1u);
                    end = hlim[hrow + tx];
                } else {
                    const u32 beg = off[hrow + tx];
                    end = off[hrow + tx + 1];
                    slot = beg + atomicAdd(&cur[hrow + tx], 1u + over) - epoch * (end - beg);
                    if (slot < beg || slot >= end) {
                        if (!loose) __hip_atomic_store(&wstat[WS_TAG], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        slot = end;
                    }
                }
                if (slot < end) list[slot] = (u32)t;
            }
        }
    }
}

// threadIdx.x as a value the compiler cannot see through: the per-pixel LDS
// and global addresses the item phases derive from it are then formed where
// they are used, inside the item loop, instead of being hoisted to the kernel
// prologue and kept live (spilled) across the whole raster -- the 4-wave
// instances' spills were mostly those hoisted addresses.
__device__ __forceinline__ int opaque_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// ---- deferred shading --------------------------------------------------
// A workgroup shades its tile after the raster.  The winners of the tile's
// pixels are few (a triangle wins ~9 pixels of the C3 mesh), so they are
// de-duplicated in an LDS hash table, each distinct winner's data is fetched
// once (one round of independent global loads, one thread per winner) and
// turned into a shading record in LDS, and the pixels are then shaded from
// LDS.  Per-pixel dependent global loads (eight rounds of latency per
// thread) were the largest cost of the fused raster.
constexpr int REC_EXTRA = 19200;   // LDS beyond the keys for shading records (k_vis stays <= 40 KB: 4 workgroups per CU)
constexpr int HTS = 512;           // hash slots (power of two)
constexpr int HTS_WIDE = 1024;     // hash slots of the 512-thread instance (its LDS holds two workgroups per CU)
constexpr int MAXPROBE = 16;       // linear-probe limit: a winner not placed / found within it loads directly
constexpr int OVF_Q = 1;           // directly loaded records in flight per thread (0: one at a time, in pass 3)

template <bool GOURAUD, int HS = HTS>
struct ShadeStage {
    // Gouraud record: sx0 sy0 e1x e1y e2x e2y inv | c0 rgb | (c1-c0) rgb | (c2-c0) rgb
    // flat record: rgb.  Alpha is not staged: every batch routed here has
    // vertex alpha 1 (and colourTransform[3] == 1), so the interpolated alpha
    // is 1 + 0*w1 + 0*w2, computed as such.
    // LDS of a k_vis workgroup: hash table | dense-index table | keys | extra.
    // The records of the shading pass overwrite the keys (each thread keeps
    // its pixels' winners in registers by then) and run on into `extra`, so
    // a tile stages RT records in KEY_BYTES + EXTRA bytes.
    static constexpr int REC = RecLen<GOURAUD>::REC;
    static constexpr int KEY_BYTES = TH * (TW + 1) * 8;
    static constexpr int EXTRA = GOURAUD ? REC_EXTRA : 0;
    static constexpr int RT_RAW = (KEY_BYTES + EXTRA) / (REC * 8);
    static constexpr int RT = RT_RAW < TH * TW ? RT_RAW : TH * TW;   // staged records per tile
    static constexpr int HT = 0, HIDX = HS * 4, DIDX = HS * 6;
    static constexpr int KEY_OFF = ((DIDX + RT * 4) + 15) & ~15;
    static constexpr int BYTES = KEY_OFF + KEY_BYTES + EXTRA;
};

template <int HS>
__device__ __forceinline__ u32 ht_hash(u32 id) { return (id * 2654435761u) >> (32 - __builtin_ctz(HS)); }

// Shades the tile from its LDS keys (`key` at row stride KS).  Pass 1: each
// thread takes its PPT pixels (p = tid + k*NT), stores their depth, keeps
// their winners in registers and enters the distinct winners in an LDS hash
// table (dense index d).  Pass 2: one record per staged winner (independent
// global loads: one latency round), written over the keys.  Pass 3: colour,
// ApplyPixel, framebuffer (+ u8 frame) written once.  A winner past the RT
// staged records (or not placed within MAXPROBE probes) loads its own record.
template <int ZMODE, bool GOURAUD, int NT, int HS>
__device__ __forceinline__ void shade_tile(const FrameParams& fp, i64 x0, i64 y0, int wlim, int hlim,
                                           const u64* key, unsigned char* lds, u32& nU) {
    using St = ShadeStage<GOURAUD, HS>;
    constexpr int PPT = TH * TW / NT;
    static_assert(PPT <= 32, "overflow bitmask");
    const int tid = opaque_tid();
    if constexpr (!GOURAUD) {
        // Flat: a winner's colour is its rgb -- no record to stage, so no
        // winner dedup: each pixel loads its winner's colour itself (the few
        // distinct winners of a tile stay in L2), FQ pixels' loads in flight
        // at a time.
        constexpr int FQ = PPT < 4 ? PPT : 4;
        static_assert(PPT % FQ == 0, "pixel groups");
#pragma unroll 1
        for (int k0 = 0; k0 < PPT; k0 += FQ) {
            u32 id[FQ];
            f64 c[FQ][3];
#pragma unroll
            for (int j = 0; j < FQ; ++j) {
                const int p = tid + (k0 + j) * NT, lx = p & (TW - 1), ly = p / TW;
                id[j] = 0;
                if (lx >= wlim || ly >= hlim) continue;
                const u64 kv = key[ly * (TW + 1) + lx];
                id[j] = (u32)kv;
                store_depth<ZMODE>(fp, (y0 + ly) * fp.W + x0 + lx, kv);
                if (id[j]) {
                    const f64* q = fp.src.rgba + ((i64)id[j] - 1) * 4;
                    const double2 rg = *reinterpret_cast<const double2*>(q);
                    c[j][0] = rg.x; c[j][1] = rg.y; c[j][2] = q[2];
                }
            }
#pragma unroll
            for (int j = 0; j < FQ; ++j) {
                const int p = tid + (k0 + j) * NT, lx = p & (TW - 1), ly = p / TW;
                if (lx >= wlim || ly >= hlim) continue;
                const i64 px = x0 + lx, py = y0 + ly;
                const i64 gp = py * fp.W + px;
                if (!id[j]) {
                    if (fp.pendColor) {
                        const f64 v = fp.pendColorValue;
                        store_colour(fp, gp, px, py, v, v, v, v);
                    }
                    continue;
                }
                f64 cr = c[j][0], cg = c[j][1], cb = c[j][2], ca = 1.0;   // (record_colour's flat case)
                apply_winner(fp, gp, cr, cg, cb, ca);
                store_colour(fp, gp, px, py, cr, cg, cb, ca);
            }
        }
        return;
    }
    u32* ht = reinterpret_cast<u32*>(lds + St::HT);
    unsigned short* hidx = reinterpret_cast<unsigned short*>(lds + St::HIDX);
    u32* didx = reinterpret_cast<u32*>(lds + St::DIDX);
    f64* rec = reinterpret_cast<f64*>(lds + St::KEY_OFF);   // over the keys, after pass 1
    for (int i = tid; i < HS; i += NT) ht[i] = 0;
    if (tid == 0) nU = 0;
    __syncthreads();
    u32 ids[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) ids[k] = 0;
    // bit k: pixel k's winner is not staged -- its record is loaded directly
    // in pass 3b, OVF_Q pixels at a time.  A dense tile (more distinct
    // winners than RT, e.g. the many-sliver tiles at a mesh's poles) stops
    // inserting once RT winners are staged instead of probing a full table.
    u32 ovf = 0;
#pragma unroll 1
    for (int k = 0; k < PPT; ++k) {
        const int p = tid + k * NT, lx = p & (TW - 1), ly = p / TW;
        if (lx >= wlim || ly >= hlim) continue;
        const u64 kv = key[ly * (TW + 1) + lx];
        const u32 id = (u32)kv;
#pragma unroll
        for (int q = 0; q < PPT; ++q)
            if (q == k) ids[q] = id;   // static register index
        store_depth<ZMODE>(fp, (y0 + ly) * fp.W + x0 + lx, kv);
        if (!id) continue;
        if (OVF_Q && __hip_atomic_load(&nU, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (u32)St::RT) {
            ovf |= 1u << k;
            continue;
        }
        u32 h = ht_hash<HS>(id);
        bool placed = false;
        for (int probe = 0; probe < MAXPROBE; ++probe, h = (h + 1) & (HS - 1)) {
            const u32 cur = ht[h];
            if (cur == id) { placed = true; break; }
            if (cur == 0) {
                const u32 old = atomicCAS(&ht[h], 0u, id);
                if (old == 0) {
                    const u32 d = atomicAdd(&nU, 1u);
                    hidx[h] = (unsigned short)(d < (u32)St::RT ? d : St::RT);
                    if (d < (u32)St::RT) didx[d] = id;
                    placed = d < (u32)St::RT;
                    break;
                }
                if (old == id) { placed = true; break; }
            }
        }
        if (OVF_Q && !placed) ovf |= 1u << k;
    }
    __syncthreads();   // every key read: the records may overwrite them
    NR_PROBE_STAMP(4);
    const u32 U = nU < (u32)St::RT ? nU : (u32)St::RT;
    // two winners per thread per round, both records' loads in flight
    for (u32 u = tid; u < U; u += 2 * NT) {
        RecordSrc<GOURAUD> s0, s1;
        const bool two = u + NT < U;
        load_record_src<GOURAUD>(fp, (i64)didx[u] - 1, s0);
        if (two) load_record_src<GOURAUD>(fp, (i64)didx[u + NT] - 1, s1);
        build_record<GOURAUD>(fp, s0, rec + u * St::REC);
        if (two) build_record<GOURAUD>(fp, s1, rec + (u + NT) * St::REC);
    }
    __syncthreads();
    NR_PROBE_STAMP(5);
#pragma unroll 1
    for (int k = 0; k < PPT; ++k) {
        const int p = tid + k * NT, lx = p & (TW - 1), ly = p / TW;
        if (lx >= wlim || ly >= hlim) continue;
        const i64 px = x0 + lx, py = y0 + ly;
        const i64 gp = py * fp.W + px;
        u32 id = 0;
#pragma unroll
        for (int q = 0; q < PPT; ++q)
            if (q == k) id = ids[q];
        if (!id) {
            if (fp.pendColor) {
                const f64 v = fp.pendColorValue;
                store_colour(fp, gp, px, py, v, v, v, v);
            }
            continue;
        }
        if ((ovf >> k) & 1u) continue;
        int d = St::RT;
        u32 h = ht_hash<HS>(id);
        for (int probe = 0; probe < MAXPROBE; ++probe, h = (h + 1) & (HS - 1)) {
            const u32 cur = ht[h];
            if (cur == id) { d = hidx[h]; break; }
            if (cur == 0) break;
        }
        f64 cr, cg, cb, ca;
        NR_DEV_CHECK(d >= St::RT || (u32)d < U, "shade_tile: pixel (%ld, %ld) reads record %d of %u staged (winner %u)",
                     (long)px, (long)py, d, U, id);
        NR_DEV_CHECK(id <= (u32)fp.src.n, "shade_tile: pixel (%ld, %ld) winner %u of %ld triangles", (long)px, (long)py, id,
                     (long)fp.src.n);
        if (d < St::RT) {
            record_colour<GOURAUD>(rec + d * St::REC, px, py, cr, cg, cb, ca);
        } else if (OVF_Q) {
            ovf |= 1u << k;
            continue;
        } else {   // overflow: load this pixel's winner directly
            f64 r[St::REC];
            make_record<GOURAUD>(fp, (i64)id - 1, r);
            record_colour<GOURAUD>(r, px, py, cr, cg, cb, ca);
        }
        apply_winner(fp, gp, cr, cg, cb, ca);
        store_colour(fp, gp, px, py, cr, cg, cb, ca);
    }
    // pass 3b: pixels whose winner is not staged, OVF_Q at a time: their
    // records' loads are independent and in flight together
    if constexpr (OVF_Q > 0) {
#pragma unroll 1
        while (ovf) {
            constexpr int Q = OVF_Q > 0 ? OVF_Q : 1;
            int kq[Q];
            RecordSrc<GOURAUD> src[Q];
#pragma unroll
            for (int j = 0; j < Q; ++j) {
                kq[j] = -1;
                if (!ovf) continue;
                kq[j] = __builtin_ctz(ovf);
                ovf &= ovf - 1;
                u32 id = 0;
#pragma unroll
                for (int q = 0; q < PPT; ++q)
                    if (q == kq[j]) id = ids[q];
                load_record_src<GOURAUD>(fp, (i64)id - 1, src[j]);
            }
#pragma unroll
            for (int j = 0; j < Q; ++j) {
                if (kq[j] < 0) continue;
                const int p = tid + kq[j] * NT, lx = p & (TW - 1), ly = p / TW;
                const i64 px = x0 + lx, py = y0 + ly;
                const i64 gp = py * fp.W + px;
                f64 r[St::REC];
                build_record<GOURAUD>(fp, src[j], r);
                f64 cr, cg, cb, ca;
                record_colour<GOURAUD>(r, px, py, cr, cg, cb, ca);
                apply_winner(fp, gp, cr, cg, cb, ca);
                store_colour(fp, gp, px, py, cr, cg, cb, ca);
            }
        }
    }
}

// ---- flattened chunk raster (k_vis FLAT) -------------------------------
// A wave's chunk (one triangle per lane) is rasterised in two flattened
// stages: its (triangle, row) pairs are dealt out 64 at a time (lane = row
// slot: the row's span), and each such window's covered pixels 64 at a time
// (lane = fragment) -- no lane idles on a short row or span beside a long one.
// The lanes fetch their triangle's and row's terms by lane permutes.

__device__ __forceinline__ int wave_scan_max(int v) {   // inclusive max scan (values >= 0)
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}

__device__ __forceinline__ int bperm(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ u32 bperm(u32 v, int src) { return (u32)__builtin_amdgcn_ds_bpermute(src << 2, (int)v); }
__device__ __forceinline__ float bperm(float v, int src) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
__device__ __forceinline__ f64 bperm(f64 v, int src) {
    const u64 b = __double_as_longlong(v);
    const u32 lo = (u32)__builtin_amdgcn_ds_bpermute(src << 2, (int)(u32)b);
    const u32 hi = (u32)__builtin_amdgcn_ds_bpermute(src << 2, (int)(u32)(b >> 32));
    return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}

// Owner of each slot of the window [wb, wb + 64) (slot wb + lane): the highest
// lane o whose run [st_o, st_o + n_o) (n_o > 0; runs in lane order, back to
// back) starts at or before it -- the runs that start in the window mark
// their first slot in the wave's 64 LDS words, an inclusive max scan carries
// each mark forward, and `carry` (the owner of slot wb - 1) fills the slots
// before the window's first mark.  (One wave, in-order LDS: the clear, the
// marks and the read need no barrier.)
__device__ __forceinline__ int window_owner(u32* mk, int lane, u32 st, u32 n, u32 wb, int carry) {
    __hip_atomic_store(&mk[lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (n && st - wb < 64u)
        __hip_atomic_fetch_max(&mk[st - wb], (u32)lane + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    const int v = (int)__hip_atomic_load(&mk[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return max(wave_scan_max(v), carry + 1) - 1;
}

static_assert(TH <= 64, "flattened raster: a fragment's row in 6 bits");
constexpr f64 COOP_PAIRS = 2.0;   // tile pairs per triangle above which k_vis takes the flattened raster
constexpr u32 HEAVY_PRIO = 512;   // work items of at least this many triangles run at raised wave priority
constexpr int KS = TW + 1;        // padded row stride of the LDS tile keys


// One workgroup per work item (tile, slice of <= SLICE triangles).  The 4
// waves share only the tile's 2048 LDS keys; each wave independently walks
// 64-triangle chunks of the slice (chunk c goes to wave c % 4) with no
// workgroup barrier: one lane per triangle, its setup in registers (screen
// vertices, edge slopes, 1/den, depths; the next chunk's loads in flight),
// then the lane walks the triangle's rows in this tile (exact span,
// row_span_slopes) and their pixels (depth + LDS atomic on the packed key,
// two pixels per step).  Then the workgroup shades the tile (shade_tile).
// FLAT: the chunk's rows and pixels are instead dealt out 64 per window
// (flattened raster, above): for batches whose triangles cover many pixels of
// a tile (C2 -17 %, profiles/r06/ab_flat.txt); for sliver meshes the permutes
// cost more than the lane raster's idle lanes (C3 +29 %).  The host picks it
// from the previous batch's pair density (COOP_PAIRS).
// NT: workgroup size (VWG, or 2 * VWG for batches with few pairs, whose dense
// items are latency-bound: more waves per item).
// The checks of a warm batch (k_bin_warm).  Batch-wide: the tag word
// wstat[WS_TAG] != this batch's tag (no tile over its range) and the plan says
// it fits (plan[3] == 0: the binning's token never came, k_gate_wait);
// otherwise the raster runs its work items over EVERY triangle of the batch
// instead of the tile lists -- slow, but the same frame bit for bit (a
// triangle that misses a tile adds nothing to it).  Per tile: the tile's
// cursor == mult * its count (mult = epoch + 1: the cursors run on across a
// schedule's warm batches, k_bin_warm); otherwise only that tile's items run
// over every triangle.  The first workgroup to see a failure (wstat[WS_REP]
// exchanged for the batch's tag) reports it in host-mapped *hfail (reason 1 a
// tile over its range, 2 token timeout, 3 a tile's count wrong, 4 a tile over
// its loose range; nr_settle latches an error and drops the schedule, or for
// 4 stops binning that buffer loose).  wstat null: a cold batch (plan[3] == 0
// there: the batch does nothing, the host re-runs it).
// Loose batches (a changed transform, loose ranges off = off2): the cursors
// start at 0 and hold the tile's pair count n, which only has to fit the
// tile's range; the tile's items then slice its n pairs afresh (item k of
// nsl: [k n / nsl, (k + 1) n / nsl)).
struct WarmCheck {
    u32* wstat;
    const u32* cur;   // the set's cursors
    const u32* off;   // the schedule's tile offsets (loose: its loose ranges)
    u32 tag, mult;
    u32* hfail;
    u32 loose;
};

// One report per failed warm batch (see WarmCheck): words 1..3 for the
// message, then the reason.
__device__ __forceinline__ void warm_report(const WarmCheck& wc, u32 why, u32 a, u32 b, u32 c) {
    if (__hip_atomic_exchange(&wc.wstat[WS_REP], wc.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == wc.tag) return;
    __hip_atomic_store(&wc.hfail[1], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&wc.hfail[2], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&wc.hfail[3], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&wc.hfail[0], why, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int ZMODE, bool COUNT, bool GOURAUD, bool FLAT, int NT>   // ZMODE 0: no test, 1: LESS+write, 2: LESS no write
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(VIS_WPE))) void k_vis(const FrameParams fp, const uint4* __restrict__ items,
                                             const u32* __restrict__ list,
                                             u64* __restrict__ kslot, u32* __restrict__ done,
                                             const u32* __restrict__ plan, const WarmCheck wc) {
    constexpr bool DEPTH = ZMODE != 0;
    constexpr int NWV = NT / 64;   // waves per workgroup
    // tile keys, rows padded to KS = 65 entries: lanes working on different
    // rows at the same column then hit different LDS banks
    // one LDS block (ShadeStage): hash tables | tile keys | extra; the
    // shading records overwrite the keys
    // the 512-thread instance has LDS to spare for a larger hash table (two
    // workgroups per CU)
    constexpr int HS = NT > VWG ? HTS_WIDE : HTS;
    __shared__ __attribute__((aligned(16))) unsigned char lds[ShadeStage<GOURAUD, HS>::BYTES];
    u64* const key = reinterpret_cast<u64*>(lds + ShadeStage<GOURAUD, HS>::KEY_OFF);
    __shared__ u32 zin[ZMODE == 2 ? TH * KS : 1];
    __shared__ u32 nU;
    __shared__ int sLast;
    __shared__ unsigned long long sFrag;
    raster_stamp_begin(fp);
    bool fb = false;   // fallback: every triangle of the batch against every tile (WarmCheck)
    if (wc.wstat) {
        const u32 wt = __hip_atomic_load(&wc.wstat[WS_TAG], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fb = !plan[3] || wt == wc.tag;
        if (fb && blockIdx.x == 0 && threadIdx.x == 0) warm_report(wc, plan[3] ? 1u : 2u, ~0u, wt, wc.tag);
    } else if (!plan[3]) {
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (uniform: the chunk loop is a scalar loop)
    const u32 nitems = plan[1];
    unsigned long long myFrags = 0;
    if (COUNT && tid == 0) sFrag = 0;
    // grid-stride over the work items (the grid is sized from a capacity
    // bound, not from the item count, so no host sync is needed)
    uint4 dnext = blockIdx.x < nitems ? items[blockIdx.x] : make_uint4(0, 0, 0, 0);
    u32 badTile = ~0u;   // a tile of this workgroup's whose cursor check failed (WarmCheck)
#if NR_PROBE
    u64 pr_t0 = 0;
    u32 pr_item = ~0u;
    uint4 pr_d = make_uint4(0, 0, 0, 0);
#endif
    for (u32 item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint4 d = dnext;
        if (item + gridDim.x < nitems) dnext = items[item + gridDim.x];
#if NR_PROBE
        if (tid == 0) {
            const u64 now = __builtin_amdgcn_s_memrealtime();
            if (pr_item != ~0u) probe_item(pr_item, pr_d, pr_t0, now, NT);
            pr_t0 = now; pr_item = item; pr_d = d;
        }
#endif
        __syncthreads();
        const int itid = opaque_tid();   // (this item's per-pixel addresses: formed here, not kept live)
        const int tile = (int)d.x;
        u32 ls = d.y, le = d.z;
        const u32 nsl = d.w & 0xFFFFu;   // slices of the tile (d.w >> 16: this item's slice)
        const bool multi = nsl > 1;
        bool fbt = fb;   // this tile's list is not trusted (WarmCheck)
        if (wc.wstat && !fb) {
            // (uniform values: scalar registers, nothing kept in VGPRs across the item)
            const u32 beg = __builtin_amdgcn_readfirstlane(wc.off[tile]);
            const u32 cnt = __builtin_amdgcn_readfirstlane(wc.off[tile + 1]) - beg;
            const u32 cu = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&wc.cur[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (!wc.loose) {
                fbt = cu != wc.mult * cnt;
            } else {
                fbt = cu > cnt;
                if (!fbt) {   // this item's slice of the tile's cu pairs
                    const u32 k = d.w >> 16;
                    ls = beg + (u32)(((u64)k * cu) / nsl);
                    le = beg + (u32)(((u64)(k + 1) * cu) / nsl);
                }
            }
            if (fbt) badTile = (u32)tile;   // (reported after the item loop: no report code live in it)
        }
        if (fbt) {   // this item's slice of all n triangles (never empty: a split tile has n >= its pairs > nsl)
            const u64 n = (u64)fp.src.n, k = d.w >> 16;
            ls = (u32)(k * n / nsl);
            le = (u32)((k + 1) * n / nsl);
        }
        constexpr int rlo = 0;
        // the longest work items (dense tiles' slices, and the slices of split
        // tiles, whose last slice merges and shades: the longest chains) set
        // the kernel's critical path: their waves win the SIMD's issue
        // arbitration over the short items that run beside them
        if (le - ls >= HEAVY_PRIO || multi) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
        const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
        const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
        const int wlim = (int)(fp.W - x0 < TW ? fp.W - x0 : TW);
        const int hlim = (int)(fp.H - y0 < TH ? fp.H - y0 : TH);
        const int rcap = hlim;   // rows [rlo, rcap) of the tile are rasterised here
        if (ls == le && !multi) {   // no triangle: only the pending clears
            if (fp.tileStamp) {
                // fast clear: the tile's framebuffer and depth keep the clear
                // pending (RenderContext::tileStamp); only the frame output,
                // which the batch hands over, is written
                if (fp.frameU8 && fp.pendColor) {
                    const f64 v = fp.pendColorValue;
                    for (int p = itid; p < TH * TW; p += NT) {
                        const int lx = p & (TW - 1), ly = p / TW;
                        if (lx < wlim && ly < hlim)
                            store_frame_out(fp, (y0 + ly) * fp.W + x0 + lx, x0 + lx, y0 + ly, v, v, v, v);
                    }
                }
                if (itid == 0) fp.tileStamp[tile] = fp.tileEpoch;
                continue;
            }
            for (int p = itid; p < TH * TW; p += NT) {
                const int lx = p & (TW - 1), ly = p / TW;
                if (lx < wlim && ly < hlim)
                    store_clear<ZMODE>(fp, (y0 + ly) * fp.W + x0 + lx, x0 + lx, y0 + ly);
            }
            continue;
        }

        for (int p = itid; p < TH * TW; p += NT) {
            const int lx = p & (TW - 1), ly = p / TW;
            u32 z0 = 0xFFFFFFFFu;
            if (DEPTH && lx < wlim && ly < hlim)
                z0 = fp.pendDepth ? fp.pendDepthValue : fp.depth[(y0 + ly) * fp.W + x0 + lx];
            key[ly * KS + lx] = ZMODE == 1 ? ((u64)z0 << 32) : 0ull;
            if (ZMODE == 2) zin[ly * KS + lx] = z0;
        }
        __syncthreads();
        NR_PROBE_STAMP(1);

        // this wave's chunks: c = wave, wave + NW, ...  One lane per triangle,
        // its setup in registers; the lane walks the triangle's rows in this
        // tile (exact span from the per-edge slopes) and their pixels -- or,
        // FLAT, the chunk's rows and then their pixels are dealt out to the
        // lanes 64 per window.  A short slice is cut into NW chunks so that
        // every wave gets a share.
        const u32 ns = le - ls;
        const u32 cs = ns >= 64u * NWV ? 64u : (ns + NWV - 1) / NWV;
        const u32 nch = (ns + cs - 1) / cs;
        // Loads run two chunks ahead for the list and one chunk ahead for the
        // triangle data: chunk c's setup issues the vertex loads of chunk
        // c + NWV from an index that arrived during chunk c - NWV, and the
        // index of chunk c + 2 NWV -- the dependent list -> vertex load pair
        // is never waited on inside a chunk (it used to stall every chunk
        // for one memory latency before the setup).
        // Every load here is unconditional, from an in-range address (a lane
        // past the chunk reads the slice's first entry, a real triangle), and
        // nothing is computed from a loaded value until it is used: a
        // conditional load, or a use right after it, makes the compiler wait
        // for the loads in flight on the spot.
        auto list_at = [&](u32 c) -> u32 {
            const int ln = opaque_tid() & 63;   // (formed here: the lane index is not kept live across the item)
            const u32 b = ls + c * cs + ln;
            const u32 i = c < nch && (u32)ln < cs && b < le ? b : ls;
            return fbt ? i : list[i];   // (fallback: the slice's triangle ids themselves)
        };
        // chunk c + NWV's triangle (loaded) and chunk c + 2 NWV's (in flight)
        u32 pt = list_at(wave), ptn = list_at(wave + NWV);
        const bool hasZ = DEPTH && fp.src.z;
        const f64* const zsrc = hasZ ? fp.src.z : fp.src.xy;   // (no z: any valid address, values unused)
        f64 pxy[6], pz[3];
        auto prefetch = [&](u32 t) {
            load_tri_xy(fp.src.xy, t, pxy);
            if (DEPTH) {
                const f64* qz = zsrc + (i64)t * 3;
                pz[0] = qz[0]; pz[1] = qz[1]; pz[2] = qz[2];
            }
        };
        // (FLAT: the chunk's vertices are loaded at its start -- a flattened
        // chunk runs long enough that its next one's loads would only hold
        // registers through it)
        if (!FLAT) prefetch(pt);
        for (u32 c = wave; c < nch; c += NWV) {
            const u32 base = ls + c * cs;
            const int cnt = (int)((le - base) < cs ? (le - base) : cs);
            if (FLAT) prefetch(pt);
            const u32 t = pt;
            f64 sx[3], sy[3], sl[3];
#pragma unroll
            for (int v = 0; v < 3; ++v) nr_xform(fp.m, pxy[2 * v], pxy[2 * v + 1], sx[v], sy[v]);
#if NR_PROBE
            if (threadIdx.x == 0 && c == (u32)wave) pr_st[6] = __builtin_amdgcn_s_memrealtime() + (sx[0] != sx[0] ? 1 : 0);
#endif
            const f64 zz0 = hasZ ? pz[0] : 0.0;
            const f64 dz1 = hasZ ? pz[1] - pz[0] : 0.0, dz2 = hasZ ? pz[2] - pz[0] : 0.0;
            pt = ptn;
            if (!FLAT) prefetch(pt);
            ptn = list_at(c + 2 * NWV);
            const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
            const f64 den = e1x * e2y - e2x * e1y;
            int r0 = 0, r1 = 0;   // rows with a straddling edge: ymin <= y < ymax (exact)
            if (lane < cnt && tri_finite(sx, sy) && den != 0) {
                const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
                r0 = (int)clampd(ceil(ymn) - (f64)y0, (f64)rlo, (f64)rcap);
                r1 = (int)clampd(ceil(ymx) - (f64)y0, (f64)rlo, (f64)rcap);
            }
            edge_slopes(sx, sy, sl);
            const f64 inv = 1.0 / den;
            const u64 id1 = (u64)t + 1;
            // f32 row spans (row_span32) with the exact f64 row_span_in for the
            // rows the f32 bound cannot decide: C2 -2 %, one rank's 8-way C3
            // share -3 % (k_vis 44 -> 40 us; profiles/r03_c3/ab_span32.txt).
            // Flat batches keep the f64 spans (the f32 ones cost the flat
            // instances 8-24 B/lane of spills).
            constexpr bool SPAN32 = GOURAUD && ZMODE != 2 && !COUNT;
            if constexpr (FLAT) {
                // rows: the chunk's (triangle, row) pairs, 64 per window
                const u32 nr = r0 < r1 ? (u32)(r1 - r0) : 0u;
                const u32 rin = wave_scan(nr, lane);
                const u32 R = (u32)__builtin_amdgcn_readlane((int)rin, 63), rex = rin - nr;
                const int r0x = r0 - (int)rex;   // (row of slot s: s + r0x of its triangle's lane)
                Span32 S32;
                if (SPAN32) S32 = span32_setup(sx, sy, sl, (f64)x0, (f64)y0);
                u32* const mk = reinterpret_cast<u32*>(lds + ShadeStage<GOURAUD, HS>::HT) + wave * 64;
                int rcar = -1;
                for (u32 rb = 0; rb < R; rb += 64) {
                    const int o = window_owner(mk, lane, rex, nr, rb, rcar);
                    rcar = __builtin_amdgcn_readlane(o, 63);
                    const u32 slot = rb + (u32)lane;
                    const int r = (int)slot + bperm(r0x, o);
                    const f64 y = (f64)(int)(y0 + r);
                    // (every permute with all lanes active: a permute reads 0 from an inactive lane)
                    Span32 S;
                    f64 ox[3], oy[3], os[3];
                    u32 oid = 0;
                    if (SPAN32) {
                        S.L = {bperm(S32.L.x, o), bperm(S32.L.yhi, o), bperm(S32.L.ylo, o), bperm(S32.L.s, o),
                               bperm(S32.L.ce, o)};
                        S.T = {bperm(S32.T.x, o), bperm(S32.T.yhi, o), bperm(S32.T.ylo, o), bperm(S32.T.s, o),
                               bperm(S32.T.ce, o)};
                        S.B = {bperm(S32.B.x, o), bperm(S32.B.yhi, o), bperm(S32.B.ylo, o), bperm(S32.B.s, o),
                               bperm(S32.B.ce, o)};
                        S.ymid = bperm(S32.ymid, o);
                        oid = bperm((u32)id1, o);
                    } else {
#pragma unroll
                        for (int v = 0; v < 3; ++v) {
                            ox[v] = bperm(sx[v], o); oy[v] = bperm(sy[v], o); os[v] = bperm(sl[v], o);
                        }
                    }
                    int xs = 0, xe = 0;
                    if (slot < R) {
                        if (SPAN32) {
                            if (!row_span32(S, r, y, (float)wlim, xs, xe)) {
                                f64 qx[3], qy[3];
                                tri_screen(fp.src, fp.m, (i64)oid - 1, qx, qy);
                                row_span_in(qx, qy, y, (f64)x0, (f64)wlim, xs, xe);
                            }
                        } else {
                            row_span_slopes(ox, oy, os, y, (f64)x0, (f64)wlim, xs, xe);
                        }
                    }
                    if (COUNT) myFrags += (unsigned long long)(xe - xs);
                    const u32 len = xe > xs ? (u32)(xe - xs) : 0u;
                    // the row's depth terms (frag_depth's e2x * dy and e1x * dy) and its
                    // triangle's, held by the row's lane: a fragment fetches all of its
                    // terms from one lane (one permute round)
                    f64 t1 = 0.0, t2 = 0.0, ox0 = 0.0, oe1y = 0.0, oe2y = 0.0, oin = 0.0, oz0 = 0.0, od1 = 0.0, od2 = 0.0;
                    const u32 rid = bperm((u32)id1, o);
                    if (ZMODE != 0) {
                        const f64 dy = y - bperm(sy[0], o);
                        t1 = bperm(e2x, o) * dy;
                        t2 = bperm(e1x, o) * dy;
                        ox0 = bperm(sx[0], o); oe1y = bperm(e1y, o); oe2y = bperm(e2y, o);
                        oin = bperm(inv, o); oz0 = bperm(zz0, o); od1 = bperm(dz1, o); od2 = bperm(dz2, o);
                    }
                    // fragments of the window's rows, 64 per step
                    const u32 fin = wave_scan(len, lane);
                    const u32 F = (u32)__builtin_amdgcn_readlane((int)fin, 63), fex = fin - len;
                    const int pk = (xs - (int)fex) * 64 + r;   // x - f, row
                    int fcar = -1;
                    for (u32 fb = 0; fb < F; fb += 64) {
                        const int q = window_owner(mk, lane, fex, len, fb, fcar);
                        fcar = __builtin_amdgcn_readlane(q, 63);
                        const int pq = bperm(pk, q);
                        const u32 fid = bperm(rid, q);
                        const int rr = pq & 63;
                        const int xx = (int)(fb + (u32)lane) + (pq >> 6);
                        if (ZMODE == 0) {
                            if (fb + (u32)lane < F) atomicMax(&key[rr * KS + xx], (u64)fid);
                            continue;
                        }
                        const f64 T1 = bperm(t1, q), T2 = bperm(t2, q);
                        const f64 qx0 = bperm(ox0, q), qe1y = bperm(oe1y, q), qe2y = bperm(oe2y, q);
                        const f64 qin = bperm(oin, q), qz0 = bperm(oz0, q), qd1 = bperm(od1, q), qd2 = bperm(od2, q);
                        if (fb + (u32)lane < F) {
                            // frag_depth with the row's products: the same operations on the same values
                            const f64 X = (f64)(int)(x0 + xx);
                            const f64 dx = X - qx0;
                            const f64 w1 = (dx * qe2y - T1) * qin;
                            const f64 w2 = (T2 - dx * qe1y) * qin;
                            const f64 zz = qz0 + qd1 * w1 + qd2 * w2;
                            const u32 zq = nr_quantize_depth_hw(zz);
                            const int kp = rr * KS + xx;
                            if (ZMODE == 1) atomicMin(&key[kp], ((u64)zq << 32) | fid);
                            else if (zq < zin[kp]) atomicMax(&key[kp], (u64)fid);
                        }
                    }
                }
                continue;
            }
            if (r0 < r1) {
                Span32 S32;
                if (SPAN32) S32 = span32_setup(sx, sy, sl, (f64)x0, (f64)y0);
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
                for (int r = r0; r < r1; ++r) {
                    const f64 y = (f64)(int)(y0 + r);
                    int xs, xe;
                    if (!SPAN32) {
                        row_span_slopes(sx, sy, sl, y, (f64)x0, (f64)wlim, xs, xe);
                    } else if (!row_span32(S32, r, y, (float)wlim, xs, xe)) {
                        // (rare: the exact statement.)  The screen vertices are
                        // formed again from the triangle's positions rather than
                        // kept live through the row loop: 8 fewer VGPRs there,
                        // the 4-wave instances' register peak
                        f64 qx[3], qy[3];
                        tri_screen(fp.src, fp.m, (i64)id1 - 1, qx, qy);
                        row_span_in(qx, qy, y, (f64)x0, (f64)wlim, xs, xe);
                    }
                    if (COUNT) myFrags += (unsigned long long)(xe - xs);
                    if (xs >= xe) continue;
                    if (ZMODE == 0) {
#pragma clang loop vectorize(disable) interleave(disable)
                        for (int lx = xs; lx < xe; ++lx) atomicMax(&key[r * KS + lx], id1);
                        continue;
                    }
                    const f64 dy = y - sy[0];   // (f64)j - pts[0][1], as the oracle
                    // two pixels per step: independent chains (ILP) and half the
                    // divergent trip count for the short spans of sliver triangles
                    f64 X = (f64)(int)(x0 + xs);   // pixel x as f64, exact (integers < 2^31)
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
                    for (int lx = xs; lx < xe; lx += 2, X += 2.0) {
                        frag_key<ZMODE>(key, zin, r * KS + lx, X, dy, sx[0], e1x, e1y, e2x, e2y, inv, zz0, dz1, dz2,
                                        id1);
                        if (lx + 1 < xe)
                            frag_key<ZMODE>(key, zin, r * KS + lx + 1, X + 1.0, dy, sx[0], e1x, e1y, e2x, e2y, inv,
                                            zz0, dz1, dz2, id1);
                    }
                }
            }
        }
        NR_PROBE_STAMP(7);
        __syncthreads();
        NR_PROBE_STAMP(2);
        if (!multi) {   // the whole list was in this slice: shade now
            if (rlo < rcap)
                shade_tile<ZMODE, GOURAUD, NT, HS>(fp, x0, y0 + rlo, wlim, rcap - rlo, key + rlo * KS, lds, nU);
            continue;
        }
        // split tile (a dense tile's slice): the slice's keys go to its own
        // slot of `kslot` (slot = item index: the split tiles' items come first
        // in the item list, plan kernels), as plain agent-coherent stores -- no
        // read-modify-write, so the slices of a tile never contend; the slice
        // that finishes last reduces every slot of the tile (min for LESS +
        // write, max of the ids otherwise: every slot starts from the same
        // initial keys) into its LDS keys and shades the tile.  The hand-off
        // needs no cache-wide fence: the slots move through agent-scope
        // (sc1) stores and loads, each wave drains its stores before the
        // barrier, and the slice counter is a relaxed device atomic.
        {
            u64* const mine = kslot + (size_t)item * (TH * TW);
            for (int p = itid; p < TH * TW; p += NT)   // (every key: pixels past the frame edge are never shaded)
                __hip_atomic_store(&mine[p], key[(p / TW) * KS + (p & (TW - 1))], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_s_waitcnt(0);   // vmcnt = lgkmcnt = 0: this wave's stores performed
        __syncthreads();
        if (tid == 0) {
            const u32 prev = __hip_atomic_fetch_add(&done[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sLast = prev + 1 == nsl;
            if (prev + 1 == nsl) __hip_atomic_store(&done[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!sLast) continue;
        {
            // each thread reduces its PR pixels together: per slot, PR
            // independent loads in flight (one latency round per slot, not
            // per pixel and slot)
            const u32 first = item - (d.w >> 16);   // the tile's first slice (its slot)
            constexpr int PR = TH * TW / NT;
            u64 kk[PR];
#pragma unroll
            for (int j = 0; j < PR; ++j) {
                const int p = itid + j * NT;
                kk[j] = key[(p / TW) * KS + (p & (TW - 1))];
            }
            // MB slots per round, all their loads in flight together (16 keys
            // per thread): a 16-slice pole tile's merge is 4 latency rounds,
            // not 16.  This slice's own slot and the padding past the last
            // slice read slot `first` again: min / max are idempotent.
            constexpr int MB = PR >= 8 ? 2 : (PR >= 4 ? 4 : 8);
            for (u32 sl = 0; sl < nsl; sl += MB) {
                u64 v[MB][PR];
#pragma unroll
                for (int b = 0; b < MB; ++b) {
                    const u32 s2 = sl + b < nsl ? sl + b : 0u;
                    const u64* slot = kslot + (size_t)(first + s2) * (TH * TW);
#pragma unroll
                    for (int j = 0; j < PR; ++j)
                        v[b][j] = __hip_atomic_load(slot + itid + j * NT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
                for (int b = 0; b < MB; ++b)
#pragma unroll
                    for (int j = 0; j < PR; ++j)
                        kk[j] = ZMODE == 1 ? (v[b][j] < kk[j] ? v[b][j] : kk[j]) : (v[b][j] > kk[j] ? v[b][j] : kk[j]);
            }
#pragma unroll
            for (int j = 0; j < PR; ++j) {
                const int p = itid + j * NT;
                key[(p / TW) * KS + (p & (TW - 1))] = kk[j];
            }
        }
        __syncthreads();
        NR_PROBE_STAMP(3);
        shade_tile<ZMODE, GOURAUD, NT, HS>(fp, x0, y0, wlim, hlim, key, lds, nU);
    }   // work items
#if NR_PROBE
    if (tid == 0 && pr_item != ~0u) probe_item(pr_item, pr_d, pr_t0, __builtin_amdgcn_s_memrealtime(), NT);
#endif
    raster_stamp_end(fp);
    if (badTile != ~0u && tid == 0)
        warm_report(wc, wc.loose ? 4u : 3u, badTile, wc.cur[badTile],
                    (wc.loose ? 1u : wc.mult) * (wc.off[badTile + 1] - wc.off[badTile]));
    if (COUNT) {
        __syncthreads();
        atomicAdd(&sFrag, myFrags);
        __syncthreads();
        if (tid == 0) atomicAdd(fp.fragCounter, sFrag);
    }
}

// k_vis runs 2 * VWG-thread workgroups when the last batch had a few dense
// tiles (>= HEAVY_PAIRS pairs), fewer than WIDE_HEAVY (half the chip's k_vis
// workgroup slots): each dense item is then latency-bound at low occupancy
// and gains from more waves (C3 sharded 8 ways -18 %, 4 ways -14 %; 2 ways
// +6 %, hence the threshold); with many dense tiles (C3 unsharded, 2 ways)
// or none (C2) the narrow workgroups are faster.  (A 3-wave-per-SIMD
// instance, which left the next batch's binning a slot beside the raster, was
// dropped in round 5: 4 waves measured faster once k_vis was spill-free, C3
// 0.147 -> 0.140 ms, profiles/r04/ab_instances.txt.)
// Round 6 re-measure (profiles/r06/ab_wide_heavy.txt): with ~226 dense tiles (C3
// 8-way share) wide is 24 % faster; with ~444 (4-way share) and ~478 (1M
// triangles at 1080p) the narrow one is 7 % faster, so the threshold moved
// from 512 to 320.
constexpr u32 WIDE_HEAVY = 320;

// The k_vis inputs of one batch: its work items, pair list and plan totals
// (a binning set's, or the warm schedule's).
struct VisArgs {
    const uint4* items;
    const u32* list;
    const u32* plan;
    WarmCheck wc;   // (a warm batch's checks; zero: a cold batch)
};

template <int Z, bool C, bool G>
void launch_vis(const FrameParams& fp, const TriScratch& sc, const VisArgs& va, u32 grid, hipStream_t s,
                hipEvent_t start, hipEvent_t stop) {
    const WarmCheck wc = va.wc;
    // the flattened raster when the previous batch had more than COOP_PAIRS
    // tiles per triangle (large triangles), or when there is no history
    const bool coop = sc.coopMode ? sc.coopMode == 1
                                  : (sc.lastN == 0 || sc.lastPairs > (u64)(COOP_PAIRS * (f64)sc.lastN));
    // wide workgroups when the last batch had few pairs (a sharded frame):
    // its dense items run at low occupancy and are latency-bound
    const bool wide = !C && sc.lastN != 0 && sc.lastHeavy > 0 && sc.lastHeavy < WIDE_HEAVY;
#define NR_VIS(CO, NTT, ...)                                                                                       \
    hipExtLaunchKernelGGL((k_vis<Z, __VA_ARGS__>), dim3(grid), dim3(NTT), 0, s, start, stop, 0, fp, va.items,    \
                          va.list, sc.kslot, sc.fdone, va.plan, wc)
    if (wide) {
        if (coop) NR_VIS(1, 2 * VWG, false, G, true, 2 * VWG);
        else NR_VIS(0, 2 * VWG, false, G, false, 2 * VWG);
    } else if (coop) {
        NR_VIS(1, VWG, C, G, true, VWG);
    } else {
        NR_VIS(0, VWG, C, G, false, VWG);
    }
#undef NR_VIS
}

template <int Z, bool G>
void launch_vis_z(const FrameParams& fp, const TriScratch& sc, const VisArgs& va, u32 grid, hipStream_t s,
                  hipEvent_t start, hipEvent_t stop) {
    if (fp.fragCounter) launch_vis<Z, true, G>(fp, sc, va, grid, s, start, stop);
    else launch_vis<Z, false, G>(fp, sc, va, grid, s, start, stop);
}

static void launch_vis_any(const FrameParams& fp, const TriScratch& sc, const VisArgs& va, u32 grid, hipStream_t s,
                           hipEvent_t start, hipEvent_t stop, int zmode, bool g) {
#define NR_VZ(ZM) (g ? launch_vis_z<ZM, true>(fp, sc, va, grid, s, start, stop) \
                     : launch_vis_z<ZM, false>(fp, sc, va, grid, s, start, stop))
    if (zmode == 1) NR_VZ(1);
    else if (zmode == 2) NR_VZ(2);
    else NR_VZ(0);
#undef NR_VZ
}

// Events of a batch carried by the kernels' own completion signals
// (hipExtLaunchKernel stop events) instead of separate marker packets: every
// packet between two rasters on the main queue costs a few microseconds.

// Everything a batch needs to be re-run after an overflow (nr_settle).
struct PendingBatch {
    TriSrc src;
    FrameParams fp;
    BinParams bp;
    int set;
    u32 seq;
    TriangleBuffer* tb;   // non-null: record the validated totals as its known sizes
    BinKey key;
    bool ordered;         // rasterised by the ordered raster (binned)
};

static BinKey bin_key(const BinParams& bp) {
    BinKey k;
    memset(&k, 0, sizeof k);   // padding too: keys are compared bytewise
    for (int i = 0; i < 6; ++i) k.m[i] = bp.m[i];
    k.W = bp.W; k.H = bp.H; k.period = bp.period; k.mask = bp.mask;
    return k;
}

static void record_known(TriangleBuffer* tb, const BinKey& key, u32 pairs, u32 heavy, u32 items, u32 split) {
    if (!tb) return;
    tb->known = true;
    tb->knownKey = key;
    tb->knownPairs = pairs;
    tb->knownHeavy = heavy;
    tb->knownItems = items;
    tb->knownSplit = split;
}

// Split limits of dense tiles (split_limits): a tile of more pairs than
// min(slice, SPLIT_AT) is split into slices of about DSLICE pairs (SetSplitLimits
// overrides them per context).
constexpr u32 SPLIT_AT = 1024, DSLICE = 1024;

// Binning output sets in rotation: with k sets the binning of batch b waits
// only for the raster of batch b - k.
constexpr int BIN_SETS = 3;

static hipEvent_t sync_event() {
    hipEvent_t e;
    NR_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    return e;
}

// A warm binning beside the raster hands off to the raster through its token
// only.  Should the raster's wait time out (a binning delayed by over a second,
// or serialised dispatch), the raster falls back and finishes while that
// binning may still be queued or running on the binning stream, and nothing
// orders later main-stream work after it.  So before the main stream writes a
// binning set or the warm schedule itself -- a binning on the main stream
// (inline warm, or a cold batch binned in line) or sched_capture's copies into
// the schedule every warm binning reads -- it waits for everything enqueued on
// the binning stream so far.  Steady state (always beside, or
// always inline) never takes this wait.
static void main_after_side_binning(RenderContext* ctx) {
    TriScratch& sc = ctx->tri;
    if (!sc.sideGated) return;
    if (!sc.evSide) sc.evSide = sync_event();
    NR_CHECK(hipEventRecord(sc.evSide, nr_bin_stream_for(ctx->device)));
    NR_CHECK(hipStreamWaitEvent(ctx->stream, sc.evSide, 0));
    sc.sideGated = false;
}

// Enqueues one batch with binning outputs in set `si`.  exact: read the
// pair/item totals back (host sync) and allocate exactly; otherwise size the
// list from the previous batch, let the plan kernel check it on the device
// and validate later (nr_settle).  pipelined: bin on the device's binning
// stream -- after the raster that last read set `si`, not after everything
// queued before on the main stream -- so that it overlaps the previous
// batch's k_vis (only for immutable inputs: a TriangleBuffer).
// Host view of a plan kernel's totals (k_free_plan*): word k = (seq << 32) | value, each
// stored by the device on its own; a batch's totals are complete once every word carries
// its sequence number.
static bool plan_ready(const TriScratch::FreeSet& F, u32 seq) {
    for (int k = 0; k < 7; ++k)
        if ((u32)(__atomic_load_n(&F.h_plan[k], __ATOMIC_ACQUIRE) >> 32) != seq) return false;
    return true;
}
static u32 plan_val(const TriScratch::FreeSet& F, int k) { return (u32)__atomic_load_n(&F.h_plan[k], __ATOMIC_ACQUIRE); }

// Returns ENQ_FAIL, ENQ_OK, or (exact, ordered) ENQ_SORTED: a tile list is
// longer than the ordered raster sorts in LDS -- nothing was rasterised; the
// caller takes the global-sort path.
enum { ENQ_FAIL = 0, ENQ_OK = 1, ENQ_SORTED = 2 };
static int free_enqueue(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp,
                        bool exact, int si, bool pipelined, u32* seqOut, u64 knownPairs = 0,
                        u32 knownItems = 0, bool idle = false, u32 knownSplit = 0, bool ordered = false) {
    hipStream_t sa = ctx->stream;
    hipStream_t sb = pipelined ? nr_bin_stream_for(ctx->device) : sa;
    TriScratch& sc = ctx->tri;
    TriScratch::FreeSet& F = sc.fset[si];
    const int ntiles = fp.tiles_x * fp.tiles_y;
    const int zmode = fp.depthTest ? (fp.depthWrite ? 1 : 2) : 0;
    const bool g = src.gouraud != 0;
    if (!F.evBin) { F.evBin = sync_event(); F.evVis = sync_event(); }
    if (sb == sa) main_after_side_binning(ctx);
    // the set's buffers are rewritten (binning stream) only after the raster
    // that last read them; a regrow frees them, so the host waits for it then
    if (F.visRecorded && sb != sa) NR_CHECK(hipStreamWaitEvent(sb, F.evVis, 0));
    auto quiesce = [&]() {
        if (F.visRecorded) NR_CHECK(hipEventSynchronize(F.evVis));
    };

    if (F.ftile_cap < std::max<size_t>((size_t)ntiles + 1, TILE_ARR) || !F.fcnt) quiesce();
    u32* tb[3] = {F.fcnt, F.foff, F.fcur};
    const size_t oldcap = F.ftile_cap;
    // (k_free_plan_r reads and writes the tile arrays as 16-byte vectors up to TILE_ARR)
    if (!grow_set(tb, &F.ftile_cap, std::max<size_t>((size_t)ntiles + 1, TILE_ARR))) return ENQ_FAIL;
    F.fcnt = tb[0]; F.foff = tb[1]; F.fcur = tb[2];
    if (F.ftile_cap != oldcap) {   // counters start at zero; k_free_plan re-zeroes them after each use
        NR_CHECK(hipMemsetAsync(F.fcnt, 0, F.ftile_cap * sizeof(u32), sb));
        NR_CHECK(hipMemsetAsync(F.fcur, 0, F.ftile_cap * sizeof(u32), sb));
    }
    u32* db[1] = {sc.fdone};
    const size_t olddone = sc.fdone_cap;
    if (!grow_set(db, &sc.fdone_cap, (size_t)ntiles + 1)) return ENQ_FAIL;
    sc.fdone = db[0];
    if (sc.fdone_cap != olddone) NR_CHECK(hipMemsetAsync(sc.fdone, 0, sc.fdone_cap * sizeof(u32), sa));
    if (!F.dplan) NR_CHECK(hipMalloc(&F.dplan, 4 * sizeof(u32)));
    if (!F.h_plan) {
        NR_CHECK(hipHostMalloc((void**)&F.h_plan, 8 * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent));
        for (int k = 0; k < 8; ++k) F.h_plan[k] = 0;
        NR_CHECK(hipHostGetDevicePointer((void**)&F.d_hplan, F.h_plan, 0));
    }
    // key slots of split tiles' slices (TH * TW keys each): sized from the
    // last validated batch; the plan kernel checks the capacity on the device
    auto grow_kslot = [&](size_t slices) {
        slices = std::max<size_t>(slices, 1);
        if (sc.kslot_cap >= slices * (TH * TW) && sc.kslot) return true;
        NR_CHECK(hipStreamSynchronize(sa));   // the running raster may still read them
        u64* kb[1] = {sc.kslot};
        const bool ok = grow_set(kb, &sc.kslot_cap, slices * (TH * TW));
        sc.kslot = kb[0];
        return ok;
    };
    auto grow_list = [&](size_t need) {
        need = std::max<size_t>(need, 1);
        if (F.flist_cap < need) quiesce();
        u32* lb[1] = {F.flist};
        const bool ok = grow_set(lb, &F.flist_cap, need);
        F.flist = lb[0];
        return ok;
    };
    auto grow_items = [&](size_t need) {
        need = std::max<size_t>(need, 1);
        if (F.fitems_cap < need) quiesce();
        uint4* ib[1] = {F.fitems};
        const bool ok = grow_set(ib, &F.fitems_cap, need);
        F.fitems = ib[0];
        return ok;
    };
    if (F.frect_cap < (size_t)src.n) quiesce();
    u64* rb[1] = {F.frect};
    if (!grow_set(rb, &F.frect_cap, (size_t)src.n)) return ENQ_FAIL;
    F.frect = rb[0];
    if (ordered) {   // the ordered raster's per-triangle setup records
        const size_t need = (size_t)std::max<i64>(src.n, 1) * ORec;
        if (F.frec_cap < need) quiesce();
        f64* rr[1] = {F.frec};
        if (!grow_set(rr, &F.frec_cap, need)) return ENQ_FAIL;
        F.frec = rr[0];
    }
    size_t cap;
    if (!exact) {
        const u64 est = std::max<u64>(std::max<u64>(std::max<u64>(sc.lastPairs + sc.lastPairs / 4, (u64)src.n * 2), 1u << 20),
                                      knownPairs);
        cap = (size_t)std::min<u64>(sc.capOverride ? sc.capOverride : est, 0xFFFFFFF0ull);
        if (!grow_list(cap)) return ENQ_FAIL;
        if (!sc.capOverride) cap = std::min<size_t>(F.flist_cap, 0xFFFFFFF0ull);
        // work items: at most one per tile + one per full slice of the list,
        // twice that with dense tiles split into row halves (NR_ROW_SPLIT)
        if (!grow_items((size_t)ntiles + cap / SLICE_MIN + 2)) return ENQ_FAIL;
        // key slots of split tiles' slices (ordered batches use none): the last validated batch's + 25 %, at
        // least one per tile (a slot per slice is needed only for tiles over the slice length)
        if (!ordered && !grow_kslot(std::max<size_t>(std::max<size_t>((size_t)sc.lastSplit + sc.lastSplit / 4, knownSplit),
                                                     std::min<size_t>((size_t)ntiles, 1024))))
            return ENQ_FAIL;
    } else {
        if (!grow_list(1) || !grow_items(1) || (!ordered && !grow_kslot(std::max<u32>(sc.lastSplit, 1)))) return ENQ_FAIL;
        cap = std::min<size_t>(F.flist_cap, 0xFFFFFFF0ull);
    }

    const int hbins = bp.hrows * fp.tiles_x;   // LDS histograms: the owned tile rows
    const bool ldsh = hbins <= LDS_HIST_MAX;
    const size_t hbytes = ldsh ? (size_t)hbins * sizeof(u32) : 0;
    const int gb = (int)((src.n + 256 * TPT - 1) / (256 * TPT));
    hipEvent_t e0, e1;
    u32 grid;
    for (int attempt = 0;; ++attempt) {
        nr_timing_begin_on(ctx, NRK_TRI_COUNT, &e0, &e1, sb);
        if (ordered) {
            if (ldsh) hipLaunchKernelGGL((k_free_count<true, true>), dim3(gb), dim3(256), hbytes, sb, bp, F.fcnt, ntiles, F.frect, F.frec);
            else hipLaunchKernelGGL((k_free_count<false, true>), dim3(gb), dim3(256), 0, sb, bp, F.fcnt, ntiles, F.frect, F.frec);
        } else if (ldsh) {
            hipLaunchKernelGGL((k_free_count<true>), dim3(gb), dim3(256), hbytes, sb, bp, F.fcnt, ntiles, F.frect, nullptr);
        } else {
            hipLaunchKernelGGL((k_free_count<false>), dim3(gb), dim3(256), 0, sb, bp, F.fcnt, ntiles, F.frect, nullptr);
        }
        NR_CHECK(hipGetLastError());
        nr_timing_end_on(ctx, NRK_TRI_COUNT, e0, e1, sb);

        const u32 seq = ++sc.planSeq;
        *seqOut = seq;
        nr_timing_begin_on(ctx, NRK_TRI_SCAN, &e0, &e1, sb);
        const u32 icap32 = (u32)std::min<size_t>(F.fitems_cap, 0xFFFFFFF0ull);
        // (an ordered batch uses no key slots, and its lists must fit the raster's LDS sort)
        const u32 kcap32 = ordered ? 0xFFFFFFFFu : (u32)std::min<size_t>(sc.kslot_cap / (TH * TW), 0xFFFFFFF0ull);
        const u32 maxc = ordered ? ORD_SORT_CAP : 0u;
        const u32 sat = sc.splitAt ? sc.splitAt : SPLIT_AT, dsl = sc.dslice ? sc.dslice : DSLICE;
        if (ntiles <= PLAN_T * PR_MAX || ordered) {   // (ordered: ntiles <= ORD_BIN_TILES)
            // the register plan: one 1024-thread workgroup, PR = tiles per
            // thread -> 4, 8 or 16 (PR 4: 107 VGPRs; PR 8 and 16 spill a few,
            // 4 and 39, at __launch_bounds__(1024)'s 128).  It needs a whole CU
            // (an ordered batch's plan beside the ordered raster therefore waits
            // for the raster's tail, which measured better than a 512-thread
            // instance that runs the chain earlier, beside it: C5 +10 %,
            // profiles/r03_c5/ab_plan512.txt).  A 256-thread multi-round plan
            // that fits beside a running k_vis was kept for large batches until
            // round 5 (C3 0.163 vs 0.172 ms then, profiles/r02_c3/ab_plan_r.txt);
            // with the faster raster the chain's count ends with the raster and
            // the wide plan is faster: a cold C3 frame (c3_animated) 0.157 ->
            // 0.150 ms (profiles/r05/ab_plan_wide.txt).
            const int per = (ntiles + PLAN_T - 1) / PLAN_T;
#define NR_PLAN_R(PP) hipLaunchKernelGGL((k_free_plan_r<PLAN_T, PP>), dim3(1), dim3(PLAN_T), 0, sb, F.fcnt, ntiles, \
                                         fp.tiles_x, fp.period, fp.mask, F.foff, F.fitems, F.fcur, F.dplan, F.d_hplan, \
                                         (u32)cap, icap32, seq, SLICE_TARGET, kcap32, sat, dsl, maxc)
            if (per <= 4) NR_PLAN_R(4); else if (per <= 8) NR_PLAN_R(8); else NR_PLAN_R(16);
#undef NR_PLAN_R
        }
        else
            hipLaunchKernelGGL(k_free_plan, dim3(1), dim3(1024), 0, sb, F.fcnt, ntiles, fp.tiles_x, fp.period,
                               fp.mask, F.foff, F.fitems, F.fcur, F.dplan, F.d_hplan, (u32)cap,
                               (u32)std::min<size_t>(F.fitems_cap, 0xFFFFFFF0ull), seq, SLICE_TARGET, kcap32, sat, dsl);
        NR_CHECK(hipGetLastError());
        nr_timing_end_on(ctx, NRK_TRI_SCAN, e0, e1, sb);

        if (!exact) {
            // grid-stride over the items.  The grid need not cover them all,
            // only fill the chip: one workgroup per item of a batch of known
            // totals, else the last validated batch's items + 25 % (>= 1024,
            // the chip's k_vis workgroup slots) -- not the capacity bound, whose
            // surplus workgroups (45 % of a C3 launch, 90 % of an 8-way share's)
            // were dispatched only to exit
            // (two or three items per workgroup in turn: C3 k_vis 138 -> 150 / 157 us,
            // profiles/r03_c3/ab_grid_div.txt)
            u64 g = F.fitems_cap;
            if (knownItems) g = knownItems;
            else if (sc.lastItems) g = std::max<u64>((u64)sc.lastItems + sc.lastItems / 4, 1024);
            grid = (u32)std::min<u64>(std::min<u64>(g, F.fitems_cap), 8192);
            break;
        }
        // exact: read the totals back; if the list or the items did not fit,
        // grow both and bin again (the plan kernel re-zeroed the counters)
        NR_CHECK(hipStreamSynchronize(sb));
        sc.lastPairs = plan_val(F, 0);
        sc.lastHeavy = plan_val(F, 5);
        sc.lastItems = plan_val(F, 1);
        sc.lastSplit = plan_val(F, 2);
        sc.lastN = (u64)src.n;
        grid = plan_val(F, 1);
        if (plan_val(F, 3)) break;
        if (ordered && plan_val(F, 6) > ORD_SORT_CAP) return ENQ_SORTED;
        if (attempt > 0 || !grow_list(plan_val(F, 0)) || !grow_items(plan_val(F, 1)) ||
            (!ordered && !grow_kslot(plan_val(F, 2)))) {
            nr_set_error_msg("triangle binning: pair list allocation failed");
            return ENQ_FAIL;
        }
        cap = std::min<size_t>(F.flist_cap, 0xFFFFFFF0ull);
    }

    nr_timing_begin_on(ctx, NRK_TRI_EMIT, &e0, &e1, sb);
    const bool xs = sb != sa && !e1;   // no timing events around the kernel
    hipEvent_t binStop = xs ? F.evBin : nullptr;
    hipEvent_t emitStop = ordered ? nullptr : binStop;   // (ordered: the list sort ends the binning)
    if (ldsh) hipExtLaunchKernelGGL(k_free_emit<true>, dim3(gb), dim3(256), (u32)hbytes, sb, nullptr, emitStop, 0, bp, F.foff, F.fcur, F.flist, ntiles, F.frect, (const u32*)F.dplan);
    else hipExtLaunchKernelGGL(k_free_emit<false>, dim3(gb), dim3(256), 0, sb, nullptr, emitStop, 0, bp, F.foff, F.fcur, F.flist, ntiles, F.frect, (const u32*)F.dplan);
    NR_CHECK(hipGetLastError());
    nr_timing_end_on(ctx, NRK_TRI_EMIT, e0, e1, sb);
    if (ordered) {   // each tile's list into submission order
        nr_timing_begin_on(ctx, NRK_TRI_SORT, &e0, &e1, sb);
        launch_tile_sort(F.foff, F.flist, F.dplan, ntiles, sb, binStop);
        NR_CHECK(hipGetLastError());
        nr_timing_end_on(ctx, NRK_TRI_SORT, e0, e1, sb);
    }
    if (sb != sa) {   // (a device-side hand-off instead, a polling kernel on the main queue, measured +15 % on
                      // an 8-way share and needs the two streams on separate hardware queues: removed in round 4)
        if (!xs) NR_CHECK(hipEventRecord(F.evBin, sb));
        NR_CHECK(hipStreamWaitEvent(sa, F.evBin, 0));
    }

    bool visDone = false;
    FrameParams fpt = fp;   // (timed: the raster stamps itself on the device clock)
    fpt.tstamp = nr_timing_stamp(ctx, NRK_TILE_RASTER);
    if (ordered) {   // one workgroup per tile, its list sorted in LDS
        launch_ordered_binned(fpt, F.flist, F.foff, F.dplan, F.frec, ntiles, sa, nullptr, F.evVis);
        NR_CHECK(hipGetLastError());
        visDone = true;
    } else if (grid > 0) {
        launch_vis_any(fpt, sc, VisArgs{F.fitems, F.flist, F.dplan, WarmCheck{nullptr, nullptr, nullptr, 0u, 0u, nullptr, 0u}},
                       grid, sa, nullptr, F.evVis, zmode, g);
        NR_CHECK(hipGetLastError());
        visDone = true;
    }
    if (!visDone) NR_CHECK(hipEventRecord(F.evVis, sa));
    F.visRecorded = true;
    return ENQ_OK;
}

// ---- warm binning ---------------------------------------------------------
// On unless SetWarmBinning(2).
static bool warm_on(const TriScratch& sc) { return sc.warmMode != 2; }
// Warm binning inline (main stream, right before the raster) or beside the
// previous raster (binning stream).  Inline when the rank's owned share of
// the batch is large and its frame share small: 1M triangles at 1080p
// 0.1001 -> 0.0985 ms per frame; beside the raster for small batches (C2
// 0.065 -> 0.058 ms), for the smaller shares, whose active binning blocks fit
// beside the raster (8-way 0.0505 -> 0.046-0.048 ms, 4-way -1 %;
// profiles/r04/ab_warm_blocks.txt), and -- since the fast clear left the
// raster HBM time to share -- for frame shares of >= 4 M pixels (C3 at 4K
// 0.130 -> 0.124 ms, its 2-way share 0.092 -> 0.077 ms;
// profiles/r05/ab_warm_beside.txt).  NR_WARM_INLINE: 1 always inline, 0
// always beside (A/B); inline by default under AMD_SERIALIZE_KERNEL.
static bool warm_inline(i64 n, int period, u64 mask, i64 W, i64 H) {
    static const int v = [] {
        const char* e = getenv("NR_WARM_INLINE");
        if (e) return atoi(e);
        // serialised dispatch: a binning beside the raster could not start
        // until the raster's token wait gave up (a second per frame)
        const char* ser = getenv("AMD_SERIALIZE_KERNEL");
        return ser && atoi(ser) != 0 ? 1 : 2;
    }();
    if (v != 2) return v != 0;
    const u64 m = period >= 64 ? mask : (mask & ((1ull << period) - 1ull));
    const f64 share = period == 1 ? 1.0 : (f64)__builtin_popcountll(m) / (f64)period;
    if ((f64)W * (f64)H * share >= 4.0e6) return false;
    return n >= 65536 && (f64)n * share >= 300000.0;
}

// Keeps the tile offsets, work items and plan totals of a validated binning
// of `tb` under `key` (binning set F, which held room for them) as the
// context's warm schedule: device copies on the main stream, after the
// batch's raster; the set's next binning waits for them (F.evVis).
static void sched_capture(RenderContext* ctx, TriScratch::FreeSet& F, const BinKey& key, const TriangleBuffer* tb,
                          int ntiles, u32 pairs, u32 items, u32 heavy, u32 split, u64 n) {
    TriScratch& sc = ctx->tri;
    if (!warm_on(sc) || !tb) return;
    auto& S = sc.sched;
    hipStream_t sa = ctx->stream;
    main_after_side_binning(ctx);   // (a late warm binning may still read S.off)
    S.valid = false;
    if (S.off_cap < (size_t)ntiles + 1 || S.items_cap < std::max<size_t>(items, 1) || !S.dplan) {
        NR_CHECK(hipStreamSynchronize(sa));   // a queued warm batch may still read the old arrays
        NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(ctx->device)));
        u32* ob[1] = {S.off};
        if (!grow_set(ob, &S.off_cap, (size_t)ntiles + 1)) return;
        S.off = ob[0];
        uint4* ib[1] = {S.items};
        if (!grow_set(ib, &S.items_cap, std::max<size_t>(items, 1))) return;
        S.items = ib[0];
        if (!S.dplan) NR_CHECK(hipMalloc(&S.dplan, 4 * sizeof(u32)));
    }
    if (!S.ready) S.ready = sync_event();
    NR_CHECK(hipMemcpyAsync(S.off, F.foff, ((size_t)ntiles + 1) * sizeof(u32), hipMemcpyDeviceToDevice, sa));
    if (items) NR_CHECK(hipMemcpyAsync(S.items, F.fitems, (size_t)items * sizeof(uint4), hipMemcpyDeviceToDevice, sa));
    NR_CHECK(hipMemcpyAsync(S.dplan, F.dplan, 4 * sizeof(u32), hipMemcpyDeviceToDevice, sa));
    NR_CHECK(hipEventRecord(S.ready, sa));
    NR_CHECK(hipEventRecord(F.evVis, sa));   // the set is rewritten only after the copies
    F.visRecorded = true;
    S.valid = true;
    S.tbUid = tb->uid;
    S.key = key;
    S.pairs = pairs; S.nitems = items; S.heavy = heavy; S.split = split; S.n = n;
    static u64 g_gen = 0;
    S.gen = ++g_gen;
    S.waitReady = true;
}

static bool sched_matches(const TriScratch& sc, const TriangleBuffer* tb, const BinKey& key) {
    return warm_on(sc) && tb && sc.sched.valid && sc.sched.tbUid == tb->uid && !sc.capOverride &&
           memcmp(&sc.sched.key, &key, sizeof key) == 0 &&
           std::find(sc.warmBanned.begin(), sc.warmBanned.end(), tb->uid) == sc.warmBanned.end();
}

// Loose binning (round 6): the buffer of the schedule drawn under another
// transform (same frame, shard pattern and depth mode), where no vertex moves
// more than LOOSE_PX on screen from where the schedule's transform put it --
// a moving or jittering scene.  Every tile's pair count then changes by the
// triangles that cross its edges; the loose ranges (loose_cap) hold them, so
// the batch bins in one pass (k_bin_warm) instead of count -> plan -> emit.
// The displacement bound: the two affine maps differ by an affine map, whose
// largest displacement over the buffer's bounding box is at one of its corners.
constexpr f64 LOOSE_PX = 2.0;
static bool loose_matches(const TriScratch& sc, const TriangleBuffer* tb, const BinKey& key) {
    const auto& S = sc.sched;
    if (!warm_on(sc) || !tb || !S.valid || S.tbUid != tb->uid || sc.capOverride) return false;
    if (S.key.W != key.W || S.key.H != key.H || S.key.period != key.period || S.key.mask != key.mask) return false;
    if (std::find(sc.warmBanned.begin(), sc.warmBanned.end(), tb->uid) != sc.warmBanned.end() ||
        std::find(sc.looseBanned.begin(), sc.looseBanned.end(), tb->uid) != sc.looseBanned.end())
        return false;
    const f64* b = tb->bbox;
    if (!(std::isfinite(b[0]) && std::isfinite(b[1]) && std::isfinite(b[2]) && std::isfinite(b[3]))) return false;
    for (int c = 0; c < 4; ++c) {
        const f64 x = b[(c & 1) ? 2 : 0], y = b[(c & 2) ? 3 : 1];
        f64 ax, ay, bx, by;
        nr_xform(S.key.m, x, y, ax, ay);
        nr_xform(key.m, x, y, bx, by);
        if (!(std::fabs(ax - bx) <= LOOSE_PX && std::fabs(ay - by) <= LOOSE_PX)) return false;
    }
    return true;
}

// A warm batch that failed its checks (k_vis WarmCheck: the raster then ran
// over every triangle, so its frame is right) -- read at the next call into
// the context: latch an error, drop the schedule (the next draw bins cold),
// and after a binning-check failure bin that buffer cold from now on.
static void warm_poll(RenderContext* ctx) {
    TriScratch& sc = ctx->tri;
    if (!sc.hfail) return;
    const u32 f = __atomic_load_n(sc.hfail, __ATOMIC_ACQUIRE);
    if (!f) return;
    const u32 w1 = __atomic_load_n(&sc.hfail[1], __ATOMIC_ACQUIRE), w2 = __atomic_load_n(&sc.hfail[2], __ATOMIC_ACQUIRE);
    const u32 w3 = __atomic_load_n(&sc.hfail[3], __ATOMIC_ACQUIRE);
    __atomic_store_n(sc.hfail, 0u, __ATOMIC_RELEASE);
    ++sc.warmFailures;
    char msg[320];
    if (f == 4) {   // a tile over its loose range: the schedule stays, the buffer is not binned loose again
        if (sc.sched.valid) sc.looseBanned.push_back(sc.sched.tbUid);
        snprintf(msg, sizeof msg, "triangle batch: a loose warm binning gave tile %u %u pairs, room for %u; that "
                                  "tile was rasterised from all the batch's triangles and the buffer is no longer "
                                  "binned loose", w1, w2, w3);
        nr_set_error_msg(msg);
        return;
    }
    if (f != 2 && sc.sched.valid) sc.warmBanned.push_back(sc.sched.tbUid);
    sc.sched.valid = false;
    if (f == 2)
        snprintf(msg, sizeof msg, "triangle batch: a raster's wait for its warm binning timed out; the batch was "
                                  "rasterised from all its triangles (under serialised kernel dispatch -- a "
                                  "profiler's counter passes, AMD_SERIALIZE_KERNEL -- set NR_WARM_INLINE=1)");
    else if (f == 1)
        snprintf(msg, sizeof msg, "triangle batch: a warm binning put a tile over its range (tag %u of batch %u); the "
                                  "batch was rasterised from all its triangles and the buffer bins cold from now on",
                 w2, w3);
    else
        snprintf(msg, sizeof msg, "triangle batch: a warm binning gave tile %u %u pairs, expected %u; that tile was "
                                  "rasterised from all the batch's triangles and the buffer bins cold from now on",
                 w1, w2, w3);
    nr_set_error_msg(msg);
}

// A warm batch: one binning kernel into the schedule's ranges (binning set
// `si`: cursors and pair list), then k_vis over the schedule's items.
// Same-queue hand-off from a warm binning beside the raster to the raster
// (NR_GATE, default on): the binning stream ends the batch's binning with
// k_gate_signal storing the set's next token, and the main stream runs
// k_gate_wait -- one thread polling the token -- right before the raster, in
// place of a cross-queue event wait, whose wake-up cost ~10 us per frame
// after a binning that had long finished (8-way share kernel trace,
// profiles/r04/ab_any_order.txt).  The binning kernel's completion (kernel
// boundary on the binning stream) makes its pairs visible before the token is
// stored.  k_gate_wait also hands the raster its plan words (a copy of the
// schedule's); should the token not arrive within a second, the copy says
// "did not fit" (the raster does nothing) and the host latches an error --
// no wave polls forever, no raster reads a half-written list.  The binning is
// enqueued before the wait on the host, so even two streams sharing one
// hardware queue cannot deadlock.  (A timed-out raster runs its fallback and
// reports, WarmCheck.)
__global__ void k_gate_signal(u32* __restrict__ gate, u32 tok) {
    if (threadIdx.x == 0) __hip_atomic_store(gate, tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Testing (SetWarmFaultInjection 4): holds the binning stream for 1.5 s before
// a warm binning, so that the raster's token wait (1 s) gives up first and the
// binning lands after the raster's fallback (one thread, bounded).
__global__ void k_delay_binning() {
    if (threadIdx.x != 0) return;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    while (__builtin_amdgcn_s_memrealtime() - t0 < 150000000ull) __builtin_amdgcn_s_sleep(127);
}
__global__ void k_gate_wait(const u32* __restrict__ gate, u32 tok, const u32* __restrict__ splan,
                            u32* __restrict__ gplan) {
    if (threadIdx.x != 0) return;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    bool ok = true;
    while (__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tok) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
            ok = false;
            break;
        }
    }
    for (int k = 0; k < 4; ++k) gplan[k] = (k == 3 && !ok) ? 0u : splan[k];   // {pairs, items, slices, fits}
}

// The binning blocks (256 * TPT triangles) of a schedule with a cluster that
// may reach an owned tile: cluster_may_touch on the host over the buffer's
// cluster boxes, widened by two rows and eight columns each side (a superset
// of the device test, which still runs per wave).  Built once per schedule:
// the warm binning of a rank then launches only these workgroups (an 8-way
// share: about 1 in 7).
static bool host_cluster_may_touch(const BinParams& bp, const f64* box) {
    f64 y0 = INFINITY, y1 = -INFINITY, x0 = INFINITY, x1 = -INFINITY;
    bool huge = false;   // (tri_tiles' full-width rule, as the device test)
    for (int c = 0; c < 4; ++c) {
        f64 sx, sy;
        nr_xform(bp.m, box[(c & 1) ? 2 : 0], box[(c & 2) ? 3 : 1], sx, sy);
        if (!std::isfinite(sx) || !std::isfinite(sy)) return true;
        huge = huge || std::fabs(sx) > 5e6 || std::fabs(sy) > 5e6;
        y0 = std::min(y0, sy); y1 = std::max(y1, sy); x0 = std::min(x0, sx); x1 = std::max(x1, sx);
    }
    if (!huge && (x1 < -12.0 || x0 > (f64)bp.W + 12.0)) return false;
    const f64 r0 = std::max(std::ceil(y0) - 3.0, 0.0), r1 = std::min(std::ceil(y1) + 3.0, (f64)bp.H);
    if (!(r0 < r1)) return false;
    if (bp.period == 1) return true;
    const int ty0 = (int)r0 / TH, ty1 = ((int)r1 - 1) / TH;
    if (ty1 >= ty0 + 64) return true;
    for (int ty = ty0; ty <= ty1; ++ty)
        if ((bp.mask >> (ty % bp.period)) & 1ull) return true;
    return false;
}
static void warm_blocks(RenderContext* ctx, const BinParams& bp, const TriangleBuffer* tb) {
    auto& S = ctx->tri.sched;
    if (S.blocksGen == S.gen) return;
    const i64 n = bp.src.n, per = 256 * TPT, nb = (n + per - 1) / per;
    const i64 nc = (i64)tb->hcbox.size() / 4;
    // (the previous upload from this vector was ordered before any warm
    // binning of the previous schedule, all of which the sync below or the
    // stream order has passed)
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    std::vector<u32>& act = S.hblocks;
    act.clear();
    act.reserve((size_t)nb);
    bool anyCull = false;
    for (i64 b = 0; b < nb; ++b) {
        bool any = false;
        for (i64 c = b * (per / NR_CLUSTER); c < std::min<i64>((b + 1) * (per / NR_CLUSTER), nc); ++c) {
            const bool t = host_cluster_may_touch(bp, tb->hcbox.data() + c * 4);
            any = any || t;
            anyCull = anyCull || !t;
        }
        if (any || nc == 0) act.push_back((u32)b);
    }
    // every cluster may reach an owned tile (an unsharded frame with the mesh
    // on screen): the device's cluster tests could cull nothing worth a test
    S.anyCull = anyCull;
    if (S.blocks_cap < std::max<size_t>(act.size(), 1)) {
        NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(ctx->device)));
        if (S.blocks) NR_CHECK(hipFree(S.blocks));
        S.blocks_cap = std::max<size_t>((size_t)nb, 1);
        NR_CHECK(hipMalloc(&S.blocks, S.blocks_cap * sizeof(u32)));
    }
    // (ordered on the main stream before any warm binning of this schedule, S.ready)
    if (!act.empty())
        NR_CHECK(hipMemcpyAsync(S.blocks, act.data(), act.size() * sizeof(u32), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipEventRecord(S.ready, ctx->stream));
    S.waitReady = true;
    S.nblocks = (u32)act.size();
    S.blocksGen = S.gen;
}

// loose: the batch's transform differs from the schedule's (loose_matches):
// bin into the schedule's loose ranges, cursors from 0 (k_bin_warm), and let
// k_vis slice each tile's actual count.
static bool warm_enqueue(RenderContext* ctx, const FrameParams& fp, const BinParams& bp, const TriangleBuffer* tb,
                         bool loose = false) {
    const f64* tbCbox = tb->cbox;
    TriScratch& sc = ctx->tri;
    auto& S = sc.sched;
    hipStream_t sa = ctx->stream;
    hipStream_t sb = warm_inline(bp.src.n, fp.period, fp.mask, fp.W, fp.H) ? sa : nr_bin_stream_for(ctx->device);
    const int ntiles = fp.tiles_x * fp.tiles_y;
    const int si = sc.fnext;
    sc.fnext = (sc.fnext + 1) % BIN_SETS;
    TriScratch::FreeSet& F = sc.fset[si];
    if (!F.evBin) { F.evBin = sync_event(); F.evVis = sync_event(); }
    if (sb == sa) main_after_side_binning(ctx);
    if (!sc.hfail) {
        NR_CHECK(hipHostMalloc((void**)&sc.hfail, 4 * sizeof(u32), hipHostMallocMapped | hipHostMallocCoherent));
        for (int k = 0; k < 4; ++k) sc.hfail[k] = 0;
        NR_CHECK(hipHostGetDevicePointer((void**)&sc.dfail, sc.hfail, 0));
    }
    // cursors [0, ntiles), then the batch checks {report tag, error tag} (WarmCheck)
    const size_t tneed = std::max<size_t>((size_t)ntiles + 2, TILE_ARR);
    if (loose && S.off2Gen != S.gen)   // (a bound of the loose list: every tile's loose_cap)
        S.pairs2 = (u64)S.pairs + S.pairs / 4 + 64ull * (u64)(ntiles + 1);
    const size_t lneed = std::max<size_t>(loose ? (size_t)S.pairs2 : (size_t)S.pairs, 1);
    if (loose && lneed >= 0xF0000000ull) return false;
    const bool grow = F.ftile_cap < tneed || !F.fcnt || F.flist_cap < lneed ||
                      sc.kslot_cap < std::max<size_t>(S.split, 1) * (TH * TW) || sc.fdone_cap < (size_t)ntiles + 1;
    if (grow) {   // (first use of a set, or a larger schedule: rare)
        NR_CHECK(hipStreamSynchronize(sa));
        NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(ctx->device)));
        u32* tb3[3] = {F.fcnt, F.foff, F.fcur};
        const size_t oldcap = F.ftile_cap;
        if (!grow_set(tb3, &F.ftile_cap, tneed)) return false;
        F.fcnt = tb3[0]; F.foff = tb3[1]; F.fcur = tb3[2];
        if (F.ftile_cap != oldcap) {
            NR_CHECK(hipMemsetAsync(F.fcnt, 0, F.ftile_cap * sizeof(u32), sa));
            F.curGen = 0;
        }
        u32* lb[1] = {F.flist};
        if (!grow_set(lb, &F.flist_cap, lneed)) return false;
        F.flist = lb[0];
        u64* kb[1] = {sc.kslot};
        if (!grow_set(kb, &sc.kslot_cap, std::max<size_t>(S.split, 1) * (TH * TW))) return false;
        sc.kslot = kb[0];
        u32* db[1] = {sc.fdone};
        const size_t olddone = sc.fdone_cap;
        if (!grow_set(db, &sc.fdone_cap, (size_t)ntiles + 1)) return false;
        sc.fdone = db[0];
        if (sc.fdone_cap != olddone) NR_CHECK(hipMemsetAsync(sc.fdone, 0, sc.fdone_cap * sizeof(u32), sa));
    }
    // (the active blocks are found under the schedule's own transform: a loose batch launches them all)
    if (tbCbox && !loose) warm_blocks(ctx, bp, tb);
    if (loose && S.off2Gen != S.gen) {   // the schedule's loose ranges, once (main stream, before S.ready)
        if (S.off2_cap < (size_t)ntiles + 1) {
            NR_CHECK(hipStreamSynchronize(sa));
            NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(ctx->device)));
            u32* ob[1] = {S.off2};
            if (!grow_set(ob, &S.off2_cap, (size_t)ntiles + 1)) return false;
            S.off2 = ob[0];
        }
        hipLaunchKernelGGL(k_loose_off, dim3(1), dim3(1024), 0, sa, (const u32*)S.off, S.off2, ntiles);
        NR_CHECK(hipGetLastError());
        NR_CHECK(hipEventRecord(S.ready, sa));
        S.waitReady = true;
        S.off2Gen = S.gen;
    }
    if (F.visRecorded && sb != sa) NR_CHECK(hipStreamWaitEvent(sb, F.evVis, 0));
    if (S.waitReady && sb != sa) NR_CHECK(hipStreamWaitEvent(sb, S.ready, 0));
    S.waitReady = false;
    // cursors: epoch e of this schedule on this set (k_bin_warm); zeroed for a
    // new schedule, after a cold batch on the set, or before they could wrap
    // (loose: from zero every batch -- they count the tile's pairs)
    if (loose || F.curGen != S.gen || (u64)(F.curEpoch + 1) * std::max<u32>(S.pairs, 1) >= 0xF0000000ull) {
        NR_CHECK(hipMemsetAsync(F.fcur, 0, ((size_t)ntiles + 2) * sizeof(u32), sb));   // (and the check words)
        F.curGen = loose ? 0 : S.gen;
        F.curEpoch = 0;
    }
    const int hbins = bp.hrows * fp.tiles_x;
    const bool ldsh = 2 * hbins <= LDS_HIST_MAX;
    const int gb = (int)((bp.src.n + 256 * TPT - 1) / (256 * TPT));
    hipEvent_t e0, e1;
    nr_timing_begin_on(ctx, NRK_TRI_EMIT, &e0, &e1, sb);
    const bool gated = sb != sa && !e1;   // same-queue hand-off (k_gate_wait) instead of an event wait
    if (gated && !F.gate) {
        NR_CHECK(hipMalloc(&F.gate, 4 * sizeof(u32)));
        NR_CHECK(hipMalloc(&F.gplan, 4 * sizeof(u32)));
        // zeroed in order on the signalling stream: a plain hipMemset (null
        // stream) may still be pending when the first signal lands and zero
        // it -- that raster's wait then times out (seen with a cold-batch gate
        // on a busy device, profiles/r05/ab_cold_gate.txt)
        NR_CHECK(hipMemsetAsync(F.gate, 0, 4 * sizeof(u32), sb));
        // and done before the first k_gate_wait (main stream) reads the word:
        // uninitialised memory holding a token would let the raster go early
        // (once per set)
        NR_CHECK(hipStreamSynchronize(sb));
        F.gateTok = 0;
    }
    const bool xs = sb != sa && !e1 && !gated;
    hipEvent_t binStop = xs ? F.evBin : nullptr;
    const u32 epoch = loose ? 0u : F.curEpoch++;
    if (++sc.warmTag == 0) sc.warmTag = 1;
    const u32 tag = sc.warmTag;
    u32* const wstat = F.fcur + ntiles;   // {report tag, error tag} (WS_REP, WS_TAG)
    const int inject = sc.warmInject;
    sc.warmInject = 0;
    // cluster culling of the rank's tile rows, and only the schedule's active blocks launched
    const f64* cbox = S.anyCull || loose ? tbCbox : nullptr;
    const bool useBlocks = cbox && !loose && S.blocksGen == S.gen;
    const u32* const binOff = loose ? S.off2 : S.off;
    const u32* blocks = useBlocks ? S.blocks : nullptr;
    const int grid = useBlocks ? (int)S.nblocks : gb;
    if (inject == 4 && gated) hipLaunchKernelGGL(k_delay_binning, dim3(1), dim3(64), 0, sb);
    if (grid > 0) {
        if (ldsh)
            hipExtLaunchKernelGGL(k_bin_warm<true>, dim3(grid), dim3(256), (u32)(2 * hbins * sizeof(u32)), sb, nullptr,
                                  binStop, 0, bp, binOff, F.fcur, F.flist, wstat, tag, epoch, cbox, blocks, (u32)inject,
                                  (u32)loose);
        else
            hipExtLaunchKernelGGL(k_bin_warm<false>, dim3(grid), dim3(256), 0, sb, nullptr, binStop, 0, bp, binOff,
                                  F.fcur, F.flist, wstat, tag, epoch, cbox, blocks, (u32)inject, (u32)loose);
    } else if (binStop) {
        NR_CHECK(hipEventRecord(F.evBin, sb));
    }
    NR_CHECK(hipGetLastError());
    nr_timing_end_on(ctx, NRK_TRI_EMIT, e0, e1, sb);
    const u32* visPlan = S.dplan;
    if (gated) {
        if (++F.gateTok == 0) F.gateTok = 1;   // (the word starts at 0)
        if (inject != 2)   // (2: the token is withheld -- tests of the timeout)
            hipLaunchKernelGGL(k_gate_signal, dim3(1), dim3(64), 0, sb, F.gate, F.gateTok);
        hipLaunchKernelGGL(k_gate_wait, dim3(1), dim3(64), 0, sa, (const u32*)F.gate, F.gateTok, (const u32*)S.dplan,
                           F.gplan);
        NR_CHECK(hipGetLastError());
        visPlan = F.gplan;
        sc.sideGated = true;
    } else if (sb != sa) {
        if (!xs) NR_CHECK(hipEventRecord(F.evBin, sb));
        NR_CHECK(hipStreamWaitEvent(sa, F.evBin, 0));
    }
    // this batch's totals pick the k_vis variant (launch_vis)
    sc.lastN = S.n; sc.lastPairs = S.pairs; sc.lastHeavy = S.heavy; sc.lastItems = S.nitems; sc.lastSplit = S.split;
    const int zmode = fp.depthTest ? (fp.depthWrite ? 1 : 2) : 0;
    bool visDone = false;
    if (S.nitems > 0) {
        FrameParams fpt = fp;   // (timed: the raster stamps itself on the device clock)
        fpt.tstamp = nr_timing_stamp(ctx, NRK_TILE_RASTER);
        const WarmCheck wc{wstat, F.fcur, binOff, tag, epoch + 1, sc.dfail, (u32)loose};
        launch_vis_any(fpt, sc, VisArgs{S.items, F.flist, visPlan, wc}, std::min<u32>(S.nitems, 8192), sa, nullptr,
                       F.evVis, zmode, fp.src.gouraud != 0);
        NR_CHECK(hipGetLastError());
        visDone = true;
    }
    if (!visDone) NR_CHECK(hipEventRecord(F.evVis, sa));
    F.visRecorded = true;
    return true;
}

}  // namespace

// ordered: the batch is rasterised by the ordered raster (blending, Z test
// without write...): the same binning, each tile's list sorted in LDS.
void draw_free(RenderContext* ctx, const TriSrc& src, TriangleBuffer* tb, bool callerOwned, bool ordered) {
    FrameParams fp = frame_params(ctx, src);
    if (ctx->frameOutput && fp.pendColor) {
        const size_t n = (size_t)nr_frame_bytes(ctx);
        if (n <= ctx->frameU8cap) fp.frameU8 = ctx->frameU8;
    }
    if (!ordered && (fp.pendColor || fp.pendDepth))   // fast clear: the empty tiles' clears stay pending (k_vis)
        fp.tileStamp = tile_stamps(ctx, (i64)fp.tiles_x * fp.tiles_y), fp.tileEpoch = ctx->tileEpoch;
    BinParams bp;
    bp.src = src;
    for (int k = 0; k < 6; ++k) bp.m[k] = ctx->m[k];
    bp.W = ctx->width; bp.H = ctx->height; bp.tiles_x = fp.tiles_x;
    bp.period = fp.period; bp.mask = fp.mask;
    set_owned_rows(bp, fp.tiles_y);
    // fragment counting reads a counter back anyway: run exact (synchronous);
    // so does a batch from the caller's device arrays: a deferred overflow
    // re-run (settle, at the next call) could read them after the caller has
    // synchronised and released or rewritten them
    const bool exact = fp.fragCounter != nullptr || callerOwned;
    TriScratch& sc = ctx->tri;
    // A TriangleBuffer drawn again under the binning key of its last validated
    // draw has the same pair total: the list is sized to hold it, so the plan's
    // capacity check cannot fail and the batch needs no validation (no host
    // wait for its plan kernel at the next call: the host runs ahead).
    const BinKey key = bin_key(bp);
    // Only unsharded batches: a sharded frame's raster is short, and a binning
    // chain issued at once runs beside it and is starved (measured: 1 GPU C3
    // 0.1640 -> 0.1614 ms, C2 0.0685 -> 0.062 ms with known sizes; an emulated
    // rank share of 4 / 8 shards 0.066 -> 0.076 / 0.054 -> 0.062 ms, where the
    // host wait on the plan paces the binning; profiles/r02_c3/ab_known.txt).
    // (ordered batches are always validated: their plan also checks the list lengths)
    const bool known = !ordered && fp.period == 1 && tb && tb->known &&
                       !sc.capOverride && memcmp(&tb->knownKey, &key, sizeof key) == 0;
    if (known && !exact) {   // this batch's totals pick the k_vis variant (launch_vis)
        sc.lastN = (u64)src.n;
        sc.lastPairs = tb->knownPairs;
        sc.lastHeavy = tb->knownHeavy;
        sc.lastItems = tb->knownItems;
        sc.lastSplit = tb->knownSplit;
    }
    // warm: the schedule kept from this buffer's last validated binning under this key
    warm_poll(ctx);
    if (!ordered && !exact && sched_matches(sc, tb, key)) {
        if (warm_enqueue(ctx, fp, bp, tb)) {
            ctx->lastPath = 1;
            ++sc.warmBatches;
            finish_batch(ctx, fp);
        }
        return;
    }
    if (!ordered && !exact && loose_matches(sc, tb, key) && warm_enqueue(ctx, fp, bp, tb, true)) {
        ctx->lastPath = 1;
        ++sc.warmBatches;
        ++sc.looseBatches;
        finish_batch(ctx, fp);
        return;
    }
    const int si = sc.fnext;
    sc.fnext = (sc.fnext + 1) % BIN_SETS;
    u32 seq = 0;
    static const bool pipeOn = [] {   // NR_BIN_PIPE=0: bin on the main stream (A/B, isolated kernel times)
        const char* e = getenv("NR_BIN_PIPE");
        return e ? atoi(e) != 0 : true;
    }();
    // A batch issued to an idle main stream (the first frame after a readback
    // or a Flush) has no raster to overlap its binning with: it bins in line
    // on the main stream, with the wide plan kernel, and k_vis follows without
    // a cross-queue wait (whose wake-up took ~15 us in the kernel trace,
    // profiles/r02h_c3).
    bool idle = false;
    if (pipeOn && tb != nullptr && !exact) {
        const hipError_t q = hipStreamQuery(ctx->stream);
        idle = q == hipSuccess;
        if (q == hipErrorNotReady) (void)hipGetLastError();   // an answer, not a failure
        else if (q != hipSuccess) NR_CHECK(q);                 // a real asynchronous error: latch it
    }
    sc.fset[si].curGen = 0;   // (its cursors will hold this batch's counts)
    const int r = free_enqueue(ctx, src, fp, bp, exact, si, pipeOn && tb != nullptr && !exact && !idle, &seq,
                               known ? tb->knownPairs : 0, known ? tb->knownItems : 0, idle, known ? tb->knownSplit : 0,
                               ordered);
    if (r == ENQ_FAIL) return;
    if (r == ENQ_SORTED) {   // (exact) a tile list too long for the LDS sort
        fp.tileStamp = nullptr;   // (the ordered raster writes every tile)
        draw_ordered_sorted(ctx, src, fp, bp);
        return;
    }
    const int ntiles = fp.tiles_x * fp.tiles_y;
    if (exact) {
        if (!ordered) {
            record_known(tb, key, (u32)sc.lastPairs, sc.lastHeavy, sc.lastItems, sc.lastSplit);
            sched_capture(ctx, sc.fset[si], key, tb, ntiles, (u32)sc.lastPairs, sc.lastItems, sc.lastHeavy,
                          sc.lastSplit, (u64)src.n);
        }
    } else if (known) {
        sched_capture(ctx, sc.fset[si], key, tb, ntiles, tb->knownPairs, tb->knownItems, tb->knownHeavy,
                      tb->knownSplit, (u64)src.n);
    } else {
        PendingBatch* pb = new PendingBatch{src, fp, bp, si, seq, tb, key, ordered};
        ctx->pendingBatch = pb;
    }
    ctx->lastPath = ordered ? 2 : 1;
    finish_batch(ctx, fp);
}

// Validates the last asynchronously sized batch of `ctx`: waits for its plan
// kernel (usually long finished), and if the pair list did not fit, re-runs
// the batch with an exact allocation.  Called at the start of every API
// entry point that enqueues work on, or reads, the context's buffers, so the
// re-run is ordered before anything that depends on the batch.
void settle(RenderContext* ctx) {
    warm_poll(ctx);
    PendingBatch* pb = reinterpret_cast<PendingBatch*>(ctx->pendingBatch);
    if (!pb) return;
    ctx->pendingBatch = nullptr;
    TriScratch& sc = ctx->tri;
    TriScratch::FreeSet& F = sc.fset[pb->set];
    // wait for the batch's plan (usually long finished): it writes its totals
    // into pinned host memory, each word tagged with the batch's sequence
    // number -- polling them avoids an event record per batch (each costs a
    // multi-microsecond bubble on the stream)
    const u32 want = pb->seq;
    for (u64 spin = 0; !plan_ready(F, want); ++spin) {
        if ((spin & 1023) == 1023) {
            const bool idle = hipStreamQuery(ctx->stream) != hipErrorNotReady &&
                              hipStreamQuery(nr_bin_stream_for(ctx->device)) != hipErrorNotReady;
            if (idle && !plan_ready(F, want)) {
                nr_set_error_msg("triangle batch: plan result missing (stream idle or failed)");
                delete pb;
                return;
            }
            std::this_thread::yield();
        }
    }
    sc.lastN = (u64)pb->src.n;
    sc.lastPairs = plan_val(F, 0);
    sc.lastHeavy = plan_val(F, 5);
    sc.lastItems = plan_val(F, 1);
    sc.lastSplit = plan_val(F, 2);
    if (!pb->ordered) {   // exact totals, fitted or not
        record_known(pb->tb, pb->key, plan_val(F, 0), plan_val(F, 5), plan_val(F, 1), plan_val(F, 2));
        if (plan_val(F, 3))   // it fitted: its offsets and items are the buffer's schedule under this key
            sched_capture(ctx, F, pb->key, pb->tb, pb->fp.tiles_x * pb->fp.tiles_y, plan_val(F, 0), plan_val(F, 1),
                          plan_val(F, 5), plan_val(F, 2), (u64)pb->src.n);
    }
    if (!plan_val(F, 3)) {
        // overflow (or, ordered, a tile list too long for the LDS sort): the
        // batch's later kernels did nothing; re-run it exactly on the main
        // stream, after everything queued so far
        NR_CHECK(hipEventSynchronize(F.evVis));
        u32 seq = 0;
        const bool sorted = pb->ordered && plan_val(F, 6) > ORD_SORT_CAP;
        int rr = ENQ_SORTED;
        if (sorted || (rr = free_enqueue(ctx, pb->src, pb->fp, pb->bp, true, pb->set, false, &seq, 0, 0, false, 0,
                                         pb->ordered)) == ENQ_SORTED)
            rerun_ordered_sorted(ctx, pb->src, pb->fp, pb->bp);   // (the context's flags are left as they are now)
        else if (rr == ENQ_OK && !pb->ordered) {   // the exact re-run's binning is the buffer's schedule under this key
            record_known(pb->tb, pb->key, (u32)sc.lastPairs, sc.lastHeavy, sc.lastItems, sc.lastSplit);
            sched_capture(ctx, F, pb->key, pb->tb, pb->fp.tiles_x * pb->fp.tiles_y, (u32)sc.lastPairs, sc.lastItems,
                          sc.lastHeavy, sc.lastSplit, (u64)pb->src.n);
        }
    }
    delete pb;
}

}  // namespace nrtri

#if NR_PROBE
extern "C" {
// probe build only: clear / read the k_vis per-item clocks (8 u64 per item)
void NrProbeReset() {
    const unsigned int z = 0;
    NR_CHECK(hipDeviceSynchronize());
    NR_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(nrtri::nr_probe_n), &z, sizeof z));
}
i64 NrProbeRead(unsigned long long* out, i64 maxItems) {
    unsigned int n = 0;
    NR_CHECK(hipDeviceSynchronize());
    NR_CHECK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(nrtri::nr_probe_n), sizeof n));
    const i64 m = std::min<i64>(std::min<i64>((i64)n, maxItems), nrtri::PROBE_MAX);
    NR_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(nrtri::nr_probe_buf), (size_t)m * 8 * sizeof(unsigned long long)));
    return m;
}
}
#endif
