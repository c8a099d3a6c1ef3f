// nr_tri_ordered.hip — in-order tiled raster: correct for every batch
// (alpha blending, Z test without write, colour transforms), the general
// path behind DrawTriangles*.
//
//   1 k_tri_count   per triangle: number of 64x32 tiles its bbox touches
//   2 scan          exclusive sum of the counts (hipcub)
//   3 k_tri_emit    (tile, triangle) pairs, written in triangle order
//   4 sort          stable radix sort by tile: each tile's list stays in
//                   submission order (painter's order is preserved)
//   5 k_tile_ranges start/end of each tile's list
//   6 k_tile_raster one 512-thread workgroup per tile; the tile's colour and
//                   Z live in registers (8 waves, each a 32 x 8 block: 4
//                   pixels per lane) for the whole list.  Per 64-triangle chunk the setup and the exact
//                   per-row coverage spans are staged in LDS, then each wave
//                   walks the chunk in order and blends its covered lanes
//                   (ApplyPixel, cpp:529-547).  The tile is read once and
//                   written once; a pending uniform clear is applied on chip.
#include "nr_tri.h"

#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

namespace nrtri {
namespace {

constexpr int RPW = 4;           // steps per wave: a lane holds RPW pixels of the tile in registers
constexpr int NWAVE = 8;         // waves per tile
constexpr int WG = NWAVE * 64;   // 512 threads
constexpr int CH = 64;           // triangles staged per chunk
// Wave blocks: a wave owns a block of BW columns x RPW * SR rows of the tile
// (BW * SR = 64 lanes; step r of lane l is the pixel (l % BW, r * SR + l / BW)
// of the block).  Square-ish blocks cut the (triangle, wave) units a large
// triangle's edges cross: C5 needs 6.28 M units with 64 x 4 blocks, 5.09 M with
// 32 x 8 and 4.77 M with 16 x 16 (counted from the scene on the CPU).  Measured
// (C5 k_tile_raster): 778 us at 64 x 4, 715 us at 32 x 8, 746 us at 16 x 16 (its
// masks take four window ballots and more span-phase work per chunk), so 32 x 8
// (profiles/r03_c5/ab_blocks.txt).
constexpr int BW = 32;           // block columns (64, 32 and 16 measured)
constexpr int SR = 64 / BW;      // rows per step
constexpr int NQ = TW / BW;      // column windows of the tile
static_assert(BW * SR == 64 && NQ * (TH / (RPW * SR)) == NWAVE, "wave blocks tile the tile");

__global__ __launch_bounds__(256) void k_tri_count(const BinParams bp, unsigned long long* __restrict__ cnt,
                                                   f64* __restrict__ rec) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= bp.src.n) return;
    f64 sx[3], sy[3];
    tri_screen(bp.src, bp.m, t, sx, sy);
    int tx0, tx1, ty0, ty1;
    unsigned long long c = 0;
    if (tri_tiles(sx, sy, bp.W, bp.H, tx0, tx1, ty0, ty1)) {
        int rows = 0;
        for (int ty = ty0; ty <= ty1; ++ty) rows += owned_row(ty, bp.period, bp.mask) ? 1 : 0;
        c = (unsigned long long)(tx1 - tx0 + 1) * rows;
    }
    cnt[t] = c;
    if (!c) return;   // never listed: no record needed
    write_ordered_record(rec, t, sx, sy, bp.src.z);   // (tri_tiles lists only finite triangles with den != 0)
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
        if (owned_row(ty, bp.period, bp.mask))
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

__device__ __forceinline__ u32 wave_min_u32(u32 v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (u32)__shfl_xor((int)v, d, 64));
    return v;
}

// LDS staging slots of a chunk (SoA, CH entries each)
enum {
    S_X0 = 0, S_Y0, S_X1, S_Y1, S_X2, S_Y2,   // screen-space vertices
    S_E1X, S_E1Y, S_E2X, S_E2Y, S_INV,         // barycentric setup
    S_Z0, S_DZ1, S_DZ2,                        // depth: z0, z1-z0, z2-z0
    S_C0,                                      // colour c0[4] (flat: the colour)
    S_D1 = S_C0 + 4,                           // c1-c0 [4] (Gouraud)
    S_D2 = S_D1 + 4,                           // c2-c0 [4] (Gouraud)
    // flat: ApplyPixel's per-triangle terms (cpp:529-535), formed once at setup
    S_FR = S_D2 + 4, S_FG, S_FB, S_FA,         // src * colourTransform
    S_OM, S_RA, S_GA, S_BA,                    // 1 - a, src * a
    S_SL0, S_SL1, S_SL2,                       // edge slopes (edge_slopes) for the division-free spans
    S_NSLOT
};

__device__ __forceinline__ u64 uniform_u64(u64 v) {   // (a wave-uniform value into scalar registers)
    return ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
           (u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)v);
}

// Bits [xs, xe) of a BW-bit window (xs, xe relative to the window, clamped).
__device__ __forceinline__ u64 window_bits(int xs, int xe) {
    xs = max(xs, 0);
    xe = min(xe, BW);
    if (xs >= xe) return 0ull;
    const int n = xe - xs;
    return (n == 64 ? ~0ull : ((1ull << n) - 1ull)) << xs;
}

// RGBA: the context has an alpha channel (ipp 4).  An RGB context never
// stores alpha, so the per-fragment alpha moves are dropped.
// BINNED: the tile's list comes from the order-free binning, sorted per tile
// by k_tile_sort (tstart = the plan's list offsets: [off[tile], off[tile + 1]));
// the batch is a no-op unless plan[3] (fits); otherwise [tstart, tend) of the
// globally sorted pairs.
// 4 waves per SIMD (6: 80 VGPRs, 85 spilled -- C5 raster 740 -> 1355 us)
template <bool GOURAUD, bool DEPTH, bool COUNT, bool RGBA, bool BINNED>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) void k_tile_raster(const FrameParams fp, const u32* __restrict__ list,
                                                    const u32* __restrict__ tstart, const u32* __restrict__ tend,
                                                    const f64* __restrict__ rec, const u32* __restrict__ plan) {
    const int tile = blockIdx.x;
    const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
    const i64 x0 = (i64)tx * TW, y0 = (i64)ty * TH;
    // (wave: uniform, so the per-wave masks and addresses below stay scalar)
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    raster_stamp_begin(fp);
    if (BINNED && !plan[3]) return;
    if (!owned_row(ty, fp.period, fp.mask)) return;
    const u32 ls = tstart[tile], le = BINNED ? tstart[tile + 1] : tend[tile];
    if (ls == le && !fp.pendColor && !(DEPTH && fp.pendDepth)) return;
    __shared__ f64 S[2][S_NSLOT][CH];   // (two chunks: one set up while the other is blended)
    // the lane masks of a wave's RPW steps for triangle k (bit l: lane l's
    // pixel of that step is covered), formed by the span phase's 512 threads
    // in VALU: the blend loop only moves them into scalar registers and sets
    // exec (it is bound by scalar issue)
    __shared__ __attribute__((aligned(16))) u64 SPM[2][CH][NWAVE][RPW];
    // span-phase ballots, one per column window q: HITQ[q][w] byte g = which of
    // triangles 8w..8w+7 touch window q of the tile rows 4g..4g+3
    __shared__ u64 HITQ[2][NQ][NWAVE];
    __shared__ iu8 ZPASS[2][CH];   // depth test known to pass on every covered pixel (see zpass_all)
    __shared__ u32 zmin_w[NWAVE];
    __shared__ unsigned long long fragSum;
    if (COUNT && tid == 0) fragSum = 0;

    // ---- the tile's pixel state, resident in registers for the whole list:
    // this wave's block (band, q), the lane's column and its row in each step
    const int band = wave / NQ, q = wave - band * NQ;
    const int lcol = q * BW + (lane % BW);               // column in the tile
    const int lrow0 = band * (RPW * SR) + lane / BW;     // row in the tile at step 0 (step r: + r * SR)
    const i64 px = x0 + lcol;
    constexpr int ipp = RGBA ? 4 : 3;
    f64 cr[RPW], cg[RPW], cb[RPW], ca[RPW];
    u32 cz[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const i64 py = y0 + lrow0 + r * SR;
        cr[r] = cg[r] = cb[r] = ca[r] = 0;
        cz[r] = 0xFFFFFFFFu;
        if (px < fp.W && py < fp.H) {
            if (fp.pendColor) {
                cr[r] = cg[r] = cb[r] = ca[r] = fp.pendColorValue;
            } else {
                const f64* p = fp.fb + (py * fp.W + px) * ipp;
                cr[r] = p[0]; cg[r] = p[1]; cb[r] = p[2];
                if (RGBA) ca[r] = p[3];
            }
            if (DEPTH) cz[r] = fp.pendDepth ? fp.pendDepthValue : fp.depth[py * fp.W + px];
        }
    }
    const f64 ct0 = fp.ct[0], ct1 = fp.ct[1], ct2 = fp.ct[2], ct3 = fp.ct[3];
    const f64 wlim = (f64)(fp.W - x0 < TW ? fp.W - x0 : TW);
    unsigned long long myFrags = 0;
    // Z test without Z write: the tile's depth is constant for the whole
    // batch, so a triangle whose every covered pixel provably quantises below
    // the tile's smallest depth passes the test everywhere (zpass_all) and its
    // fragments skip the depth expression -- the same result, bit for bit.
    u32 zTileMin = 0;
    if (DEPTH && !fp.depthWrite) {
        u32 m = min(min(cz[0], cz[1]), min(cz[2], cz[3]));
        m = wave_min_u32(m);
        if (lane == 0) zmin_w[wave] = m;
        __syncthreads();
        zTileMin = zmin_w[0];
#pragma unroll
        for (int w = 1; w < NWAVE; ++w) zTileMin = min(zTileMin, zmin_w[w]);
    }

    // Chunks are double-buffered (round 6): while the waves blend chunk c
    // (buffer buf), one wave -- a different one each chunk -- sets chunk c + 1
    // up into buffer buf ^ 1 before its own blend, and after one barrier every
    // wave forms chunk c + 1's spans: two barriers per chunk instead of three,
    // and the setup's dependent global loads no longer keep seven waves waiting.
    //
    // (a) triangle setup of the chunk at cb into buffer sb, one lane of the
    // calling wave per triangle: the record k_tri_count formed (zpass_bound)
    // and the per-tile parts.  Returns the lane's vote for the blend-only loop
    // (a chunk of flat translucent triangles whose depth test is proven to pass,
    // or off: C5's common case).
    auto setup = [&](u32 cb, int sb) -> bool {
        const int cnt = (le - cb) < (u32)CH ? (int)(le - cb) : CH;
        bool blendOnly = !GOURAUD;
        if (lane < cnt) {
            const int k = lane;
            const i64 t = list[cb + k];
            const double2* r = reinterpret_cast<const double2*>(rec + t * ORec);
            const double2 v0 = r[0], v1 = r[1], v2 = r[2], v3 = r[3], v4 = r[4];
            const f64 sx[3] = {v0.x, v1.x, v2.x}, sy[3] = {v0.y, v1.y, v2.y};
            const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
            S[sb][S_X0][k] = sx[0]; S[sb][S_Y0][k] = sy[0];
            S[sb][S_X1][k] = sx[1]; S[sb][S_Y1][k] = sy[1];
            S[sb][S_X2][k] = sx[2]; S[sb][S_Y2][k] = sy[2];
            S[sb][S_E1X][k] = e1x; S[sb][S_E1Y][k] = e1y; S[sb][S_E2X][k] = e2x; S[sb][S_E2Y][k] = e2y;
            S[sb][S_INV][k] = v4.y;
            S[sb][S_SL0][k] = v3.x; S[sb][S_SL1][k] = v3.y; S[sb][S_SL2][k] = v4.x;
            bool zok = !DEPTH;
            if (DEPTH) {
                const double2 v5 = r[5], v6 = r[6];
                const f64 z0 = v5.x, z1 = v5.y, z2 = v6.x;
                S[sb][S_Z0][k] = z0; S[sb][S_DZ1][k] = z1 - z0; S[sb][S_DZ2][k] = z2 - z0;
                const u32 zb = (u32)((u64)__double_as_longlong(v6.y) >> 32);
                zok = !fp.depthWrite && zb < zTileMin;   // zpass_all
                ZPASS[sb][k] = zok;
            }
            if (GOURAUD) {
                const f64* c = fp.src.rgba + t * 12;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    S[sb][S_C0 + j][k] = c[j];
                    S[sb][S_D1 + j][k] = c[4 + j] - c[j];
                    S[sb][S_D2 + j][k] = c[8 + j] - c[j];
                }
            } else {
                const f64* c = fp.src.rgba + t * 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) S[sb][S_C0 + j][k] = c[j];
                const f64 fR = c[0] * ct0, fG = c[1] * ct1, fB = c[2] * ct2, fA = c[3] * ct3;
                S[sb][S_FR][k] = fR; S[sb][S_FG][k] = fG; S[sb][S_FB][k] = fB; S[sb][S_FA][k] = fA;
                S[sb][S_OM][k] = 1 - fA;
                S[sb][S_RA][k] = fR * fA; S[sb][S_GA][k] = fG * fA; S[sb][S_BA][k] = fB * fA;
                blendOnly = zok && fA != 1;
            }
        }
        return blendOnly;
    };
    // (b) exact coverage spans of the chunk at cb (buffer sb)
    auto spans = [&](u32 cb, int sb) {
        const int cnt = (le - cb) < (u32)CH ? (int)(le - cb) : CH;
        // ---- (b) exact coverage spans: thread = (triangle k, row group rg =
        // tile rows 4rg..4rg+3); wave w takes triangles 8w..8w+7, lane = rg * 8
        // + (k - 8w).  Its 4 rows are 4 / SR steps of the waves of band rg / SR
        // (one per column window): it writes those 4 lane masks, and the
        // wave's ballot per window holds one byte per row group
        {
            const int k = (wave << 3) | (lane & 7), rg = lane >> 3;
            bool touch[NQ];
#pragma unroll
            for (int qq = 0; qq < NQ; ++qq) touch[qq] = false;
            if (k < cnt) {
                const bool ok = true;   // (only valid triangles are listed)
                const f64 sx[3] = {S[sb][S_X0][k], S[sb][S_X1][k], S[sb][S_X2][k]};
                const f64 sy[3] = {S[sb][S_Y0][k], S[sb][S_Y1][k], S[sb][S_Y2][k]};
                const f64 sl[3] = {S[sb][S_SL0][k], S[sb][S_SL1][k], S[sb][S_SL2][k]};
                // rows with a straddling edge: ymin <= y < ymax, where exactly
                // two edges straddle (row_span_slopes = row_span there); none
                // elsewhere (row_span's empty span)
                const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
                u64 mk[RPW];   // [j * NQ + qq]: step (4 rg % (RPW SR)) / SR + j of window qq
#pragma unroll
                for (int i = 0; i < RPW; ++i) mk[i] = 0;
                // (f32 row spans as in k_vis measured slower here: 786 vs 740 us,
                // profiles/r03_c5/ab_span32_wpe.txt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = rg * 4 + r;
                    const i64 gy = y0 + row;
                    int xs = 0, xe = 0;
                    if (ok && gy < fp.H && ymn <= (f64)gy && (f64)gy < ymx) {
                        row_span_slopes(sx, sy, sl, (f64)gy, (f64)x0, wlim, xs, xe);
                    }
                    if (COUNT) myFrags += (unsigned long long)(xe - xs);
#pragma unroll
                    for (int qq = 0; qq < NQ; ++qq)
                        mk[(r / SR) * NQ + qq] |= window_bits(xs - qq * BW, xe - qq * BW) << ((r % SR) * BW);
                }
                const int b = rg / SR;                        // band of these rows
                const int st0 = ((rg * 4) % (RPW * SR)) / SR; // their first step
#pragma unroll
                for (int j = 0; j < 4 / SR; ++j)
#pragma unroll
                    for (int qq = 0; qq < NQ; ++qq) {
                        SPM[sb][k][b * NQ + qq][st0 + j] = mk[j * NQ + qq];
                        touch[qq] |= mk[j * NQ + qq] != 0;
                    }
            }
#pragma unroll
            for (int qq = 0; qq < NQ; ++qq) {
                const u64 hit = __ballot(touch[qq]);
                if (lane == 0) HITQ[sb][qq][wave] = hit;
            }
        }
    };
    // (c) in-order raster of the chunk in buffer sb
    auto blend = [&](int sb, bool allBlend) {
        // this wave's triangles of the chunk (bit k: triangle k touches its
        // block): the bytes of its band's SR row groups in its window's ballots
        u64 hm = 0;
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) {
            const u64 h = uniform_u64(HITQ[sb][q][w]) >> (8 * band * SR);
            u64 m = 0;
#pragma unroll
            for (int i = 0; i < SR; ++i) m |= h >> (8 * i);
            hm |= (m & 0xFFull) << (8 * w);
        }
        // ---- (c) in-order raster of the chunk; each wave owns its block.
        // Every product of the per-pixel expressions that is constant along
        // a column (dx * e2y, dx * e1y), along a row (e2x * dy, e1x * dy) or
        // over the triangle (flat: src * colourTransform, src * a, 1 - a) is
        // formed once there: the same rounded values in the same expression
        // trees, so the result is bit-identical to the per-pixel form.
        if (!GOURAUD && allBlend) {
            // every triangle of the chunk: ApplyPixel from the per-triangle
            // terms on the covered lanes (a loop with one path, so the pixel
            // registers are updated in place), only the triangles touching
            // this wave's block
            for (; hm; hm &= hm - 1) {
                const int k = (int)__builtin_ctzll(hm);
                const f64 om = S[sb][S_OM][k], RA = S[sb][S_RA][k], GA = S[sb][S_GA][k], BA = S[sb][S_BA][k];
                const f64 fA = RGBA ? S[sb][S_FA][k] : 0.0;
                u64 lm[RPW];
                const ulonglong2 m01 = *reinterpret_cast<const ulonglong2*>(&SPM[sb][k][wave][0]);
                const ulonglong2 m23 = *reinterpret_cast<const ulonglong2*>(&SPM[sb][k][wave][2]);
                lm[0] = uniform_u64(m01.x); lm[1] = uniform_u64(m01.y);
                lm[2] = uniform_u64(m23.x); lm[3] = uniform_u64(m23.y);
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    if (__builtin_amdgcn_inverse_ballot_w64(lm[r])) {
                        cr[r] = cr[r] * om + RA;
                        cg[r] = cg[r] * om + GA;
                        cb[r] = cb[r] * om + BA;
                        if (RGBA) ca[r] = fA;
                    }
                }
            }
            return;
        }
        const f64 X = (f64)px;
        for (; hm; hm &= hm - 1) {
            const int k = (int)__builtin_ctzll(hm);
            u64 lm[RPW];
            {
                const ulonglong2 m01 = *reinterpret_cast<const ulonglong2*>(&SPM[sb][k][wave][0]);
                const ulonglong2 m23 = *reinterpret_cast<const ulonglong2*>(&SPM[sb][k][wave][2]);
                lm[0] = uniform_u64(m01.x); lm[1] = uniform_u64(m01.y);
                lm[2] = uniform_u64(m23.x); lm[3] = uniform_u64(m23.y);
            }
            // (uniform: read into scalar registers, so the branches below are scalar)
            const bool ztest = DEPTH && !__builtin_amdgcn_readfirstlane((int)ZPASS[sb][k]);   // the depth expression is needed
            if (!GOURAUD && !ztest) {
                // flat colour, no per-pixel depth: ApplyPixel from the
                // per-triangle terms on the covered lanes of each step
                const f64 fA = __longlong_as_double((long long)uniform_u64((u64)__double_as_longlong(S[sb][S_FA][k])));
                if (fA != 1) {
                    const f64 om = S[sb][S_OM][k], RA = S[sb][S_RA][k], GA = S[sb][S_GA][k], BA = S[sb][S_BA][k];
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        if (__builtin_amdgcn_inverse_ballot_w64(lm[r])) {
                            cr[r] = cr[r] * om + RA;
                            cg[r] = cg[r] * om + GA;
                            cb[r] = cb[r] * om + BA;
                            if (RGBA) ca[r] = fA;
                        }
                    }
                } else {
                    const f64 fR = S[sb][S_FR][k], fG = S[sb][S_FG][k], fB = S[sb][S_FB][k];
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        if (__builtin_amdgcn_inverse_ballot_w64(lm[r])) {
                            cr[r] = fR; cg[r] = fG; cb[r] = fB;
                            if (RGBA) ca[r] = fA;
                        }
                    }
                }
                continue;
            }
            const f64 sx0 = S[sb][S_X0][k], sy0 = S[sb][S_Y0][k];
            const f64 e1x = S[sb][S_E1X][k], e1y = S[sb][S_E1Y][k], e2x = S[sb][S_E2X][k], e2y = S[sb][S_E2Y][k];
            const f64 inv = S[sb][S_INV][k];
            f64 pa = 0, pb = 0;   // dx * e2y, dx * e1y of this lane's column
            if (ztest || GOURAUD) {
                const f64 dx = X - sx0;
                pa = dx * e2y;
                pb = dx * e1y;
            }
            f64 fR = 0, fG = 0, fB = 0, fA = 1, om = 0, RA = 0, GA = 0, BA = 0;
            if (!GOURAUD) {   // ApplyPixel's per-triangle terms (cpp:529-535), formed at setup
                fR = S[sb][S_FR][k]; fG = S[sb][S_FG][k]; fB = S[sb][S_FB][k]; fA = S[sb][S_FA][k];
                om = S[sb][S_OM][k];
                RA = S[sb][S_RA][k]; GA = S[sb][S_GA][k]; BA = S[sb][S_BA][k];
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                if (!__builtin_amdgcn_inverse_ballot_w64(lm[r])) continue;
                f64 w1 = 0, w2 = 0;
                if (ztest || GOURAUD) {
                    const f64 dy = (f64)(y0 + lrow0 + r * SR) - sy0;
                    w1 = (pa - e2x * dy) * inv;
                    w2 = (e1x * dy - pb) * inv;
                }
                u32 zq = 0;
                if (ztest) {
                    const f64 zz = S[sb][S_Z0][k] + S[sb][S_DZ1][k] * w1 + S[sb][S_DZ2][k] * w2;
                    zq = nr_quantize_depth_hw(zz);
                    if (!(zq < cz[r])) continue;
                }
                if (GOURAUD) {
                    f64 R = S[sb][S_C0 + 0][k] + S[sb][S_D1 + 0][k] * w1 + S[sb][S_D2 + 0][k] * w2;
                    f64 G = S[sb][S_C0 + 1][k] + S[sb][S_D1 + 1][k] * w1 + S[sb][S_D2 + 1][k] * w2;
                    f64 B = S[sb][S_C0 + 2][k] + S[sb][S_D1 + 2][k] * w1 + S[sb][S_D2 + 2][k] * w2;
                    f64 A = S[sb][S_C0 + 3][k] + S[sb][S_D1 + 3][k] * w1 + S[sb][S_D2 + 3][k] * w2;
                    // ApplyPixel (cpp:529-547) on the register-resident pixel
                    R *= ct0; G *= ct1; B *= ct2; A *= ct3;
                    if (A != 1) {
                        R = cr[r] * (1 - A) + R * A;
                        G = cg[r] * (1 - A) + G * A;
                        B = cb[r] * (1 - A) + B * A;
                    }
                    cr[r] = R; cg[r] = G; cb[r] = B;
                    if (RGBA) ca[r] = A;
                } else if (fA != 1) {
                    cr[r] = cr[r] * om + RA;
                    cg[r] = cg[r] * om + GA;
                    cb[r] = cb[r] * om + BA;
                    if (RGBA) ca[r] = fA;
                } else {
                    cr[r] = fR; cg[r] = fG; cb[r] = fB;
                    if (RGBA) ca[r] = fA;
                }
                if (DEPTH && fp.depthWrite) cz[r] = zq;
            }
        }
    };

    int buf = 0;
    bool allB = false;
    if (ls < le) {   // the first chunk: set up by wave 0
        const bool bo = wave == 0 ? setup(ls, 0) : !GOURAUD;
        allB = __syncthreads_and(bo ? 1 : 0) != 0;
        spans(ls, 0);
        __syncthreads();
    }
    u32 ci = 0;
    for (u32 base = ls; base < le; base += CH, buf ^= 1, ++ci) {
        const u32 nb = base + CH;
        const bool more = nb < le;
        bool bo = !GOURAUD;
        if (more && wave == (int)((ci + 1) & (NWAVE - 1))) bo = setup(nb, buf ^ 1);
        blend(buf, allB);
        if (more) {
            allB = __syncthreads_and(bo ? 1 : 0) != 0;
            spans(nb, buf ^ 1);
        }
        __syncthreads();
    }

    // ---- write the tile back once
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const i64 py = y0 + lrow0 + r * SR;
        if (px < fp.W && py < fp.H) {
            f64* p = fp.fb + (py * fp.W + px) * ipp;
            out_store<f64>(p, cr[r]); out_store<f64>(p + 1, cg[r]); out_store<f64>(p + 2, cb[r]);
            if (RGBA) out_store<f64>(p + 3, ca[r]);
            if (DEPTH && (fp.depthWrite || fp.pendDepth)) out_store<u32>(fp.depth + py * fp.W + px, cz[r]);
            store_frame_out(fp, py * fp.W + px, px, py, cr[r], cg[r], cb[r], RGBA ? ca[r] : 1.0);
        }
    }
    raster_stamp_end(fp);
    if (COUNT) {
        atomicAdd(&fragSum, myFrags);
        __syncthreads();
        if (tid == 0) atomicAdd(fp.fragCounter, fragSum);
    }
}

// Sorts each tile's list of a binned ordered batch into submission order, in
// place: one workgroup per tile, the list (<= ORD_SORT_CAP entries: the plan
// guarantees it, or the batch is a no-op) bitonic-sorted in LDS.  It runs on
// the binning stream after k_free_emit, beside the previous batch's raster.
constexpr int SORT_T = 512;
__global__ __launch_bounds__(SORT_T) void k_tile_sort(const u32* __restrict__ off, u32* __restrict__ list,
                                                      const u32* __restrict__ plan) {
    if (!plan[3]) return;
    const u32 ls = off[blockIdx.x], n = off[blockIdx.x + 1] - ls;
    if (n < 2) return;
    __shared__ u32 SL[ORD_SORT_CAP];
    const u32 tid = threadIdx.x;
    u32 np2 = 2;
    while (np2 < n) np2 <<= 1;
    for (u32 i = tid; i < np2; i += SORT_T) SL[i] = i < n ? list[ls + i] : 0xFFFFFFFFu;
    __syncthreads();
    for (u32 k = 2; k <= np2; k <<= 1)
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            for (u32 i = tid; i < (np2 >> 1); i += SORT_T) {
                const u32 lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;   // (lo has bit j clear)
                const u32 a = SL[lo], b = SL[hi];
                if ((a > b) == ((lo & k) == 0)) { SL[lo] = b; SL[hi] = a; }
            }
            __syncthreads();
        }
    for (u32 i = tid; i < n; i += SORT_T) list[ls + i] = SL[i];
}

template <bool G, bool D, bool C, bool B>
void launch_raster(const FrameParams& fp, const u32* list, const u32* ts, const u32* te, int ntiles, hipStream_t s,
                   const f64* rec, const u32* plan, hipEvent_t start, hipEvent_t stop) {
    if (fp.ipp == 4)
        hipExtLaunchKernelGGL((k_tile_raster<G, D, C, true, B>), dim3(ntiles), dim3(WG), 0, s, start, stop, 0, fp, list,
                              ts, te, rec, plan);
    else
        hipExtLaunchKernelGGL((k_tile_raster<G, D, C, false, B>), dim3(ntiles), dim3(WG), 0, s, start, stop, 0, fp,
                              list, ts, te, rec, plan);
}

template <bool C, bool B>
void launch_raster_c(const FrameParams& fp, const u32* list, const u32* ts, const u32* te, int ntiles,
                     hipStream_t s, const f64* rec, const u32* plan = nullptr, hipEvent_t start = nullptr,
                     hipEvent_t stop = nullptr) {
    const bool g = fp.src.gouraud != 0, d = fp.depthTest != 0;
    if (g && d) launch_raster<true, true, C, B>(fp, list, ts, te, ntiles, s, rec, plan, start, stop);
    else if (g) launch_raster<true, false, C, B>(fp, list, ts, te, ntiles, s, rec, plan, start, stop);
    else if (d) launch_raster<false, true, C, B>(fp, list, ts, te, ntiles, s, rec, plan, start, stop);
    else launch_raster<false, false, C, B>(fp, list, ts, te, ntiles, s, rec, plan, start, stop);
}

}  // namespace

void launch_tile_sort(const u32* off, u32* list, const u32* plan, int ntiles, hipStream_t s, hipEvent_t stop) {
    hipExtLaunchKernelGGL(k_tile_sort, dim3(ntiles), dim3(SORT_T), 0, s, nullptr, stop, 0, off, list, plan);
}

void launch_ordered_binned(const FrameParams& fp, const u32* list, const u32* off, const u32* plan, const f64* rec,
                           int ntiles, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (fp.fragCounter) launch_raster_c<true, true>(fp, list, off, nullptr, ntiles, s, rec, plan, start, stop);
    else launch_raster_c<false, true>(fp, list, off, nullptr, ntiles, s, rec, plan, start, stop);
}

void draw_ordered(RenderContext* ctx, const TriSrc& src, TriangleBuffer* tb, bool callerOwned) {
    const i64 ntiles = (i64)((ctx->width + TW - 1) / TW) * ((ctx->height + TH - 1) / TH);
    if (ntiles <= ORD_BIN_TILES) {
        draw_free(ctx, src, tb, callerOwned, true);
        return;
    }
    FrameParams fp = frame_params(ctx, src);
    BinParams bp;
    bp.src = src;
    for (int k = 0; k < 6; ++k) bp.m[k] = ctx->m[k];
    bp.W = ctx->width; bp.H = ctx->height; bp.tiles_x = fp.tiles_x;
    bp.period = fp.period; bp.mask = fp.mask;
    set_owned_rows(bp, fp.tiles_y);
    draw_ordered_sorted(ctx, src, fp, bp);
}

namespace {

// The global-sort ordered path for a batch with its state snapshot (fp, bp):
// per-triangle tile counts -> scan -> (tile, triangle) pairs in triangle order
// -> stable radix sort by tile -> tile ranges -> k_tile_raster.  Only enqueues
// kernels: the context's flags are the caller's business (draw_ordered_sorted
// consumes them; a deferred re-run, rerun_ordered_sorted, must leave them as
// the calls after the batch set them).
void ordered_sorted_kernels(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp) {
    hipStream_t s = ctx->stream;
    TriScratch& sc = ctx->tri;
    const int ntiles = fp.tiles_x * fp.tiles_y;

    u64* tri_bufs[2] = {sc.cnt, sc.off};
    if (!grow_set(tri_bufs, &sc.tri_cap, (size_t)src.n)) return;
    sc.cnt = tri_bufs[0]; sc.off = tri_bufs[1];
    f64* rec_bufs[1] = {sc.orec};
    if (!grow_set(rec_bufs, &sc.orec_cap, (size_t)std::max<i64>(src.n, 1) * ORec)) return;
    sc.orec = rec_bufs[0];
    u32* tile_bufs[2] = {sc.tile_start, sc.tile_end};
    if (!grow_set(tile_bufs, &sc.tile_cap, (size_t)ntiles)) return;
    sc.tile_start = tile_bufs[0]; sc.tile_end = tile_bufs[1];

    const int g1 = (int)((src.n + 255) / 256);
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_TRI_COUNT, &e0, &e1);
    hipLaunchKernelGGL(k_tri_count, dim3(g1), dim3(256), 0, s, bp, sc.cnt, sc.orec);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_TRI_COUNT, e0, e1);

    size_t need = 0;
    NR_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, sc.cnt, sc.off, (int)src.n, s));
    if (!grow_temp(sc, need)) return;
    nr_timing_begin(ctx, NRK_TRI_SCAN, &e0, &e1);
    NR_CHECK(hipcub::DeviceScan::ExclusiveSum(sc.temp, need, sc.cnt, sc.off, (int)src.n, s));
    nr_timing_end(ctx, NRK_TRI_SCAN, e0, e1);

    // total pair count: sizes the sort (host sync)
    NR_CHECK(hipMemcpyAsync(&sc.h_total[0], sc.off + (src.n - 1), sizeof(u64), hipMemcpyDeviceToHost, s));
    NR_CHECK(hipMemcpyAsync(&sc.h_total[1], sc.cnt + (src.n - 1), sizeof(u64), hipMemcpyDeviceToHost, s));
    NR_CHECK(hipStreamSynchronize(s));
    const u64 P = sc.h_total[0] + sc.h_total[1];

    if (P > (1ull << 31) && src.n > 1) {
        // too many pairs for one pass: split the batch; submission order kept
        TriSrc a = src, b = src;
        a.n = src.n / 2;
        b.n = src.n - a.n;
        b.xy = src.xy + a.n * 6;
        b.z = src.z ? src.z + a.n * 3 : nullptr;
        b.rgba = src.rgba + a.n * (src.gouraud ? 12 : 4);
        BinParams ba = bp, bb = bp;
        ba.src = a; bb.src = b;
        FrameParams fa = fp, fb = fp;
        fa.src = a; fb.src = b;
        // (fb keeps the frame output: the second half rewrites the tiles it covers)
        ordered_sorted_kernels(ctx, a, fa, ba);
        if (fa.fragCounter) {   // fragments of the first half, then the counter restarts for the second
            NR_CHECK(hipMemcpyAsync(&sc.h_total[2], fa.fragCounter, sizeof(u64), hipMemcpyDeviceToHost, s));
            NR_CHECK(hipStreamSynchronize(s));
            ctx->fragTotal += sc.h_total[2];
            NR_CHECK(hipMemsetAsync(fb.fragCounter, 0, sizeof(u64), s));
        }
        fb.pendColor = 0;   // (the first half applied the pending clears)
        fb.pendDepth = 0;
        ordered_sorted_kernels(ctx, b, fb, bb);
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

    FrameParams fpt = fp;   // (timed: the raster stamps itself on the device clock)
    fpt.tstamp = nr_timing_stamp(ctx, NRK_TILE_RASTER);
    if (fp.fragCounter) launch_raster_c<true, false>(fpt, list, sc.tile_start, sc.tile_end, ntiles, s, sc.orec);
    else launch_raster_c<false, false>(fpt, list, sc.tile_start, sc.tile_end, ntiles, s, sc.orec);
    NR_CHECK(hipGetLastError());
}

}  // namespace

void draw_ordered_sorted(RenderContext* ctx, const TriSrc& src, const FrameParams& fp0, const BinParams& bp) {
    FrameParams fp = fp0;
    // with a pending clear every owned tile is rasterised and written back,
    // so the write-back also produces the frame output (as k_vis does)
    if (ctx->frameOutput && fp.pendColor) {
        const size_t n = (size_t)nr_frame_bytes(ctx);
        if (n <= ctx->frameU8cap) fp.frameU8 = ctx->frameU8;
    }
    ordered_sorted_kernels(ctx, src, fp, bp);
    ctx->lastPath = 2;
    finish_batch(ctx, fp);
}

// The deferred re-run of a batch whose binned ordered raster was a no-op (a
// tile list over ORD_SORT_CAP, found at nr_settle): the batch's own snapshot
// (its pending clears and frame output as they were when it was drawn), and
// nothing of the context's current state -- the calls made since (ClearDepth,
// SetColor, ...) have already set the flags for what comes next.  Only its
// fragments are accounted.
void rerun_ordered_sorted(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp) {
    ordered_sorted_kernels(ctx, src, fp, bp);
    if (fp.fragCounter) {
        TriScratch& sc = ctx->tri;
        NR_CHECK(hipMemcpyAsync(&sc.h_total[2], fp.fragCounter, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
        NR_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->fragTotal += sc.h_total[2];
    }
}

}  // namespace nrtri
