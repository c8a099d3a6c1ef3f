// nr_tri.h — shared pieces of the triangle / depth / Gouraud path.
//
// Semantics (no reference implementation exists; defined
// in the reference's idiom, DESIGN.md §3, restated by the CPU oracle):
//   vertices -> context transform (cpp:446-453) -> screen space;
//   coverage = even-odd pointInPolygon (cpp:822-845) at integer pixels;
//   w1,w2 barycentric in f64, attr = a0 + (a1-a0)*w1 + (a2-a0)*w2;
//   depth u32 LESS, written only when test+write are on;
//   blend = ApplyPixel (cpp:515-549) in submission order.
//
// Two rasterisers share the screen tiling (64x32 tiles) and these helpers:
//   nr_tri_ordered.hip  in-order tile raster (any batch: blending, Z w/o write)
//   nr_tri_free.hip     visibility-buffer raster (opaque batches: every
//                       fragment overwrites, so per-pixel results are an
//                       order-independent min/max over packed keys)
#pragma once

#include "nr_common.h"

namespace nrtri {

constexpr int TW = 64;   // tile width  (= one wave's lanes)
constexpr int TH = 32;   // tile height

struct TriSrc {
    const f64* xy;    // n*6
    const f64* z;     // n*3 or null
    const f64* rgba;  // n*4 flat / n*12 Gouraud
    int gouraud;
    i64 n;
};

struct BinParams {
    TriSrc src;
    f64 m[6];
    i64 W, H;
    int tiles_x;
    int period;           // owned tile rows: bit (ty % period) of mask (SetShard / SetShardSlots)
    u64 mask;
    // the owned tile rows, numbered 0.. (the binning kernels' LDS histograms
    // hold only those): pc owned slots per period, slotOf[k] = the k-th
    // owned slot; hrows = owned rows of the frame (set_owned_rows)
    int pc, hrows;
    unsigned char slotOf[64];
};

// Ordinal of owned tile row ty among the owned rows, and its inverse
// (unsharded: the identity, no division).
__device__ __forceinline__ int owned_ord(const BinParams& bp, int ty) {
    if (bp.period == 1) return ty;
    const int q = ty / bp.period, s = ty - q * bp.period;
    return q * bp.pc + __builtin_popcountll(bp.mask & ((1ull << s) - 1ull));
}
__device__ __forceinline__ int owned_row_of(const BinParams& bp, int ord) {
    if (bp.period == 1) return ord;
    const int q = ord / bp.pc;
    return q * bp.period + bp.slotOf[ord - q * bp.pc];
}
inline void set_owned_rows(BinParams& bp, int tiles_y) {
    bp.pc = 0;
    for (int s = 0; s < bp.period && s < 64; ++s)
        if ((bp.mask >> s) & 1ull) bp.slotOf[bp.pc++] = (unsigned char)s;
    bp.hrows = 0;
    for (int ty = 0; ty < tiles_y; ++ty)
        if (bp.period == 1 || ((bp.mask >> (ty % bp.period)) & 1ull)) ++bp.hrows;
}

// (unsharded: no integer division -- it costs ~30 VALU instructions)
__device__ __forceinline__ bool owned_row(int ty, int period, u64 mask) {
    return period == 1 || ((mask >> (ty % period)) & 1ull);
}

__device__ __forceinline__ f64 clampd(f64 v, f64 lo, f64 hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Triangle arrays are 16-byte aligned (hipMalloc'd, or staged by the draw
// entry points): a triangle's 6 positions / 12 or 4 colours load as 16-byte
// vectors, 3 or 6 or 2 loads instead of 6 or 12 or 4.
__device__ __forceinline__ void load_tri_xy(const f64* xy, i64 t, f64 (&v)[6]) {
    const double2* q = reinterpret_cast<const double2*>(xy + t * 6);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double2 a = q[k];
        v[2 * k] = a.x; v[2 * k + 1] = a.y;
    }
}

template <int N>   // 4 (flat) or 12 (Gouraud)
__device__ __forceinline__ void load_tri_rgba(const f64* rgba, i64 t, f64 (&c)[N]) {
    const double2* q = reinterpret_cast<const double2*>(rgba + t * N);
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
        const double2 a = q[k];
        c[2 * k] = a.x; c[2 * k + 1] = a.y;
    }
}

// Screen-space vertices of triangle t (cpp:446-453 applied to each vertex).
__device__ __forceinline__ void tri_screen(const TriSrc& s, const f64* m, i64 t, f64 (&sx)[3], f64 (&sy)[3]) {
    f64 p[6];
    load_tri_xy(s.xy, t, p);
#pragma unroll
    for (int v = 0; v < 3; ++v) nr_xform(m, p[2 * v], p[2 * v + 1], sx[v], sy[v]);
}

__device__ __forceinline__ bool tri_finite(const f64 (&sx)[3], const f64 (&sy)[3]) {
    return isfinite(sx[0]) && isfinite(sy[0]) && isfinite(sx[1]) && isfinite(sy[1]) && isfinite(sx[2]) &&
           isfinite(sy[2]);
}

// Tile rectangle touched by a triangle; false if it produces no fragment.
// Rows: a row y has a straddling edge iff ymin <= y < ymax (exact), so
// [ceil(ymin), ceil(ymax)).  Columns: crossings lie in [xmin, xmax] up to
// rounding, so [floor(xmin)-2, ceil(xmax)+2]; for |coord| > 1e7 the full width.
__device__ __forceinline__ bool tri_tiles(const f64 (&sx)[3], const f64 (&sy)[3], i64 W, i64 H, int& tx0, int& tx1,
                                          int& ty0, int& ty1) {
    bool huge = false;
#pragma unroll
    for (int v = 0; v < 3; ++v) huge = huge || fabs(sx[v]) > 1e7 || fabs(sy[v]) > 1e7;
    if (!tri_finite(sx, sy)) return false;
    const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
    const f64 den = e1x * e2y - e2x * e1y;
    if (den == 0) return false;
    const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
    const i64 r0 = (i64)clampd(ceil(ymn), 0.0, (f64)H);
    const i64 r1 = (i64)clampd(ceil(ymx), 0.0, (f64)H);
    if (r0 >= r1) return false;
    i64 c0 = 0, c1 = W - 1;
    if (!huge) {
        const f64 xmn = fmin(fmin(sx[0], sx[1]), sx[2]), xmx = fmax(fmax(sx[0], sx[1]), sx[2]);
        if (ceil(xmx) + 2 < 0 || floor(xmn) - 2 > (f64)(W - 1)) return false;
        c0 = (i64)clampd(floor(xmn) - 2, 0.0, (f64)(W - 1));
        c1 = (i64)clampd(ceil(xmx) + 2, 0.0, (f64)(W - 1));
    }
    tx0 = (int)(c0 / TW); tx1 = (int)(c1 / TW);
    ty0 = (int)(r0 / TH); ty1 = (int)((r1 - 1) / TH);
    return true;
}

// Exact covered columns [xs, xe) of screen row y, relative to x0 and clamped
// to [0, wlim].  The two edges straddling y (pointInPolygon's edge order
// (i=0,j=2) (i=1,j=0) (i=2,j=1) and crossing expression, cpp:832-839) give
// crossings ca, cb; (x < ca) != (x < cb)  <=>  ceil(min) <= x < ceil(max).
__device__ __forceinline__ void row_span(const f64 (&sx)[3], const f64 (&sy)[3], f64 y, f64 x0, f64 wlim, int& xs,
                                         int& xe) {
    f64 c0 = 0, c1 = 0;
    int nc = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 2) % 3;
        if ((sy[i] > y) != (sy[j] > y)) {
            const f64 cc = (sx[j] - sx[i]) * (y - sy[i]) / (sy[j] - sy[i]) + sx[i];
            if (nc == 0) c0 = cc; else c1 = cc;
            ++nc;
        }
    }
    xs = xe = 0;
    if (nc == 2) {
        const f64 lo = fmin(c0, c1), hi = fmax(c0, c1);
        xs = (int)clampd(ceil(lo) - x0, 0.0, wlim);
        xe = (int)clampd(ceil(hi) - x0, 0.0, wlim);
        if (xe < xs) xe = xs;
    }
}

// row_span for a row known to lie in [ceil(ymin), ceil(ymax)) (ymin <= y <
// ymax), without branches.  There exactly one vertex v is on its own side of
// y (sy[v] > y differs from the other two), and the two straddling edges are
// the two edges at v; in pointInPolygon's (i, j) orientation those are
// v=0: (0,2) (1,0)   v=1: (2,1) (1,0)   v=2: (0,2) (2,1).
// The crossings are evaluated with the same expression, and min/max does not
// depend on which edge comes first, so the span equals row_span's.
__device__ __forceinline__ void row_span_in(const f64 (&sx)[3], const f64 (&sy)[3], f64 y, f64 x0, f64 wlim,
                                            int& xs, int& xe) {
    const bool b0 = sy[0] > y, b1 = sy[1] > y, b2 = sy[2] > y;
    const bool v1 = (b1 != b0) && (b1 != b2);
    const bool v2 = (b2 != b0) && (b2 != b1);
    // edge A: v==1 ? (2,1) : (0,2);  edge B: v==2 ? (2,1) : (1,0)
    const f64 aix = v1 ? sx[2] : sx[0], aiy = v1 ? sy[2] : sy[0];
    const f64 ajx = v1 ? sx[1] : sx[2], ajy = v1 ? sy[1] : sy[2];
    const f64 bix = v2 ? sx[2] : sx[1], biy = v2 ? sy[2] : sy[1];
    const f64 bjx = v2 ? sx[1] : sx[0], bjy = v2 ? sy[1] : sy[0];
    const f64 ca = (ajx - aix) * (y - aiy) / (ajy - aiy) + aix;
    const f64 cb = (bjx - bix) * (y - biy) / (bjy - biy) + bix;
    const f64 lo = fmin(ca, cb), hi = fmax(ca, cb);
    xs = (int)clampd(ceil(lo) - x0, 0.0, wlim);
    xe = (int)clampd(ceil(hi) - x0, 0.0, wlim);
    if (xe < xs) xe = xs;
}

// Edge slopes for row_span_slopes, one per pointInPolygon edge (i, j) in its
// orientation: e0 = (0,2), e1 = (1,0), e2 = (2,1); slope = (sx[j]-sx[i]) /
// (sy[j]-sy[i]) (inf/NaN for a horizontal edge, which never straddles a row).
__device__ __forceinline__ void edge_slopes(const f64 (&sx)[3], const f64 (&sy)[3], f64 (&sl)[3]) {
    sl[0] = (sx[2] - sx[0]) / (sy[2] - sy[0]);
    sl[1] = (sx[0] - sx[1]) / (sy[0] - sy[1]);
    sl[2] = (sx[1] - sx[2]) / (sy[1] - sy[2]);
}

// One crossing without a division.  The exact crossing is
//   cc  = fl(fl(fl(a*b) / d) + c)      a = sx[j]-sx[i], b = y-sy[i], d = sy[j]-sy[i], c = sx[i]
// and with the per-edge slope s = fl(a/d):
//   cc' = fl(fl(b*s) + c).
// With unit roundoff u = 2^-53 both products are A(1+e)(1+e') for A = a*b/d,
// so |fl(a*b)/d - fl(b*s)| <= (4u + 2u^2)|A|, and the two final roundings add
// u|cc| + u|cc'|; hence |cc - cc'| <= 4.001u|v| + 2.001u|cc'| (v = fl(b*s))
// < 2^-50 (|v| + |cc'|) = eps (plus 2^-1000 for underflow).  ceil is what the
// span needs: if cc' is more than eps away from the integers on both sides of
// it, ceil(cc) == ceil(cc').  The lane reports `safe`; otherwise the caller
// evaluates the exact expression (integer-aligned vertices hit that path,
// arbitrary geometry essentially never).
__device__ __forceinline__ f64 crossing_ceil(f64 b, f64 s, f64 c, bool& safe) {
    const f64 v = b * s;
    const f64 cc = v + c;
    const f64 k = ceil(cc);
    const f64 eps = (fabs(v) + fabs(cc)) * 0x1p-50 + 0x1p-1000;
    safe = safe && (cc - (k - 1.0) > eps) && (k - cc > eps);
    return k;
}

// row_span_in with the per-edge slopes (no division unless a crossing lies
// within eps of an integer, see crossing_ceil): the same [xs, xe).  (k_vis
// uses this form; row_span_in is its reference statement, and both are
// checked against row_span in tests/test_oracle.py.)
__device__ __forceinline__ void row_span_slopes(const f64 (&sx)[3], const f64 (&sy)[3], const f64 (&sl)[3], f64 y,
                                                f64 x0, f64 wlim, int& xs, int& xe) {
    const bool b0 = sy[0] > y, b1 = sy[1] > y, b2 = sy[2] > y;
    const bool v1 = (b1 != b0) && (b1 != b2);
    const bool v2 = (b2 != b0) && (b2 != b1);
    const f64 aix = v1 ? sx[2] : sx[0], aiy = v1 ? sy[2] : sy[0], sa = v1 ? sl[2] : sl[0];
    const f64 bix = v2 ? sx[2] : sx[1], biy = v2 ? sy[2] : sy[1], sb = v2 ? sl[2] : sl[1];
    bool safe = true;
    f64 ka = crossing_ceil(y - aiy, sa, aix, safe);
    f64 kb = crossing_ceil(y - biy, sb, bix, safe);
    if (!safe) {   // exact expression (cpp:832-839 order of operations)
        const f64 ajx = v1 ? sx[1] : sx[2], ajy = v1 ? sy[1] : sy[2];
        const f64 bjx = v2 ? sx[1] : sx[0], bjy = v2 ? sy[1] : sy[0];
        ka = ceil((ajx - aix) * (y - aiy) / (ajy - aiy) + aix);
        kb = ceil((bjx - bix) * (y - biy) / (bjy - biy) + bix);
    }
    xs = (int)clampd(fmin(ka, kb) - x0, 0.0, wlim);
    xe = (int)clampd(fmax(ka, kb) - x0, 0.0, wlim);
}

// ---- f32 fast path of row_span_slopes (k_vis) -----------------------------
// The two straddling edges of a row are the two edges at the vertex alone on
// its side of the row: the edges at the lowest-y vertex above the middle
// vertex's y (L = min-max, T = min-mid), at the highest-y vertex from there on
// (L, B = mid-max) -- row_span_in's selection, made once per triangle.  Each
// crossing cc = (y - yi) * s + xi is evaluated in f32 relative to the tile
// origin (xi - x0, yi - y0: exact in f64, small), which is cheap (f32 issues at
// twice the f64 rate) and whose error bound is small:
//   |cc32 - cc| <= 2^-24 (|cc| + 4|v| + |xr|) + |s| (|yr| 2^-48 + |yi| 2^-53)
//                  + |xi| 2^-53 + (the f64 expression's own rounding, 2^-50 (|v| + |cc|))
// (v = (y - yi) s; the bound used, eps = 2^-22 |cc32| + 2^-20 |v32| + ce, has a
// factor 4 of margin and ce per edge).  When cc32 is further than eps from the
// integers on both sides, ceil(cc32) is the exact expression's ceil; otherwise
// (or for non-finite / huge values: eps or cc32 not finite) the row takes
// row_span_slopes, which is itself exact.
struct Edge32 {
    float x, yhi, ylo, s, ce;   // anchor vertex relative to the tile origin (y as hi + lo), slope, error term
};

__device__ __forceinline__ Edge32 edge32(f64 xi, f64 yi, f64 s, f64 x0, f64 y0) {
    Edge32 e;
    const f64 xr = xi - x0, yr = yi - y0;
    e.x = (float)xr;
    e.yhi = (float)yr;
    e.ylo = (float)(yr - (f64)e.yhi);
    e.s = (float)s;
    const float as = fabsf(e.s);
    e.ce = fabsf(e.x) * 0x1p-21f + as * (fabsf(e.yhi) * 0x1p-46f + (float)(fabs(yi) * 0x1p-51)) +
           (float)(fabs(xi) * 0x1p-51) + 0x1p-23f;
    return e;
}

// Per-triangle edge selection: L (min-y vertex to max-y vertex), T (min-mid),
// B (mid-max), each as pointInPolygon's edge k anchored at vertex k (edge_slopes);
// ymid = the middle vertex's y (rows y < ymid use L and T, the others L and B).
struct Span32 {
    Edge32 L, T, B;
    f64 ymid;
};

__device__ __forceinline__ Span32 span32_setup(const f64 (&sx)[3], const f64 (&sy)[3], const f64 (&sl)[3], f64 x0,
                                               f64 y0) {
    const f64 a = sy[0], b = sy[1], c = sy[2];
    const int imin = (b < a) ? ((c < b) ? 2 : 1) : ((c < a) ? 2 : 0);
    const int imax = (b >= a) ? ((c >= b) ? 2 : 1) : ((c >= a) ? 2 : 0);
    const int imid = 3 - imin - imax;
    // edge id of vertex pair {p, q}: {0,2} -> 0, {0,1} -> 1, {1,2} -> 2 (sums 2, 1, 3)
    auto eid = [](int p, int q) { const int s = p + q; return s == 2 ? 0 : (s == 1 ? 1 : 2); };
    auto pick = [&](int k) {
        const f64 xi = k == 0 ? sx[0] : (k == 1 ? sx[1] : sx[2]);
        const f64 yi = k == 0 ? sy[0] : (k == 1 ? sy[1] : sy[2]);
        const f64 si = k == 0 ? sl[0] : (k == 1 ? sl[1] : sl[2]);
        return edge32(xi, yi, si, x0, y0);
    };
    Span32 S;
    S.L = pick(eid(imin, imax));
    S.T = pick(eid(imin, imid));
    S.B = pick(eid(imid, imax));
    S.ymid = imid == 0 ? a : (imid == 1 ? b : c);
    return S;
}

__device__ __forceinline__ float crossing32(const Edge32& e, float rf, bool& ok) {
    const float bb = (rf - e.yhi) - e.ylo;
    const float v = bb * e.s;
    const float cc = v + e.x;
    const float k = ceilf(cc);
    const float d = k - cc;   // in [0, 1), exact
    const float eps = fmaf(fabsf(cc), 0x1p-22f, fmaf(fabsf(v), 0x1p-20f, e.ce));
    ok = ok && (d > eps) && ((1.0f - d) > eps);
    return k;
}

// Row r of the tile (y = y0 + r, a row with exactly two straddling edges):
// the span [xs, xe) relative to x0, clamped to [0, wlim], when the f32 bound
// proves it (returns true); false: the caller evaluates row_span_slopes.
__device__ __forceinline__ bool row_span32(const Span32& S, int r, f64 y, float wlim, int& xs, int& xe) {
    const bool top = y < S.ymid;
    const Edge32& E = top ? S.T : S.B;
    const float rf = (float)r;
    bool ok = true;
    const float ka = crossing32(S.L, rf, ok);
    const float kb = crossing32(E, rf, ok);
    const float lo = fminf(ka, kb), hi = fmaxf(ka, kb);
    xs = (int)fminf(fmaxf(lo, 0.0f), wlim);
    xe = (int)fminf(fmaxf(hi, 0.0f), wlim);
    return ok;
}

// State snapshot of one draw call (passed by value to the kernels).
struct FrameParams {
    TriSrc src;
    f64 m[6];
    f64 ct[4];
    f64* fb;
    u32* depth;
    i64 W, H;
    int ipp;
    int tiles_x, tiles_y;
    int period;   // owned tile rows (BinParams)
    u64 mask;
    int depthTest, depthWrite;
    int pendColor;
    f64 pendColorValue;
    int pendDepth;
    u32 pendDepthValue;
    unsigned long long* fragCounter;   // non-null: count covered fragments
    iu8* frameU8;                      // non-null: resolve also writes the frame output: the u8
                                       // image (cpp:52-57), or with frameYUV its YUV420P planes
    int frameYUV;
    u32* tileStamp;   // non-null: k_vis leaves an empty tile's pending clears pending (stamps it tileEpoch,
    u32 tileEpoch;    // RenderContext::tileStamp) and writes only its frame output
    u64* tstamp;      // non-null (kernel timing): {~first start, last end} of the raster on the device's
                      // 100 MHz clock (raster_stamp_begin / _end, nr_timing_stamp)
};

// Kernel timing of the rasters by the device's constant 100 MHz clock
// (s_memrealtime): the first workgroups dispatched on each XCD (blockIdx < 8)
// max-in the inverted start time, every workgroup the end time -- the
// kernel's execution span, as rocprofv3's kernel trace measures it, with no
// packet on the stream (events around or bound to the launch add the launch
// gap to the time; profiles/r06/ab_event_every.txt).
__device__ __forceinline__ void raster_stamp_begin(const FrameParams& fp) {
    if (fp.tstamp && threadIdx.x == 0 && blockIdx.x < 8)
        atomicMax(reinterpret_cast<unsigned long long*>(&fp.tstamp[0]), ~__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void raster_stamp_end(const FrameParams& fp) {
    if (fp.tstamp && threadIdx.x == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(&fp.tstamp[1]), __builtin_amdgcn_s_memrealtime());
}

// Frame output of pixel p = (px, py) from its framebuffer value, written by
// the rasters' own write-back when they cover every owned pixel (a pending
// clear): the u8 image (cpp:52-57) or, with fp.frameYUV, its YUV420P planes --
// Y of every pixel, U and V from the even pixel of each 2x2 block (tiles have
// even sizes and origins, so a block never straddles two).
// Output stores of the rasters' shading passes (framebuffer, depth, frame
// output): written once per frame and not read again by the kernel, so
// non-temporal (streaming) stores -- round 6, with the fast clear and the
// binning beside the raster: C3 -2.5 %, an 8-way share -2.6 %, 1080p and C2
// within 1 % (profiles/r06/ab_ntst.txt; round 3, frame outputs only: +-2 %).
template <class T>
__device__ __forceinline__ void out_store(T* p, T v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void store_frame_out(const FrameParams& fp, i64 p, i64 px, i64 py, f64 cr, f64 cg, f64 cb,
                                                f64 ca) {
    if (!fp.frameU8) return;
    const int r8 = nr_to_u8(cr), g8 = nr_to_u8(cg), b8 = nr_to_u8(cb);
    if (fp.frameYUV) {
        out_store<iu8>(fp.frameU8 + p, (iu8)nr_y_of(r8, g8, b8));
        if (!((px | py) & 1)) {
            const i64 cw = fp.W >> 1;
            iu8* up = fp.frameU8 + fp.W * fp.H + (py >> 1) * cw + (px >> 1);
            out_store<iu8>(up, (iu8)nr_u_of(r8, g8, b8));
            out_store<iu8>(up + cw * (fp.H >> 1), (iu8)nr_v_of(r8, g8, b8));
        }
    } else {
        iu8* d8 = fp.frameU8 + p * fp.ipp;
        out_store<iu8>(d8, (iu8)r8); out_store<iu8>(d8 + 1, (iu8)g8); out_store<iu8>(d8 + 2, (iu8)b8);
        if (fp.ipp == 4) out_store<iu8>(d8 + 3, (iu8)nr_to_u8(ca));
    }
}

// Per-triangle setup record of the ordered raster, formed once per triangle
// by the counting kernel (k_tri_count, or k_free_count for a binned ordered batch) (a triangle of C5 lies in ~100 tiles; the raster used to set
// it up again in each): screen vertices, edge slopes, 1/den, depths and the
// depth-pass bound (zpass_bound).  16 doubles, 128 B, 16-B aligned.
enum { R_X0 = 0, R_Y0, R_X1, R_Y1, R_X2, R_Y2, R_SL0, R_SL1, R_SL2, R_INV, R_Z0, R_Z1, R_Z2, R_FLAGS, ORec = 16 };

// Depth-pass proof (zpass_all): with the Z test on and Z write off, a
// triangle passes the LESS test on every pixel the exact span rule covers when
// all of them quantise (nr_quantize_depth) strictly below the tile's smallest
// depth zmin.  For a triangle with G = max|edge| / |den|, bbox extent S and
// coordinate magnitude M, G*S <= 1e4 and G*M <= 1e4 bound the computed
// barycentrics of covered pixels to [-1e-10, 1 + 1e-10] (span-rule crossings
// and the w1/w2 expressions both err by O(u (G S + G M)), u = 2^-53; den's
// cancellation by O(u G S) relative), so with |z| <= 2 the computed depth is at
// most max(z) + 1e-9 (< max(z) + 1e-8, the bound used).  The triangle-only
// part is this bound, quantised, or 0xFFFFFFFF when the analysis does not
// apply (no tile minimum lies above it): zpass_all == (zpass_bound < zmin).
__device__ __forceinline__ u32 zpass_bound(const f64 (&sx)[3], const f64 (&sy)[3], f64 e1x, f64 e1y, f64 e2x, f64 e2y,
                                           f64 den, f64 z0, f64 z1, f64 z2) {
    if (!tri_finite(sx, sy) || den == 0) return 0xFFFFFFFFu;
    if (!(fabs(z0) <= 2 && fabs(z1) <= 2 && fabs(z2) <= 2)) return 0xFFFFFFFFu;   // (NaN: no bound)
    const f64 xmn = fmin(fmin(sx[0], sx[1]), sx[2]), xmx = fmax(fmax(sx[0], sx[1]), sx[2]);
    const f64 ymn = fmin(fmin(sy[0], sy[1]), sy[2]), ymx = fmax(fmax(sy[0], sy[1]), sy[2]);
    const f64 e = fmax(fmax(fabs(e1x), fabs(e1y)), fmax(fabs(e2x), fabs(e2y)));
    const f64 G = e / fabs(den);
    const f64 S = (xmx - xmn) + (ymx - ymn) + 4.0;
    const f64 M = fmax(fmax(fabs(xmn), fabs(xmx)), fmax(fabs(ymn), fabs(ymx))) + 1.0;
    if (!(G * S <= 1e4 && G * M <= 1e4)) return 0xFFFFFFFFu;
    return nr_quantize_depth(fmax(fmax(z0, z1), z2) + 1e-8);
}

// Setup record of triangle t (screen vertices sx, sy, valid: finite, den != 0).
__device__ __forceinline__ void write_ordered_record(f64* rec, i64 t, const f64 (&sx)[3], const f64 (&sy)[3],
                                                     const f64* zsrc) {
    const f64 e1x = sx[1] - sx[0], e1y = sy[1] - sy[0], e2x = sx[2] - sx[0], e2y = sy[2] - sy[0];
    const f64 den = e1x * e2y - e2x * e1y;
    f64 sl[3];
    edge_slopes(sx, sy, sl);
    f64 z0 = 0, z1 = 0, z2 = 0;
    if (zsrc) { z0 = zsrc[t * 3]; z1 = zsrc[t * 3 + 1]; z2 = zsrc[t * 3 + 2]; }
    const u64 flags = 1ull | ((u64)zpass_bound(sx, sy, e1x, e1y, e2x, e2y, den, z0, z1, z2) << 32);
    double2* r = reinterpret_cast<double2*>(rec + t * ORec);
    r[0] = make_double2(sx[0], sy[0]);
    r[1] = make_double2(sx[1], sy[1]);
    r[2] = make_double2(sx[2], sy[2]);
    r[3] = make_double2(sl[0], sl[1]);
    r[4] = make_double2(sl[2], 1.0 / den);
    r[5] = make_double2(z0, z1);
    r[6] = make_double2(z2, __longlong_as_double((long long)flags));
}

enum Opacity { OPQ_UNKNOWN = 0, OPQ_OPAQUE, OPQ_BLENDED };

template <typename T, size_t K>
bool grow_set(T* (&ptrs)[K], size_t* cap, size_t need) {
    if (*cap >= need && ptrs[0]) return true;
    size_t n = need > *cap * 3 / 2 ? need : *cap * 3 / 2;
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
bool grow_temp(TriScratch& sc, size_t need);

FrameParams frame_params(RenderContext* ctx, const TriSrc& src);
void finish_batch(RenderContext* ctx, const FrameParams& fp);
u32* tile_stamps(RenderContext* ctx, i64 ntiles);   // the context's tile stamps, next epoch (nr_tri.hip)

// the two rasterisers (host side)
// ordered batches: binned like the order-free ones (count / plan / emit, on the
// binning stream beside the previous raster) when the frame has at most
// ORD_BIN_TILES tiles, each tile's list sorted in LDS (k_tile_sort); the
// global-sort path (draw_ordered_sorted) otherwise, and for a batch with a tile
// of more than ORD_SORT_CAP triangles (detected by the plan, re-run)
void draw_ordered(RenderContext* ctx, const TriSrc& src, TriangleBuffer* tb, bool callerOwned);
void draw_ordered_sorted(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp);
// the same kernels for a deferred re-run (nr_settle): the batch's snapshot only, context flags untouched
void rerun_ordered_sorted(RenderContext* ctx, const TriSrc& src, const FrameParams& fp, const BinParams& bp);
constexpr u32 ORD_SORT_CAP = 8192;    // longest tile list the ordered raster sorts in LDS
constexpr int ORD_BIN_TILES = 16384;  // tiles of the binned ordered path (the register plan kernel's limit)
// binned ordered batches: k_tile_sort sorts each tile's list [off[t], off[t + 1])
// in place (binning stream), then the raster runs one workgroup per tile; both
// are no-ops unless plan[3] (fits)
void launch_tile_sort(const u32* off, u32* list, const u32* plan, int ntiles, hipStream_t s, hipEvent_t stop);
void launch_ordered_binned(const FrameParams& fp, const u32* list, const u32* off, const u32* plan, const f64* rec,
                           int ntiles, hipStream_t s, hipEvent_t start, hipEvent_t stop);
// tb: the batch is that (immutable) TriangleBuffer, so its binning may overlap
// the previous raster and a repeat draw is sized from its known totals;
// callerOwned: the arrays are the caller's device memory (DrawTrianglesDevice),
// so the batch is sized exactly in the call -- an overflow re-run never reads
// them after it returns
void draw_free(RenderContext* ctx, const TriSrc& src, TriangleBuffer* tb, bool callerOwned, bool ordered = false);
void settle(RenderContext* ctx);

}  // namespace nrtri
