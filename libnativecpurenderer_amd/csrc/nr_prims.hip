// nr_prims.hip — the reference's per-pixel primitives as HIP kernels for
// gfx950: DrawRect / DrawTexture (both paths) / DrawSplittedTexture /
// DrawVerticalGrd / DrawCircle / DrawLine
// (/root/reference/src/libNativeCPURenderer.cpp:720-948, 1285-1316).
//
// Each reference `for i / for j` nest becomes one launch over the same pixel
// set: a 64x4 workgroup covers 64 consecutive pixels of 4 rows, so a wave
// touches one contiguous 64*ipp*8-byte run of a framebuffer row (coalesced).
// The per-pixel arithmetic is the reference's, expression for expression,
// compiled with -ffp-contract=off, so results are bit-identical.  Loop bounds
// are computed on the host exactly as the reference computes them (GetBoarder
// truncation, the IsNoTransform fast-path bounds).
#include "nr_common.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace {

enum PrimMode { PM_RECT = 0, PM_TEX, PM_SPLIT, PM_VGRD, PM_CIRCLE, PM_LINE, PM_TEX_FAST };

struct PrimParams {
    f64* buf;
    i64 W;
    int ipp;
    f64 ct[4];
    f64 inv[6];
    i64 i0, j0, ni, nj;      // pixel range [i0, i0+ni) x [j0, j0+nj)
    f64 x, y, w, h;          // quad in user space (circle: centre in x, y)
    f64 c[4];                // flat colour / gradient top
    f64 c2[4];               // gradient bottom
    const f64* tex;
    i64 tw, th;
    int talpha;
    f64 sx, sy;              // tex->width / width, tex->height / height
    f64 uS, uE, vS, vE;
    f64 radius;
    f64 pts[4][2];           // DrawLine polygon (user space)
};

template <int MODE>
__global__ __launch_bounds__(256) void k_prim(const PrimParams p) {
    const i64 li = (i64)blockIdx.x * 64 + threadIdx.x;
    const i64 lj = (i64)blockIdx.y * 4 + threadIdx.y;
    if (li >= p.ni || lj >= p.nj) return;
    const i64 i = p.i0 + li, j = p.j0 + lj;
    f64 r, g, b, a;
    if constexpr (MODE == PM_TEX_FAST) {
        // cpp:741-750 (IsNoTransform path; the transform is ignored)
        f64 u = ((f64)i - p.x) * p.sx;
        f64 v = ((f64)j - p.y) * p.sy;
        nr_sample(p.tex, p.tw, p.th, p.talpha, u, v, r, g, b, a);
    } else {
        f64 ix, iy;
        nr_xform(p.inv, (f64)i, (f64)j, ix, iy);   // cpp:446-453 on the inverse
        if constexpr (MODE == PM_CIRCLE) {
            // cpp:937-946
            f64 dx = ix - p.x, dy = iy - p.y;
            f64 dist = sqrt(dx * dx + dy * dy);
            if (dist > p.radius) return;
            r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
        } else if constexpr (MODE == PM_LINE) {
            // cpp:908-917
            if (!nr_point_in_polygon<4>(ix, iy, p.pts)) return;
            r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
        } else {
            // inclusive quad test, cpp:866-869 / 764-767 / 806-809 / 1302-1305
            if (ix < p.x) return;
            if (ix > p.x + p.w) return;
            if (iy < p.y) return;
            if (iy > p.y + p.h) return;
            if constexpr (MODE == PM_RECT) {
                r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
            } else if constexpr (MODE == PM_VGRD) {
                // cpp:1307-1312
                f64 t = (iy - p.y) / p.h;
                r = p.c[0] + (p.c2[0] - p.c[0]) * t;
                g = p.c[1] + (p.c2[1] - p.c[1]) * t;
                b = p.c[2] + (p.c2[2] - p.c[2]) * t;
                a = p.c[3] + (p.c2[3] - p.c[3]) * t;
            } else {
                f64 u = (ix - p.x) * p.sx;
                f64 v = (iy - p.y) * p.sy;
                if constexpr (MODE == PM_SPLIT) {
                    // cpp:812-813
                    u = (p.uS + (p.uE - p.uS) * u / (f64)p.tw) * (f64)p.tw;
                    v = (p.vS + (p.vE - p.vS) * v / (f64)p.th) * (f64)p.th;
                }
                nr_sample(p.tex, p.tw, p.th, p.talpha, u, v, r, g, b, a);
            }
        }
    }
    nr_apply_pixel(p.buf + (j * p.W + i) * p.ipp, p.ipp, r, g, b, a, p.ct[0], p.ct[1], p.ct[2], p.ct[3]);
}

static inline f64 dmin(f64 a, f64 b) { return (b < a) ? b : a; }   // std::min
static inline f64 dmax(f64 a, f64 b) { return (a < b) ? b : a; }   // std::max
static inline i64 lmin(i64 a, i64 b) { return (b < a) ? b : a; }
static inline i64 lmax(i64 a, i64 b) { return (a < b) ? b : a; }

// cpp:693-718
static void get_boarder(const f64* m, f64 x, f64 y, f64 w, f64 h, i64* l, i64* r, i64* t, i64* b, f64 mw, f64 mh) {
    f64 ltx, lty, rtx, rty, lbx, lby, rbx, rby;
    nr_xform(m, x, y, ltx, lty);
    nr_xform(m, x + w, y, rtx, rty);
    nr_xform(m, x, y + h, lbx, lby);
    nr_xform(m, x + w, y + h, rbx, rby);
    *l = nr_f2i64(dmin(dmin(ltx, rtx), dmin(lbx, rbx)));
    *r = nr_f2i64(dmax(dmax(ltx, rtx), dmax(lbx, rbx)));
    *t = nr_f2i64(dmin(dmin(lty, rty), dmin(lby, rby)));
    *b = nr_f2i64(dmax(dmax(lty, rty), dmax(lby, rby)));
    *l = lmax(0L, lmin(nr_f2i64(mw), *l));
    *r = lmax(0L, lmin(nr_f2i64(mw), *r));
    *t = lmax(0L, lmin(nr_f2i64(mh), *t));
    *b = lmax(0L, lmin(nr_f2i64(mh), *b));
}

// cpp:472-492
static void inverse_of(const f64* m, f64* out) {
    f64 a = m[0], b = m[1], c = m[2], d = m[3], e = m[4], f = m[5];
    f64 det = a * d - b * c;
    f64 inv_det = det != 0 ? 1 / det : 1e9;
    out[0] = d * inv_det;
    out[1] = -b * inv_det;
    out[2] = -c * inv_det;
    out[3] = a * inv_det;
    out[4] = (c * f - d * e) * inv_det;
    out[5] = (b * e - a * f) * inv_det;
}

// cpp:551-553 (signed sum, Appendix A.4)
static bool is_no_transform(const f64* m) {
    return m[0] - 1 + m[1] + m[2] + m[3] - 1 + m[4] + m[5] < 1e-5;
}

static PrimParams base_params(RenderContext* ctx) {
    PrimParams p;
    memset(&p, 0, sizeof p);
    p.buf = ctx->buffer;
    p.W = ctx->width;
    p.ipp = ctx->enableAlpha ? 4 : 3;
    for (int k = 0; k < 4; ++k) p.ct[k] = ctx->ct[k];
    inverse_of(ctx->m, p.inv);
    return p;
}

template <int MODE>
static void launch(RenderContext* ctx, PrimParams& p, i64 i0, i64 i1, i64 j0, i64 j1) {
    if (i1 <= i0 || j1 <= j0) return;
    p.i0 = i0; p.j0 = j0; p.ni = i1 - i0; p.nj = j1 - j0;
    dim3 grid((unsigned)((p.ni + 63) / 64), (unsigned)((p.nj + 3) / 4));
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_PRIM, &e0, &e1);
    hipLaunchKernelGGL(k_prim<MODE>, grid, dim3(64, 4), 0, ctx->stream, p);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_PRIM, e0, e1);
}

static void prepare(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    ctx->frameU8Valid = false;
}

// Texture source for a draw.  An alias of the destination framebuffer is read
// while being written in the reference (order-dependent result); here the
// draw samples a snapshot taken before it starts.
struct TexSrc {
    const f64* ptr = nullptr;
    f64* tmp = nullptr;
};
static TexSrc tex_source(RenderContext* ctx, Texture* tex) {
    TexSrc s;
    if (tex->aliasOf) nr_materialize_color(tex->aliasOf);
    s.ptr = tex->buffer;
    if (tex->buffer == ctx->buffer) {
        size_t bytes = (size_t)(tex->width * tex->height * (tex->enableAlpha ? 4 : 3)) * sizeof(f64);
        NR_CHECK(hipMalloc((void**)&s.tmp, bytes));
        NR_CHECK(hipMemcpyAsync(s.tmp, tex->buffer, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        s.ptr = s.tmp;
    }
    return s;
}
static void tex_release(RenderContext* ctx, TexSrc& s) {
    if (!s.tmp) return;
    NR_CHECK(hipStreamSynchronize(ctx->stream));   // rare path: a texture aliasing its own target
    NR_CHECK(hipFree(s.tmp));
}

// Fast-path loop bounds of cpp:741-742: i from (i64)x while (f64)i < x + w,
// intersected with the screen (ApplyPixel clips everything else).
static void fast_range(f64 x, f64 w, i64 limit, i64* lo, i64* hi) {
    f64 lim = x + w;
    i64 s = nr_f2i64(x);
    *lo = 0; *hi = 0;
    if (!((f64)s < lim)) return;
    i64 e;
    if (!(lim < 9.0e15)) e = LONG_MAX;
    else {
        e = (i64)std::ceil(lim);
        while ((f64)(e - 1) >= lim) --e;
        while ((f64)e < lim) ++e;
    }
    *lo = lmax(s, 0);
    *hi = lmin(e, limit);
}

}  // namespace

extern "C" {

// cpp:720-779
void DrawTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height) {
    if (width == 0 || height == 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    TexSrc src = tex_source(ctx, tex);
    p.tex = src.ptr; p.tw = tex->width; p.th = tex->height; p.talpha = tex->enableAlpha;
    p.sx = tex->width / width;
    p.sy = tex->height / height;
    p.x = x; p.y = y; p.w = width; p.h = height;
    if (is_no_transform(ctx->m)) {
        i64 i0, i1, j0, j1;
        fast_range(x, width, ctx->width, &i0, &i1);
        fast_range(y, height, ctx->height, &j0, &j1);
        launch<PM_TEX_FAST>(ctx, p, i0, i1, j0, j1);
    } else {
        i64 l, r, t, b;
        get_boarder(ctx->m, x, y, width, height, &l, &r, &t, &b, (f64)ctx->width, (f64)ctx->height);
        launch<PM_TEX>(ctx, p, l, r, t, b);
    }
    tex_release(ctx, src);
}

// cpp:781-820
void DrawSplittedTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height, f64 uStart,
                         f64 uEnd, f64 vStart, f64 vEnd) {
    if (width == 0 || height == 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    TexSrc src = tex_source(ctx, tex);
    p.tex = src.ptr; p.tw = tex->width; p.th = tex->height; p.talpha = tex->enableAlpha;
    p.sx = tex->width / width;
    p.sy = tex->height / height;
    p.x = x; p.y = y; p.w = width; p.h = height;
    p.uS = uStart; p.uE = uEnd; p.vS = vStart; p.vE = vEnd;
    i64 l, r, t, b;
    get_boarder(ctx->m, x, y, width, height, &l, &r, &t, &b, (f64)ctx->width, (f64)ctx->height);
    launch<PM_SPLIT>(ctx, p, l, r, t, b);
    tex_release(ctx, src);
}

// cpp:847-874
void DrawRect(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height, f64 r, f64 g, f64 b, f64 a) {
    if (width <= 0 || height <= 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    p.x = x; p.y = y; p.w = width; p.h = height;
    p.c[0] = r; p.c[1] = g; p.c[2] = b; p.c[3] = a;
    i64 l, rr, t, bb;
    get_boarder(ctx->m, x, y, width, height, &l, &rr, &t, &bb, (f64)ctx->width, (f64)ctx->height);
    launch<PM_RECT>(ctx, p, l, rr, t, bb);
}

// cpp:1285-1316
void DrawVerticalGrd(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height, f64 top_r, f64 top_g, f64 top_b,
                     f64 top_a, f64 bottom_r, f64 bottom_g, f64 bottom_b, f64 bottom_a) {
    if (width <= 0 || height <= 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    p.x = x; p.y = y; p.w = width; p.h = height;
    p.c[0] = top_r; p.c[1] = top_g; p.c[2] = top_b; p.c[3] = top_a;
    p.c2[0] = bottom_r; p.c2[1] = bottom_g; p.c2[2] = bottom_b; p.c2[3] = bottom_a;
    i64 l, r, t, b;
    get_boarder(ctx->m, x, y, width, height, &l, &r, &t, &b, (f64)ctx->width, (f64)ctx->height);
    launch<PM_VGRD>(ctx, p, l, r, t, b);
}

// cpp:920-948 (bbox from GetBoarder(x-r, y-r, 2r, 2r))
void DrawCircle(RenderContext* ctx, f64 x, f64 y, f64 radius, f64 r, f64 g, f64 b, f64 a) {
    if (radius <= 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    p.x = x; p.y = y; p.radius = radius;
    p.c[0] = r; p.c[1] = g; p.c[2] = b; p.c[3] = a;
    i64 l, rr, t, bb;
    get_boarder(ctx->m, x - radius, y - radius, 2 * radius, 2 * radius, &l, &rr, &t, &bb, (f64)ctx->width,
                (f64)ctx->height);
    launch<PM_CIRCLE>(ctx, p, l, rr, t, bb);
}

// cpp:876-918.  The reference scans all W*H pixels.  A pixel outside the
// polygon's screen-space bounding box (plus a margin) maps, through the
// inverse transform, to a point outside the polygon's x- or y-range, where
// the even-odd count is 0 (Appendix A.9), so scanning only that box gives the
// same pixels.  A singular or non-finite transform falls back to the full scan.
void DrawLine(RenderContext* ctx, f64 x1, f64 y1, f64 x2, f64 y2, f64 width, f64 r, f64 g, f64 b, f64 a) {
    if (width <= 0) return;
    f64 dx = x2 - x1, dy = y2 - y1;
    f64 len = sqrt(dx * dx + dy * dy);
    if (len == 0) return;
    prepare(ctx);
    PrimParams p = base_params(ctx);
    f64 ux = dx / len, uy = dy / len;
    f64 vx = -uy, vy = ux;
    f64 hw = width / 2;
    f64 pts[4][2] = {
        {x1 - vx * hw, y1 - vy * hw},
        {x1 + vx * hw, y1 + vy * hw},
        {x2 + vx * hw, y2 + vy * hw},
        {x2 - vx * hw, y2 - vy * hw},
    };
    for (int k = 0; k < 4; ++k) { p.pts[k][0] = pts[k][0]; p.pts[k][1] = pts[k][1]; }
    p.c[0] = r; p.c[1] = g; p.c[2] = b; p.c[3] = a;
    i64 i0 = 0, i1 = ctx->width, j0 = 0, j1 = ctx->height;
    const f64* m = ctx->m;
    f64 det = m[0] * m[3] - m[1] * m[2];
    bool full = !(det != 0) || !std::isfinite(det);
    f64 mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY;
    for (int k = 0; k < 4 && !full; ++k) {
        f64 sx, sy;
        nr_xform(m, pts[k][0], pts[k][1], sx, sy);
        if (!std::isfinite(sx) || !std::isfinite(sy)) full = true;
        mnx = std::min(mnx, sx); mxx = std::max(mxx, sx);
        mny = std::min(mny, sy); mxy = std::max(mxy, sy);
    }
    if (!full) {
        f64 mag = std::max(std::max(std::fabs(mnx), std::fabs(mxx)), std::max(std::fabs(mny), std::fabs(mxy)));
        f64 margin = 2.0 + mag * 1e-9;
        f64 fx0 = std::floor(mnx - margin), fx1 = std::ceil(mxx + margin) + 1;
        f64 fy0 = std::floor(mny - margin), fy1 = std::ceil(mxy + margin) + 1;
        i0 = (i64)std::max(0.0, std::min((f64)ctx->width, fx0));
        i1 = (i64)std::max(0.0, std::min((f64)ctx->width, fx1));
        j0 = (i64)std::max(0.0, std::min((f64)ctx->height, fy0));
        j1 = (i64)std::max(0.0, std::min((f64)ctx->height, fy1));
    }
    launch<PM_LINE>(ctx, p, i0, i1, j0, j1);
}

}  // extern "C"
