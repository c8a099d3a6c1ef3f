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
#include <vector>

namespace {

enum PrimMode { PM_RECT = 0, PM_TEX, PM_SPLIT, PM_VGRD, PM_CIRCLE, PM_LINE, PM_TEX_FAST, PM_FILL, PM_SETPIX };

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

// Colour of pixel (i, j) under draw p; false when the draw does not cover it.
template <int MODE>
__device__ __forceinline__ bool prim_pixel(const PrimParams& p, i64 i, i64 j, f64& r, f64& g, f64& b, f64& a) {
    if constexpr (MODE == PM_FILL) {
        r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
    } else if constexpr (MODE == PM_TEX_FAST) {
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
            if (dist > p.radius) return false;
            r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
        } else if constexpr (MODE == PM_LINE) {
            // cpp:908-917
            if (!nr_point_in_polygon<4>(ix, iy, p.pts)) return false;
            r = p.c[0]; g = p.c[1]; b = p.c[2]; a = p.c[3];
        } else {
            // inclusive quad test, cpp:866-869 / 764-767 / 806-809 / 1302-1305
            if (ix < p.x) return false;
            if (ix > p.x + p.w) return false;
            if (iy < p.y) return false;
            if (iy > p.y + p.h) return false;
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
    return true;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_prim(const PrimParams p) {
    const i64 li = (i64)blockIdx.x * 64 + threadIdx.x;
    const i64 lj = (i64)blockIdx.y * 4 + threadIdx.y;
    if (li >= p.ni || lj >= p.nj) return;
    const i64 i = p.i0 + li, j = p.j0 + lj;
    f64 r, g, b, a;
    if (!prim_pixel<MODE>(p, i, j, r, g, b, a)) return;
    nr_apply_pixel(p.buf + (j * p.W + i) * p.ipp, p.ipp, r, g, b, a, p.ct[0], p.ct[1], p.ct[2], p.ct[3]);
}

// ---- deferred command list ----------------------------------------------
// Recorded draws (the same PrimParams the immediate launches take, bounds
// included) run in one launch: a workgroup owns a CL_W x CL_H screen tile,
// each thread CL_R pixels of one column, held in registers from the first
// command to the last.  Commands are applied in recording order per pixel,
// with the same per-pixel arithmetic (prim_pixel + ApplyPixel), so the result
// equals the immediate sequence bit for bit, while the framebuffer is read and
// written once per list instead of once per draw.  A tile skips a command
// whose pixel range misses it (wave-uniform test on scalar loads).
struct NrCmd {
    int mode;
    PrimParams p;
};
constexpr int CL_W = 64, CL_H = 16, CL_R = CL_H / 4;

// ApplyPixel (cpp:515-549) on a register-resident pixel (nr_apply_pixel's
// expressions).
__device__ __forceinline__ void apply_reg(f64 (&px)[4], int ipp, f64 r, f64 g, f64 b, f64 a, const f64* ct) {
    r *= ct[0]; g *= ct[1]; b *= ct[2]; a *= ct[3];
    if (a != 1) {
        r = px[0] * (1 - a) + r * a;
        g = px[1] * (1 - a) + g * a;
        b = px[2] * (1 - a) + b * a;
    }
    px[0] = r; px[1] = g; px[2] = b;
    if (ipp == 4) px[3] = a;
}

template <int MODE>
__device__ __forceinline__ void cmd_apply(const PrimParams& p, i64 i, i64 j0, int ipp, f64 (&px)[CL_R][4],
                                          bool (&dirty)[CL_R], i64 W, i64 H) {
    const bool colIn = i >= p.i0 && i < p.i0 + p.ni;
#pragma unroll
    for (int r = 0; r < CL_R; ++r) {
        const i64 j = j0 + 4 * r;
        if (!colIn || j < p.j0 || j >= p.j0 + p.nj) continue;
        if constexpr (MODE == PM_SETPIX) {
            // SetPixel (cpp:494-513): raw store of the target pixel; for RGB the
            // reference also writes index+3 = channel 0 of the next pixel (A.6)
            if (i == (i64)p.x && j == (i64)p.y) {
                px[r][0] = p.c[0]; px[r][1] = p.c[1]; px[r][2] = p.c[2];
                if (ipp == 4) px[r][3] = p.c[3];
                dirty[r] = true;
            } else if (ipp == 3 && i == (i64)p.sx && j == (i64)p.sy) {
                px[r][0] = p.c[3];
                dirty[r] = true;
            }
        } else {
            f64 cr, cg, cb, ca;
            if (!prim_pixel<MODE>(p, i, j, cr, cg, cb, ca)) continue;
            apply_reg(px[r], ipp, cr, cg, cb, ca, p.ct);
            dirty[r] = true;
        }
    }
}

template <int IPP>
__global__ __launch_bounds__(256) void k_cmd_list(const NrCmd* __restrict__ cmds, int ncmd, f64* __restrict__ buf,
                                                  i64 W, i64 H, int pend, f64 pendValue) {
    const i64 tx0 = (i64)blockIdx.x * CL_W, ty0 = (i64)blockIdx.y * CL_H;
    const i64 i = tx0 + threadIdx.x;
    const i64 j0 = ty0 + threadIdx.y;
    f64 px[CL_R][4];
    bool dirty[CL_R];
#pragma unroll
    for (int r = 0; r < CL_R; ++r) {
        const i64 j = j0 + 4 * r;
        dirty[r] = pend != 0;
        px[r][0] = px[r][1] = px[r][2] = px[r][3] = pendValue;
        if (!pend && i < W && j < H) {
            const f64* q = buf + (j * W + i) * IPP;
            px[r][0] = q[0]; px[r][1] = q[1]; px[r][2] = q[2];
            if (IPP == 4) px[r][3] = q[3];
        }
    }
    // the commands are taken 256 at a time: each thread tests one against the
    // tile, and the hits are compacted in order (ballot + wave sums) into
    // LDS, so the apply loop visits only the commands that touch the tile
    __shared__ int sIdx[256];
    __shared__ int sWave[4];
    const int tid = threadIdx.y * 64 + threadIdx.x, lane = threadIdx.x, wave = threadIdx.y;
    for (int base = 0; base < ncmd; base += 256) {
        const int cidx = base + tid;
        bool hit = false;
        if (cidx < ncmd) {
            const PrimParams& q = cmds[cidx].p;
            hit = !(q.i0 >= tx0 + CL_W || q.i0 + q.ni <= tx0 || q.j0 >= ty0 + CL_H || q.j0 + q.nj <= ty0);
        }
        const unsigned long long m = __ballot(hit);
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (lane == 0) sWave[wave] = (int)__builtin_popcountll(m);
        __syncthreads();
        int off = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            off += w < wave ? sWave[w] : 0;
            total += sWave[w];
        }
        if (hit) sIdx[off + pre] = cidx;
        __syncthreads();
        for (int k = 0; k < total; ++k) {
        const int c = __builtin_amdgcn_readfirstlane(sIdx[k]);
        const PrimParams& p = cmds[c].p;
        switch (cmds[c].mode) {
            case PM_RECT: cmd_apply<PM_RECT>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_TEX: cmd_apply<PM_TEX>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_SPLIT: cmd_apply<PM_SPLIT>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_VGRD: cmd_apply<PM_VGRD>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_CIRCLE: cmd_apply<PM_CIRCLE>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_LINE: cmd_apply<PM_LINE>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_TEX_FAST: cmd_apply<PM_TEX_FAST>(p, i, j0, IPP, px, dirty, W, H); break;
            case PM_FILL: cmd_apply<PM_FILL>(p, i, j0, IPP, px, dirty, W, H); break;
            default: cmd_apply<PM_SETPIX>(p, i, j0, IPP, px, dirty, W, H); break;
        }
        }
        __syncthreads();   // sIdx / sWave are reused by the next round
    }
#pragma unroll
    for (int r = 0; r < CL_R; ++r) {
        const i64 j = j0 + 4 * r;
        if (!dirty[r] || i >= W || j >= H) continue;
        f64* q = buf + (j * W + i) * IPP;
        q[0] = px[r][0]; q[1] = px[r][1]; q[2] = px[r][2];
        if (IPP == 4) q[3] = px[r][3];
    }
}

struct CmdList {
    std::vector<NrCmd> cmds;
    NrCmd* dev = nullptr;
    size_t devCap = 0;
};

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

static CmdList* cmd_list(RenderContext* ctx) {
    if (!ctx->cmdList) ctx->cmdList = new CmdList();
    return reinterpret_cast<CmdList*>(ctx->cmdList);
}

template <int MODE>
static void launch(RenderContext* ctx, PrimParams& p, i64 i0, i64 i1, i64 j0, i64 j1) {
    if (i1 <= i0 || j1 <= j0) return;
    p.i0 = i0; p.j0 = j0; p.ni = i1 - i0; p.nj = j1 - j0;
    if (ctx->recording) {   // queued; runs with the rest of the list
        cmd_list(ctx)->cmds.push_back(NrCmd{MODE, p});
        return;
    }
    dim3 grid((unsigned)((p.ni + 63) / 64), (unsigned)((p.nj + 3) / 4));
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_PRIM, &e0, &e1);
    hipLaunchKernelGGL(k_prim<MODE>, grid, dim3(64, 4), 0, ctx->stream, p);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_PRIM, e0, e1);
}

static void prepare(RenderContext* ctx) {
    ctx->frameU8Valid = false;
    if (ctx->recording) return;   // a pending clear is applied by the list launch
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
}

// A texture that aliases a framebuffer (CreateTextureFromRenderContextShared)
// is read as it is at the draw: a recorded draw would see it later, so such a
// draw runs immediately, after the list recorded so far.
struct ImmediateScope {
    RenderContext* ctx;
    bool was;
    ImmediateScope(RenderContext* c, const Texture* tex) : ctx(c), was(c->recording) {
        if (was && tex->aliasOf) {
            NR_CHECK(hipSetDevice(ctx->device));
            nr_flush_commands(ctx);
            ctx->recording = false;
        }
    }
    ~ImmediateScope() { ctx->recording = was; }
};

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
    ImmediateScope imm(ctx, tex);
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
    ImmediateScope imm(ctx, tex);
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

// ---- deferred command list: host side ------------------------------------
void nr_flush_commands(RenderContext* ctx) {
    CmdList* L = reinterpret_cast<CmdList*>(ctx->cmdList);
    if (!L || L->cmds.empty()) return;
    const size_t n = L->cmds.size();
    if (L->devCap < n) {
        if (L->dev) NR_CHECK(hipFree(L->dev));
        L->devCap = std::max(n, L->devCap * 2);
        L->dev = nullptr;
        if (hipMalloc((void**)&L->dev, L->devCap * sizeof(NrCmd)) != hipSuccess) {
            nr_set_error_msg("command list: hipMalloc failed");
            L->devCap = 0;
            L->cmds.clear();
            return;
        }
    }
    // pageable source: the copy is staged before the call returns, so the
    // vector can be reused at once
    NR_CHECK(hipMemcpyAsync(L->dev, L->cmds.data(), n * sizeof(NrCmd), hipMemcpyHostToDevice, ctx->stream));
    nr_materialize_tiles(ctx, true, false);
    const int pend = ctx->pendColor ? 1 : 0;
    const f64 pv = ctx->pendColorValue;
    ctx->pendColor = false;   // the launch writes every pixel when a clear is pending
    ctx->frameU8Valid = false;
    if (ctx->width > 0 && ctx->height > 0) {
        dim3 grid((unsigned)((ctx->width + CL_W - 1) / CL_W), (unsigned)((ctx->height + CL_H - 1) / CL_H));
        hipEvent_t e0, e1;
        nr_timing_begin(ctx, NRK_PRIM, &e0, &e1);
        if (ctx->enableAlpha)
            hipLaunchKernelGGL(k_cmd_list<4>, grid, dim3(64, 4), 0, ctx->stream, L->dev, (int)n, ctx->buffer,
                               ctx->width, ctx->height, pend, pv);
        else
            hipLaunchKernelGGL(k_cmd_list<3>, grid, dim3(64, 4), 0, ctx->stream, L->dev, (int)n, ctx->buffer,
                               ctx->width, ctx->height, pend, pv);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_PRIM, e0, e1);
    }
    L->cmds.clear();
}

void nr_drop_commands(RenderContext* ctx) {
    CmdList* L = reinterpret_cast<CmdList*>(ctx->cmdList);
    if (L) L->cmds.clear();
}

void nr_free_commands(RenderContext* ctx) {
    CmdList* L = reinterpret_cast<CmdList*>(ctx->cmdList);
    if (!L) return;
    if (L->dev) {
        NR_CHECK(hipStreamSynchronize(ctx->stream));   // a launch may still read it
        NR_CHECK(hipFree(L->dev));
    }
    delete L;
    ctx->cmdList = nullptr;
}

bool nr_record_fill(RenderContext* ctx, i64 i0, i64 i1, i64 j0, i64 j1, f64 r, f64 g, f64 b, f64 a) {
    PrimParams p = base_params(ctx);
    p.c[0] = r; p.c[1] = g; p.c[2] = b; p.c[3] = a;
    launch<PM_FILL>(ctx, p, i0, i1, j0, j1);
    return true;
}

bool nr_record_set_pixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a) {
    PrimParams p = base_params(ctx);
    p.c[0] = r; p.c[1] = g; p.c[2] = b; p.c[3] = a;
    p.x = (f64)x; p.y = (f64)y;
    // RGB: the pixel whose channel 0 the reference's index+3 store hits (none
    // past the end of the buffer)
    i64 ox = x + 1, oy = y;
    if (ox == ctx->width) { ox = 0; oy = y + 1; }
    p.sx = (f64)ox; p.sy = (f64)(oy < ctx->height ? oy : -1);
    if (ox == 0) launch<PM_SETPIX>(ctx, p, 0, ctx->width, y, std::min<i64>(y + 2, ctx->height));
    else launch<PM_SETPIX>(ctx, p, x, x + 2, y, y + 1);
    return true;
}

extern "C" {

// Starts recording: primitive draws (DrawTexture, DrawSplittedTexture,
// DrawRect, DrawLine, DrawCircle, DrawVerticalGrd, FillColor, ApplyPixel,
// SetPixel) are queued and run together by EndCommandList (or by any call
// that reads or otherwise touches the framebuffer), in recording order and
// with the results of the immediate calls.  Transform and colour-transform
// calls take effect as usual (each queued draw keeps the state it was
// recorded with).  Replaces the reference's recording proxy
// MultiThreadedVideoRenderContextPreparer (Pybind:302-367).
void BeginCommandList(RenderContext* ctx) {
    if (!ctx) return;
    ctx->recording = true;
}

// Runs the queued draws (one launch) and stops recording.
void EndCommandList(RenderContext* ctx) {
    if (!ctx) return;
    NR_CHECK(hipSetDevice(ctx->device));
    nr_settle(ctx);
    ctx->recording = false;
}

// Runs the queued draws and keeps recording (one frame of a recorded stream).
void FlushCommandList(RenderContext* ctx) {
    if (!ctx) return;
    NR_CHECK(hipSetDevice(ctx->device));
    nr_settle(ctx);
}

i64 GetCommandListLength(RenderContext* ctx) {
    CmdList* L = ctx ? reinterpret_cast<CmdList*>(ctx->cmdList) : nullptr;
    return L ? (i64)L->cmds.size() : 0;
}

bool IsRecordingCommands(RenderContext* ctx) { return ctx && ctx->recording; }

}  // extern "C"
