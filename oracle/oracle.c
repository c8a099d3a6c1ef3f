/*
 * oracle.c — CPU restatement of libNativeCPURenderer's raster path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in libnativecpurenderer_amd/ links, loads
 * or calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * It exports the reference's own C ABI names (/root/reference/src/
 * libNativeCPURenderer.h:83-152) so the same scene driver can run a scene on
 * the oracle and on the HIP library and compare the framebuffers bit for bit.
 * Every function cites the reference lines it restates.  Built with the
 * reference's flags (-O3 -g, compile.sh:1) plus -ffp-contract=off; baseline
 * x86-64 has no FMA, so the arithmetic is SSE2 double, left to right, exactly
 * like the reference build.
 *
 * Parity pinning: the reference itself cannot be built in this image (its
 * header includes FFmpeg headers that are absent, libNativeCPURenderer.h:20-25)
 * and ships no tests or golden vectors.  This restatement is
 * pinned by the reference behaviours recorded in SURVEY.md Appendix A (checked
 * in tests/test_oracle.py) and by hand-derived known answers.  The triangle /
 * depth / Gouraud entry points (DrawTriangles & co.) have NO reference
 * implementation: their semantics are defined here in the reference's idiom
 * (pointInPolygon coverage cpp:822-845, ApplyPixel blend cpp:515-549,
 * DrawVerticalGrd-style interpolation cpp:1308-1312) — "parity unpinned by
 * the reference" for those, see DESIGN.md §3.
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <limits.h>

typedef long i64;
typedef double f64;
typedef unsigned char iu8;

typedef struct { f64 m[6]; f64 ct[4]; } State;

typedef struct RenderContext {
    i64 width, height;
    bool enableAlpha;
    f64 *buffer;
    f64 m[6];          /* transformMatrix, h:39 */
    f64 ct[4];         /* colorTransform, h:40 */
    State *stack; i64 nstack, capstack;   /* std::stack<RenderContextState>, h:41 */
    /* depth state (new; no reference counterpart) */
    uint32_t *depth;
    bool depthTest, depthWrite;
} RenderContext;

typedef struct Texture {
    i64 width, height;
    bool enableAlpha;
    f64 *buffer;
    bool shared;
} Texture;

static i64 g_last_fragments = 0;

/* x86-64 cvttsd2si semantics for (i64)double: out of range / NaN -> INT64_MIN. */
static inline i64 f2i64(f64 v) {
    if (!(v >= -9223372036854775808.0 && v < 9223372036854775808.0)) return LONG_MIN;
    return (i64)v;
}
static inline f64 dmin(f64 a, f64 b) { return (b < a) ? b : a; }   /* std::min */
static inline f64 dmax(f64 a, f64 b) { return (a < b) ? b : a; }   /* std::max */
static inline i64 lmin(i64 a, i64 b) { return (b < a) ? b : a; }
static inline i64 lmax(i64 a, i64 b) { return (a < b) ? b : a; }

/* cpp:3-5 */
i64 GetBufferSize(RenderContext *ctx) {
    return ctx->width * ctx->height * (ctx->enableAlpha ? 4 : 3);
}

static void alloc_depth(RenderContext *ctx) {
    i64 n = ctx->width * ctx->height;
    ctx->depth = (uint32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint32_t));
    for (i64 i = 0; i < n; ++i) ctx->depth[i] = 0xFFFFFFFFu;
}

/* cpp:7-31.  The reference leaves the buffer uninitialised (Appendix A.11);
 * the oracle zeroes it — any content is a valid restatement. */
RenderContext *CreateRenderContext(i64 width, i64 height, bool enableAlpha) {
    RenderContext *ctx = (RenderContext *)calloc(1, sizeof(RenderContext));
    ctx->width = width; ctx->height = height; ctx->enableAlpha = enableAlpha;
    i64 n = GetBufferSize(ctx);
    ctx->buffer = (f64 *)calloc((size_t)(n > 0 ? n : 1), sizeof(f64));
    ctx->m[0] = 1; ctx->m[1] = 0; ctx->m[2] = 0; ctx->m[3] = 1; ctx->m[4] = 0; ctx->m[5] = 0;
    ctx->ct[0] = 1; ctx->ct[1] = 1; ctx->ct[2] = 1; ctx->ct[3] = 1;
    alloc_depth(ctx);
    return ctx;
}

/* cpp:33-37 is a no-op leak in the reference; the oracle frees. */
void DestroyRenderContext(RenderContext *ctx) {
    if (!ctx) return;
    free(ctx->buffer); free(ctx->stack); free(ctx->depth); free(ctx);
}

/* cpp:39-45 */
void ResizeRenderContext(RenderContext *ctx, i64 width, i64 height) {
    i64 n = width * height * (ctx->enableAlpha ? 4 : 3);
    free(ctx->buffer);
    ctx->buffer = (f64 *)calloc((size_t)(n > 0 ? n : 1), sizeof(f64));
    ctx->width = width; ctx->height = height;
    free(ctx->depth);
    alloc_depth(ctx);
}

/* cpp:52-57 — (iu8)(v*255) is cvttsd2si to int32 then the low byte
 * (Appendix A.5); NaN / out of int32 range gives 0x80000000 -> 0. */
void GetBufferAsUInt8(RenderContext *ctx, iu8 *out) {
    i64 size = GetBufferSize(ctx);
    for (i64 i = 0; i < size; ++i) {
        f64 t = ctx->buffer[i] * 255;
        out[i] = (t > -2147483649.0 && t < 2147483648.0) ? (iu8)((int)t & 0xFF) : 0;
    }
}

/* cpp:277-289 */
void SaveContextState(RenderContext *ctx) {
    if (ctx->nstack == ctx->capstack) {
        ctx->capstack = ctx->capstack ? 2 * ctx->capstack : 16;
        ctx->stack = (State *)realloc(ctx->stack, (size_t)ctx->capstack * sizeof(State));
    }
    memcpy(ctx->stack[ctx->nstack].m, ctx->m, sizeof ctx->m);
    memcpy(ctx->stack[ctx->nstack].ct, ctx->ct, sizeof ctx->ct);
    ctx->nstack++;
}

/* cpp:291-309 */
bool RestoreContextState(RenderContext *ctx) {
    if (ctx->nstack == 0) return false;
    ctx->nstack--;
    memcpy(ctx->m, ctx->stack[ctx->nstack].m, sizeof ctx->m);
    memcpy(ctx->ct, ctx->stack[ctx->nstack].ct, sizeof ctx->ct);
    return true;
}

/* cpp:311-316 */
void GetBuffer(RenderContext *ctx, f64 *out) {
    memcpy(out, ctx->buffer, (size_t)GetBufferSize(ctx) * sizeof(f64));
}

/* cpp:318-335 */
Texture *CreateTexture(i64 width, i64 height, bool enableAlpha, f64 *buffer) {
    Texture *t = (Texture *)calloc(1, sizeof(Texture));
    t->width = width; t->height = height; t->enableAlpha = enableAlpha;
    i64 size = width * height * (enableAlpha ? 4 : 3);
    t->buffer = (f64 *)malloc((size_t)(size > 0 ? size : 1) * sizeof(f64));
    for (i64 i = 0; i < size; ++i) t->buffer[i] = buffer[i];
    return t;
}

/* cpp:337-354 */
Texture *CreateTextureUInt8(i64 width, i64 height, bool enableAlpha, iu8 *buffer) {
    Texture *t = (Texture *)calloc(1, sizeof(Texture));
    t->width = width; t->height = height; t->enableAlpha = enableAlpha;
    i64 size = width * height * (enableAlpha ? 4 : 3);
    t->buffer = (f64 *)malloc((size_t)(size > 0 ? size : 1) * sizeof(f64));
    for (i64 i = 0; i < size; ++i) t->buffer[i] = buffer[i] / 255.0;
    return t;
}

/* cpp:356-360 (no-op in the reference) */
void DestroyTexture(Texture *t) {
    if (!t) return;
    if (!t->shared) free(t->buffer);
    free(t);
}

/* cpp:362-375 */
Texture *CreateTextureFromRenderContext(RenderContext *ctx) {
    Texture *t = (Texture *)calloc(1, sizeof(Texture));
    t->width = ctx->width; t->height = ctx->height; t->enableAlpha = ctx->enableAlpha;
    i64 size = GetBufferSize(ctx);
    t->buffer = (f64 *)malloc((size_t)(size > 0 ? size : 1) * sizeof(f64));
    memcpy(t->buffer, ctx->buffer, (size_t)size * sizeof(f64));
    return t;
}

/* cpp:377-384 — non-owning alias of the framebuffer */
Texture *CreateTextureFromRenderContextShared(RenderContext *ctx) {
    Texture *t = (Texture *)calloc(1, sizeof(Texture));
    t->width = ctx->width; t->height = ctx->height; t->enableAlpha = ctx->enableAlpha;
    t->buffer = ctx->buffer; t->shared = true;
    return t;
}

/* cpp:386-396 */
void SetTransform(RenderContext *ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f) {
    ctx->m[0] = a; ctx->m[1] = b; ctx->m[2] = c; ctx->m[3] = d; ctx->m[4] = e; ctx->m[5] = f;
}

/* cpp:398-411 */
void ApplyTransform(RenderContext *ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f) {
    f64 o[6];
    for (int i = 0; i < 6; ++i) o[i] = ctx->m[i];
    ctx->m[0] = o[0] * a + o[2] * b;
    ctx->m[1] = o[1] * a + o[3] * b;
    ctx->m[2] = o[0] * c + o[2] * d;
    ctx->m[3] = o[1] * c + o[3] * d;
    ctx->m[4] = o[0] * e + o[2] * f + o[4];
    ctx->m[5] = o[1] * e + o[3] * f + o[5];
}

/* cpp:420-426 */
void Scale(RenderContext *ctx, f64 sx, f64 sy) { ApplyTransform(ctx, sx, 0, 0, sy, 0, 0); }
/* cpp:428-434 */
void Translate(RenderContext *ctx, f64 tx, f64 ty) { ApplyTransform(ctx, 1, 0, 0, 1, tx, ty); }
/* cpp:436-444 */
void Rotate(RenderContext *ctx, f64 angle) {
    f64 s = sin(angle), c = cos(angle);
    ApplyTransform(ctx, c, s, -s, c, 0, 0);
}

/* cpp:446-453 */
static inline void xform(const f64 m[6], f64 x, f64 y, f64 *ox, f64 *oy) {
    *ox = m[0] * x + m[2] * y + m[4];
    *oy = m[1] * x + m[3] * y + m[5];
}

/* cpp:455-461 (inline in the reference, exported here) */
void TransformPoint(RenderContext *ctx, f64 x, f64 y, f64 *ox, f64 *oy) { xform(ctx->m, x, y, ox, oy); }

/* cpp:463-470 */
void GetTransform(RenderContext *ctx, f64 out[6]) { for (int i = 0; i < 6; ++i) out[i] = ctx->m[i]; }

/* cpp:472-492 — singular matrices use inv_det = 1e9 (Appendix A.10) */
static void inverse_of(const f64 m[6], f64 out[6]) {
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
void GetInverseTransform(RenderContext *ctx, f64 out[6]) { inverse_of(ctx->m, out); }

/* cpp:494-513 — raw store, no colour transform; writes index+3 even when
 * ipp == 3 (Appendix A.6).  The store past the end of the buffer (last pixel
 * of an RGB context) is UB in the reference and is skipped here. */
bool SetPixel(RenderContext *ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a) {
    if (x < 0 || x >= ctx->width || y < 0 || y >= ctx->height) return false;
    i64 ipp = ctx->enableAlpha ? 4 : 3;
    i64 index = y * ctx->width * ipp + x * ipp;
    ctx->buffer[index + 0] = r;
    ctx->buffer[index + 1] = g;
    ctx->buffer[index + 2] = b;
    if (index + 3 < GetBufferSize(ctx)) ctx->buffer[index + 3] = a;
    return true;
}

/* cpp:515-549 — colour transform then "over"; RGBA stores dst.a = a
 * (Appendix A.8; the composite at cpp:545 is dead). */
bool ApplyPixel(RenderContext *ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a) {
    if (x < 0 || x >= ctx->width || y < 0 || y >= ctx->height) return false;
    r *= ctx->ct[0];
    g *= ctx->ct[1];
    b *= ctx->ct[2];
    a *= ctx->ct[3];
    i64 ipp = ctx->enableAlpha ? 4 : 3;
    i64 index = y * ctx->width * ipp + x * ipp;
    f64 *p = ctx->buffer + index;
    if (a != 1) {
        r = p[0] * (1 - a) + r * a;
        g = p[1] * (1 - a) + g * a;
        b = p[2] * (1 - a) + b * a;
    }
    p[0] = r; p[1] = g; p[2] = b;
    if (ctx->enableAlpha) p[3] = a;
    return true;
}

/* cpp:551-553 — signed sum, not an abs test (Appendix A.4) */
static bool IsNoTransform(const f64 m[6]) {
    return m[0] - 1 + m[1] + m[2] + m[3] - 1 + m[4] + m[5] < 1e-5;
}

/* cpp:555-573 — nearest texel; clamp to [0, w-2] x [0, h-2] (Appendix A.3).
 * RGB textures leave alpha uninitialised in the reference (A.2); defined 1. */
static inline void sample(const Texture *t, f64 x, f64 y, f64 *r, f64 *g, f64 *b, f64 *a) {
    if (x < 0) x = 0;
    if (x >= t->width - 1) x = t->width - 2;
    if (y < 0) y = 0;
    if (y >= t->height - 1) y = t->height - 2;
    i64 ipp = t->enableAlpha ? 4 : 3;
    i64 index = (i64)y * t->width * ipp + (i64)x * ipp;
    *r = t->buffer[index + 0];
    *g = t->buffer[index + 1];
    *b = t->buffer[index + 2];
    *a = t->enableAlpha ? t->buffer[index + 3] : 1.0;
}

/* cpp:623-631 */
void SetColorTransform(RenderContext *ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->ct[0] = r; ctx->ct[1] = g; ctx->ct[2] = b; ctx->ct[3] = a;
}
/* cpp:633-641 */
void ApplyColorTransform(RenderContext *ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->ct[0] *= r; ctx->ct[1] *= g; ctx->ct[2] *= b; ctx->ct[3] *= a;
}

/* cpp:643-657 — uniform clear fills every channel with r; otherwise SetPixel
 * x-outer / y-inner (the order makes the A.6 overrun visible in column 0). */
void SetColor(RenderContext *ctx, f64 r, f64 g, f64 b, f64 a) {
    if (r == g && g == b && b == a) {
        i64 n = GetBufferSize(ctx);
        for (i64 i = 0; i < n; ++i) ctx->buffer[i] = r;
        return;
    }
    for (i64 i = 0; i < ctx->width; ++i)
        for (i64 j = 0; j < ctx->height; ++j)
            SetPixel(ctx, i, j, r, g, b, a);
}

/* cpp:659-680 (the reference Python binding passes c_long here and crashes,
 * SURVEY §8b; the C signature takes f64). */
void GetColor(RenderContext *ctx, f64 x, f64 y, f64 *r, f64 *g, f64 *b, f64 *a) {
    if (x < 0) x = 0;
    if (x >= ctx->width) x = ctx->width - 1;
    if (y < 0) y = 0;
    if (y >= ctx->height) y = ctx->height - 1;
    i64 ix = (i64)x, iy = (i64)y;
    i64 ipp = ctx->enableAlpha ? 4 : 3;
    i64 index = iy * ctx->width * ipp + ix * ipp;
    *r = ctx->buffer[index + 0];
    *g = ctx->buffer[index + 1];
    *b = ctx->buffer[index + 2];
    if (ctx->enableAlpha) *a = ctx->buffer[index + 3];
}

/* cpp:682-691 */
void FillColor(RenderContext *ctx, f64 r, f64 g, f64 b, f64 a) {
    for (i64 i = 0; i < ctx->width; ++i)
        for (i64 j = 0; j < ctx->height; ++j)
            ApplyPixel(ctx, i, j, r, g, b, a);
}

/* cpp:693-718 — truncating bbox, right/bottom exclusive in the callers */
static void GetBoarder(const f64 m[6], f64 x, f64 y, f64 w, f64 h,
                       i64 *l, i64 *r, i64 *t, i64 *b, f64 mw, f64 mh) {
    f64 ltx, lty, rtx, rty, lbx, lby, rbx, rby;
    xform(m, x, y, &ltx, &lty);
    xform(m, x + w, y, &rtx, &rty);
    xform(m, x, y + h, &lbx, &lby);
    xform(m, x + w, y + h, &rbx, &rby);
    *l = f2i64(dmin(dmin(ltx, rtx), dmin(lbx, rbx)));
    *r = f2i64(dmax(dmax(ltx, rtx), dmax(lbx, rbx)));
    *t = f2i64(dmin(dmin(lty, rty), dmin(lby, rby)));
    *b = f2i64(dmax(dmax(lty, rty), dmax(lby, rby)));
    *l = lmax(0L, lmin(f2i64(mw), *l));
    *r = lmax(0L, lmin(f2i64(mw), *r));
    *t = lmax(0L, lmin(f2i64(mh), *t));
    *b = lmax(0L, lmin(f2i64(mh), *b));
}

/* cpp:720-779 */
void DrawTexture(RenderContext *ctx, Texture *tex, f64 x, f64 y, f64 width, f64 height) {
    if (width == 0 || height == 0) return;
    f64 scaleX = tex->width / width;
    f64 scaleY = tex->height / height;
    if (IsNoTransform(ctx->m)) {
        /* fast path: the transform is ignored (A.4); loop bounds i64 i = x
         * (truncation) while i < x + width (f64 compare); ApplyPixel clips. */
        /* Pixels with i < 0, j < 0, i >= W or j >= H are clipped by
         * ApplyPixel, so skipping them leaves the result unchanged. */
        for (i64 i = lmax(f2i64(x), 0); i < x + width; ++i) {
            if (i >= ctx->width) break;
            for (i64 j = lmax(f2i64(y), 0); j < y + height; ++j) {
                if (j >= ctx->height) break;
                f64 u = (i - x) * scaleX;
                f64 v = (j - y) * scaleY;
                f64 r, g, b, a;
                sample(tex, u, v, &r, &g, &b, &a);
                ApplyPixel(ctx, i, j, r, g, b, a);
            }
        }
    } else {
        f64 inv[6];
        inverse_of(ctx->m, inv);
        i64 left, right, top, bottom;
        GetBoarder(ctx->m, x, y, width, height, &left, &right, &top, &bottom,
                   (f64)ctx->width, (f64)ctx->height);
        for (i64 i = left; i < right; ++i)
            for (i64 j = top; j < bottom; ++j) {
                f64 ix, iy;
                xform(inv, (f64)i, (f64)j, &ix, &iy);
                if (ix < x) continue;
                if (ix > x + width) continue;
                if (iy < y) continue;
                if (iy > y + height) continue;
                f64 u = (ix - x) * scaleX;
                f64 v = (iy - y) * scaleY;
                f64 r, g, b, a;
                sample(tex, u, v, &r, &g, &b, &a);
                ApplyPixel(ctx, i, j, r, g, b, a);
            }
    }
}

/* cpp:781-820 */
void DrawSplittedTexture(RenderContext *ctx, Texture *tex, f64 x, f64 y, f64 width, f64 height,
                         f64 uStart, f64 uEnd, f64 vStart, f64 vEnd) {
    if (width == 0 || height == 0) return;
    f64 inv[6];
    inverse_of(ctx->m, inv);
    f64 scaleX = tex->width / width;
    f64 scaleY = tex->height / height;
    i64 left, right, top, bottom;
    GetBoarder(ctx->m, x, y, width, height, &left, &right, &top, &bottom,
               (f64)ctx->width, (f64)ctx->height);
    for (i64 i = left; i < right; ++i)
        for (i64 j = top; j < bottom; ++j) {
            f64 ix, iy;
            xform(inv, (f64)i, (f64)j, &ix, &iy);
            if (ix < x) continue;
            if (ix > x + width) continue;
            if (iy < y) continue;
            if (iy > y + height) continue;
            f64 u = (ix - x) * scaleX;
            f64 v = (iy - y) * scaleY;
            u = (uStart + (uEnd - uStart) * u / tex->width) * tex->width;
            v = (vStart + (vEnd - vStart) * v / tex->height) * tex->height;
            f64 r, g, b, a;
            sample(tex, u, v, &r, &g, &b, &a);
            ApplyPixel(ctx, i, j, r, g, b, a);
        }
}

/* cpp:822-845 — even-odd crossing test */
static inline bool pointInPolygon(f64 x, f64 y, const f64 pts[][2], i64 n) {
    i64 j = n - 1;
    bool res = false;
    for (i64 i = 0; i < n; ++i) {
        if ((pts[i][1] > y) != (pts[j][1] > y) &&
            (x < (pts[j][0] - pts[i][0]) * (y - pts[i][1]) / (pts[j][1] - pts[i][1]) + pts[i][0]))
            res = !res;
        j = i;
    }
    return res;
}

/* cpp:847-874 */
void DrawRect(RenderContext *ctx, f64 x, f64 y, f64 width, f64 height, f64 r, f64 g, f64 b, f64 a) {
    if (width <= 0 || height <= 0) return;
    f64 inv[6];
    inverse_of(ctx->m, inv);
    i64 left, right, top, bottom;
    GetBoarder(ctx->m, x, y, width, height, &left, &right, &top, &bottom,
               (f64)ctx->width, (f64)ctx->height);
    for (i64 i = left; i < right; ++i)
        for (i64 j = top; j < bottom; ++j) {
            f64 ix, iy;
            xform(inv, (f64)i, (f64)j, &ix, &iy);
            if (ix < x) continue;
            if (ix > x + width) continue;
            if (iy < y) continue;
            if (iy > y + height) continue;
            ApplyPixel(ctx, i, j, r, g, b, a);
        }
}

/* cpp:876-918 — scans every pixel of the screen (Appendix A.9) */
void DrawLine(RenderContext *ctx, f64 x1, f64 y1, f64 x2, f64 y2, f64 width,
              f64 r, f64 g, f64 b, f64 a) {
    if (width <= 0) return;
    f64 inv[6];
    inverse_of(ctx->m, inv);
    f64 dx = x2 - x1, dy = y2 - y1;
    f64 len = sqrt(dx * dx + dy * dy);
    if (len == 0) return;
    f64 ux = dx / len, uy = dy / len;
    f64 vx = -uy, vy = ux;
    f64 hw = width / 2;
    f64 pts[4][2] = {
        {x1 - vx * hw, y1 - vy * hw},
        {x1 + vx * hw, y1 + vy * hw},
        {x2 + vx * hw, y2 + vy * hw},
        {x2 - vx * hw, y2 - vy * hw},
    };
    for (i64 i = 0; i < ctx->width; ++i)
        for (i64 j = 0; j < ctx->height; ++j) {
            f64 ix, iy;
            xform(inv, (f64)i, (f64)j, &ix, &iy);
            if (!pointInPolygon(ix, iy, pts, 4)) continue;
            ApplyPixel(ctx, i, j, r, g, b, a);
        }
}

/* cpp:920-948 */
void DrawCircle(RenderContext *ctx, f64 x, f64 y, f64 radius, f64 r, f64 g, f64 b, f64 a) {
    if (radius <= 0) return;
    f64 inv[6];
    inverse_of(ctx->m, inv);
    i64 left, right, top, bottom;
    GetBoarder(ctx->m, x - radius, y - radius, 2 * radius, 2 * radius,
               &left, &right, &top, &bottom, (f64)ctx->width, (f64)ctx->height);
    for (i64 i = left; i < right; ++i)
        for (i64 j = top; j < bottom; ++j) {
            f64 ix, iy;
            xform(inv, (f64)i, (f64)j, &ix, &iy);
            f64 dx = ix - x, dy = iy - y;
            f64 dist = sqrt(dx * dx + dy * dy);
            if (dist > radius) continue;
            ApplyPixel(ctx, i, j, r, g, b, a);
        }
}

/* cpp:950-976 */
Texture *ResampleTexture(Texture *tex, i64 width, i64 height) {
    Texture *res = (Texture *)calloc(1, sizeof(Texture));
    res->width = width; res->height = height; res->enableAlpha = tex->enableAlpha;
    i64 ipp = tex->enableAlpha ? 4 : 3;
    res->buffer = (f64 *)malloc((size_t)(width * height * ipp > 0 ? width * height * ipp : 1) * sizeof(f64));
    for (i64 i = 0; i < width; ++i)
        for (i64 j = 0; j < height; ++j) {
            f64 r, g, b, a;
            sample(tex, (f64)i / width * tex->width, (f64)j / height * tex->height, &r, &g, &b, &a);
            f64 *p = res->buffer + j * res->width * ipp + i * ipp;
            p[0] = r; p[1] = g; p[2] = b;
            if (tex->enableAlpha) p[3] = a;
        }
    return res;
}

/* cpp:978-988 */
i64 GetTextureWidth(Texture *t) { return t->width; }
i64 GetTextureHeight(Texture *t) { return t->height; }
bool GetTextureEnableAlpha(Texture *t) { return t->enableAlpha; }

/* ---- texture preparation: the procedural hit-effect shader, cpp:1318-1440 ----
 * ShaderUtils in f64, left to right, no FMA.  `abs(atan2(...))` (cpp:1388) is
 * the double overload in the reference build: its header includes FFmpeg's,
 * libavutil/common.h includes <math.h>, and libstdc++'s <math.h> brings
 * std::abs(double) into the global namespace (so fabs here). */
static f64 sh_fract(f64 x) { return x - floor(x); }                                    /* cpp:1333-1335 */
static f64 sh_rand(f64 nx, f64 ny) { return sh_fract(sin(nx * 12.9898 + ny * 78.233) * 43758.5453); } /* :1341 */
static f64 sh_mix(f64 a, f64 b, f64 t) { return a + (b - a) * t; }                    /* cpp:1357-1359 */
static f64 sh_noise(f64 px, f64 py) {                                                   /* cpp:1370-1381 */
    f64 ipx = floor(px), ipy = floor(py);
    f64 ux = sh_fract(px), uy = sh_fract(py);
    f64 a = sh_rand(ipx, ipy);
    f64 b = sh_rand(ipx + 1.0, ipy + 0.0);
    f64 c = sh_rand(ipx + 0.0, ipy + 1.0);
    f64 d = sh_rand(ipx + 1.0, ipy + 1.0);
    f64 sx = ux * ux * (3.0 - 2.0 * ux), sy = uy * uy * (3.0 - 2.0 * uy);
    return sh_mix(sh_mix(a, b, sx), sh_mix(c, d, sx), sy);
}
static f64 sh_circular_noise(f64 uvx, f64 uvy, f64 density, f64 seed) {                /* cpp:1384-1401 */
    f64 cx = uvx - 0.5, cy = uvy - 0.5;
    f64 radius = sqrt(cx * cx + cy * cy) * density;
    f64 angle = fabs(atan2(cy, cx));
    if (uvy > 0.5) angle += sin(angle) * 2.0;
    f64 px = radius + seed * 100.0, py = angle + seed * 100.0;
    f64 n = 0.0;
    n += sh_noise(px, py) * 0.7;
    n += sh_noise(px * 2.0, py * 2.0) * 0.3;
    n += sh_noise(px * 4.0, py * 4.0) * 0.1;
    return n;
}

/* cpp:1405-1410 (inline in the reference) */
void GetMilthmHitEffectPixel(f64 seed, f64 t, f64 x, f64 y, f64 *a) {
    f64 n = sh_circular_noise(x, y, 50.0, seed);
    *a = (n < t) ? 0.0 : 1.0;
}

/* cpp:1416-1438: texel (i, j) at (i * h + j) * 4, the mask read at the same
 * index (GetPixelChannel, cpp:1412-1414) — column-major; NULL without alpha */
Texture *CreateMilthmHitEffectTexture(Texture *mask, f64 seed, f64 t, f64 r, f64 g, f64 b) {
    if (!mask->enableAlpha) return NULL;
    Texture *tex = (Texture *)calloc(1, sizeof(Texture));
    tex->width = mask->width; tex->height = mask->height; tex->enableAlpha = true;
    tex->buffer = (f64 *)malloc((size_t)(mask->width * mask->height * 4 > 0 ? mask->width * mask->height * 4 : 1)
                                * sizeof(f64));
    for (i64 i = 0; i < mask->width; ++i)
        for (i64 j = 0; j < mask->height; ++j) {
            f64 a;
            GetMilthmHitEffectPixel(seed, t, (f64)i / mask->width, (f64)j / mask->height, &a);
            f64 mask_a = mask->buffer[i * mask->height * 4 + j * 4 + 3];
            f64 *o = tex->buffer + i * mask->height * 4 + j * 4;
            o[0] = r; o[1] = g; o[2] = b; o[3] = a * mask_a;
        }
    return tex;
}

/* Oracle-only: a texture's texels (tests compare them with the GPU's). */
void OracleGetTextureBuffer(Texture *t, f64 *out) {
    memcpy(out, t->buffer, (size_t)(t->width * t->height * (t->enableAlpha ? 4 : 3)) * sizeof(f64));
}

/* h:9 / cpp GetVersion */
i64 GetVersion(void) { return 1; }

/* cpp:1285-1316 — linear interpolation along the quad's local y */
void DrawVerticalGrd(RenderContext *ctx, f64 x, f64 y, f64 width, f64 height,
                     f64 tr, f64 tg, f64 tb, f64 ta, f64 br, f64 bg, f64 bb, f64 ba) {
    if (width <= 0 || height <= 0) return;
    f64 inv[6];
    inverse_of(ctx->m, inv);
    i64 left, right, top, bottom;
    GetBoarder(ctx->m, x, y, width, height, &left, &right, &top, &bottom,
               (f64)ctx->width, (f64)ctx->height);
    for (i64 i = left; i < right; ++i)
        for (i64 j = top; j < bottom; ++j) {
            f64 ix, iy;
            xform(inv, (f64)i, (f64)j, &ix, &iy);
            if (ix < x) continue;
            if (ix > x + width) continue;
            if (iy < y) continue;
            if (iy > y + height) continue;
            f64 p = (iy - y) / height;
            f64 r = tr + (br - tr) * p;
            f64 g = tg + (bg - tg) * p;
            f64 b = tb + (bb - tb) * p;
            f64 a = ta + (ba - ta) * p;
            ApplyPixel(ctx, i, j, r, g, b, a);
        }
}

/* ------------------------------------------------------------------------
 * New entry points: triangles, depth, Gouraud.  No reference counterpart;
 * semantics defined in the reference idiom:
 *  - vertices go through the context transform (TransformPointFromMatrix,
 *    cpp:446-453) into screen space;
 *  - coverage = pointInPolygon(i, j, tri, 3) (cpp:822-845) at integer pixel
 *    coordinates; triangles with a non-finite vertex or zero signed area
 *    are skipped;
 *  - attributes: w1, w2 barycentric in f64, attr = a0 + (a1-a0)*w1 +
 *    (a2-a0)*w2 (the `top + (bottom-top)*p` form of cpp:1309), no FMA;
 *  - depth: u32, zq = z<=0 ? 0 : z>=1 ? 0xFFFFFFFF : (u32)(z*4294967295.0),
 *    test LESS against the buffer, write only when test+write are enabled;
 *  - blend: ApplyPixel (cpp:515-549) in submission order.
 * ------------------------------------------------------------------------ */

void SetDepthState(RenderContext *ctx, bool test, bool write) {
    ctx->depthTest = test; ctx->depthWrite = write;
}

void ClearDepth(RenderContext *ctx, uint32_t value) {
    i64 n = ctx->width * ctx->height;
    for (i64 i = 0; i < n; ++i) ctx->depth[i] = value;
}

void GetDepthBuffer(RenderContext *ctx, uint32_t *out) {
    memcpy(out, ctx->depth, (size_t)(ctx->width * ctx->height) * sizeof(uint32_t));
}

static inline uint32_t quantize_depth(f64 z) {
    if (!(z > 0.0)) return 0u;
    if (z >= 1.0) return 0xFFFFFFFFu;
    return (uint32_t)(z * 4294967295.0);
}

void DrawTriangles(RenderContext *ctx, const f64 *xy, const f64 *z, const f64 *rgba,
                   i64 n, bool gouraud) {
    i64 W = ctx->width, H = ctx->height;
    i64 frags = 0;
    for (i64 t = 0; t < n; ++t) {
        f64 pts[3][2];
        bool finite = true, huge = false;
        for (int v = 0; v < 3; ++v) {
            xform(ctx->m, xy[t * 6 + 2 * v], xy[t * 6 + 2 * v + 1], &pts[v][0], &pts[v][1]);
            if (!isfinite(pts[v][0]) || !isfinite(pts[v][1])) finite = false;
            if (fabs(pts[v][0]) > 1e7 || fabs(pts[v][1]) > 1e7) huge = true;
        }
        if (!finite) continue;
        f64 e1x = pts[1][0] - pts[0][0], e1y = pts[1][1] - pts[0][1];
        f64 e2x = pts[2][0] - pts[0][0], e2y = pts[2][1] - pts[0][1];
        f64 den = e1x * e2y - e2x * e1y;
        if (den == 0) continue;
        f64 inv = 1.0 / den;
        i64 i0 = 0, i1 = W, j0 = 0, j1 = H;
        if (!huge) {
            f64 xmn = dmin(dmin(pts[0][0], pts[1][0]), pts[2][0]);
            f64 xmx = dmax(dmax(pts[0][0], pts[1][0]), pts[2][0]);
            f64 ymn = dmin(dmin(pts[0][1], pts[1][1]), pts[2][1]);
            f64 ymx = dmax(dmax(pts[0][1], pts[1][1]), pts[2][1]);
            i0 = lmax(0, (i64)floor(xmn) - 2); i1 = lmin(W, (i64)ceil(xmx) + 3);
            j0 = lmax(0, (i64)floor(ymn) - 2); j1 = lmin(H, (i64)ceil(ymx) + 3);
        }
        f64 z0 = 0, z1 = 0, z2 = 0;
        if (z) { z0 = z[t * 3 + 0]; z1 = z[t * 3 + 1]; z2 = z[t * 3 + 2]; }
        const f64 *c = gouraud ? rgba + t * 12 : rgba + t * 4;
        for (i64 j = j0; j < j1; ++j)
            for (i64 i = i0; i < i1; ++i) {
                if (!pointInPolygon((f64)i, (f64)j, pts, 3)) continue;
                ++frags;
                f64 dx = (f64)i - pts[0][0], dy = (f64)j - pts[0][1];
                f64 w1 = (dx * e2y - e2x * dy) * inv;
                f64 w2 = (e1x * dy - dx * e1y) * inv;
                uint32_t zq = 0;
                i64 p = j * W + i;
                if (ctx->depthTest) {
                    f64 zz = z0 + (z1 - z0) * w1 + (z2 - z0) * w2;
                    zq = quantize_depth(zz);
                    if (!(zq < ctx->depth[p])) continue;
                }
                f64 r, g, b, a;
                if (gouraud) {
                    r = c[0] + (c[4] - c[0]) * w1 + (c[8] - c[0]) * w2;
                    g = c[1] + (c[5] - c[1]) * w1 + (c[9] - c[1]) * w2;
                    b = c[2] + (c[6] - c[2]) * w1 + (c[10] - c[2]) * w2;
                    a = c[3] + (c[7] - c[3]) * w1 + (c[11] - c[3]) * w2;
                } else {
                    r = c[0]; g = c[1]; b = c[2]; a = c[3];
                }
                ApplyPixel(ctx, i, j, r, g, b, a);
                if (ctx->depthTest && ctx->depthWrite) ctx->depth[p] = zq;
            }
    }
    g_last_fragments = frags;
}

/* Oracle-only: covered on-screen pixel x triangle pairs of the last
 * DrawTriangles call (the "shaded+Z-tested fragments" work count, §8d). */
i64 OracleLastFragmentCount(void) { return g_last_fragments; }

/* ------------------------------------------------------------------------
 * Audio clips, cpp:990-1283, restated loop for loop.  Where the
 * reference reads or writes outside a buffer (undefined behaviour) the result
 * is defined here exactly as libnativecpurenderer_amd/csrc/nr_audio.hip
 * defines it: overlay frames before the target are skipped; resample reads of
 * a negative index give 0.0; cut frames outside the source are 0.0 and a
 * negative length / negative resampled length gives an empty clip.  Parity
 * unpinned by the reference (no reference test, fixture or decodable audio
 * input exists here; the .ogg inputs in test_files need FFmpeg/pydub, absent).
 * ------------------------------------------------------------------------ */
typedef struct AudioClip { i64 sampleRate, channels, numFrames; f64 *buffer; } AudioClip;  /* h:70-75 */
typedef struct WapperedBytes { iu8 *data; i64 size; } WapperedBytes;                       /* h:77-80 */

static AudioClip *new_clip(i64 rate, i64 ch, i64 frames) {
    AudioClip *a = (AudioClip *)malloc(sizeof(AudioClip));
    i64 n = frames * ch;
    a->sampleRate = rate; a->channels = ch; a->numFrames = frames;
    a->buffer = (f64 *)calloc((size_t)(n > 0 ? n : 1), sizeof(f64));
    return a;
}

i64 GetAudioClipBufferSizeFromData(i64 numFrames, i64 channels) { return numFrames * channels; }   /* cpp:990 */
i64 GetAudioClipBufferSize(AudioClip *clip) { return clip->numFrames * clip->channels; }             /* cpp:994 */

AudioClip *CreateAudioClipFromBuffer(i64 sampleRate, i64 channels, i64 numFrames, f64 *buffer) {  /* cpp:998-1014 */
    AudioClip *a = new_clip(sampleRate, channels, numFrames);
    for (i64 i = 0; i < numFrames * channels; ++i) a->buffer[i] = buffer[i];
    return a;
}

AudioClip *CreateAudioClipFromInt16Buffer(i64 sampleRate, i64 channels, i64 numFrames, int16_t *buffer) { /* cpp:1016-1034 */
    AudioClip *a = new_clip(sampleRate, channels, numFrames);
    for (i64 i = 0; i < numFrames; ++i)
        for (i64 j = 0; j < channels; ++j) a->buffer[i * channels + j] = (f64)buffer[i * channels + j] / 32768.0;
    return a;
}

AudioClip *CreateSilentAudioClip(i64 sampleRate, i64 channels, i64 numFrames) {  /* cpp:1036-1046 */
    return new_clip(sampleRate, channels, numFrames);
}

void DestroyAudioClip(AudioClip *clip) {   /* cpp:1048-1052 is a no-op; freed here */
    if (!clip) return;
    free(clip->buffer);
    free(clip);
}

AudioClip *CloneAudioClip(AudioClip *clip) {   /* cpp:1054-1061 */
    return CreateAudioClipFromBuffer(clip->sampleRate, clip->channels, clip->numFrames, clip->buffer);
}

f64 GetAudioClipDuration(AudioClip *clip) { return (f64)clip->numFrames / (f64)clip->sampleRate; }  /* cpp:1242 */

static inline f64 clip_sample(const AudioClip *c, i64 idx) { return idx >= 0 ? c->buffer[idx] : 0.0; }

void ApplyResampleAudioClip(AudioClip *clip, i64 sampleRate, i64 channels) {   /* cpp:1063-1120 */
    if (clip->sampleRate == sampleRate && clip->channels == channels) return;
    f64 dur = GetAudioClipDuration(clip);
    i64 newNum = f2i64(dur * sampleRate);
    if (newNum < 0) newNum = 0;
    i64 newSize = newNum * channels;
    f64 *nb = (f64 *)calloc((size_t)(newSize > 0 ? newSize : 1), sizeof(f64));
    for (i64 i = 0; i < newNum; ++i) {
        f64 secT = (f64)i / sampleRate;
        f64 old = secT * clip->sampleRate;
        i64 fl = (i64)floor(old);
        i64 ce = (i64)ceil(old);
        if (fl < 0) fl = 0;
        if (fl >= clip->numFrames - clip->channels) fl = clip->numFrames - clip->channels - 1;
        if (ce < 0) ce = 0;
        if (ce >= clip->numFrames - clip->channels) ce = clip->numFrames - clip->channels - 1;
        f64 frac = old - fl;
        if (clip->channels == channels) {
            for (i64 c = 0; c < channels; ++c) {
                f64 vf = clip_sample(clip, fl * clip->channels + c);
                f64 vc = clip_sample(clip, ce * clip->channels + c);
                nb[i * channels + c] = vf + (vc - vf) * frac;
            }
        } else {
            f64 sf = 0, sc = 0;
            for (i64 c = 0; c < clip->channels; ++c) {
                sf += clip_sample(clip, fl * clip->channels + c);
                sc += clip_sample(clip, ce * clip->channels + c);
            }
            for (i64 c = 0; c < channels; ++c)
                nb[i * channels + c] = sf / clip->channels + (sc / clip->channels - sf / clip->channels) * frac;
        }
    }
    free(clip->buffer);
    clip->buffer = nb;
    clip->sampleRate = sampleRate;
    clip->channels = channels;
    clip->numFrames = newNum;
}

void ResampleAudioClipLike(AudioClip *clip, AudioClip *like) {   /* cpp:1122-1127 */
    ApplyResampleAudioClip(clip, like->sampleRate, like->channels);
}

i64 OverlayAudioClip(AudioClip *target, AudioClip *source, i64 startFrame, bool autoResample) {   /* cpp:1129-1154 */
    AudioClip *tmp = NULL;
    if (autoResample && (target->sampleRate != source->sampleRate || target->channels != source->channels)) {
        tmp = source = CloneAudioClip(source);
        ResampleAudioClipLike(source, target);
    }
    i64 rc = 0;
    if (target->sampleRate != source->sampleRate) rc = -1;
    else if (target->channels != source->channels) rc = -2;
    else
        for (i64 i = 0; i < source->numFrames; ++i) {
            if (startFrame + i >= target->numFrames) break;
            i64 ti = startFrame + i;
            if (ti < 0) continue;
            for (i64 c = 0; c < source->channels; ++c)
                target->buffer[ti * source->channels + c] += source->buffer[i * source->channels + c];
        }
    DestroyAudioClip(tmp);
    return rc;
}

i64 OverlayAudioClipSecond(AudioClip *target, AudioClip *source, f64 startSecond, bool autoResample) {  /* cpp:1156-1163 */
    return OverlayAudioClip(target, source, f2i64(startSecond * target->sampleRate), autoResample);
}

WapperedBytes *SaveAudioClipAsWav(AudioClip *clip) {   /* cpp:1165-1228 */
    i64 n = GetAudioClipBufferSize(clip);
    i64 size = 44 + n * 2;
    iu8 *d = (iu8 *)malloc((size_t)size);
    int32_t v32; int16_t v16;
    memcpy(d, "RIFF", 4);
    v32 = (int32_t)(size - 8); memcpy(d + 4, &v32, 4);
    memcpy(d + 8, "WAVE", 4);
    memcpy(d + 12, "fmt ", 4);
    v32 = 0x10; memcpy(d + 16, &v32, 4);
    v16 = 1; memcpy(d + 20, &v16, 2);
    v16 = (int16_t)clip->channels; memcpy(d + 22, &v16, 2);
    v32 = (int32_t)clip->sampleRate; memcpy(d + 24, &v32, 4);
    v32 = (int32_t)(clip->sampleRate * clip->channels * 2); memcpy(d + 28, &v32, 4);
    v16 = (int16_t)(clip->channels * 2); memcpy(d + 32, &v16, 2);
    v16 = 16; memcpy(d + 34, &v16, 2);
    memcpy(d + 36, "data", 4);
    v32 = (int32_t)(n * 2); memcpy(d + 40, &v32, 4);
    for (i64 i = 0; i < n; ++i) {
        f64 v = clip->buffer[i];
        f64 x = (v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v)) * 32767.0;
        /* x86 cvttsd2si to int32, low 16 bits: NaN -> 0x80000000 -> 0 */
        int16_t s = (x != x) ? 0 : (int16_t)(int32_t)x;
        memcpy(d + 44 + 2 * i, &s, 2);
    }
    WapperedBytes *w = (WapperedBytes *)malloc(sizeof(WapperedBytes));
    w->data = d;
    w->size = size;
    return w;
}

i64 GetAudioClipSampleRate(AudioClip *clip) { return clip->sampleRate; }    /* cpp:1230 */
i64 GetAudioClipChannels(AudioClip *clip) { return clip->channels; }        /* cpp:1234 */
i64 GetAudioClipNumFrames(AudioClip *clip) { return clip->numFrames; }      /* cpp:1238 */
iu8 *GetWapperedBytesDataPtr(WapperedBytes *b) { return b->data; }          /* cpp:1246 */
i64 GetWapperedBytesDataSize(WapperedBytes *b) { return b->size; }          /* cpp:1250 */
void DestroyWapperedBytes(WapperedBytes *b) { if (b) { free(b->data); free(b); } }

void ApplyVolumeGain(AudioClip *clip, f64 gain) {   /* cpp:1254-1259 */
    for (i64 i = 0; i < GetAudioClipBufferSize(clip); ++i) clip->buffer[i] *= gain;
}

void ApplyCutAudioClip(AudioClip *clip, i64 startFrame, i64 endFrame) {   /* cpp:1265-1279 */
    i64 frames = endFrame - startFrame;
    if (frames < 0) frames = 0;
    f64 *nb = (f64 *)calloc((size_t)(frames * clip->channels > 0 ? frames * clip->channels : 1), sizeof(f64));
    for (i64 i = 0; i < frames; ++i) {
        if (startFrame + i >= clip->numFrames) break;
        if (startFrame + i < 0) continue;
        for (i64 c = 0; c < clip->channels; ++c)
            nb[i * clip->channels + c] = clip->buffer[(startFrame + i) * clip->channels + c];
    }
    free(clip->buffer);
    clip->buffer = nb;
    clip->numFrames = frames;
}

void ApplySpeedAudioClip(AudioClip *clip, f64 speed) {   /* cpp:1281-1283: i64 *= f64 */
    clip->sampleRate = f2i64(clip->sampleRate * speed);
}

void GetAudioClipBuffer(AudioClip *clip, f64 *out) {
    memcpy(out, clip->buffer, (size_t)GetAudioClipBufferSize(clip) * sizeof(f64));
}
