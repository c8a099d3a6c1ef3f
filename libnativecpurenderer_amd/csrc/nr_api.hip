// nr_api.hip — render context, state stack, textures and readback of the
// MI355X raster library: the extern "C" surface of
// /root/reference/src/libNativeCPURenderer.h:83-152 (render part), plus the
// error/timing/device entry points declared in include/libNativeCPURenderer.h.
//
// Host-side state (transform, colour transform, save/restore stack) stays on
// the host exactly as in the reference (cpp:277-309, 386-492, 623-641): the
// caller reads it back synchronously (milrenderer.py:983), so it is never
// moved to the device.  Pixel data lives in HBM; every draw is an async
// kernel launch on the device's stream, readback is the only sync point.
#include "nr_common.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static std::mutex g_err_mu;
static std::string g_err;
static long g_err_count = 0;

void nr_set_error(const char* where, hipError_t e) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    if (g_err_count++ < 8) fprintf(stderr, "[libNativeCPURenderer-amd] HIP error in %s\n", g_err.c_str());
}
void nr_set_error_msg(const char* msg) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = msg;
    if (g_err_count++ < 8) fprintf(stderr, "[libNativeCPURenderer-amd] %s\n", msg);
}

extern "C" {
// Non-empty string when a HIP call failed since the last ClearLastError().
const char* GetLastErrorString() {
    std::lock_guard<std::mutex> lk(g_err_mu);
    return g_err.c_str();
}
void ClearLastError() {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err.clear();
}
}

// ---------------------------------------------------------------------------
// device / stream registry: one non-blocking stream per device shared by all
// contexts and textures of that device, so cross-object ordering (texture
// uploads, render-to-texture) is the reference's single-threaded order.
// ---------------------------------------------------------------------------
// Stream priorities: the main stream at the greatest, the binning stream at
// the least (the next batch's binning fills the gaps the current raster
// leaves instead of competing with it).
static std::mutex g_dev_mu;
static std::vector<hipStream_t> g_streams;

hipStream_t nr_stream_for(int device) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if ((int)g_streams.size() <= device) g_streams.resize(device + 1, nullptr);
    if (!g_streams[device]) {
        NR_CHECK(hipSetDevice(device));
        int least = 0, greatest = 0;
        NR_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        NR_CHECK(hipStreamCreateWithPriority(&g_streams[device], hipStreamNonBlocking,
                                             greatest));
    }
    return g_streams[device];
}

static std::vector<hipStream_t> g_bin_streams;
hipStream_t nr_bin_stream_for(int device) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if ((int)g_bin_streams.size() <= device) g_bin_streams.resize(device + 1, nullptr);
    if (!g_bin_streams[device]) {
        NR_CHECK(hipSetDevice(device));
        int least = 0, greatest = 0;
        NR_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        NR_CHECK(hipStreamCreateWithPriority(&g_bin_streams[device], hipStreamNonBlocking,
                                             least));
    }
    return g_bin_streams[device];
}

// live contexts (nr_settle_all validates every pending batch)
static std::mutex g_ctx_mu;
static std::vector<RenderContext*> g_ctxs;

void nr_settle_all() {
    std::vector<RenderContext*> v;
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        v = g_ctxs;
    }
    int prev = 0;
    NR_CHECK(hipGetDevice(&prev));
    for (RenderContext* c : v)
        if (c->pendingBatch || c->cmdList) {
            NR_CHECK(hipSetDevice(c->device));
            nr_settle(c);
        }
    NR_CHECK(hipSetDevice(prev));
}

static int current_device() {
    int d = 0;
    NR_CHECK(hipGetDevice(&d));
    return d;
}

// ---------------------------------------------------------------------------
// small kernels
// ---------------------------------------------------------------------------
__global__ void k_fill_f64(f64* __restrict__ p, i64 n, f64 v) {
    i64 i = ((i64)blockIdx.x * blockDim.x + threadIdx.x) * 2;
    i64 stride = (i64)gridDim.x * blockDim.x * 2;
    for (; i + 1 < n; i += stride) {
        double2 w; w.x = v; w.y = v;
        *reinterpret_cast<double2*>(p + i) = w;   // 16-B stores
    }
    if (i < n) p[i] = v;
}

__global__ void k_fill_u32(u32* __restrict__ p, i64 n, u32 v) {
    i64 i = ((i64)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    i64 stride = (i64)gridDim.x * blockDim.x * 4;
    for (; i + 3 < n; i += stride) {
        uint4 w; w.x = v; w.y = v; w.z = v; w.w = v;
        *reinterpret_cast<uint4*>(p + i) = w;
    }
    for (; i < n; ++i) p[i] = v;
}

static int fill_grid(i64 n, int per_thread) {
    i64 g = (n / per_thread + 255) / 256;
    if (g < 1) g = 1;
    if (g > 8192) g = 8192;
    return (int)g;
}

void nr_fill_f64(hipStream_t s, f64* p, i64 n, f64 v) {
    if (n <= 0) return;
    // buffers come from hipMalloc (256-B aligned): the double2 path is aligned
    hipLaunchKernelGGL(k_fill_f64, dim3(fill_grid(n, 2)), dim3(256), 0, s, p, n, v);
    NR_CHECK(hipGetLastError());
}
void nr_fill_u32(hipStream_t s, u32* p, i64 n, u32 v) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill_u32, dim3(fill_grid(n, 4)), dim3(256), 0, s, p, n, v);
    NR_CHECK(hipGetLastError());
}

// cpp:52-57 f64 -> u8 readback conversion
__global__ void k_to_u8(const f64* __restrict__ src, iu8* __restrict__ dst, i64 n) {
    i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    i64 stride = (i64)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = nr_to_u8(src[i]);
}

// cpp:337-354: tex[i] = u8/255.0
__global__ void k_u8_to_f64(const iu8* __restrict__ src, f64* __restrict__ dst, i64 n) {
    i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    i64 stride = (i64)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = src[i] / 255.0;
}

// cpp:643-657 non-uniform clear through SetPixel (cpp:494-513).  On an RGB
// context SetPixel also stores `a` into index+3 = the next pixel's R; with
// the reference's x-outer loop the only surviving overrun is column 0 of rows
// >= 1 (R = a) when W >= 2 (Appendix A.6).
__global__ void k_set_color(f64* __restrict__ buf, i64 W, i64 H, int ipp, f64 r, f64 g, f64 b, f64 a) {
    i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    i64 n = W * H;
    i64 stride = (i64)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        i64 x = i % W, y = i / W;
        f64* p = buf + i * ipp;
        p[0] = (ipp == 3 && x == 0 && y >= 1 && W >= 2) ? a : r;
        p[1] = g;
        p[2] = b;
        if (ipp == 4) p[3] = a;
    }
}

// cpp:682-691 FillColor = ApplyPixel on every pixel
__global__ void k_fill_color(f64* __restrict__ buf, i64 npix, int ipp, f64 r, f64 g, f64 b, f64 a,
                             f64 ct0, f64 ct1, f64 ct2, f64 ct3) {
    i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    i64 stride = (i64)gridDim.x * blockDim.x;
    for (; i < npix; i += stride) nr_apply_pixel(buf + i * ipp, ipp, r, g, b, a, ct0, ct1, ct2, ct3);
}

// cpp:950-976 ResampleTexture
__global__ void k_resample(const f64* __restrict__ src, i64 tw, i64 th, bool talpha,
                           f64* __restrict__ dst, i64 W, i64 H) {
    i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    i64 n = W * H;
    i64 stride = (i64)gridDim.x * blockDim.x;
    int ipp = talpha ? 4 : 3;
    for (; i < n; i += stride) {
        i64 x = i % W, y = i / W;
        f64 r, g, b, a;
        nr_sample(src, tw, th, talpha, (f64)x / W * tw, (f64)y / H * th, r, g, b, a);
        f64* p = dst + i * ipp;
        p[0] = r; p[1] = g; p[2] = b;
        if (talpha) p[3] = a;
    }
}

static int grid_for(i64 n) { return fill_grid(n, 1); }

// ---------------------------------------------------------------------------
// pending clears
// ---------------------------------------------------------------------------
void nr_ensure_depth(RenderContext* ctx) {
    if (ctx->depth) return;
    i64 n = ctx->width * ctx->height;
    NR_CHECK(hipMalloc(&ctx->depth, (size_t)(n > 0 ? n : 1) * sizeof(u32)));
    nr_fill_u32(ctx->stream, ctx->depth, n, 0xFFFFFFFFu);
}

void nr_materialize_color(RenderContext* ctx) {
    nr_settle(ctx);
    nr_materialize_tiles(ctx, true, false);
    if (!ctx->pendColor) return;
    ctx->pendColor = false;
    ctx->frameU8Valid = false;
    hipEvent_t a, b;
    nr_timing_begin(ctx, NRK_FILL, &a, &b);
    nr_fill_f64(ctx->stream, ctx->buffer, ctx->width * ctx->height * (ctx->enableAlpha ? 4 : 3),
                ctx->pendColorValue);
    nr_timing_end(ctx, NRK_FILL, a, b);
}

void nr_materialize_depth(RenderContext* ctx) {
    nr_settle(ctx);
    nr_materialize_tiles(ctx, false, true);
    if (!ctx->pendDepth) return;
    ctx->pendDepth = false;
    nr_ensure_depth(ctx);
    nr_fill_u32(ctx->stream, ctx->depth, ctx->width * ctx->height, ctx->pendDepthValue);
}

void nr_materialize(RenderContext* ctx) {
    nr_materialize_color(ctx);
    nr_materialize_depth(ctx);
}

// ---------------------------------------------------------------------------
// per-kernel timing (HIP events on the launch stream)
// ---------------------------------------------------------------------------
static hipEvent_t ev_get(RenderContext* ctx) {
    if (!ctx->evPool.empty()) {
        hipEvent_t e = ctx->evPool.back();
        ctx->evPool.pop_back();
        return e;
    }
    // timing only: no system-scope fence at record (a fenced record leaves a
    // multi-microsecond bubble between the kernels it separates)
    hipEvent_t e;
    NR_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    return e;
}

void nr_timing_begin_on(RenderContext* ctx, int kid, hipEvent_t* a, hipEvent_t* b, hipStream_t s) {
    *a = *b = nullptr;
    if (!ctx->timing || !((ctx->timingMask >> kid) & 1ull)) return;
    *a = ev_get(ctx);
    *b = ev_get(ctx);
    NR_CHECK(hipEventRecord(*a, s));
}
void nr_timing_end_on(RenderContext* ctx, int kid, hipEvent_t a, hipEvent_t b, hipStream_t s) {
    if (!ctx->timing || !a) return;
    NR_CHECK(hipEventRecord(b, s));
    ctx->evPending.push_back({kid, {a, b}});
}
void nr_timing_begin(RenderContext* ctx, int kid, hipEvent_t* a, hipEvent_t* b) {
    nr_timing_begin_on(ctx, kid, a, b, ctx->stream);
}
void nr_timing_end(RenderContext* ctx, int kid, hipEvent_t a, hipEvent_t b) {
    nr_timing_end_on(ctx, kid, a, b, ctx->stream);
}


constexpr int TS_PAIRS = 4096;   // timed raster launches between two collections
static void timing_collect(RenderContext* ctx) {
    if (ctx->evPending.empty() && ctx->tsPending.empty()) return;
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    if (!ctx->tsPending.empty()) {   // device-clock pairs: ~start (max of inverted), end; 100 MHz
        std::vector<u64> h(ctx->tsPending.size() * 2);
        NR_CHECK(hipMemcpy(h.data(), ctx->tsDev, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
        for (auto& p : ctx->tsPending) {
            const u64 s = ~h[2 * p.second], e = h[2 * p.second + 1];
            if (!h[2 * p.second] || e < s) continue;   // (a launch that did no work)
            ctx->kTimeMs[p.first] += (f64)(e - s) * 1e-5;
            ctx->kCount[p.first] += 1;
        }
        NR_CHECK(hipMemsetAsync(ctx->tsDev, 0, h.size() * sizeof(u64), ctx->stream));
        NR_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->tsPending.clear();
    }
    for (auto& p : ctx->evPending) {
        float ms = 0;
        NR_CHECK(hipEventElapsedTime(&ms, p.second.first, p.second.second));
        ctx->kTimeMs[p.first] += ms;
        ctx->kCount[p.first] += 1;
        ctx->evPool.push_back(p.second.first);
        ctx->evPool.push_back(p.second.second);
    }
    ctx->evPending.clear();
}

u64* nr_timing_stamp(RenderContext* ctx, int kid) {
    if (!ctx->timing || !((ctx->timingMask >> kid) & 1ull)) return nullptr;
    if ((int)ctx->tsPending.size() >= TS_PAIRS) timing_collect(ctx);
    if (!ctx->tsDev) {
        NR_CHECK(hipMalloc(&ctx->tsDev, (size_t)TS_PAIRS * 2 * sizeof(u64)));
        NR_CHECK(hipMemsetAsync(ctx->tsDev, 0, (size_t)TS_PAIRS * 2 * sizeof(u64), ctx->stream));
    }
    const int i = (int)ctx->tsPending.size();
    ctx->tsPending.push_back({kid, i});
    return ctx->tsDev + 2 * i;
}


static const char* kKernelNames[NRK_COUNT_] = {"tri_count", "tri_scan",    "tri_emit", "tri_sort",
                                               "tile_ranges", "tile_raster", "prim",     "fill",
                                               "resolve",   "vis_init",    "output",   "gather"};

extern "C" {

// ---------------------------------------------------------------------------
// context (cpp:3-45)
// ---------------------------------------------------------------------------
i64 GetBufferSize(RenderContext* ctx) {
    return ctx->width * ctx->height * (ctx->enableAlpha ? 4 : 3);
}

// cpp:7-31 on the calling thread's current HIP device.  Returns NULL (and
// latches an error) when no GPU is usable: there is no CPU fallback.
RenderContext* CreateRenderContext(i64 width, i64 height, bool enableAlpha) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        nr_set_error_msg("CreateRenderContext: no HIP device available (this library has no CPU path)");
        return nullptr;
    }
    RenderContext* ctx = new RenderContext();
    ctx->width = width;
    ctx->height = height;
    ctx->enableAlpha = enableAlpha;
    ctx->device = current_device();
    ctx->stream = nr_stream_for(ctx->device);
    i64 n = GetBufferSize(ctx);
    if (hipMalloc(&ctx->buffer, (size_t)(n > 0 ? n : 1) * sizeof(f64)) != hipSuccess) {
        nr_set_error_msg("CreateRenderContext: hipMalloc failed");
        delete ctx;
        return nullptr;
    }
    // The reference leaves the buffer uninitialised (A.11); zero it once.
    NR_CHECK(hipMemsetAsync(ctx->buffer, 0, (size_t)(n > 0 ? n : 1) * sizeof(f64), ctx->stream));
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        g_ctxs.push_back(ctx);
    }
    return ctx;
}

// cpp:33-37 is a deliberate leak in the reference; here handles own memory.
void DestroyRenderContext(RenderContext* ctx) {
    if (!ctx) return;
    NR_CHECK(hipSetDevice(ctx->device));
    nr_free_commands(ctx);   // queued draws of a destroyed context are dead
    nr_settle(ctx);
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        for (size_t i = 0; i < g_ctxs.size(); ++i)
            if (g_ctxs[i] == ctx) { g_ctxs.erase(g_ctxs.begin() + i); break; }
    }
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(ctx->device)));
    nr_dist_release(ctx);
    TriScratch& t = ctx->tri;
    void* ptrs[] = {ctx->buffer, ctx->depth, t.cnt,  t.off,        t.keys[0], t.keys[1], t.vals[0],
                    t.vals[1],   t.tile_start, t.tile_end, t.temp, t.stage, t.d_frag, t.d_flag, ctx->u8buf,
                    t.fdone,     t.kslot, t.orec, ctx->tileStamp};
    for (void* p : ptrs)
        if (p) NR_CHECK(hipFree(p));
    for (auto& F : t.fset) {
        void* fp[] = {F.fcnt, F.foff, F.fcur, F.fitems, F.frect, F.frec, F.flist, F.dplan, F.gate, F.gplan};
        for (void* p : fp)
            if (p) NR_CHECK(hipFree(p));
        if (F.h_plan) NR_CHECK(hipHostFree(F.h_plan));
        if (F.evBin) NR_CHECK(hipEventDestroy(F.evBin));
        if (F.evVis) NR_CHECK(hipEventDestroy(F.evVis));
    }
    if (t.h_total) NR_CHECK(hipHostFree(t.h_total));
    if (t.hfail) NR_CHECK(hipHostFree(t.hfail));
    {   // the warm-binning schedule
        auto& S = t.sched;
        void* sp[] = {S.off, S.items, S.dplan, S.blocks, S.off2};
        for (void* p : sp)
            if (p) NR_CHECK(hipFree(p));
        if (S.ready) NR_CHECK(hipEventDestroy(S.ready));
    }
    for (auto& p : ctx->evPending) {
        NR_CHECK(hipEventDestroy(p.second.first));
        NR_CHECK(hipEventDestroy(p.second.second));
    }
    for (auto e : ctx->evPool) NR_CHECK(hipEventDestroy(e));
    if (ctx->tsDev) NR_CHECK(hipFree(ctx->tsDev));
    delete ctx;
}

// cpp:39-45 (new buffer; content unspecified in the reference, zeroed here)
void ResizeRenderContext(RenderContext* ctx, i64 width, i64 height) {
    ctx->frameU8Valid = false;
    NR_CHECK(hipSetDevice(ctx->device));
    nr_settle(ctx);
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    NR_CHECK(hipFree(ctx->buffer));
    if (ctx->depth) NR_CHECK(hipFree(ctx->depth));
    ctx->depth = nullptr;
    // the gathered frame (old size) is dropped: GetFrameU8 fails until the next GatherFrameU8
    nr_dist_sync(ctx);
    ctx->frameLast = -1;
    for (bool& g : ctx->gatherPending) g = false;
    ctx->width = width;
    ctx->height = height;
    if (ctx->frameFormat == 1 && ((width & 1) || (height & 1))) {   // YUV420P needs even sizes (SetFrameFormat)
        ctx->frameFormat = 0;
        nr_set_error_msg("ResizeRenderContext: odd size, frame output format reset from YUV420P to the u8 image");
    }
    ctx->pendColor = ctx->pendDepth = false;
    ctx->tileColor = ctx->tileDepth = false;
    i64 n = GetBufferSize(ctx);
    NR_CHECK(hipMalloc(&ctx->buffer, (size_t)(n > 0 ? n : 1) * sizeof(f64)));
    NR_CHECK(hipMemsetAsync(ctx->buffer, 0, (size_t)(n > 0 ? n : 1) * sizeof(f64), ctx->stream));
}

// cpp:277-289
void SaveContextState(RenderContext* ctx) {
    NRState s;
    memcpy(s.m, ctx->m, sizeof s.m);
    memcpy(s.ct, ctx->ct, sizeof s.ct);
    ctx->stack.push_back(s);
}

// cpp:291-309
bool RestoreContextState(RenderContext* ctx) {
    if (ctx->stack.empty()) return false;
    const NRState& s = ctx->stack.back();
    memcpy(ctx->m, s.m, sizeof s.m);
    memcpy(ctx->ct, s.ct, sizeof s.ct);
    ctx->stack.pop_back();
    return true;
}

// cpp:311-316: D2H copy (the sync point)
void GetBuffer(RenderContext* ctx, f64* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    NR_CHECK(hipMemcpyAsync(out, ctx->buffer, (size_t)GetBufferSize(ctx) * sizeof(f64),
                            hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
}

// cpp:52-57: converted on the GPU, 1/8 of the bytes cross PCIe.  The u8
// staging buffer is owned by the context (no stream-ordered allocator).
void GetBufferAsUInt8(RenderContext* ctx, iu8* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    i64 n = GetBufferSize(ctx);
    if (n <= 0) return;
    if ((size_t)n > ctx->u8cap) {
        if (ctx->u8buf) NR_CHECK(hipFree(ctx->u8buf));
        ctx->u8buf = nullptr;
        if (hipMalloc((void**)&ctx->u8buf, (size_t)n) != hipSuccess) {
            nr_set_error_msg("GetBufferAsUInt8: hipMalloc failed");
            ctx->u8cap = 0;
            return;
        }
        ctx->u8cap = (size_t)n;
    }
    hipLaunchKernelGGL(k_to_u8, dim3(grid_for(n)), dim3(256), 0, ctx->stream, ctx->buffer, ctx->u8buf, n);
    NR_CHECK(hipGetLastError());
    NR_CHECK(hipMemcpyAsync(out, ctx->u8buf, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
}

// New: device-side u8 conversion into a caller-provided device buffer (the
// frame-output step of §8f-2 without the PCIe hop).
void GetBufferAsUInt8Device(RenderContext* ctx, iu8* dev_out) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    i64 n = GetBufferSize(ctx);
    hipLaunchKernelGGL(k_to_u8, dim3(grid_for(n)), dim3(256), 0, ctx->stream, ctx->buffer, dev_out, n);
    NR_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// textures (cpp:318-384, 950-988)
// ---------------------------------------------------------------------------
static Texture* new_texture(i64 w, i64 h, bool alpha) {
    Texture* t = new Texture();
    t->width = w; t->height = h; t->enableAlpha = alpha;
    t->device = current_device();
    i64 size = w * h * (alpha ? 4 : 3);
    NR_CHECK(hipMalloc(&t->buffer, (size_t)(size > 0 ? size : 1) * sizeof(f64)));
    return t;
}

// cpp:318-335
Texture* CreateTexture(i64 width, i64 height, bool enableAlpha, f64* buffer) {
    Texture* t = new_texture(width, height, enableAlpha);
    hipStream_t s = nr_stream_for(t->device);
    i64 size = width * height * (enableAlpha ? 4 : 3);
    if (size > 0) NR_CHECK(hipMemcpyAsync(t->buffer, buffer, (size_t)size * sizeof(f64), hipMemcpyHostToDevice, s));
    NR_CHECK(hipStreamSynchronize(s));   // caller owns `buffer`
    return t;
}

// cpp:337-354 (u8 -> f64 on the GPU: IEEE division, same result as the host)
Texture* CreateTextureUInt8(i64 width, i64 height, bool enableAlpha, iu8* buffer) {
    Texture* t = new_texture(width, height, enableAlpha);
    hipStream_t s = nr_stream_for(t->device);
    i64 size = width * height * (enableAlpha ? 4 : 3);
    if (size > 0) {
        iu8* d = nullptr;
        NR_CHECK(hipMalloc((void**)&d, (size_t)size));
        NR_CHECK(hipMemcpyAsync(d, buffer, (size_t)size, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_u8_to_f64, dim3(grid_for(size)), dim3(256), 0, s, d, t->buffer, size);
        NR_CHECK(hipGetLastError());
        NR_CHECK(hipStreamSynchronize(s));
        NR_CHECK(hipFree(d));
    }
    NR_CHECK(hipStreamSynchronize(s));
    return t;
}

// cpp:356-360 (no-op in the reference); aliases never free the framebuffer
void DestroyTexture(Texture* t) {
    if (!t) return;
    nr_settle_all();   // recorded draws that sample this texture run first
    if (t->owns && t->buffer) {
        NR_CHECK(hipSetDevice(t->device));
        NR_CHECK(hipStreamSynchronize(nr_stream_for(t->device)));
        NR_CHECK(hipFree(t->buffer));
    }
    delete t;
}

// cpp:362-375: device-to-device snapshot of the framebuffer
Texture* CreateTextureFromRenderContext(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    Texture* t = new_texture(ctx->width, ctx->height, ctx->enableAlpha);
    NR_CHECK(hipMemcpyAsync(t->buffer, ctx->buffer, (size_t)GetBufferSize(ctx) * sizeof(f64),
                            hipMemcpyDeviceToDevice, ctx->stream));
    return t;
}

// cpp:377-384: non-owning alias of the framebuffer (dangles after a resize,
// as in the reference)
Texture* CreateTextureFromRenderContextShared(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    Texture* t = new Texture();
    t->width = ctx->width; t->height = ctx->height; t->enableAlpha = ctx->enableAlpha;
    t->buffer = ctx->buffer; t->owns = false; t->aliasOf = ctx; t->device = ctx->device;
    return t;
}

// cpp:950-976
Texture* ResampleTexture(Texture* tex, i64 width, i64 height) {
    NR_CHECK(hipSetDevice(tex->device));
    if (tex->aliasOf) nr_materialize_color(tex->aliasOf);
    Texture* t = new_texture(width, height, tex->enableAlpha);
    hipStream_t s = nr_stream_for(t->device);
    i64 n = width * height;
    if (n > 0) {
        hipLaunchKernelGGL(k_resample, dim3(grid_for(n)), dim3(256), 0, s, tex->buffer, tex->width,
                           tex->height, tex->enableAlpha, t->buffer, width, height);
        NR_CHECK(hipGetLastError());
    }
    return t;
}

i64 GetTextureWidth(Texture* t) { return t->width; }
i64 GetTextureHeight(Texture* t) { return t->height; }
bool GetTextureEnableAlpha(Texture* t) { return t->enableAlpha; }

// New: copy a texture's f64 texels to the host (tests / debugging).
void GetTextureBuffer(Texture* t, f64* out) {
    NR_CHECK(hipSetDevice(t->device));
    hipStream_t s = nr_stream_for(t->device);
    if (t->aliasOf) nr_materialize_color(t->aliasOf);
    NR_CHECK(hipMemcpyAsync(out, t->buffer, (size_t)(t->width * t->height * (t->enableAlpha ? 4 : 3)) * sizeof(f64),
                            hipMemcpyDeviceToHost, s));
    NR_CHECK(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------------------
// transform & colour-transform state (host only; cpp:386-492, 623-641)
// ---------------------------------------------------------------------------
void SetTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f) {
    ctx->m[0] = a; ctx->m[1] = b; ctx->m[2] = c; ctx->m[3] = d; ctx->m[4] = e; ctx->m[5] = f;
}

// cpp:398-411 (post-multiply)
void ApplyTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f) {
    f64 o[6];
    for (int i = 0; i < 6; ++i) o[i] = ctx->m[i];
    ctx->m[0] = o[0] * a + o[2] * b;
    ctx->m[1] = o[1] * a + o[3] * b;
    ctx->m[2] = o[0] * c + o[2] * d;
    ctx->m[3] = o[1] * c + o[3] * d;
    ctx->m[4] = o[0] * e + o[2] * f + o[4];
    ctx->m[5] = o[1] * e + o[3] * f + o[5];
}

void Scale(RenderContext* ctx, f64 sx, f64 sy) { ApplyTransform(ctx, sx, 0, 0, sy, 0, 0); }    // cpp:420-426
void Translate(RenderContext* ctx, f64 tx, f64 ty) { ApplyTransform(ctx, 1, 0, 0, 1, tx, ty); } // cpp:428-434
void Rotate(RenderContext* ctx, f64 angle) {                                                   // cpp:436-444
    // The reference is built with g++ -O3 (src/compile.sh), which merges the
    // sin/cos pair of cpp:440-441 into one glibc sincos() call; sincos differs
    // from separate sin and cos in the last bit for some angles (found by
    // tests/test_command_list.py's random mixes), so call it explicitly.
    f64 s, c;
    sincos(angle, &s, &c);
    ApplyTransform(ctx, c, s, -s, c, 0, 0);
}

// cpp:455-461 (inline in the reference; exported here)
void TransformPoint(RenderContext* ctx, f64 x, f64 y, f64* ox, f64* oy) { nr_xform(ctx->m, x, y, *ox, *oy); }

void GetTransform(RenderContext* ctx, f64 out[6]) {
    for (int i = 0; i < 6; ++i) out[i] = ctx->m[i];
}

// cpp:472-492
void GetInverseTransform(RenderContext* ctx, f64 out[6]) {
    f64 a = ctx->m[0], b = ctx->m[1], c = ctx->m[2], d = ctx->m[3], e = ctx->m[4], f = ctx->m[5];
    f64 det = a * d - b * c;
    f64 inv_det = det != 0 ? 1 / det : 1e9;
    out[0] = d * inv_det;
    out[1] = -b * inv_det;
    out[2] = -c * inv_det;
    out[3] = a * inv_det;
    out[4] = (c * f - d * e) * inv_det;
    out[5] = (b * e - a * f) * inv_det;
}

// cpp:623-641
void SetColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->ct[0] = r; ctx->ct[1] = g; ctx->ct[2] = b; ctx->ct[3] = a;
}
void ApplyColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->ct[0] *= r; ctx->ct[1] *= g; ctx->ct[2] *= b; ctx->ct[3] *= a;
}

// ---------------------------------------------------------------------------
// pixel ops (cpp:494-549, 643-691)
// ---------------------------------------------------------------------------
// cpp:494-513 (single-pixel store incl. the RGB overrun into index+3)
bool SetPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a) {
    if (x < 0 || x >= ctx->width || y < 0 || y >= ctx->height) return false;
    ctx->frameU8Valid = false;
    if (ctx->recording) return nr_record_set_pixel(ctx, x, y, r, g, b, a);
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    i64 ipp = ctx->enableAlpha ? 4 : 3;
    i64 index = y * ctx->width * ipp + x * ipp;
    f64 v[4] = {r, g, b, a};
    i64 cnt = (index + 3 < GetBufferSize(ctx)) ? 4 : 3;   // last RGB pixel: the reference writes past the end (UB)
    NR_CHECK(hipMemcpyAsync(ctx->buffer + index, v, (size_t)cnt * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));   // `v` is on this stack frame
    return true;
}

// cpp:515-549 (inline in the reference; exported here as a 1-pixel kernel)
__global__ void k_apply_one(f64* p, int ipp, f64 r, f64 g, f64 b, f64 a, f64 c0, f64 c1, f64 c2, f64 c3) {
    nr_apply_pixel(p, ipp, r, g, b, a, c0, c1, c2, c3);
}
bool ApplyPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a) {
    if (x < 0 || x >= ctx->width || y < 0 || y >= ctx->height) return false;
    ctx->frameU8Valid = false;
    if (ctx->recording) return nr_record_fill(ctx, x, x + 1, y, y + 1, r, g, b, a);
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    int ipp = ctx->enableAlpha ? 4 : 3;
    hipLaunchKernelGGL(k_apply_one, dim3(1), dim3(1), 0, ctx->stream, ctx->buffer + (y * ctx->width + x) * ipp,
                       ipp, r, g, b, a, ctx->ct[0], ctx->ct[1], ctx->ct[2], ctx->ct[3]);
    NR_CHECK(hipGetLastError());
    return true;
}

// cpp:643-657
void SetColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->frameU8Valid = false;
    NR_CHECK(hipSetDevice(ctx->device));
    nr_drop_commands(ctx);   // every value of the buffer is overwritten: queued draws are dead
    nr_settle(ctx);
    if (r == g && g == b && b == a) {
        // uniform clear: kept pending, consumed on chip by the tiled raster
        ctx->pendColor = true;
        ctx->pendColorValue = r;
        ctx->tileColor = false;   // (superseded)
        return;
    }
    ctx->pendColor = false;   // fully overwritten
    ctx->tileColor = false;
    int ipp = ctx->enableAlpha ? 4 : 3;
    i64 n = ctx->width * ctx->height;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_set_color, dim3(grid_for(n)), dim3(256), 0, ctx->stream, ctx->buffer, ctx->width,
                       ctx->height, ipp, r, g, b, a);
    NR_CHECK(hipGetLastError());
}

// cpp:659-680 (takes f64 coordinates; the reference Python binding's c_long
// declaration crashes)
void GetColor(RenderContext* ctx, f64 x, f64 y, f64* r, f64* g, f64* b, f64* a) {
    if (x < 0) x = 0;
    if (x >= ctx->width) x = ctx->width - 1;
    if (y < 0) y = 0;
    if (y >= ctx->height) y = ctx->height - 1;
    i64 ix = (i64)x, iy = (i64)y;
    i64 ipp = ctx->enableAlpha ? 4 : 3;
    i64 index = iy * ctx->width * ipp + ix * ipp;
    f64 v[4] = {0, 0, 0, 0};
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    NR_CHECK(hipMemcpyAsync(v, ctx->buffer + index, (size_t)ipp * sizeof(f64), hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    *r = v[0]; *g = v[1]; *b = v[2];
    if (ctx->enableAlpha) *a = v[3];
}

// cpp:682-691
void FillColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a) {
    ctx->frameU8Valid = false;
    if (ctx->recording) {
        nr_record_fill(ctx, 0, ctx->width, 0, ctx->height, r, g, b, a);
        return;
    }
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize_color(ctx);
    i64 n = ctx->width * ctx->height;
    if (n <= 0) return;
    int ipp = ctx->enableAlpha ? 4 : 3;
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_PRIM, &e0, &e1);
    hipLaunchKernelGGL(k_fill_color, dim3(grid_for(n)), dim3(256), 0, ctx->stream, ctx->buffer, n, ipp, r, g, b,
                       a, ctx->ct[0], ctx->ct[1], ctx->ct[2], ctx->ct[3]);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_PRIM, e0, e1);
}

i64 GetVersion() { return 1; }   // h:9

// ---------------------------------------------------------------------------
// new: device, sync, timing
// ---------------------------------------------------------------------------
// Selects the HIP device for objects created afterwards on this thread.
bool SetDevice(i64 device) { return hipSetDevice((int)device) == hipSuccess; }
i64 GetDeviceCount() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
i64 GetContextDevice(RenderContext* ctx) { return ctx->device; }

// Blocks until every queued draw of the context has finished.
void Flush(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_settle(ctx);
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    nr_dist_sync(ctx);
}

// Materialises deferred clears (tests use it to compare device state).
void ResolvePending(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize(ctx);
}

// Raw device pointers / stream, for RCCL or torch interop (no torch types).
// (the pending clears -- whole-frame and per-tile, the fast clear -- are
// written first, so the bytes behind the pointer are the framebuffer's value
// once the stream has drained: Flush)
void* GetDeviceBufferPtr(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize(ctx);
    return ctx->buffer;
}
void* GetStreamPtr(RenderContext* ctx) { return (void*)ctx->stream; }

// Switching off does not synchronise: recorded pairs are read at the next
// GetKernelTiming (or once 4096 are pending), so timing can be toggled per
// frame inside a timed loop.
void EnableKernelTiming(RenderContext* ctx, bool on) {
    ctx->timing = on;
    if (ctx->evPending.size() >= 4096 || ctx->tsPending.size() >= TS_PAIRS - 64) timing_collect(ctx);
}

// Sum and count of the named kernel's durations since the last reset
// (names: tri_count tri_scan tri_emit tri_sort tile_ranges tile_raster prim fill resolve vis_init).
bool GetKernelTiming(RenderContext* ctx, const char* name, f64* total_ms, i64* count) {
    NR_CHECK(hipSetDevice(ctx->device));
    timing_collect(ctx);
    for (int k = 0; k < NRK_COUNT_; ++k)
        if (strcmp(name, kKernelNames[k]) == 0) {
            *total_ms = ctx->kTimeMs[k];
            *count = ctx->kCount[k];
            return true;
        }
    return false;
}

// Restricts EnableKernelTiming to the named kernels (comma-separated; "" = all).
void SetKernelTimingFilter(RenderContext* ctx, const char* names) {
    if (!names || !*names) {
        ctx->timingMask = ~0ull;
        return;
    }
    ctx->timingMask = 0;
    std::string all(names);
    size_t pos = 0;
    while (pos <= all.size()) {
        size_t e = all.find(',', pos);
        if (e == std::string::npos) e = all.size();
        const std::string n = all.substr(pos, e - pos);
        for (int k = 0; k < NRK_COUNT_; ++k)
            if (n == kKernelNames[k]) ctx->timingMask |= 1ull << k;
        pos = e + 1;
    }
}

void ResetKernelTiming(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    timing_collect(ctx);
    for (int k = 0; k < NRK_COUNT_; ++k) { ctx->kTimeMs[k] = 0; ctx->kCount[k] = 0; }
}

}  // extern "C"

Texture* nr_new_texture(i64 w, i64 h, bool alpha) { return new_texture(w, h, alpha); }
