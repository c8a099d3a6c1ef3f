// nr_tri.hip — host API of the triangle / depth / Gouraud path (the
// north-star hot path) and the choice between its two rasterisers:
//   opaque batch (every vertex alpha == 1, colourTransform[3] == 1)
//       -> nr_tri_free.hip    visibility buffer, order-free, load-balanced
//   anything else
//       -> nr_tri_ordered.hip in-order tile raster (blending, painter's order)
// Both produce the oracle's bits; tests/test_parity_gpu.py checks both and
// checks that they agree with each other.
#include "nr_tri.h"

#include <algorithm>
#include <vector>
#include <atomic>
#include <cmath>

namespace nrtri {

bool grow_temp(TriScratch& sc, size_t need) {
    if (need <= sc.temp_bytes && sc.temp) return true;
    if (sc.temp) NR_CHECK(hipFree(sc.temp));
    if (hipMalloc(&sc.temp, need) != hipSuccess) {
        nr_set_error_msg("triangle scratch: hipMalloc failed");
        sc.temp = nullptr;
        sc.temp_bytes = 0;
        return false;
    }
    sc.temp_bytes = need;
    return true;
}

FrameParams frame_params(RenderContext* ctx, const TriSrc& src) {
    TriScratch& sc = ctx->tri;
    if (!sc.h_total) NR_CHECK(hipHostMalloc((void**)&sc.h_total, 4 * sizeof(u64)));
    if (ctx->depthTest) nr_ensure_depth(ctx);
    nr_materialize_tiles(ctx, true, true);   // (a batch starts from whole-frame clear state)
    FrameParams fp;
    fp.src = src;
    for (int k = 0; k < 6; ++k) fp.m[k] = ctx->m[k];
    for (int k = 0; k < 4; ++k) fp.ct[k] = ctx->ct[k];
    fp.fb = ctx->buffer;
    fp.depth = ctx->depth;
    fp.W = ctx->width;
    fp.H = ctx->height;
    fp.ipp = ctx->enableAlpha ? 4 : 3;
    fp.tiles_x = (int)((ctx->width + TW - 1) / TW);
    fp.tiles_y = (int)((ctx->height + TH - 1) / TH);
    fp.period = ctx->shardPeriod;
    fp.mask = nr_shard_mask(ctx, ctx->shard);
    fp.depthTest = ctx->depthTest;
    fp.depthWrite = ctx->depthWrite;
    fp.pendColor = ctx->pendColor;
    fp.pendColorValue = ctx->pendColorValue;
    fp.pendDepth = ctx->depthTest && ctx->pendDepth;
    fp.pendDepthValue = ctx->pendDepthValue;
    fp.fragCounter = nullptr;
    fp.frameU8 = nullptr;
    fp.frameYUV = ctx->frameFormat == 1;
    fp.tileStamp = nullptr;
    fp.tileEpoch = 0;
    fp.tstamp = nullptr;
    if (ctx->countFragments) {
        if (!sc.d_frag) NR_CHECK(hipMalloc(&sc.d_frag, sizeof(u64)));
        NR_CHECK(hipMemsetAsync(sc.d_frag, 0, sizeof(u64), ctx->stream));
        fp.fragCounter = sc.d_frag;
    }
    return fp;
}

// After the raster: account fragments, and mark the deferred clears consumed.
void finish_batch(RenderContext* ctx, const FrameParams& fp) {
    TriScratch& sc = ctx->tri;
    // the u8 mirror is current only when this batch's resolve wrote it for
    // every owned pixel (it does exactly when a clear was pending)
    ctx->frameU8Valid = fp.frameU8 != nullptr;
    if (fp.fragCounter) {
        NR_CHECK(hipMemcpyAsync(&sc.h_total[2], sc.d_frag, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
        NR_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->fragTotal += sc.h_total[2];
    }
    if (fp.tileStamp) {   // the empty tiles' clears stay pending (k_vis stamped them)
        ctx->tileColor = fp.pendColor != 0;
        ctx->tileColorValue = fp.pendColorValue;
        ctx->tileDepth = fp.pendDepth != 0;
        ctx->tileDepthValue = fp.pendDepthValue;
    }
    ctx->pendColor = false;
    if (ctx->depthTest) ctx->pendDepth = false;
}

namespace {

// Writes the pending clears of the tiles stamped `epoch` (one workgroup per tile).
__global__ __launch_bounds__(256) void k_tile_clear(f64* __restrict__ fb, u32* __restrict__ depth, i64 W, i64 H,
                                                    int tiles_x, int ipp, const u32* __restrict__ stamp, u32 epoch,
                                                    int doColor, f64 cv, int doDepth, u32 dv) {
    const int tile = blockIdx.x;
    if (stamp[tile] != epoch) return;
    const i64 x0 = (i64)(tile % tiles_x) * TW, y0 = (i64)(tile / tiles_x) * TH;
    for (int p = threadIdx.x; p < TW * TH; p += 256) {
        const i64 px = x0 + (p & (TW - 1)), py = y0 + p / TW;
        if (px >= W || py >= H) continue;
        const i64 q = py * W + px;
        if (doColor)
            for (int c = 0; c < ipp; ++c) fb[q * ipp + c] = cv;
        if (doDepth) depth[q] = dv;
    }
}

}  // namespace

// Stamp array of at least `ntiles` entries (zero = no epoch).
u32* tile_stamps(RenderContext* ctx, i64 ntiles) {
    if (ctx->tileStampCap < ntiles) {
        if (ctx->tileStamp) NR_CHECK(hipFree(ctx->tileStamp));
        NR_CHECK(hipMalloc(&ctx->tileStamp, (size_t)ntiles * sizeof(u32)));
        NR_CHECK(hipMemsetAsync(ctx->tileStamp, 0, (size_t)ntiles * sizeof(u32), ctx->stream));
        ctx->tileStampCap = ntiles;
    }
    if (++ctx->tileEpoch == 0) {   // (wrapped: no stale stamp may equal a new epoch)
        NR_CHECK(hipMemsetAsync(ctx->tileStamp, 0, (size_t)ctx->tileStampCap * sizeof(u32), ctx->stream));
        ctx->tileEpoch = 1;
    }
    return ctx->tileStamp;
}

namespace {

// User-space bounding boxes of the NR_CLUSTER-triangle clusters (TriangleBuffer::cbox).
std::vector<f64> host_cluster_boxes(const f64* xy, i64 n) {
    const i64 nc = (n + NR_CLUSTER - 1) / NR_CLUSTER;
    std::vector<f64> cb((size_t)nc * 4);
    for (i64 c = 0; c < nc; ++c) {
        f64 x0 = INFINITY, y0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY;
        bool bad = false;
        for (i64 t = c * NR_CLUSTER; t < std::min<i64>(n, (c + 1) * NR_CLUSTER); ++t)
            for (int v = 0; v < 3; ++v) {
                const f64 x = xy[t * 6 + 2 * v], y = xy[t * 6 + 2 * v + 1];
                if (!std::isfinite(x) || !std::isfinite(y)) bad = true;
                x0 = std::min(x0, x); x1 = std::max(x1, x);
                y0 = std::min(y0, y); y1 = std::max(y1, y);
            }
        if (bad) x0 = y0 = x1 = y1 = NAN;
        cb[c * 4] = x0; cb[c * 4 + 1] = y0; cb[c * 4 + 2] = x1; cb[c * 4 + 3] = y1;
    }
    return cb;
}

Opacity host_opacity(const f64* rgba, i64 n, bool gouraud) {
    const i64 stride = gouraud ? 12 : 4;
    for (i64 t = 0; t < n; ++t)
        for (int v = 0; v < (gouraud ? 3 : 1); ++v)
            if (rgba[t * stride + v * 4 + 3] != 1) return OPQ_BLENDED;
    return OPQ_OPAQUE;
}

// Opacity of a device-resident batch the host cannot inspect.
__global__ __launch_bounds__(256) void k_opacity(const f64* __restrict__ rgba, i64 n, int gouraud,
                                                 u32* __restrict__ nonopaque) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    bool bad = false;
    if (t < n) {
        if (gouraud) {
            const f64* a = rgba + t * 12;
            bad = a[3] != 1 || a[7] != 1 || a[11] != 1;
        } else {
            bad = rgba[t * 4 + 3] != 1;
        }
    }
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1)) atomicOr(nonopaque, 1u);
}

Opacity device_opacity(RenderContext* ctx, const TriSrc& src) {
    TriScratch& sc = ctx->tri;
    if (!sc.d_flag) NR_CHECK(hipMalloc(&sc.d_flag, sizeof(u32)));
    if (!sc.h_total) NR_CHECK(hipHostMalloc((void**)&sc.h_total, 4 * sizeof(u64)));
    NR_CHECK(hipMemsetAsync(sc.d_flag, 0, sizeof(u32), ctx->stream));
    hipLaunchKernelGGL(k_opacity, dim3((unsigned)((src.n + 255) / 256)), dim3(256), 0, ctx->stream, src.rgba, src.n,
                       src.gouraud, sc.d_flag);
    NR_CHECK(hipGetLastError());
    u32* h = reinterpret_cast<u32*>(&sc.h_total[3]);
    NR_CHECK(hipMemcpyAsync(h, sc.d_flag, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    return *h ? OPQ_BLENDED : OPQ_OPAQUE;
}

void draw(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud, Opacity opq,
          TriangleBuffer* tb = nullptr, bool callerOwned = false) {
    NR_CHECK(hipSetDevice(ctx->device));
    settle(ctx);
    if (n <= 0 || ctx->width <= 0 || ctx->height <= 0) return;
    if (!ctx->depthTest) nr_materialize_depth(ctx);
    TriSrc src{xy, z, rgba, gouraud ? 1 : 0, n};
    const bool freeEligible = ctx->ct[3] == 1 && ctx->forceOrdered == 0;
    if (freeEligible && opq == OPQ_UNKNOWN) opq = device_opacity(ctx, src);
    if (freeEligible && opq == OPQ_OPAQUE) draw_free(ctx, src, tb, callerOwned);
    else draw_ordered(ctx, src, tb, callerOwned);
}

}  // namespace
}  // namespace nrtri

using namespace nrtri;

void nr_materialize_tiles(RenderContext* ctx, bool color, bool depth) {
    const bool c = color && ctx->tileColor, d = depth && ctx->tileDepth && ctx->depth;
    if (!c && !d) return;
    if (c) ctx->tileColor = false;
    if (d) ctx->tileDepth = false;
    const i64 tx = (ctx->width + TW - 1) / TW, ty = (ctx->height + TH - 1) / TH;
    if (tx * ty <= 0) return;
    hipEvent_t a, b;
    nr_timing_begin(ctx, NRK_FILL, &a, &b);
    hipLaunchKernelGGL(k_tile_clear, dim3((unsigned)(tx * ty)), dim3(256), 0, ctx->stream, ctx->buffer, ctx->depth,
                       ctx->width, ctx->height, (int)tx, ctx->enableAlpha ? 4 : 3, ctx->tileStamp, ctx->tileEpoch,
                       c ? 1 : 0, ctx->tileColorValue, d ? 1 : 0, ctx->tileDepthValue);
    NR_CHECK(hipGetLastError());
    nr_timing_end(ctx, NRK_FILL, a, b);
}

void nr_settle(RenderContext* ctx) {
    nrtri::settle(ctx);
    nr_flush_commands(ctx);   // recorded draws come after the last batch in program order
}

extern "C" {

// New (no reference counterpart): depth-test LESS on/off, depth write on/off.
void SetDepthState(RenderContext* ctx, bool test, bool write) {
    ctx->depthTest = test;
    ctx->depthWrite = write;
}

// New: clear the u32 depth buffer (deferred; consumed by the raster).
void ClearDepth(RenderContext* ctx, u32 value) {
    ctx->pendDepth = true;
    ctx->pendDepthValue = value;
    ctx->tileDepth = false;   // (superseded)
}

// New: copy the W*H u32 depth buffer to the host.
void GetDepthBuffer(RenderContext* ctx, u32* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    settle(ctx);
    nr_ensure_depth(ctx);
    nr_materialize_depth(ctx);
    NR_CHECK(hipMemcpyAsync(out, ctx->depth, (size_t)(ctx->width * ctx->height) * sizeof(u32), hipMemcpyDeviceToHost,
                            ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
}

// New: triangles from device-resident arrays (xy n*6, z n*3 or NULL,
// rgba n*4 flat / n*12 Gouraud), in the context's transform.  Asynchronous
// like any kernel launch: the arrays must stay valid and unchanged until the
// batch has executed (Flush, a readback, or any device synchronisation).  The
// visibility path sizes such a batch exactly inside this call (a host wait for
// its binning), so nothing reads the arrays after that point.
void DrawTrianglesDevice(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud) {
    // the kernels load positions and colours as 16-byte vectors: re-stage
    // arrays that are not 16-byte aligned (device-to-device copy)
    if ((((uintptr_t)xy | (uintptr_t)rgba) & 15) && n > 0) {
        NR_CHECK(hipSetDevice(ctx->device));
        settle(ctx);
        const size_t ncol = gouraud ? 12 : 4, zn = ((size_t)n * 3 + 1) & ~(size_t)1;
        f64* stage_buf[1] = {ctx->tri.stage};
        if (!grow_set(stage_buf, &ctx->tri.stage_cap, (size_t)n * (6 + ncol) + zn)) return;
        ctx->tri.stage = stage_buf[0];
        f64* dxy = ctx->tri.stage;
        f64* dz = dxy + (size_t)n * 6;
        f64* dc = dz + zn;
        NR_CHECK(hipMemcpyAsync(dxy, xy, (size_t)n * 6 * sizeof(f64), hipMemcpyDeviceToDevice, ctx->stream));
        NR_CHECK(hipMemcpyAsync(dc, rgba, (size_t)n * ncol * sizeof(f64), hipMemcpyDeviceToDevice, ctx->stream));
        draw(ctx, dxy, z, dc, n, gouraud, OPQ_UNKNOWN, nullptr, z != nullptr);   // z stays the caller's
        return;
    }
    draw(ctx, xy, z, rgba, n, gouraud, OPQ_UNKNOWN, nullptr, true);
}

// New: triangles from host arrays (copied to HBM first).
void DrawTriangles(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba, i64 n, bool gouraud) {
    NR_CHECK(hipSetDevice(ctx->device));
    settle(ctx);   // a pending batch may still read the staging buffer
    if (n <= 0) return;
    const size_t ncol = gouraud ? 12 : 4;
    const size_t zn = ((size_t)n * 3 + 1) & ~(size_t)1;   // keeps the colours 16-byte aligned
    const size_t need = (size_t)n * (6 + ncol) + zn;
    f64* stage_buf[1] = {ctx->tri.stage};
    if (!grow_set(stage_buf, &ctx->tri.stage_cap, need)) return;
    ctx->tri.stage = stage_buf[0];
    f64* dxy = ctx->tri.stage;
    f64* dz = dxy + (size_t)n * 6;
    f64* dc = dz + zn;
    NR_CHECK(hipMemcpyAsync(dxy, xy, (size_t)n * 6 * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    if (z) NR_CHECK(hipMemcpyAsync(dz, z, (size_t)n * 3 * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipMemcpyAsync(dc, rgba, (size_t)n * ncol * sizeof(f64), hipMemcpyHostToDevice, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));   // caller may reuse its arrays on return
    draw(ctx, dxy, z ? dz : nullptr, dc, n, gouraud, host_opacity(rgba, n, gouraud), nullptr, false);
}

// New: a device-resident triangle soup (the H2D point; drawn many times).
TriangleBuffer* CreateTriangleBuffer(i64 n, const f64* xy, const f64* z, const f64* rgba, bool gouraud) {
    static std::atomic<u64> g_uid{0};
    TriangleBuffer* tb = new TriangleBuffer();
    tb->uid = ++g_uid;
    tb->n = n;
    tb->gouraud = gouraud;
    tb->opaque = n > 0 && host_opacity(rgba, n, gouraud) == OPQ_OPAQUE;
    std::vector<f64> cb;
    if (n > 0) cb = host_cluster_boxes(xy, n);
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
        NR_CHECK(hipMalloc(&tb->cbox, cb.size() * sizeof(f64)));
        NR_CHECK(hipMemcpyAsync(tb->cbox, cb.data(), cb.size() * sizeof(f64), hipMemcpyHostToDevice, s));
        NR_CHECK(hipStreamSynchronize(s));
        f64 b[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
        for (size_t c = 0; c + 3 < cb.size(); c += 4) {
            if (std::isnan(cb[c])) { b[0] = b[1] = b[2] = b[3] = NAN; break; }
            b[0] = std::min(b[0], cb[c]); b[1] = std::min(b[1], cb[c + 1]);
            b[2] = std::max(b[2], cb[c + 2]); b[3] = std::max(b[3], cb[c + 3]);
        }
        for (int k = 0; k < 4; ++k) tb->bbox[k] = b[k];
        tb->hcbox = std::move(cb);
    }
    return tb;
}

void DestroyTriangleBuffer(TriangleBuffer* tb) {
    if (!tb) return;
    // a context's pending batch may reference tb: the stream sync below
    // completes it; an overflow re-run would need tb, so settle all first
    nr_settle_all();
    NR_CHECK(hipSetDevice(tb->device));
    NR_CHECK(hipStreamSynchronize(nr_stream_for(tb->device)));
    NR_CHECK(hipStreamSynchronize(nr_bin_stream_for(tb->device)));
    if (tb->xy) NR_CHECK(hipFree(tb->xy));
    if (tb->z) NR_CHECK(hipFree(tb->z));
    if (tb->rgba) NR_CHECK(hipFree(tb->rgba));
    if (tb->cbox) NR_CHECK(hipFree(tb->cbox));
    delete tb;
}

i64 GetTriangleBufferCount(TriangleBuffer* tb) { return tb->n; }

void DrawTriangleBuffer(RenderContext* ctx, TriangleBuffer* tb) {
    // a TriangleBuffer never changes: its binning may overlap the previous batch's raster
    draw(ctx, tb->xy, tb->z, tb->rgba, tb->n, tb->gouraud, tb->opaque ? OPQ_OPAQUE : OPQ_BLENDED, tb, false);
}

// New: count covered on-screen pixel x triangle pairs (the "shaded+Z-tested
// fragments" work count of the Mpixels/s metric).  Counting uses a separate
// kernel variant and syncs per draw: enable it outside timed regions.
void SetFragmentCounting(RenderContext* ctx, bool on) {
    ctx->countFragments = on;
    ctx->fragTotal = 0;
}
i64 GetFragmentCount(RenderContext* ctx) { return (i64)ctx->fragTotal; }

// New (testing / A-B measurement): the whole-frame visibility buffer for
// opaque Z LESS + write batches, 0 automatic (small triangles, NR_GVIS), 1
// every such batch, 2 never (the tiled k_vis path).


// New (testing / A-B measurement): warm binning of a TriangleBuffer drawn
// again under the key of its last validated binning (one binning pass into
// the kept tile ranges), 0 automatic (NR_WARM), 1 on, 2 off.
void SetWarmBinning(RenderContext* ctx, i64 mode) { ctx->tri.warmMode = (int)(mode >= 0 && mode <= 2 ? mode : 0); }
// New (testing): number of batches of this context binned warm so far.
i64 GetWarmBatchCount(RenderContext* ctx) { return (i64)ctx->tri.warmBatches; }
// New (testing): of those, batches binned into the loose ranges (a changed transform).
i64 GetLooseBatchCount(RenderContext* ctx) { return (i64)ctx->tri.looseBatches; }
// New (testing): a fault in the next warm batch -- 1 its binning finds its
// tiles over their ranges, 2 (a batch binned beside the raster) its token is
// withheld (the raster's wait times out after 1 s), 3 it drops a workgroup's
// pairs, 4 (beside the raster) its binning is held back 1.5 s, so that it
// lands after the raster's fallback.  The raster must then run its fallback (k_vis WarmCheck): the frame
// stays exact and the failure is latched (GetWarmFailureCount, the error).
void SetWarmFaultInjection(RenderContext* ctx, i64 mode) { ctx->tri.warmInject = (int)(mode >= 0 && mode <= 4 ? mode : 0); }
// New (testing): warm batches whose checks failed so far (read at API calls).
i64 GetWarmFailureCount(RenderContext* ctx) {
    NR_CHECK(hipSetDevice(ctx->device));
    nrtri::settle(ctx);
    return (i64)ctx->tri.warmFailures;
}

// New: which raster the last batch took (1 = order-free tiled, 2 = ordered, 3 = order-free frame buffer).
i64 GetLastRasterPath(RenderContext* ctx) { return ctx->lastPath; }

// New (testing): cap the visibility path's pair list (0 = automatic), to
// exercise the overflow re-run of nr_settle.
void SetPairCapacityOverride(RenderContext* ctx, i64 pairs) { ctx->tri.capOverride = (u64)(pairs > 0 ? pairs : 0); }

// New (testing / A-B measurement): force the ordered raster for every batch.
void SetForceOrderedRaster(RenderContext* ctx, bool on) { ctx->forceOrdered = on ? 1 : 0; }

// New (testing / A-B measurement): k_vis variant, 0 automatic (previous
// batch's pair density), 1 with the wave-cooperative pass for large
// triangles, 2 without it.
void SetCoopRaster(RenderContext* ctx, i64 mode) { ctx->tri.coopMode = (int)(mode >= 0 && mode <= 2 ? mode : 0); }
// NEW (testing / tuning): a tile of more than min(slice, splitAt) pairs is split
// into slices of about dslice pairs (k_vis); 0 restores the defaults.
void SetSplitLimits(RenderContext* ctx, i64 splitAt, i64 dslice) {
    ctx->tri.splitAt = (u32)(splitAt > 0 ? splitAt : 0);
    ctx->tri.dslice = (u32)(dslice > 0 ? dslice : 0);
}

}  // extern "C"
