// nr_dist.hip — multi-GPU frames: screen tile-row sharding + RCCL assembly
// over xGMI.
//
// One process per GPU.  A context with SetShard(N, r) owns the 32-pixel tile
// rows ty with ty % N == r (interleaved, so a centred mesh loads every rank
// evenly); its triangle binning and raster skip every other row, so the
// ranks split the frame's raster work with no data-path collective.  The
// final image is assembled on the root by one grouped RCCL send/recv of the
// owned 32-row bands (each band is contiguous in the row-major framebuffer),
// written straight into place: the u8 frame the video encoder consumes
// (GatherFrameU8, cpp:237-239's conversion done per band on its owner), or
// the f64 framebuffer + depth (GatherFramebuffer) for exactness checks.
//
// RCCL is bound at run time with dlopen/dlsym, so the library loads (and the
// single-GPU path runs) where RCCL is absent, and a process that already
// loaded torch's RCCL reuses that copy instead of loading a second one.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include "nr_common.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;
bool g_rccl_tried = false;

Rccl* rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl_tried) return g_rccl.ok ? &g_rccl : nullptr;
    g_rccl_tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    void* h = nullptr;
    for (const char* n : names)
        if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
        nr_set_error_msg("RCCL not found (dlopen librccl.so.1 failed): multi-GPU assembly unavailable");
        return nullptr;
    }
    Rccl r;
    r.GetUniqueId = (decltype(r.GetUniqueId))dlsym(h, "ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))dlsym(h, "ncclCommInitRank");
    r.CommDestroy = (decltype(r.CommDestroy))dlsym(h, "ncclCommDestroy");
    r.GroupStart = (decltype(r.GroupStart))dlsym(h, "ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))dlsym(h, "ncclGroupEnd");
    r.Send = (decltype(r.Send))dlsym(h, "ncclSend");
    r.Recv = (decltype(r.Recv))dlsym(h, "ncclRecv");
    r.GetErrorString = (decltype(r.GetErrorString))dlsym(h, "ncclGetErrorString");
    r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.GroupStart && r.GroupEnd && r.Send && r.Recv &&
           r.GetErrorString;
    if (!r.ok) nr_set_error_msg("RCCL found but a required symbol is missing");
    g_rccl = r;
    return g_rccl.ok ? &g_rccl : nullptr;
}

bool nccl_ok(Rccl* r, ncclResult_t e, const char* what) {
    if (e == ncclSuccess) return true;
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, r->GetErrorString(e));
    nr_set_error_msg(buf);
    return false;
}

// Band ownership of a sharded frame, by value into the kernels: band b
// belongs to rank pattern[b % period].
struct ShardMap {
    int period;
    unsigned char pattern[64];
};

// Position of band b among the bands of its owner (bands packed back to back).
__device__ __forceinline__ i64 band_index(const ShardMap& sm, i64 b, int owner) {
    const int slot = (int)(b % sm.period);
    int per = 0, before = 0;
    for (int k = 0; k < sm.period; ++k) {
        const bool mine = sm.pattern[k] == owner;
        per += mine;
        before += (mine && k < slot);
    }
    return (b / sm.period) * per + before;
}

// f64 -> u8 (cpp:52-57) over the owned tile rows only (grid.y = every band)
__global__ void k_to_u8_rows(const f64* __restrict__ src, iu8* __restrict__ dst, i64 rowElems, i64 H, int TH,
                             int period, u64 mask) {
    const i64 band = blockIdx.y;
    if (period > 1 && !((mask >> (band % period)) & 1ull)) return;
    const i64 r0 = band * TH;
    if (r0 >= H) return;
    const i64 rows = (H - r0) < TH ? (H - r0) : TH;
    const i64 n = rows * rowElems;
    const i64 base = r0 * rowElems;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        dst[base + i] = nr_to_u8(src[base + i]);
}

// f64 -> YUV420P (SetFrameFormat(1)) over the owned tile rows: one thread per
// 2x2 block, u8 per channel as cpp:52-57, then nr_y_of / nr_u_of / nr_v_of.
__global__ void k_to_yuv_rows(const f64* __restrict__ src, iu8* __restrict__ dst, i64 W, i64 H, int ipp, int TH,
                              int period, u64 mask) {
    const i64 band = blockIdx.y;
    if (period > 1 && !((mask >> (band % period)) & 1ull)) return;
    const i64 r0 = band * TH;
    if (r0 >= H) return;
    const i64 rows = (H - r0) < TH ? (H - r0) : TH;
    const i64 cw = W / 2, nb = (rows / 2) * cw;
    iu8* up = dst + W * H;
    iu8* vp = up + cw * (H / 2);
    for (i64 q = (i64)blockIdx.x * blockDim.x + threadIdx.x; q < nb; q += (i64)gridDim.x * blockDim.x) {
        const i64 cy = r0 / 2 + q / cw, cx = q % cw;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const i64 x = 2 * cx + (k & 1), y = 2 * cy + (k >> 1);
            const f64* px = src + (y * W + x) * ipp;
            const int r = nr_to_u8(px[0]), g = nr_to_u8(px[1]), b = nr_to_u8(px[2]);
            dst[y * W + x] = nr_y_of(r, g, b);
            if (k == 0) {
                up[cy * cw + cx] = nr_u_of(r, g, b);
                vp[cy * cw + cx] = nr_v_of(r, g, b);
            }
        }
    }
}

// YUV420P from the u8 frame (GetFrameYUV420P): one thread per 2x2 block.
__global__ void k_yuv420p(const iu8* __restrict__ rgb, int ipp, i64 W, i64 H, iu8* __restrict__ yp,
                          iu8* __restrict__ up, iu8* __restrict__ vp) {
    const i64 cw = W / 2, n = cw * (H / 2);
    for (i64 q = (i64)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (i64)gridDim.x * blockDim.x) {
        const i64 cy = q / cw, cx = q - cy * cw;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const i64 x = 2 * cx + (k & 1), y = 2 * cy + (k >> 1);
            const iu8* px = rgb + (y * W + x) * ipp;
            const int r = px[0], g = px[1], b = px[2];
            yp[y * W + x] = nr_y_of(r, g, b);
            if (k == 0) {
                up[q] = nr_u_of(r, g, b);
                vp[q] = nr_v_of(r, g, b);
            }
        }
    }
}

constexpr int BAND = 32;   // = nrtri::TH, the tile height

ShardMap shard_map(const RenderContext* ctx) {
    ShardMap m;
    m.period = ctx->shardPeriod;
    memcpy(m.pattern, ctx->shardPattern, sizeof m.pattern);
    return m;
}

// Frame output geometry (nr_frame_bytes): the u8 image is one plane of
// W*ipp bytes per row; YUV420P is Y (W per row) + U and V (W/2 per chroma
// row, one chroma row per two rows).  Band b = rows [32b, 32b + 32) holds, in
// the frame, up to three segments: its rows of each plane.
struct FrameGeom {
    i64 W, H;
    int ipp;
    int yuv;
};

FrameGeom frame_geom(const RenderContext* ctx) {
    return FrameGeom{ctx->width, ctx->height, ctx->enableAlpha ? 4 : 3, ctx->frameFormat == 1 ? 1 : 0};
}

__host__ __device__ __forceinline__ int band_segments(const FrameGeom& g, i64 b, i64 (&off)[3], i64 (&len)[3]) {
    const i64 r0 = b * BAND, rows = (g.H - r0) < BAND ? (g.H - r0) : BAND;
    if (!g.yuv) {
        off[0] = r0 * g.W * g.ipp;
        len[0] = rows * g.W * g.ipp;
        return 1;
    }
    const i64 cw = g.W / 2, c0 = r0 / 2, crows = rows / 2;
    off[0] = r0 * g.W;                               len[0] = rows * g.W;
    off[1] = g.W * g.H + c0 * cw;                    len[1] = crows * cw;
    off[2] = g.W * g.H + (g.H / 2) * cw + c0 * cw;   len[2] = crows * cw;
    return 3;
}

// Bytes of a full band (every band but possibly the frame's last).
__host__ __device__ __forceinline__ i64 full_band_bytes(const FrameGeom& g) {
    return g.yuv ? BAND * g.W + 2 * (BAND / 2) * (g.W / 2) : BAND * g.W * g.ipp;
}

// Bytes of the frame output owned by `rank` under the context's band pattern.
i64 owned_bytes(const RenderContext* ctx, int rank) {
    const FrameGeom g = frame_geom(ctx);
    i64 bytes = 0;
    for (i64 b = 0; b * BAND < ctx->height; ++b)
        if (ctx->shardPattern[b % ctx->shardPeriod] == rank) {
            i64 off[3], len[3];
            const int ns = band_segments(g, b, off, len);
            for (int k = 0; k < ns; ++k) bytes += len[k];
        }
    return bytes;
}

i64 max_owned_bytes(const RenderContext* ctx, int n) {
    i64 m = 0;
    for (int p = 0; p < n; ++p) m = std::max(m, owned_bytes(ctx, p));
    return m;
}

// Packed band layout of the gather: a rank's owned bands back to back (its
// k-th band at k * full_band_bytes, its segments one after another; only the
// frame's last band can be short, and it is the last of its owner).  Pack
// (!UNPACK): the bands of `sel` from the frame into `stage`.  Unpack: the
// bands of every rank but `root` from its slot of `stage` (rank p at
// p * peerStride) into the frame.
template <typename V, bool UNPACK>
__global__ void k_band_copy(iu8* __restrict__ frame, iu8* __restrict__ stage, FrameGeom g, ShardMap sm, int sel,
                            i64 peerStride) {
    const i64 b = blockIdx.y;
    const int owner = sm.pattern[b % sm.period];
    if (UNPACK ? owner == sel : owner != sel) return;
    i64 off[3], len[3];
    const int ns = band_segments(g, b, off, len);
    iu8* sb = stage + (UNPACK ? owner * peerStride : 0) + band_index(sm, b, owner) * full_band_bytes(g);
    for (int k = 0; k < ns; ++k) {
        V* f = reinterpret_cast<V*>(frame + off[k]);
        V* st = reinterpret_cast<V*>(sb);
        const i64 n = len[k] / (i64)sizeof(V);
        for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
            if (UNPACK) f[i] = st[i];
            else st[i] = f[i];
        }
        sb += len[k];
    }
}

// Launches k_band_copy over every band on `st` (16-byte vectors when every
// segment offset and length is a multiple of 16).
void band_copy(RenderContext* ctx, iu8* frame, iu8* stage, hipStream_t st, bool unpack, int sel, i64 peerStride) {
    const ShardMap sm = shard_map(ctx);
    const FrameGeom g = frame_geom(ctx);
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    bool vec = full_band_bytes(g) % 16 == 0;
    for (i64 b = 0; b < bands && vec; ++b) {
        i64 off[3], len[3];
        const int ns = band_segments(g, b, off, len);
        for (int k = 0; k < ns; ++k) vec = vec && off[k] % 16 == 0 && len[k] % 16 == 0;
    }
    const i64 per = full_band_bytes(g) / (vec ? 16 : 1);
    dim3 grid((unsigned)std::min<i64>((per + 255) / 256, 1024), (unsigned)bands);
    if (vec) {
        if (unpack) hipLaunchKernelGGL((k_band_copy<uint4, true>), grid, dim3(256), 0, st, frame, stage, g, sm, sel,
                                       peerStride);
        else hipLaunchKernelGGL((k_band_copy<uint4, false>), grid, dim3(256), 0, st, frame, stage, g, sm, sel,
                                peerStride);
    } else {
        if (unpack) hipLaunchKernelGGL((k_band_copy<iu8, true>), grid, dim3(256), 0, st, frame, stage, g, sm, sel,
                                       peerStride);
        else hipLaunchKernelGGL((k_band_copy<iu8, false>), grid, dim3(256), 0, st, frame, stage, g, sm, sel,
                                peerStride);
    }
    NR_CHECK(hipGetLastError());
}

// The context's gather stream and events (created on first use).  The
// transfer of frame k runs there while the main stream renders frame k+1.
void ensure_comm_stream(RenderContext* ctx) {
    if (ctx->commStream) return;
    NR_CHECK(hipStreamCreateWithFlags(&ctx->commStream, hipStreamNonBlocking));
    const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
    NR_CHECK(hipEventCreateWithFlags(&ctx->evFrameReady, fl));
    for (auto& e : ctx->evGatherDone) NR_CHECK(hipEventCreateWithFlags(&e, fl));
}

// Staging buffer `x` of the packed gather (a non-root rank's own bands, or on
// the root one slot of the largest share per rank).
bool ensure_stage(RenderContext* ctx, int x, size_t need) {
    if (need <= ctx->stageCap[x]) return true;
    if (ctx->stageBuf[x]) {
        if (ctx->commStream) NR_CHECK(hipStreamSynchronize(ctx->commStream));
        NR_CHECK(hipFree(ctx->stageBuf[x]));
    }
    ctx->stageBuf[x] = nullptr;
    ctx->stageCap[x] = 0;
    if (hipMalloc((void**)&ctx->stageBuf[x], need) != hipSuccess) {
        nr_set_error_msg("GatherFrameU8: hipMalloc of the staging buffer failed");
        return false;
    }
    ctx->stageCap[x] = need;
    return true;
}

// After frame buffer x went out for assembly: the next frame renders into
// the other buffer, once the transfer that last read it (two frames back) is
// done -- the main stream waits for that on the device, the host never does.
void rotate_frame(RenderContext* ctx, int x) {
    NR_CHECK(hipEventRecord(ctx->evGatherDone[x], ctx->commStream));
    ctx->gatherPending[x] = true;
    ctx->frameLast = x;
    const int y = 1 - x;
    ctx->frameCur = y;
    ctx->frameU8 = ctx->frameBuf[y];
    ctx->frameU8Valid = false;
    if (ctx->gatherPending[y]) NR_CHECK(hipStreamWaitEvent(ctx->stream, ctx->evGatherDone[y], 0));
}

// The u8 image of the owned bands (the first half of GatherFrameU8), converted
// only when the mirror the resolves write is not current.
bool frame_u8_local(RenderContext* ctx) {
    nr_settle(ctx);   // (the buffer's pending clears are written only if the f64 frame is converted below)
    const int ipp = ctx->enableAlpha ? 4 : 3;
    const i64 n = nr_frame_bytes(ctx);
    if (n <= 0) return true;
    if ((size_t)n > ctx->frameU8cap) {   // both frame buffers (the assembly alternates between them)
        if (ctx->commStream) NR_CHECK(hipStreamSynchronize(ctx->commStream));
        for (int x = 0; x < 2; ++x) {
            if (ctx->frameBuf[x]) NR_CHECK(hipFree(ctx->frameBuf[x]));
            ctx->frameBuf[x] = nullptr;
            ctx->gatherPending[x] = false;
        }
        ctx->frameU8 = nullptr;
        ctx->frameU8cap = 0;
        ctx->frameLast = -1;
        for (int x = 0; x < 2; ++x)
            if (hipMalloc((void**)&ctx->frameBuf[x], (size_t)n) != hipSuccess) {
                nr_set_error_msg("GatherFrameU8: hipMalloc failed");
                return false;
            }
        ctx->frameU8cap = (size_t)n;
        ctx->frameU8 = ctx->frameBuf[ctx->frameCur];
        ctx->frameU8Valid = false;
    }
    const i64 rowElems = ctx->width * ipp;
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    const i64 owned = owned_bytes(ctx, ctx->shard);
    // later triangle resolves write the frame output themselves (no re-read
    // of the f64 frame); convert here only when that mirror is not current
    ctx->frameOutput = true;
    if (owned > 0 && !ctx->frameU8Valid) {
        nr_materialize_color(ctx);
        hipEvent_t e0, e1;
        nr_timing_begin(ctx, NRK_OUTPUT, &e0, &e1);
        if (ctx->frameFormat == 1) {
            const i64 blocks = (BAND / 2) * (ctx->width / 2);
            dim3 grid((unsigned)std::min<i64>((blocks + 255) / 256, 4096), (unsigned)bands);
            hipLaunchKernelGGL(k_to_yuv_rows, grid, dim3(256), 0, ctx->stream, ctx->buffer, ctx->frameU8, ctx->width,
                               ctx->height, ipp, BAND, ctx->shardPeriod, nr_shard_mask(ctx, ctx->shard));
        } else {
            dim3 grid((unsigned)std::min<i64>((BAND * rowElems + 255) / 256, 4096), (unsigned)bands);
            hipLaunchKernelGGL(k_to_u8_rows, grid, dim3(256), 0, ctx->stream, ctx->buffer, ctx->frameU8, rowElems,
                               ctx->height, BAND, ctx->shardPeriod, nr_shard_mask(ctx, ctx->shard));
        }
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_OUTPUT, e0, e1);
    }
    ctx->frameU8Valid = true;
    ctx->frameLast = ctx->frameCur;
    return true;
}

}  // namespace

struct NrComm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
};

extern "C" {

// NEW: 128-byte RCCL unique id (rank 0 creates it; the caller distributes it).
bool GetCommUniqueId(iu8* out128) {
    Rccl* r = rccl();
    if (!r) return false;
    ncclUniqueId id;
    if (!nccl_ok(r, r->GetUniqueId(&id), "ncclGetUniqueId")) return false;
    memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return true;
}

// NEW: communicator over the calling thread's current HIP device.
NrComm* CreateComm(i64 nranks, i64 rank, const iu8* id128) {
    Rccl* r = rccl();
    if (!r) return nullptr;
    NrComm* c = new NrComm();
    c->nranks = (int)nranks;
    c->rank = (int)rank;
    NR_CHECK(hipGetDevice(&c->device));
    ncclUniqueId id;
    memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    if (!nccl_ok(r, r->CommInitRank(&c->comm, (int)nranks, id, (int)rank), "ncclCommInitRank")) {
        delete c;
        return nullptr;
    }
    return c;
}

void DestroyComm(NrComm* c) {
    if (!c) return;
    Rccl* r = rccl();
    if (r && c->comm) r->CommDestroy(c->comm);
    delete c;
}

// NEW: this context renders only tile rows ty with ty % nshards == shard.
void SetShard(RenderContext* ctx, i64 nshards, i64 shard) {
    if (nshards < 1 || shard < 0 || shard >= nshards) {
        nr_set_error_msg("SetShard: need 0 <= shard < nshards");
        return;
    }
    if (nshards > 64) {
        nr_set_error_msg("SetShard: at most 64 shards");
        return;
    }
    ctx->nshards = (int)nshards;
    ctx->shard = (int)shard;
    ctx->shardPeriod = (int)nshards;
    for (int k = 0; k < 64; ++k) ctx->shardPattern[k] = (unsigned char)(k < nshards ? k : 0);
    ctx->frameU8Valid = false;
}

// NEW: weighted shards.  Rank p owns slots[p] of every sum(slots) (<= 64)
// consecutive bands, spread by smooth weighted round robin (each step every
// rank gains its slots, the rank with the most credit -- lowest rank on ties
// -- takes the band and pays the period), so a rank's bands are interleaved
// over the frame.  Equal slots give SetShard's pattern.  Every rank of a
// frame must make the same call (with its own `shard`).
void SetShardSlots(RenderContext* ctx, i64 nshards, i64 shard, const i64* slots) {
    if (nshards < 1 || nshards > 64 || shard < 0 || shard >= nshards) {
        nr_set_error_msg("SetShardSlots: need 0 <= shard < nshards <= 64");
        return;
    }
    i64 period = 0;
    for (i64 p = 0; p < nshards; ++p) {
        if (slots[p] < 1) {
            nr_set_error_msg("SetShardSlots: every rank needs at least one slot");
            return;
        }
        period += slots[p];
    }
    if (period > 64) {
        nr_set_error_msg("SetShardSlots: sum(slots) must be <= 64");
        return;
    }
    i64 credit[64] = {0};
    for (i64 k = 0; k < period; ++k) {
        int best = 0;
        for (i64 p = 0; p < nshards; ++p) {
            credit[p] += slots[p];
            if (credit[p] > credit[best]) best = (int)p;
        }
        credit[best] -= period;
        ctx->shardPattern[k] = (unsigned char)best;
    }
    ctx->nshards = (int)nshards;
    ctx->shard = (int)shard;
    ctx->shardPeriod = (int)period;
    ctx->frameU8Valid = false;
}

// NEW: the band pattern (period entries, owner rank per band slot).
i64 GetShardPattern(RenderContext* ctx, iu8* out64) {
    memcpy(out64, ctx->shardPattern, 64);
    return ctx->shardPeriod;
}

// NEW: the u8 image of the frame (cpp:52-57 per element) assembled on `root`
// in a context-owned device buffer: every rank converts its owned bands, then
// one grouped send/recv moves them into place.  comm == NULL: local only.
bool GatherFrameU8(RenderContext* ctx, NrComm* comm, i64 root) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (!frame_u8_local(ctx)) return false;
    if (!comm || comm->nranks == 1) return true;
    if (comm->nranks != ctx->nshards || comm->rank != ctx->shard) {
        nr_set_error_msg("GatherFrameU8: the context's shard must match the communicator (SetShard(nranks, rank))");
        return false;
    }
    if (root < 0 || root >= comm->nranks) {
        nr_set_error_msg("GatherFrameU8: root out of range");
        return false;
    }
    Rccl* r = rccl();
    if (!r) return false;
    // One message per rank: every non-root rank packs its bands back to back
    // and sends them; the root receives each rank's pack into its own slot
    // and scatters all of them into place with one kernel (a send/recv per
    // band would cost RCCL's per-operation latency ~H/32 times on the root).
    // The transfer and the unpack run on the context's gather stream, so they
    // overlap the next frame, which renders into the other frame buffer.
    const int n = comm->nranks, me = comm->rank, x = ctx->frameCur;
    const i64 peerStride = max_owned_bytes(ctx, n);
    ensure_comm_stream(ctx);
    if (!ensure_stage(ctx, x, (size_t)(me == root ? n * peerStride : owned_bytes(ctx, me))))
        return false;
    iu8* frame = ctx->frameBuf[x];
    iu8* stage = ctx->stageBuf[x];
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_GATHER, &e0, &e1);
    if (me != root) band_copy(ctx, frame, stage, ctx->stream, false, me, 0);
    nr_timing_end(ctx, NRK_GATHER, e0, e1);
    NR_CHECK(hipEventRecord(ctx->evFrameReady, ctx->stream));
    NR_CHECK(hipStreamWaitEvent(ctx->commStream, ctx->evFrameReady, 0));
    bool ok = nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (int p = 0; p < n && ok; ++p) {
        const size_t cnt = (size_t)owned_bytes(ctx, p);
        if (cnt == 0) continue;
        if (me == root && p != root)
            ok = nccl_ok(r, r->Recv(stage + p * peerStride, cnt, ncclUint8, p, comm->comm, ctx->commStream),
                         "ncclRecv");
        else if (me != root && p == me)
            ok = nccl_ok(r, r->Send(stage, cnt, ncclUint8, (int)root, comm->comm, ctx->commStream), "ncclSend");
    }
    ok = nccl_ok(r, r->GroupEnd(), "ncclGroupEnd") && ok;
    if (ok && me == root) band_copy(ctx, frame, stage, ctx->commStream, true, (int)root, peerStride);
    rotate_frame(ctx, x);
    return ok;
}

// NEW (testing): GatherFrameU8 for n contexts of ONE process (ctxs[p] renders
// shard p of n) with device copies in place of the RCCL send/recv: the same
// packing, slot layout, unpack kernel, gather stream and frame-buffer
// rotation, so the multi-GPU assembly (and its overlap with the next frame)
// is checked on a single GPU.
static bool gather_local(RenderContext** ctxs, i64 n, i64 root, NrComm* self);

bool GatherFrameU8Local(RenderContext** ctxs, i64 n, i64 root) { return gather_local(ctxs, n, root, nullptr); }

// NEW (testing): GatherFrameU8Local with the peers' packs moved by RCCL
// instead of device copies: one ncclGroupStart/End of a send and a receive
// per peer over a one-rank communicator of this process (`self`, a
// send/receive pair to its own rank), on the root's gather stream -- the RCCL
// calls of GatherFrameU8 exercised on one GPU.
bool GatherFrameU8LocalRccl(RenderContext** ctxs, i64 n, i64 root, NrComm* self) {
    if (!self || self->nranks != 1) {
        nr_set_error_msg("GatherFrameU8LocalRccl: need a one-rank communicator");
        return false;
    }
    return gather_local(ctxs, n, root, self);
}

}  // extern "C"

static bool gather_local(RenderContext** ctxs, i64 n, i64 root, NrComm* self) {
    if (n < 1 || root < 0 || root >= n) {
        nr_set_error_msg("GatherFrameU8Local: need 0 <= root < n");
        return false;
    }
    RenderContext* rc = ctxs[root];
    for (i64 p = 0; p < n; ++p) {
        RenderContext* c = ctxs[p];
        if (c->nshards != n || c->shard != p || c->width != rc->width || c->height != rc->height ||
            c->enableAlpha != rc->enableAlpha || c->frameFormat != rc->frameFormat || c->device != rc->device ||
            c->shardPeriod != rc->shardPeriod ||
            memcmp(c->shardPattern, rc->shardPattern, 64) != 0) {
            nr_set_error_msg("GatherFrameU8Local: ctxs[p] must be shard p of n (one pattern), all of one size and device");
            return false;
        }
        NR_CHECK(hipSetDevice(c->device));
        if (!frame_u8_local(c)) return false;
    }
    if (n == 1) return true;
    const i64 peerStride = max_owned_bytes(rc, (int)n);
    NR_CHECK(hipSetDevice(rc->device));
    ensure_comm_stream(rc);
    const int xr = rc->frameCur;
    if (!ensure_stage(rc, xr, (size_t)(n * peerStride))) return false;
    for (i64 p = 0; p < n; ++p) {   // peers: pack on their stream, the root's gather stream waits
        if (p == root) continue;
        RenderContext* c = ctxs[p];
        ensure_comm_stream(c);
        const int xp = c->frameCur;
        const size_t cnt = (size_t)owned_bytes(c, (int)p);
        if (!ensure_stage(c, xp, cnt)) return false;
        band_copy(c, c->frameBuf[xp], c->stageBuf[xp], c->stream, false, (int)p, 0);
        NR_CHECK(hipEventRecord(c->evFrameReady, c->stream));
        NR_CHECK(hipStreamWaitEvent(rc->commStream, c->evFrameReady, 0));
    }
    Rccl* r = self ? rccl() : nullptr;
    if (self && !r) return false;
    bool ok = !self || nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (i64 p = 0; p < n && ok; ++p) {   // the packs into the root's slots
        if (p == root) continue;
        RenderContext* c = ctxs[p];
        const size_t cnt = (size_t)owned_bytes(c, (int)p);
        if (cnt == 0) continue;
        iu8* dst = rc->stageBuf[xr] + p * peerStride;
        const iu8* src = c->stageBuf[c->frameCur];
        if (!self) {
            NR_CHECK(hipMemcpyAsync(dst, src, cnt, hipMemcpyDeviceToDevice, rc->commStream));
            continue;
        }
        ok = nccl_ok(r, r->Send(src, cnt, ncclUint8, 0, self->comm, rc->commStream), "ncclSend") &&
             nccl_ok(r, r->Recv(dst, cnt, ncclUint8, 0, self->comm, rc->commStream), "ncclRecv");
    }
    if (self) ok = nccl_ok(r, r->GroupEnd(), "ncclGroupEnd") && ok;
    if (!ok) return false;
    NR_CHECK(hipEventRecord(rc->evFrameReady, rc->stream));
    NR_CHECK(hipStreamWaitEvent(rc->commStream, rc->evFrameReady, 0));
    band_copy(rc, rc->frameBuf[xr], rc->stageBuf[xr], rc->commStream, true, (int)root, peerStride);
    // the peers' stages were read on the root's gather stream: their own
    // gather streams (whose events guard the buffers' reuse) wait for it
    NR_CHECK(hipEventRecord(rc->evGatherDone[xr], rc->commStream));
    for (i64 p = 0; p < n; ++p) {
        if (p == root) continue;
        RenderContext* c = ctxs[p];
        NR_CHECK(hipStreamWaitEvent(c->commStream, rc->evGatherDone[xr], 0));
        rotate_frame(c, c->frameCur);
    }
    rotate_frame(rc, xr);
    return true;
}

extern "C" {

// NEW: copy the frame of the last GatherFrameU8 to the host (the assembled
// image on the root; a rank's own bands elsewhere).  False (and nothing
// written) when there is no gathered frame: none yet, or SetFrameFormat /
// ResizeRenderContext dropped it.
bool GetFrameU8(RenderContext* ctx, iu8* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (ctx->frameLast < 0 || !ctx->frameBuf[ctx->frameLast]) {
        nr_set_error_msg("GetFrameU8: no gathered frame (GatherFrameU8 first; a resize or format change drops it)");
        return false;
    }
    if (ctx->commStream) NR_CHECK(hipStreamSynchronize(ctx->commStream));
    NR_CHECK(hipMemcpyAsync(out, ctx->frameBuf[ctx->frameLast], (size_t)nr_frame_bytes(ctx), hipMemcpyDeviceToHost,
                            ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    return true;
}

// NEW: the frame of the last GatherFrameU8 as YUV420P planes
// (Y W*H, then U and V (W/2)*(H/2) each, W and H even), the encoder input of
// PutRendererContextFrame (cpp:232-275, sws_scale RGB24/RGBA -> YUV420P).
// Converted on the GPU so the host receives 1.5 bytes per pixel instead of
// 3 or 4.  Arithmetic: swscale's unscaled RGB -> YV12 converter (rgb2rgb's
// rgb24toyv12): BT.601 limited range, 15-bit fixed-point coefficients
// (0.299/0.587/0.114 x 219/255, chroma x 224/255, rounded), Y/U/V =
// (c . rgb >> 15) + 16/128/128, chroma point-sampled at the even pixel of each
// 2x2 block.  Parity unpinned: FFmpeg is absent here, and which of swscale's
// converters a given FFmpeg build picks (this one or the bilinear scaler path)
// depends on its version.  Returns false for odd sizes.
bool GetFrameYUV420P(RenderContext* ctx, iu8* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    const i64 W = ctx->width, H = ctx->height;
    if ((W & 1) || (H & 1)) {
        nr_set_error_msg("GetFrameYUV420P: width and height must be even");
        return false;
    }
    if (ctx->frameLast < 0 || !ctx->frameBuf[ctx->frameLast] || W * H == 0) return W * H == 0;
    if (ctx->commStream) NR_CHECK(hipStreamSynchronize(ctx->commStream));
    const size_t bytes = (size_t)(W * H + 2 * (W / 2) * (H / 2));
    if (ctx->frameFormat == 1) {   // the frame output already is YUV420P
        NR_CHECK(hipMemcpyAsync(out, ctx->frameBuf[ctx->frameLast], bytes, hipMemcpyDeviceToHost, ctx->stream));
        NR_CHECK(hipStreamSynchronize(ctx->stream));
        return true;
    }
    if (bytes > ctx->yuvCap) {   // the context keeps its plane buffer (the stream has drained above)
        NR_CHECK(hipStreamSynchronize(ctx->stream));
        if (ctx->yuvBuf) NR_CHECK(hipFree(ctx->yuvBuf));
        ctx->yuvBuf = nullptr;
        ctx->yuvCap = 0;
        if (hipMalloc((void**)&ctx->yuvBuf, bytes) != hipSuccess) {
            nr_set_error_msg("GetFrameYUV420P: hipMalloc failed");
            ctx->yuvBuf = nullptr;
            return false;
        }
        ctx->yuvCap = bytes;
    }
    iu8* d = ctx->yuvBuf;
    const i64 blocks = (W / 2) * (H / 2);
    hipLaunchKernelGGL(k_yuv420p, dim3((unsigned)std::min<i64>((blocks + 255) / 256, 16384)), dim3(256), 0,
                       ctx->stream, ctx->frameBuf[ctx->frameLast], ctx->enableAlpha ? 4 : 3, W, H, d, d + W * H,
                       d + W * H + blocks);
    NR_CHECK(hipGetLastError());
    NR_CHECK(hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
    return true;
}

// NEW: format of the frame output of GatherFrameU8 / GatherFrameU8Local:
// 0 = the u8 image (cpp:52-57, default), 1 = its YUV420P planes (the encoder
// input of PutRendererContextFrame, cpp:232-275; 1.5 bytes per pixel instead
// of 3 or 4 through the gather and to the host).  The raster writes it
// directly.  Every rank of a frame must use the same format;
// YUV420P needs even W and H.
bool SetFrameFormat(RenderContext* ctx, i64 format) {
    if (format != 0 && format != 1) {
        nr_set_error_msg("SetFrameFormat: 0 (u8 image) or 1 (YUV420P)");
        return false;
    }
    if (format == 1 && ((ctx->width & 1) || (ctx->height & 1))) {
        nr_set_error_msg("SetFrameFormat: YUV420P needs even width and height");
        return false;
    }
    if (ctx->frameFormat != (int)format) {
        NR_CHECK(hipSetDevice(ctx->device));
        nr_settle(ctx);
        nr_dist_sync(ctx);
        ctx->frameFormat = (int)format;
        ctx->frameU8Valid = false;
        ctx->frameLast = -1;
        for (bool& g : ctx->gatherPending) g = false;
    }
    return true;
}

i64 GetFrameFormat(RenderContext* ctx) { return ctx->frameFormat; }

// NEW (§8f-2, frame delivery): the video caller hands every frame to the
// encoder on the host (milrenderer.py:1038 -> PutRendererContextFrame,
// cpp:232-275).  This copies the frame output of the last GatherFrameU8 (u8
// image or YUV420P planes) into `host` -- pinned memory from AllocHostBuffer,
// so the copy is one DMA -- on the gather stream, and returns at once: the
// next frame renders into the other frame buffer meanwhile, and a frame buffer
// is rendered into again only after its copy is done (device-side wait).
// Returns a ticket for WaitFrameDelivered, or -1 when there is no gathered
// frame.  `host` must hold nr_frame_bytes and stay untouched until the wait.
i64 DeliverFrameU8(RenderContext* ctx, iu8* host) {
    NR_CHECK(hipSetDevice(ctx->device));
    const int x = ctx->frameLast;
    if (x < 0 || !ctx->frameBuf[x]) {
        nr_set_error_msg("DeliverFrameU8: no gathered frame (GatherFrameU8 first)");
        return -1;
    }
    ensure_comm_stream(ctx);
    if (!ctx->evDeliver[x]) NR_CHECK(hipEventCreateWithFlags(&ctx->evDeliver[x], hipEventDisableTiming));
    const bool local = ctx->frameCur == x;   // a local gather (no assembly): buffer x was written on the main stream
    if (local) {
        NR_CHECK(hipEventRecord(ctx->evFrameReady, ctx->stream));
        NR_CHECK(hipStreamWaitEvent(ctx->commStream, ctx->evFrameReady, 0));
    }   // else: the assembly into x is already queued on the gather stream
    // (the runtime's copy: one blit workgroup; DMA-engine and wider copy kernels measured slower beside the
    // raster, profiles/r05/ab_d2h.txt)
    NR_CHECK(hipMemcpyAsync(host, ctx->frameBuf[x], (size_t)nr_frame_bytes(ctx), hipMemcpyDeviceToHost,
                            ctx->commStream));
    NR_CHECK(hipEventRecord(ctx->evDeliver[x], ctx->commStream));
    if (local) {
        rotate_frame(ctx, x);   // the next frame renders into the other buffer
    } else {                    // buffer x is reused only after this copy too
        NR_CHECK(hipEventRecord(ctx->evGatherDone[x], ctx->commStream));
        ctx->gatherPending[x] = true;
    }
    return x;
}

// NEW: wait until the DeliverFrameU8 with this ticket has landed on the host.
bool WaitFrameDelivered(RenderContext* ctx, i64 ticket) {
    if (ticket < 0 || ticket > 1 || !ctx->evDeliver[ticket]) return false;
    NR_CHECK(hipSetDevice(ctx->device));
    return hipEventSynchronize(ctx->evDeliver[ticket]) == hipSuccess;
}

// NEW (§8e, the ingress-free assembly): this rank's bands of the frame
// output (u8 image or YUV420P planes) copied from the GPU straight into their
// places in a host frame -- every rank of a sharded frame delivers into the
// same host frame (one process per GPU: a SharedHostBuffer, AllocSharedHostBuffer),
// so the frame is assembled in host memory by each GPU's own PCIe link and no
// GPU receives the others' bands (GatherFrameU8 + DeliverFrameU8 moves 7/8 of
// the frame into the root over xGMI and then all of it over the root's PCIe
// link).  Converts the owned bands first when the raster has not written them
// (as GatherFrameU8's first half), then one strided copy per plane segment and
// owned band slot of the pattern (3 per frame for equal shards of a YUV420P
// frame), on the gather stream, overlapped with the next frame as
// DeliverFrameU8.  Returns a ticket for WaitFrameDelivered, or -1.
// Band delivery copies: a rank owning at most BAND_KERNEL_MAX bytes of the frame
// output writes them with one kernel of BAND_WG workgroups into the host frame's
// device address; larger shares take one strided runtime copy per plane segment
// and owned slot of the pattern.  Measured with the copies beside the next frame
// (C3 YUV420P, bench.py --deliver bands, profiles/r05/ab_band_copy.txt): an 8-way
// share (1.55 MB) 0.0804 -> 0.0723 ms with the kernel (32 workgroups: 0.0733);
// a 2-way share (6.2 MB) 0.1617 with the strided copies against 0.1727.
constexpr i64 BAND_KERNEL_MAX = 3 << 20;
constexpr int BAND_WG = 8;
}  // extern "C"
namespace {
// This rank's bands of `frame` to the same offsets of the host frame (its
// device address): BAND_WG workgroups stride over every owned segment.
template <typename V>
__global__ __launch_bounds__(256) void k_bands_to_host(const iu8* __restrict__ frame, iu8* __restrict__ host,
                                                       FrameGeom g, ShardMap sm, int sel, i64 bands) {
    for (i64 b = 0; b < bands; ++b) {
        if (sm.pattern[b % sm.period] != sel) continue;
        i64 off[3], len[3];
        const int ns = band_segments(g, b, off, len);
        for (int k = 0; k < ns; ++k) {
            const V* src = reinterpret_cast<const V*>(frame + off[k]);
            V* dst = reinterpret_cast<V*>(host + off[k]);
            const i64 n = len[k] / (i64)sizeof(V);
            for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
                dst[i] = src[i];
        }
    }
}
}  // namespace
extern "C" {

i64 DeliverFrameBands(RenderContext* ctx, iu8* host) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (!host) {
        nr_set_error_msg("DeliverFrameBands: null host frame");
        return -1;
    }
    if (!frame_u8_local(ctx)) return -1;
    const int x = ctx->frameCur;
    iu8* const frame = ctx->frameBuf[x];
    if (!frame) {
        nr_set_error_msg("DeliverFrameBands: no frame output");
        return -1;
    }
    ensure_comm_stream(ctx);
    if (!ctx->evDeliver[x]) NR_CHECK(hipEventCreateWithFlags(&ctx->evDeliver[x], hipEventDisableTiming));
    NR_CHECK(hipEventRecord(ctx->evFrameReady, ctx->stream));
    NR_CHECK(hipStreamWaitEvent(ctx->commStream, ctx->evFrameReady, 0));
    const FrameGeom g = frame_geom(ctx);
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    const int P = ctx->shardPeriod;
    const i64 full = ctx->height / BAND;   // bands [0, full) have BAND rows; band `full` (if any) is short
    // The copy kernel writes through the host frame's device address, which
    // only pinned (hipHostMalloc'd / registered) memory has: for any other host
    // pointer (a numpy or malloc buffer) the runtime copies below take over
    // (the failed lookup used to leave a null address to write to).
    void* hdev = nullptr;
    bool viaKernel = owned_bytes(ctx, ctx->shard) <= BAND_KERNEL_MAX;
    if (viaKernel && (hipHostGetDevicePointer(&hdev, host, 0) != hipSuccess || !hdev)) {
        (void)hipGetLastError();   // (an answer: not pinned -- not a failure to latch)
        viaKernel = false;
    }
    if (viaKernel) {
        bool vec = (reinterpret_cast<uintptr_t>(hdev) | reinterpret_cast<uintptr_t>(frame)) % 16 == 0;
        for (i64 b = 0; b < bands && vec; ++b) {
            i64 off[3], len[3];
            const int ns = band_segments(g, b, off, len);
            for (int k = 0; k < ns; ++k) vec = vec && off[k] % 16 == 0 && len[k] % 16 == 0;
        }
        if (vec)
            hipLaunchKernelGGL(k_bands_to_host<uint4>, dim3(BAND_WG), dim3(256), 0, ctx->commStream, frame,
                               (iu8*)hdev, g, shard_map(ctx), ctx->shard, bands);
        else
            hipLaunchKernelGGL(k_bands_to_host<iu8>, dim3(BAND_WG), dim3(256), 0, ctx->commStream, frame,
                               (iu8*)hdev, g, shard_map(ctx), ctx->shard, bands);
        NR_CHECK(hipGetLastError());
    }
    for (int sl = 0; sl < P && sl < bands && !viaKernel; ++sl) {
        if (ctx->shardPattern[sl] != ctx->shard) continue;
        const i64 nb = sl < full ? (full - 1 - sl) / P + 1 : 0;   // full bands sl, sl + P, ...
        i64 off[3], len[3], offn[3], lenn[3];
        const int ns = band_segments(g, sl, off, len);
        band_segments(g, sl + P, offn, lenn);
        if (nb > 0)
            for (int k = 0; k < ns; ++k) {
                const size_t pitch = (size_t)(offn[k] - off[k]);   // the same segment one period on
                NR_CHECK(hipMemcpy2DAsync(host + off[k], pitch, frame + off[k], pitch, (size_t)len[k], (size_t)nb,
                                          hipMemcpyDeviceToHost, ctx->commStream));
            }
        if (full < bands && full % P == sl) {   // the frame's short last band
            const int nl = band_segments(g, full, off, len);
            for (int k = 0; k < nl; ++k)
                if (len[k] > 0)
                    NR_CHECK(hipMemcpyAsync(host + off[k], frame + off[k], (size_t)len[k], hipMemcpyDeviceToHost,
                                            ctx->commStream));
        }
    }
    NR_CHECK(hipEventRecord(ctx->evDeliver[x], ctx->commStream));
    rotate_frame(ctx, x);   // the next frame renders into the other buffer (this one after the copies)
    return x;
}

// NEW: pinned host memory shared between processes (POSIX shared memory
// `name`, "/..."; every process maps and registers the same bytes): the host
// frame the ranks' DeliverFrameBands assemble.  FreeSharedHostBuffer unmaps
// it in this process; UnlinkSharedHostBuffer removes the name (once, by the
// creator, after the others have mapped it or are done).
void* AllocSharedHostBuffer(const char* name, i64 bytes) {
    if (!name || name[0] != '/' || bytes <= 0) {
        nr_set_error_msg("AllocSharedHostBuffer: name must start with '/' and bytes be > 0");
        return nullptr;
    }
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        nr_set_error_msg("AllocSharedHostBuffer: shm_open failed");
        return nullptr;
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || (st.st_size < bytes && ftruncate(fd, (off_t)bytes) != 0)) {
        close(fd);
        nr_set_error_msg("AllocSharedHostBuffer: could not size the shared memory");
        return nullptr;
    }
    void* p = mmap(nullptr, (size_t)bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        nr_set_error_msg("AllocSharedHostBuffer: mmap failed");
        return nullptr;
    }
    // (mapped: DeliverFrameBands' copy kernel writes through its device address)
    if (hipHostRegister(p, (size_t)bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        munmap(p, (size_t)bytes);
        nr_set_error_msg("AllocSharedHostBuffer: hipHostRegister failed");
        return nullptr;
    }
    return p;
}

void FreeSharedHostBuffer(void* p, i64 bytes) {
    if (!p) return;
    NR_CHECK(hipHostUnregister(p));
    munmap(p, (size_t)bytes);
}

bool UnlinkSharedHostBuffer(const char* name) { return name && shm_unlink(name) == 0; }

// NEW: pinned (page-locked) host memory for DeliverFrameU8, and its release.
void* AllocHostBuffer(i64 bytes) {
    void* p = nullptr;
    if (bytes <= 0 || hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault) != hipSuccess) {
        nr_set_error_msg("AllocHostBuffer: hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

void FreeHostBuffer(void* p) {
    if (p) NR_CHECK(hipHostFree(p));
}

// NEW: device pointer of that frame (complete once Flush returns).
void* GetFrameU8DevicePtr(RenderContext* ctx) {
    return ctx->frameLast >= 0 ? ctx->frameBuf[ctx->frameLast] : ctx->frameU8;
}

// NEW: assemble the owned bands of the f64 framebuffer (and, with withDepth,
// of the u32 depth buffer) into the root's buffers — byte-exact N-GPU =
// 1-GPU.  Every rank must pass the same withDepth: the send/recv pairs of the
// group are posted from it alone, never from a rank's own allocation state
// (depth is allocated lazily, so ranks may differ there); a rank without a
// depth buffer allocates its cleared one (all 0xFFFFFFFF) first.
bool GatherFramebufferEx(RenderContext* ctx, NrComm* comm, i64 root, bool withDepth) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize(ctx);
    if (!comm || comm->nranks == 1) return true;
    if (comm->nranks != ctx->nshards || comm->rank != ctx->shard) {
        nr_set_error_msg("GatherFramebuffer: the context's shard must match the communicator");
        return false;
    }
    if (root < 0 || root >= comm->nranks) {
        nr_set_error_msg("GatherFramebuffer: root out of range");
        return false;
    }
    Rccl* r = rccl();
    if (!r) return false;
    if (withDepth) nr_ensure_depth(ctx);
    const int ipp = ctx->enableAlpha ? 4 : 3;
    const i64 rowElems = ctx->width * ipp;
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    bool ok = nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (i64 b = 0; b < bands && ok; ++b) {
        const int owner = ctx->shardPattern[b % ctx->shardPeriod];
        const i64 rows = std::min<i64>(BAND, ctx->height - b * BAND);
        f64* p = ctx->buffer + b * BAND * rowElems;
        u32* d = withDepth ? ctx->depth + b * BAND * ctx->width : nullptr;
        if (comm->rank == root && owner != root) {
            ok = nccl_ok(r, r->Recv(p, (size_t)(rows * rowElems), ncclFloat64, owner, comm->comm, ctx->stream), "ncclRecv");
            if (d && ok) ok = nccl_ok(r, r->Recv(d, (size_t)(rows * ctx->width), ncclUint32, owner, comm->comm, ctx->stream), "ncclRecv");
        } else if (comm->rank != root && owner == comm->rank) {
            ok = nccl_ok(r, r->Send(p, (size_t)(rows * rowElems), ncclFloat64, (int)root, comm->comm, ctx->stream), "ncclSend");
            if (d && ok) ok = nccl_ok(r, r->Send(d, (size_t)(rows * ctx->width), ncclUint32, (int)root, comm->comm, ctx->stream), "ncclSend");
        }
    }
    ok = nccl_ok(r, r->GroupEnd(), "ncclGroupEnd") && ok;
    return ok;
}

// NEW: GatherFramebufferEx with the depth bands always included.
bool GatherFramebuffer(RenderContext* ctx, NrComm* comm, i64 root) {
    return GatherFramebufferEx(ctx, comm, root, true);
}

}  // extern "C"

// Waits for the gather stream (Flush) / frees the frame-output state
// (DestroyRenderContext).
void nr_dist_sync(RenderContext* ctx) {
    if (ctx->commStream) NR_CHECK(hipStreamSynchronize(ctx->commStream));
}

void nr_dist_release(RenderContext* ctx) {
    nr_dist_sync(ctx);
    for (int x = 0; x < 2; ++x) {
        if (ctx->frameBuf[x]) NR_CHECK(hipFree(ctx->frameBuf[x]));
        if (ctx->stageBuf[x]) NR_CHECK(hipFree(ctx->stageBuf[x]));
        if (ctx->evGatherDone[x]) NR_CHECK(hipEventDestroy(ctx->evGatherDone[x]));
        if (ctx->evDeliver[x]) NR_CHECK(hipEventDestroy(ctx->evDeliver[x]));
        ctx->frameBuf[x] = ctx->stageBuf[x] = nullptr;
        ctx->evGatherDone[x] = ctx->evDeliver[x] = nullptr;
    }
    ctx->frameU8 = nullptr;
    if (ctx->yuvBuf) NR_CHECK(hipFree(ctx->yuvBuf));
    ctx->yuvBuf = nullptr;
    ctx->yuvCap = 0;
    if (ctx->evFrameReady) NR_CHECK(hipEventDestroy(ctx->evFrameReady));
    if (ctx->commStream) NR_CHECK(hipStreamDestroy(ctx->commStream));
    ctx->evFrameReady = nullptr;
    ctx->commStream = nullptr;
}

u64 nr_shard_mask(const RenderContext* ctx, int rank) {
    if (ctx->shardPeriod <= 1) return 1ull;
    u64 m = 0;
    for (int k = 0; k < ctx->shardPeriod; ++k)
        if (ctx->shardPattern[k] == rank) m |= 1ull << k;
    return m;
}
