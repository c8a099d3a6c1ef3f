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

// f64 -> u8 (cpp:52-57) over the owned tile rows only
__global__ void k_to_u8_rows(const f64* __restrict__ src, iu8* __restrict__ dst, i64 rowElems, i64 H, int TH,
                             int nshards, int shard) {
    const i64 band = (i64)blockIdx.y * nshards + shard;   // owned band index
    const i64 r0 = band * TH;
    if (r0 >= H) return;
    const i64 rows = (H - r0) < TH ? (H - r0) : TH;
    const i64 n = rows * rowElems;
    const i64 base = r0 * rowElems;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        dst[base + i] = nr_to_u8(src[base + i]);
}

constexpr int BAND = 32;   // = nrtri::TH, the tile height

// Rows of the frame owned by `rank` of n (bands b with b % n == rank).
i64 owned_rows(i64 H, int n, int rank) {
    i64 rows = 0;
    for (i64 b = rank; b * BAND < H; b += n) rows += std::min<i64>(BAND, H - b * BAND);
    return rows;
}

// Packed band layout of the gather: a rank's owned bands back to back (its
// k-th band at k * BAND rows; only the frame's last band can be short, and it
// is the last of its owner).  Pack (!UNPACK): the bands of `sel` from the
// frame into `stage`.  Unpack: the bands of every rank but `root` from its
// slot of `stage` (rank p at p * peerStride) into the frame.
template <typename V, bool UNPACK>
__global__ void k_band_copy(iu8* __restrict__ frame, iu8* __restrict__ stage, i64 rowElems, i64 H, int nranks,
                            int sel, i64 peerStride) {
    const i64 b = blockIdx.y;
    const int owner = (int)(b % nranks);
    if (UNPACK ? owner == sel : owner != sel) return;
    const i64 r0 = b * BAND;
    const i64 rows = (H - r0) < BAND ? (H - r0) : BAND;
    const i64 n = rows * rowElems / (i64)sizeof(V);
    V* f = reinterpret_cast<V*>(frame + r0 * rowElems);
    V* s = reinterpret_cast<V*>(stage + (UNPACK ? owner * peerStride : 0) + (b / nranks) * BAND * rowElems);
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        if (UNPACK) f[i] = s[i];
        else s[i] = f[i];
    }
}

// Launches k_band_copy over every band (16-byte vectors when the row length
// keeps every band 16-byte aligned).
void band_copy(RenderContext* ctx, bool unpack, int nranks, int sel, i64 peerStride, i64 rowElems) {
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    const bool vec = rowElems % 16 == 0;
    const i64 per = BAND * rowElems / (vec ? 16 : 1);
    dim3 grid((unsigned)std::min<i64>((per + 255) / 256, 1024), (unsigned)bands);
    if (vec) {
        if (unpack) hipLaunchKernelGGL((k_band_copy<uint4, true>), grid, dim3(256), 0, ctx->stream, ctx->frameU8,
                                       ctx->frameStage, rowElems, ctx->height, nranks, sel, peerStride);
        else hipLaunchKernelGGL((k_band_copy<uint4, false>), grid, dim3(256), 0, ctx->stream, ctx->frameU8,
                                ctx->frameStage, rowElems, ctx->height, nranks, sel, peerStride);
    } else {
        if (unpack) hipLaunchKernelGGL((k_band_copy<iu8, true>), grid, dim3(256), 0, ctx->stream, ctx->frameU8,
                                       ctx->frameStage, rowElems, ctx->height, nranks, sel, peerStride);
        else hipLaunchKernelGGL((k_band_copy<iu8, false>), grid, dim3(256), 0, ctx->stream, ctx->frameU8,
                                ctx->frameStage, rowElems, ctx->height, nranks, sel, peerStride);
    }
    NR_CHECK(hipGetLastError());
}

// Staging of the packed gather: a non-root rank's own bands, or on the root
// one slot of the largest share per rank.
bool ensure_stage(RenderContext* ctx, size_t need) {
    if (need <= ctx->frameStageCap) return true;
    if (ctx->frameStage) NR_CHECK(hipFree(ctx->frameStage));
    ctx->frameStage = nullptr;
    ctx->frameStageCap = 0;
    if (hipMalloc((void**)&ctx->frameStage, need) != hipSuccess) {
        nr_set_error_msg("GatherFrameU8: hipMalloc of the staging buffer failed");
        return false;
    }
    ctx->frameStageCap = need;
    return true;
}

// The u8 image of the owned bands (the first half of GatherFrameU8), converted
// only when the mirror the resolves write is not current.
bool frame_u8_local(RenderContext* ctx) {
    nr_materialize_color(ctx);
    const int ipp = ctx->enableAlpha ? 4 : 3;
    const i64 n = ctx->width * ctx->height * ipp;
    if (n <= 0) return true;
    if ((size_t)n > ctx->frameU8cap) {
        if (ctx->frameU8) NR_CHECK(hipFree(ctx->frameU8));
        ctx->frameU8 = nullptr;
        if (hipMalloc((void**)&ctx->frameU8, (size_t)n) != hipSuccess) {
            nr_set_error_msg("GatherFrameU8: hipMalloc failed");
            ctx->frameU8cap = 0;
            return false;
        }
        ctx->frameU8cap = (size_t)n;
    }
    const i64 rowElems = ctx->width * ipp;
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    const i64 owned = (bands - ctx->shard + ctx->nshards - 1) / ctx->nshards;
    // later triangle resolves write the u8 frame themselves (no re-read of
    // the f64 frame); convert here only when that mirror is not current
    ctx->frameOutput = true;
    if (owned > 0 && !ctx->frameU8Valid) {
        dim3 grid((unsigned)std::min<i64>((BAND * rowElems + 255) / 256, 4096), (unsigned)owned);
        hipEvent_t e0, e1;
        nr_timing_begin(ctx, NRK_OUTPUT, &e0, &e1);
        hipLaunchKernelGGL(k_to_u8_rows, grid, dim3(256), 0, ctx->stream, ctx->buffer, ctx->frameU8, rowElems,
                           ctx->height, BAND, ctx->nshards, ctx->shard);
        NR_CHECK(hipGetLastError());
        nr_timing_end(ctx, NRK_OUTPUT, e0, e1);
    }
    ctx->frameU8Valid = true;
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
    ctx->nshards = (int)nshards;
    ctx->shard = (int)shard;
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
    // one message per rank: every non-root rank packs its bands back to back
    // and sends them; the root receives each rank's pack into its own slot
    // and scatters all of them into place with one kernel (a send/recv per
    // band would cost RCCL's per-operation latency ~H/32 times on the root)
    const int n = comm->nranks, me = comm->rank;
    const i64 rowElems = ctx->width * (ctx->enableAlpha ? 4 : 3);
    const i64 maxRows = owned_rows(ctx->height, n, 0);   // rank 0 owns the most bands
    const i64 peerStride = maxRows * rowElems;
    if (!ensure_stage(ctx, (size_t)(me == root ? n * peerStride : owned_rows(ctx->height, n, me) * rowElems)))
        return false;
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_GATHER, &e0, &e1);
    if (me != root) band_copy(ctx, false, n, me, 0, rowElems);
    bool ok = nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (int p = 0; p < n && ok; ++p) {
        const size_t cnt = (size_t)(owned_rows(ctx->height, n, p) * rowElems);
        if (cnt == 0) continue;
        if (me == root && p != root)
            ok = nccl_ok(r, r->Recv(ctx->frameStage + p * peerStride, cnt, ncclUint8, p, comm->comm, ctx->stream),
                         "ncclRecv");
        else if (me != root && p == me)
            ok = nccl_ok(r, r->Send(ctx->frameStage, cnt, ncclUint8, (int)root, comm->comm, ctx->stream), "ncclSend");
    }
    ok = nccl_ok(r, r->GroupEnd(), "ncclGroupEnd") && ok;
    if (ok && me == root) band_copy(ctx, true, n, (int)root, peerStride, rowElems);
    nr_timing_end(ctx, NRK_GATHER, e0, e1);
    return ok;
}

// NEW (testing): the packed gather of GatherFrameU8 for n contexts of ONE
// process (ctxs[p] renders shard p of n), with device copies in place of the
// RCCL send/recv -- the same pack, slot layout and unpack kernels, so the
// multi-GPU assembly is checked on a single GPU.
bool GatherFrameU8Local(RenderContext** ctxs, i64 n, i64 root) {
    if (n < 1 || root < 0 || root >= n) {
        nr_set_error_msg("GatherFrameU8Local: need 0 <= root < n");
        return false;
    }
    RenderContext* rc = ctxs[root];
    for (i64 p = 0; p < n; ++p) {
        RenderContext* c = ctxs[p];
        if (c->nshards != n || c->shard != p || c->width != rc->width || c->height != rc->height ||
            c->enableAlpha != rc->enableAlpha) {
            nr_set_error_msg("GatherFrameU8Local: ctxs[p] must be shard p of n, all of one size");
            return false;
        }
        NR_CHECK(hipSetDevice(c->device));
        if (!frame_u8_local(c)) return false;
    }
    if (n == 1) return true;
    const i64 rowElems = rc->width * (rc->enableAlpha ? 4 : 3);
    const i64 peerStride = owned_rows(rc->height, (int)n, 0) * rowElems;
    NR_CHECK(hipSetDevice(rc->device));
    if (!ensure_stage(rc, (size_t)(n * peerStride))) return false;
    for (i64 p = 0; p < n; ++p) {
        if (p == root) continue;
        RenderContext* c = ctxs[p];
        NR_CHECK(hipSetDevice(c->device));
        const size_t cnt = (size_t)(owned_rows(c->height, (int)n, (int)p) * rowElems);
        if (!ensure_stage(c, cnt)) return false;
        band_copy(c, false, (int)n, (int)p, 0, rowElems);
        NR_CHECK(hipStreamSynchronize(c->stream));
        // on the root's (non-blocking) stream, so the unpack is ordered after it
        NR_CHECK(hipMemcpyAsync(rc->frameStage + p * peerStride, c->frameStage, cnt, hipMemcpyDefault, rc->stream));
    }
    NR_CHECK(hipSetDevice(rc->device));
    band_copy(rc, true, (int)n, (int)root, peerStride, rowElems);
    NR_CHECK(hipStreamSynchronize(rc->stream));
    return true;
}

// NEW: copy the assembled u8 frame to the host (valid on the root).
void GetFrameU8(RenderContext* ctx, iu8* out) {
    NR_CHECK(hipSetDevice(ctx->device));
    if (!ctx->frameU8) return;
    NR_CHECK(hipMemcpyAsync(out, ctx->frameU8, (size_t)(ctx->width * ctx->height * (ctx->enableAlpha ? 4 : 3)),
                            hipMemcpyDeviceToHost, ctx->stream));
    NR_CHECK(hipStreamSynchronize(ctx->stream));
}

void* GetFrameU8DevicePtr(RenderContext* ctx) { return ctx->frameU8; }

// NEW: assemble the owned bands of the f64 framebuffer (and of the depth
// buffer, when allocated) into the root's buffers — byte-exact N-GPU = 1-GPU.
bool GatherFramebuffer(RenderContext* ctx, NrComm* comm, i64 root) {
    NR_CHECK(hipSetDevice(ctx->device));
    nr_materialize(ctx);
    if (!comm || comm->nranks == 1) return true;
    if (comm->nranks != ctx->nshards || comm->rank != ctx->shard) {
        nr_set_error_msg("GatherFramebuffer: the context's shard must match the communicator");
        return false;
    }
    Rccl* r = rccl();
    if (!r) return false;
    const int ipp = ctx->enableAlpha ? 4 : 3;
    const i64 rowElems = ctx->width * ipp;
    const i64 bands = (ctx->height + BAND - 1) / BAND;
    bool ok = nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (i64 b = 0; b < bands && ok; ++b) {
        const int owner = (int)(b % comm->nranks);
        const i64 rows = std::min<i64>(BAND, ctx->height - b * BAND);
        f64* p = ctx->buffer + b * BAND * rowElems;
        u32* d = ctx->depth ? ctx->depth + b * BAND * ctx->width : nullptr;
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

}  // extern "C"
