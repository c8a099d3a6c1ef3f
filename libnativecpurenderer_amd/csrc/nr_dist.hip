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
    if (!comm || comm->nranks == 1) return true;
    if (comm->nranks != ctx->nshards || comm->rank != ctx->shard) {
        nr_set_error_msg("GatherFrameU8: the context's shard must match the communicator (SetShard(nranks, rank))");
        return false;
    }
    Rccl* r = rccl();
    if (!r) return false;
    hipEvent_t e0, e1;
    nr_timing_begin(ctx, NRK_GATHER, &e0, &e1);
    bool ok = nccl_ok(r, r->GroupStart(), "ncclGroupStart");
    for (i64 b = 0; b < bands && ok; ++b) {
        const int owner = (int)(b % comm->nranks);
        const i64 rows = std::min<i64>(BAND, ctx->height - b * BAND);
        iu8* p = ctx->frameU8 + b * BAND * rowElems;
        const size_t cnt = (size_t)(rows * rowElems);
        if (comm->rank == root && owner != root)
            ok = nccl_ok(r, r->Recv(p, cnt, ncclUint8, owner, comm->comm, ctx->stream), "ncclRecv");
        else if (comm->rank != root && owner == comm->rank)
            ok = nccl_ok(r, r->Send(p, cnt, ncclUint8, (int)root, comm->comm, ctx->stream), "ncclSend");
    }
    ok = nccl_ok(r, r->GroupEnd(), "ncclGroupEnd") && ok;
    nr_timing_end(ctx, NRK_GATHER, e0, e1);
    return ok;
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
