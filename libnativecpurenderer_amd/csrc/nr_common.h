// nr_common.h — shared types and device helpers of the MI355X raster library.
//
// Every device helper restates one reference routine bit for bit
// (/root/reference/src/libNativeCPURenderer.cpp:<lines> cited per helper).
// The whole library is compiled with -ffp-contract=off: the reference build
// has no FMA, so neither may we.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <vector>
#include <climits>

typedef long i64;
typedef double f64;
typedef unsigned char iu8;
typedef uint32_t u32;

// ---------------------------------------------------------------------------
// error latch (no exceptions cross the ABI; SURVEY §8b "Errors")
// ---------------------------------------------------------------------------
void nr_set_error(const char* where, hipError_t e);
void nr_set_error_msg(const char* msg);
#define NR_CHECK(call)                                              \
    do {                                                            \
        hipError_t nr_e_ = (call);                                  \
        if (nr_e_ != hipSuccess) nr_set_error(#call, nr_e_);        \
    } while (0)

// ---------------------------------------------------------------------------
// host objects
// ---------------------------------------------------------------------------
struct NRState { f64 m[6]; f64 ct[4]; };
typedef unsigned long long u64;

// Binning geometry of a draw: the positions' transform, the frame and the
// owned tile rows.  The same buffer binned under the same key gives the same
// (tile, triangle) pairs, work items and dense tiles.
struct BinKey {
    f64 m[6];
    i64 W, H;
    int period;
    u64 mask;
};

// Scratch of the triangle pipeline, grown on demand (never shrunk).
struct TriScratch {
    u64* cnt = nullptr; u64* off = nullptr; size_t tri_cap = 0;          // per triangle
    f64* orec = nullptr; size_t orec_cap = 0;   // ordered raster: per-triangle setup records (ORec doubles each)
    u32* keys[2] = {nullptr, nullptr}; u32* vals[2] = {nullptr, nullptr}; size_t pair_cap = 0;
    u32* tile_start = nullptr; u32* tile_end = nullptr; size_t tile_cap = 0;
    void* temp = nullptr; size_t temp_bytes = 0;                        // hipcub scratch
    u64* h_total = nullptr;                 // pinned readback: [0] pairs, [1] last count, [2] fragments
    u64* d_frag = nullptr;                  // device fragment counter
    u32* d_flag = nullptr;                  // device non-opaque flag
    // visibility-buffer raster (nr_tri_free.hip).  The binning outputs are
    // double-buffered (FreeSet): a batch drawn from a TriangleBuffer is binned
    // on the device's binning stream while the previous batch's k_vis runs.
    struct FreeSet {
        u32* fcnt = nullptr; u32* foff = nullptr; u32* fcur = nullptr; size_t ftile_cap = 0;
        uint4* fitems = nullptr; size_t fitems_cap = 0;
        u64* frect = nullptr; size_t frect_cap = 0;   // per-triangle tile rectangle (count -> emit)
        f64* frec = nullptr; size_t frec_cap = 0;     // ordered batches: per-triangle setup records (ORec doubles each)
        u32* flist = nullptr; size_t flist_cap = 0;
        u32* dplan = nullptr;
        u64* h_plan = nullptr;              // pinned, device-mapped copy of the plan totals, (seq << 32) | value
        u64* d_hplan = nullptr;             // its device address
        hipEvent_t evBin = nullptr;         // binning done (binning stream)
        hipEvent_t evVis = nullptr;         // k_vis done reading the set (main stream)
        bool visRecorded = false;
        u64 curGen = 0;                     // fcur = curEpoch x the counts of schedule curGen (0: unknown)
        u32 curEpoch = 0;
        // warm binning beside the raster: same-queue hand-off (k_gate_signal / k_gate_wait)
        u32* gate = nullptr;                // [0] token of the set's last finished binning
        u32* gplan = nullptr;               // the raster's plan words (k_gate_wait copies the schedule's)
        u32 gateTok = 0;
    } fset[3];
    int fnext = 0;                          // set of the next batch
    u32* fdone = nullptr; size_t fdone_cap = 0;   // split-tile slice counters (k_vis only)
    u64* kslot = nullptr; size_t kslot_cap = 0;   // split-tile key slots, TH*TW keys per slice (k_vis)
    u32 lastSplit = 0;                      // split-tile slices of the last validated batch (slot estimate)
    u32 planSeq = 0;                        // sequence number of the last async plan
    u64 lastPairs = 0;                      // capacity estimate for the next batch
    u32 lastItems = 0;                      // k_vis work items of the last validated batch (grid estimate)
    u32 lastHeavy = 0;                      // dense tiles of the last batch (k_vis workgroup size)
    u64 lastN = 0;                          // its triangle count (k_vis variant choice)
    u64 capOverride = 0;                    // testing: force this pair capacity
    int coopMode = 0;                       // k_vis variant: 0 auto, 1 coop, 2 lane-only (SetCoopRaster)
    u32 splitAt = 0, dslice = 0;            // dense-tile split limits (SetSplitLimits; 0: NR_SPLIT_AT / NR_DSLICE)
    f64* stage = nullptr; size_t stage_cap = 0;   // DrawTriangles() with host arrays
    // warm binning (nr_tri_free.hip): the tile offsets, k_vis work items and
    // plan totals of the last validated binning of one TriangleBuffer under
    // one binning key -- a later draw of the same buffer under the same key
    // has the same (tile, triangle) pairs, so it bins in one pass into these
    // ranges (no count pass, no plan, no validation)
    struct Schedule {
        bool valid = false;
        u64 tbUid = 0;
        BinKey key;
        u32* off = nullptr; size_t off_cap = 0;          // ntiles + 1 list offsets
        uint4* items = nullptr; size_t items_cap = 0;    // k_vis work items
        u32* dplan = nullptr;                            // the plan's device totals {pairs, items, slices, fits}
        u32 pairs = 0, nitems = 0, heavy = 0, split = 0;
        u64 n = 0;
        u64 gen = 0;                                     // process-unique generation of this schedule
        hipEvent_t ready = nullptr;                      // the copies above are done (main stream)
        bool waitReady = false;                          // the next warm binning on the binning stream waits for it
        // the binning blocks (1024 triangles) with a cluster that may reach an
        // owned tile under this key: the warm binning launches only those
        u32* blocks = nullptr; size_t blocks_cap = 0;
        std::vector<u32> hblocks;                        // (host source of the last upload, kept alive)
        u32 nblocks = 0;
        u64 blocksGen = 0;                               // gen the list was built for (0: none)
        bool anyCull = true;                             // some cluster may lie off the owned tiles (else no device test)
        // loose ranges (round 6): every tile's range widened to loose_cap(count)
        // pairs, for a draw of the same buffer under a transform that moves no
        // vertex more than LOOSE_PX from the key's (a moving scene: k_bin_warm
        // into these ranges, k_vis slices each tile's actual count)
        u32* off2 = nullptr; size_t off2_cap = 0;        // ntiles + 1 loose list offsets
        u64 off2Gen = 0;                                 // gen they were formed for (0: none)
        u64 pairs2 = 0;                                  // a bound of off2[ntiles] (list capacity)
    } sched;
    int warmMode = 0;                       // 0 automatic (NR_WARM), 1 on, 2 off (SetWarmBinning)
    u64 warmBatches = 0;                    // batches binned warm (GetWarmBatchCount)
    u64 looseBatches = 0;                   // of those, into the loose ranges (GetLooseBatchCount)
    std::vector<u64> looseBanned;           // buffers whose loose binning overflowed a tile: not binned loose again
    // warm-batch checks (k_vis WarmCheck): host-mapped word a raster sets when
    // a warm batch failed them (1 binning check, 2 token timeout), read by
    // nr_settle; the batch itself was rasterised from all its triangles
    u32* hfail = nullptr; u32* dfail = nullptr;   // [0] reason, [1..3] the words it read (the message)
    u32 warmTag = 0;                        // tag of the last warm batch (k_bin_warm's error word)
    u64 warmFailures = 0;                   // warm batches that failed their checks (GetWarmFailureCount)
    std::vector<u64> warmBanned;            // buffers (uid) whose warm binning failed a check: binned cold
    int warmInject = 0;                     // testing: fault injected into the next warm batch (SetWarmFaultInjection)
    // a warm binning beside the raster was handed off by its token only (no
    // event the main stream waits on): before the main stream next writes a
    // binning set or the schedule, it waits for the binning stream (evSide)
    bool sideGated = false;
    hipEvent_t evSide = nullptr;
};

enum NRKernelId { NRK_TRI_COUNT = 0, NRK_TRI_SCAN, NRK_TRI_EMIT, NRK_TRI_SORT, NRK_TILE_RANGES,
                  NRK_TILE_RASTER, NRK_PRIM, NRK_FILL, NRK_RESOLVE, NRK_VIS_INIT, NRK_OUTPUT, NRK_GATHER,
                  NRK_COUNT_ };

struct RenderContext {
    i64 width = 0, height = 0;
    bool enableAlpha = false;
    f64* buffer = nullptr;            // device, row-major interleaved, W*H*ipp (cpp:3-5)
    f64 m[6] = {1, 0, 0, 1, 0, 0};    // transformMatrix (h:39)
    f64 ct[4] = {1, 1, 1, 1};         // colorTransform (h:40)
    std::vector<NRState> stack;       // stateStack (h:41)
    int device = 0;
    hipStream_t stream = nullptr;
    // depth (new)
    u32* depth = nullptr;
    bool depthTest = false, depthWrite = false;
    // deferred clears: a uniform SetColor / ClearDepth is kept pending and
    // consumed on chip by the tiled raster, or materialised before any
    // other operation that touches the buffer.
    bool pendColor = false; f64 pendColorValue = 0;
    bool pendDepth = false; u32 pendDepthValue = 0xFFFFFFFFu;
    // tile-granular pending clears (a fast clear): an order-free batch that
    // consumed a pending clear leaves the tiles no triangle touched holding it
    // in name only -- their framebuffer / depth pixels are not written; tile t
    // is such a tile while tileStamp[t] == tileEpoch (written by k_vis).  Any
    // later use of the buffers writes them first (nr_materialize_tiles), a new
    // clear of the same buffer drops them.
    bool tileColor = false; f64 tileColorValue = 0;
    bool tileDepth = false; u32 tileDepthValue = 0xFFFFFFFFu;
    u32* tileStamp = nullptr; i64 tileStampCap = 0; u32 tileEpoch = 0;
    TriScratch tri;
    // per-kernel HIP-event timing (bench.py's live roofline measurement)
    bool timing = false;
    unsigned long long timingMask = ~0ull;   // which NRKernelId are timed
    std::vector<hipEvent_t> evPool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> evPending;
    u64* tsDev = nullptr;                    // device-clock stamp pairs of timed raster launches
    std::vector<std::pair<int, int>> tsPending;   // (kernel id, pair index)
    f64 kTimeMs[NRK_COUNT_] = {0};
    i64 kCount[NRK_COUNT_] = {0};
    // covered-fragment counting (the work count of the Mpixels/s metric)
    bool countFragments = false;
    bool fragPending = false;
    u64 fragTotal = 0;
    int lastPath = 0;                 // raster of the last triangle batch (1 order-free, 2 ordered)
    int forceOrdered = 0;             // testing: always take the ordered raster
    iu8* u8buf = nullptr; size_t u8cap = 0;   // GetBufferAsUInt8 staging
    // multi-GPU: owned tile rows ty % nshards == shard (nr_dist.hip)
    int nshards = 1, shard = 0;
    // band ownership: band b belongs to rank shardPattern[b % shardPeriod]
    // (SetShard: period nshards, pattern 0..n-1; SetShardSlots: a weighted
    // interleave); every rank of a frame holds the same pattern
    int shardPeriod = 1;
    unsigned char shardPattern[64] = {0};
    // u8 frame output (GatherFrameU8, nr_dist.hip): two frame buffers, the
    // next frame renders into one while the other is assembled on the gather
    // stream; frameU8 = frameBuf[frameCur]
    iu8* frameU8 = nullptr; size_t frameU8cap = 0;
    iu8* frameBuf[2] = {nullptr, nullptr};
    int frameCur = 0, frameLast = -1;            // buffer being rendered / of the last GatherFrameU8
    iu8* stageBuf[2] = {nullptr, nullptr}; size_t stageCap[2] = {0, 0};   // packed bands per buffer
    iu8* yuvBuf = nullptr; size_t yuvCap = 0;    // GetFrameYUV420P planes (device)
    hipStream_t commStream = nullptr;            // RCCL transfers + the root's unpack
    hipEvent_t evFrameReady = nullptr, evGatherDone[2] = {nullptr, nullptr};
    hipEvent_t evDeliver[2] = {nullptr, nullptr};   // DeliverFrameU8: D2H of frame buffer x done
    bool gatherPending[2] = {false, false};
    bool frameOutput = false;   // set by GatherFrameU8: resolves also write the u8 frame
    bool frameU8Valid = false;  // frameU8 holds the u8 image of every owned pixel
    // frame output format (SetFrameFormat): 0 = the u8 image (cpp:52-57,
    // W*H*ipp bytes), 1 = its YUV420P planes (Y W*H, U and V (W/2)*(H/2);
    // W and H even), the encoder input of PutRendererContextFrame
    int frameFormat = 0;
    void* pendingBatch = nullptr;   // last visibility batch awaiting validation (nr_settle)
    // deferred command list (BeginCommandList / EndCommandList, nr_prims.hip):
    // while recording, primitive draws are queued and run together, in
    // order, by one launch (every pixel read and written once)
    bool recording = false;
    void* cmdList = nullptr;
};

struct Texture {
    i64 width = 0, height = 0;
    bool enableAlpha = false;
    f64* buffer = nullptr;            // device
    bool owns = true;                 // false: alias of a context framebuffer (cpp:377-384)
    RenderContext* aliasOf = nullptr;
    int device = 0;
};

struct TriangleBuffer {
    i64 n = 0;
    bool gouraud = false;
    f64* xy = nullptr;    // n*6   (x0,y0,x1,y1,x2,y2)
    f64* z = nullptr;     // n*3 or null
    f64* rgba = nullptr;  // n*4 (flat) or n*12 (Gouraud)
    bool opaque = false;  // every vertex alpha == 1 (known at upload)
    int device = 0;
    // totals of the last validated binning of this buffer (nr_tri_free.hip):
    // a draw under the same key is sized from them and needs no validation
    bool known = false;
    BinKey knownKey;
    u32 knownPairs = 0, knownHeavy = 0, knownItems = 0, knownSplit = 0;
    u64 uid = 0;          // process-unique id (a context's warm schedule names its buffer by it)
    // per cluster of CLUSTER consecutive triangles (one wave of the binning
    // kernels): its user-space bounding box {xmin, ymin, xmax, ymax} (NaN when
    // a vertex is not finite: never culled), computed at upload -- the warm
    // binning of a sharded frame skips the clusters that lie outside the
    // rank's tile rows without loading their triangles
    f64* cbox = nullptr;
    std::vector<f64> hcbox;   // (host copy: the warm schedule's active binning blocks are found on the host)
    // user-space bounding box of every vertex {xmin, ymin, xmax, ymax} (NaN: a
    // vertex is not finite): bounds how far a change of transform moves any
    // vertex on screen (loose binning, nr_tri_free.hip)
    f64 bbox[4] = {NAN, NAN, NAN, NAN};
};
constexpr int NR_CLUSTER = 64;

// host helpers shared across translation units
Texture* nr_new_texture(i64 w, i64 h, bool alpha);   // device texels, current device
void nr_dist_sync(RenderContext* ctx);      // wait for the frame-assembly stream
u64 nr_shard_mask(const RenderContext* ctx, int rank);   // bit k: pattern slot k belongs to rank
void nr_dist_release(RenderContext* ctx);   // free the frame-output buffers
hipStream_t nr_stream_for(int device);
hipStream_t nr_bin_stream_for(int device);        // second stream: triangle binning overlapped with the raster
void nr_timing_begin_on(RenderContext* ctx, int kid, hipEvent_t* a, hipEvent_t* b, hipStream_t s);
void nr_timing_end_on(RenderContext* ctx, int kid, hipEvent_t a, hipEvent_t b, hipStream_t s);
void nr_materialize(RenderContext* ctx);          // flush pending clears
void nr_materialize_color(RenderContext* ctx);
void nr_materialize_depth(RenderContext* ctx);
void nr_materialize_tiles(RenderContext* ctx, bool color, bool depth);   // tile-granular pending clears
void nr_ensure_depth(RenderContext* ctx);
void nr_timing_begin(RenderContext* ctx, int kid, hipEvent_t* a, hipEvent_t* b);
// The rasters time themselves on the device clock (FrameParams::tstamp,
// raster_stamp_begin / _end): a zeroed {start, end} pair for one timed launch,
// or null when not timed.  (Events bound to the launch, hipExtLaunchKernel
// start/stop, measured the launch gap too: profiles/r06/ab_event_every.txt.)
u64* nr_timing_stamp(RenderContext* ctx, int kid);
void nr_timing_end(RenderContext* ctx, int kid, hipEvent_t a, hipEvent_t b);
void nr_fill_f64(hipStream_t s, f64* p, i64 n, f64 v);
void nr_fill_u32(hipStream_t s, u32* p, i64 n, u32 v);
void nr_settle(RenderContext* ctx);               // validate an asynchronously sized batch, run queued commands
void nr_settle_all();                             // ... of every live context
void nr_flush_commands(RenderContext* ctx);       // run the recorded primitive draws (nr_prims.hip)
void nr_drop_commands(RenderContext* ctx);        // discard them (the whole buffer is overwritten next)
void nr_free_commands(RenderContext* ctx);        // discard and release the list storage
bool nr_record_fill(RenderContext* ctx, i64 i0, i64 i1, i64 j0, i64 j1, f64 r, f64 g, f64 b, f64 a);  // ApplyPixel over a range
bool nr_record_set_pixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a);

// x86-64 cvttsd2si semantics for (i64)double: out of range / NaN -> INT64_MIN
static inline i64 nr_f2i64(f64 v) {
    if (!(v >= -9223372036854775808.0 && v < 9223372036854775808.0)) return LONG_MIN;
    return (i64)v;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
// cpp:446-453, expression order kept: (m0*x + m2*y) + m4
__host__ __device__ __forceinline__ void nr_xform(const f64* m, f64 x, f64 y, f64& ox, f64& oy) {
    ox = m[0] * x + m[2] * y + m[4];
    oy = m[1] * x + m[3] * y + m[5];
}

// cpp:515-549 body on an already-located pixel: colour transform, then "over"
// unless a == 1; RGBA stores dst.a = a.
__device__ __forceinline__ void nr_apply_pixel(f64* p, int ipp, f64 r, f64 g, f64 b, f64 a,
                                               f64 ct0, f64 ct1, f64 ct2, f64 ct3) {
    r *= ct0; g *= ct1; b *= ct2; a *= ct3;
    if (a != 1) {
        r = p[0] * (1 - a) + r * a;
        g = p[1] * (1 - a) + g * a;
        b = p[2] * (1 - a) + b * a;
    }
    p[0] = r; p[1] = g; p[2] = b;
    if (ipp == 4) p[3] = a;
}

// cpp:555-573 nearest-texel sampler (clamp to [0,w-2]x[0,h-2]); alpha of an RGB
// texture is uninitialised in the reference (Appendix A.2) and defined as 1.
__device__ __forceinline__ void nr_sample(const f64* tb, i64 tw, i64 th, bool talpha, f64 x, f64 y,
                                          f64& r, f64& g, f64& b, f64& a) {
    if (x < 0) x = 0;
    if (x >= (f64)(tw - 1)) x = (f64)(tw - 2);
    if (y < 0) y = 0;
    if (y >= (f64)(th - 1)) y = (f64)(th - 2);
    i64 ipp = talpha ? 4 : 3;
    i64 index = (i64)y * tw * ipp + (i64)x * ipp;
    if (index < 0) index = 0;   // 1-px-wide textures read index -1 in the reference (UB)
    r = tb[index + 0];
    g = tb[index + 1];
    b = tb[index + 2];
    a = talpha ? tb[index + 3] : 1.0;
}

// cpp:822-845 even-odd crossing test
template <int N>
__device__ __forceinline__ bool nr_point_in_polygon(f64 x, f64 y, const f64 (&pts)[N][2]) {
    int j = N - 1;
    bool res = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if ((pts[i][1] > y) != (pts[j][1] > y) &&
            (x < (pts[j][0] - pts[i][0]) * (y - pts[i][1]) / (pts[j][1] - pts[i][1]) + pts[i][0]))
            res = !res;
        j = i;
    }
    return res;
}

// depth quantisation (new)
__host__ __device__ __forceinline__ u32 nr_quantize_depth(f64 z) {
    if (!(z > 0.0)) return 0u;
    if (z >= 1.0) return 0xFFFFFFFFu;
    return (u32)(z * 4294967295.0);
}

// The same function without branches: clamping the product to
// [0, 4294967295] maps z <= 0 (and NaN: fmax drops it) to 0 and z >= 1 (and
// +inf) to 0xFFFFFFFF, and leaves every in-range product (hence its
// truncation) unchanged.
__device__ __forceinline__ u32 nr_quantize_depth_bl(f64 z) {
    return (u32)fmin(fmax(z * 4294967295.0, 0.0), 4294967295.0);
}

// The same function in one conversion: gfx950's v_cvt_u32_f64 truncates and
// saturates (negative and -inf to 0, >= 2^32 and +inf to 0xFFFFFFFF, NaN to
// 0), which is exactly the clamp above -- two f64 VALU operations fewer per
// fragment.  (In C++ an out-of-range cast is undefined, hence the asm.)
// Pinned against nr_quantize_depth on NaN, infinities, huge and boundary
// values by tests/test_depth_edges_gpu.py.
__device__ __forceinline__ u32 nr_quantize_depth_hw(f64 z) {
    const f64 p = z * 4294967295.0;
    u32 r;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(p));
    return r;
}

// Bytes of the context's frame output (frameFormat: u8 image or YUV420P).
static inline i64 nr_frame_bytes(const RenderContext* ctx) {
    const i64 W = ctx->width, H = ctx->height;
    return ctx->frameFormat == 1 ? W * H + 2 * (W / 2) * (H / 2) : W * H * (ctx->enableAlpha ? 4 : 3);
}

// YUV420P of the u8 image (GetFrameYUV420P, SetFrameFormat): swscale's
// unscaled RGB -> YV12 arithmetic (rgb2rgb rgb24toyv12): BT.601 limited
// range, 15-bit coefficients (0.299/0.587/0.114 x 219/255, chroma x 224/255,
// rounded), arithmetic shift, + 16 / 128; chroma point-sampled at the even
// pixel of each 2x2 block.  Parity unpinned (FFmpeg absent).
constexpr int NR_YRY = 8414, NR_YGY = 16519, NR_YBY = 3208;
constexpr int NR_YRU = -4864, NR_YGU = -9527, NR_YBU = 14392;
constexpr int NR_YRV = 14392, NR_YGV = -12060, NR_YBV = -2331;
__host__ __device__ __forceinline__ iu8 nr_y_of(int r, int g, int b) {
    return (iu8)(((NR_YRY * r + NR_YGY * g + NR_YBY * b) >> 15) + 16);
}
__host__ __device__ __forceinline__ iu8 nr_u_of(int r, int g, int b) {
    return (iu8)(((NR_YRU * r + NR_YGU * g + NR_YBU * b) >> 15) + 128);
}
__host__ __device__ __forceinline__ iu8 nr_v_of(int r, int g, int b) {
    return (iu8)(((NR_YRV * r + NR_YGV * g + NR_YBV * b) >> 15) + 128);
}

// cpp:52-57: (iu8)(v*255) = cvttsd2si to int32, keep the low byte (A.5)
__device__ __forceinline__ iu8 nr_to_u8(f64 v) {
    f64 t = v * 255;
    if (!(t > -2147483649.0 && t < 2147483648.0)) return 0;
    return (iu8)((int)t & 0xFF);
}
