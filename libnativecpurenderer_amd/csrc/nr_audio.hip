// nr_audio.hip — audio clips: the sample buffers of
// milrenderer's hit-sound mix (milrenderer.py:803-815, hjm_mixer.py:67-97)
// kept in HBM, and the reference's clip operations (cpp:990-1283) as kernels.
//
// Layout: the reference's interleaved f64 samples, `buffer[frame * channels
// + c]` (cpp:1007-1011), so a clip's readback and its WAV export are one copy.
// Every per-sample expression is the reference's, in its order, in f64 with
// no FMA (-ffp-contract=off), so results are bit-identical.
//
// The mix is the hot part: thousands of OverlayAudioClip calls, each adding a
// short clip into the song at a note time.  Sequential f64 adds do not
// commute, so OverlayAudioClipMany (new) keeps the call order per sample: a
// workgroup owns 1024 consecutive samples of the target, finds the overlays
// touching them 256 starts at a time (ballot + prefix count into LDS, in call
// order) and each thread adds its samples' contributions in that order —
// identical to n calls of OverlayAudioClip, in one launch.
//
// Where the reference reads or writes outside a buffer (undefined behaviour)
// this library defines the result, and the oracle does the same:
//  * OverlayAudioClip with startFrame < 0: frames landing before the target
//    are skipped (the reference writes before the buffer);
//  * ApplyResampleAudioClip reads index `numFrames - channels - 1` at most
//    (cpp:1081-1084, the frame count compared with the channel count): a
//    negative index (clips of <= channels frames) reads 0.0;
//  * ApplyCutAudioClip leaves frames past the source uninitialised
//    (cpp:1265-1279): they are 0.0 here, as are frames before a negative start;
//    a negative length gives an empty clip (the reference's `new f64[n < 0]`
//    throws);
//  * a negative resampled length gives an empty clip.
#include "nr_common.h"

#include <algorithm>
#include <cstring>
#include <atomic>
#include <mutex>
#include <unordered_set>

struct AudioClip {   // h:70-75, samples in HBM
    i64 sampleRate;
    i64 channels;
    i64 numFrames;
    f64* buffer;     // device, numFrames * channels (at least one element allocated)
    int device;
    u64 uid;         // never reused (keys the resample cache)
    u64 version;     // bumped by every change of the samples or the rate
    bool external;   // its device pointer was handed out: never cached
};

struct WapperedBytes {   // h:77-80, host bytes
    iu8* data;
    i64 size;
};

namespace {

constexpr int AWG = 256;

int grid_for(i64 n) {
    i64 g = (n + AWG - 1) / AWG;
    if (g < 1) g = 1;
    if (g > 65535) g = 65535;
    return (int)g;
}

// Sample and scratch buffers.  Every clip operation runs on the clip's
// device stream (nr_stream_for) and every host-visible result is read back
// after a synchronisation of that stream, so a buffer is only ever touched in
// that one stream's order: no other library stream or the null stream reads
// or writes it.  Default allocator: plain hipMalloc, freed after a stream
// synchronisation; SetAudioStreamOrderedAlloc(true) switches to hipMallocAsync
// / hipFreeAsync on the same stream (tests/test_audio.py runs the whole mix
// under both).
//
// Round 1 saw one mix run (stream-ordered allocator) read back a stale 32 MiB
// span of a clip.  Every device-side access of a clip is in one stream's
// order, so the one step that was not under the library's control is the
// readback itself: hipMemcpyAsync into the caller's PAGEABLE host memory
// (a numpy array), which the HIP runtime does not copy as one stream-ordered
// DMA but stages chunk by chunk through its own pinned buffers
// (GPU_PINNED_XFER_SIZE / GPU_STAGING_BUFFER_SIZE; a 32 MiB span is one such
// chunk), with a separate path when the source is stream-ordered pool memory.
// One chunk landing from before the producing kernel finished is the
// observed symptom.  The readbacks (GetAudioClipBuffer, SaveAudioClipAsWav)
// therefore no longer hand pageable memory to the runtime: d2h_pinned copies
// through library-owned pinned buffers, each chunk a plain stream-ordered
// DMA that the host waits for before it touches the bytes.  This explanation
// is inferred from the evidence (span size, allocator, pageable target); the
// failure was never reproduced, before or after.
std::atomic<bool> g_async_alloc{false};
std::mutex g_async_mu;
std::unordered_set<void*> g_async_ptrs;   // buffers from hipMallocAsync

void* alloc_bytes(size_t bytes, hipStream_t s) {
    void* p = nullptr;
    if (bytes == 0) bytes = 8;
    if (g_async_alloc.load()) {
        NR_CHECK(hipMallocAsync(&p, bytes, s));
        std::lock_guard<std::mutex> lk(g_async_mu);
        g_async_ptrs.insert(p);
    } else {
        NR_CHECK(hipMalloc(&p, bytes));
    }
    return p;
}

f64* alloc_samples(i64 n, hipStream_t s) {
    return static_cast<f64*>(alloc_bytes((size_t)(n > 0 ? n : 1) * sizeof(f64), s));
}

// Device -> pageable host copy through two library-owned pinned buffers
// (chunk k+1's DMA in flight while chunk k is copied out on the host); the
// host reads a chunk only after the event of its DMA.
constexpr size_t PIN_CHUNK = 8u << 20;
constexpr int PIN_DEVICES = 64;
std::mutex g_pin_mu;
// per device (a clip's stream belongs to the clip's device, and an event can
// only be recorded on a stream of the device it was created on)
struct PinPair {
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
};
PinPair g_pin[PIN_DEVICES];

// The caller has made the clip's device current (clip_stream).
void d2h_pinned(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return;
    int dev = 0;
    NR_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= PIN_DEVICES) {   // (no pinned pair: a plain synchronous copy)
        NR_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
        NR_CHECK(hipStreamSynchronize(s));
        return;
    }
    std::lock_guard<std::mutex> lk(g_pin_mu);
    PinPair& P = g_pin[dev];
    for (int k = 0; k < 2; ++k)
        if (!P.buf[k]) {
            NR_CHECK(hipHostMalloc(&P.buf[k], PIN_CHUNK, hipHostMallocDefault));
            NR_CHECK(hipEventCreateWithFlags(&P.ev[k], hipEventDisableTiming));
        }
    const size_t nch = (bytes + PIN_CHUNK - 1) / PIN_CHUNK;
    auto issue = [&](size_t c) {
        const size_t off = c * PIN_CHUNK, len = std::min(PIN_CHUNK, bytes - off);
        NR_CHECK(hipMemcpyAsync(P.buf[c & 1], static_cast<const iu8*>(src) + off, len, hipMemcpyDeviceToHost, s));
        NR_CHECK(hipEventRecord(P.ev[c & 1], s));
    };
    issue(0);
    for (size_t c = 0; c < nch; ++c) {
        if (c + 1 < nch) issue(c + 1);   // the other buffer: its previous chunk was copied out below
        NR_CHECK(hipEventSynchronize(P.ev[c & 1]));
        const size_t off = c * PIN_CHUNK, len = std::min(PIN_CHUNK, bytes - off);
        std::memcpy(static_cast<iu8*>(dst) + off, P.buf[c & 1], len);
    }
}

// cpp:1029: (f64)v / 32768.0
__global__ void k_i16_to_f64(const short* __restrict__ in, f64* __restrict__ out, i64 n) {
    for (i64 i = (i64)blockIdx.x * AWG + threadIdx.x; i < n; i += (i64)gridDim.x * AWG) out[i] = (f64)in[i] / 32768.0;
}

// cpp:1254-1259
__global__ void k_gain(f64* __restrict__ p, i64 n, f64 gain) {
    for (i64 i = (i64)blockIdx.x * AWG + threadIdx.x; i < n; i += (i64)gridDim.x * AWG) p[i] *= gain;
}

__device__ __forceinline__ f64 sample_at(const f64* b, i64 idx) { return idx >= 0 ? b[idx] : 0.0; }

// cpp:1063-1120, one thread per new frame
__global__ void k_resample(const f64* __restrict__ src, i64 oldFrames, i64 oldCh, i64 oldRate, f64* __restrict__ dst,
                           i64 newFrames, i64 newCh, i64 newRate) {
    for (i64 i = (i64)blockIdx.x * AWG + threadIdx.x; i < newFrames; i += (i64)gridDim.x * AWG) {
        const f64 secT = (f64)i / (f64)newRate;
        const f64 old = secT * (f64)oldRate;
        i64 fl = (i64)floor(old), ce = (i64)ceil(old);
        const i64 lim = oldFrames - oldCh;
        if (fl < 0) fl = 0;
        if (fl >= lim) fl = lim - 1;
        if (ce < 0) ce = 0;
        if (ce >= lim) ce = lim - 1;
        const f64 frac = old - (f64)fl;
        if (oldCh == newCh) {
            for (i64 c = 0; c < newCh; ++c) {
                const f64 vf = sample_at(src, fl * oldCh + c), vc = sample_at(src, ce * oldCh + c);
                dst[i * newCh + c] = vf + (vc - vf) * frac;
            }
        } else {
            f64 sf = 0, sc = 0;
            for (i64 c = 0; c < oldCh; ++c) {
                sf += sample_at(src, fl * oldCh + c);
                sc += sample_at(src, ce * oldCh + c);
            }
            const f64 dc = (f64)oldCh;
            const f64 v = sf / dc + (sc / dc - sf / dc) * frac;
            for (i64 c = 0; c < newCh; ++c) dst[i * newCh + c] = v;
        }
    }
}

// cpp:1145-1151, one thread per source sample
__global__ void k_overlay(f64* __restrict__ tgt, i64 tgtFrames, const f64* __restrict__ src, i64 srcFrames, i64 ch,
                          i64 start) {
    const i64 n = srcFrames * ch;
    for (i64 e = (i64)blockIdx.x * AWG + threadIdx.x; e < n; e += (i64)gridDim.x * AWG) {
        const i64 i = e / ch, c = e - i * ch;
        const i64 t = start + i;
        if (t < 0 || t >= tgtFrames) continue;
        tgt[t * ch + c] += src[e];
    }
}

// A clip overlaid onto itself at start 0: every sample is read once, then
// written (cpp:1145-1151 with target == source), i.e. x + x.  Its own kernel:
// k_overlay's __restrict__ operands must not alias.
__global__ void k_overlay_same(f64* __restrict__ b, i64 n) {
    for (i64 e = (i64)blockIdx.x * AWG + threadIdx.x; e < n; e += (i64)gridDim.x * AWG) {
        const f64 v = b[e];
        b[e] = v + v;
    }
}

// A clip overlaid onto itself at start s > 0 (an echo): the reference's
// loop reads samples it has already added to (cpp:1145-1151), so frame
// s + i gets the updated frame i -- a recurrence along each chain r, r + s,
// r + 2s, ... of stride s.  One thread per (chain, channel), sequential along
// its chain; chains are independent.  f64 adds in the reference's order do
// not reassociate, so a chain is inherently serial and latency-bound: ~0.2 us
// per chain step (a 1-frame delay over 20000 frames: 3.9 ms; a 0.1 s echo on a
// 114 s stereo song: 7.6 ms including the 80 MB readback; tools/exp/echo_time.py).
__global__ void k_overlay_self(f64* __restrict__ b, i64 frames, i64 ch, i64 s) {
    const i64 n = s * ch;
    for (i64 q = (i64)blockIdx.x * AWG + threadIdx.x; q < n; q += (i64)gridDim.x * AWG) {
        const i64 r = q / ch, c = q - r * ch;
        // source frame i = r + k*s updates target frame i + s, in increasing i
        for (i64 i = r; i + s < frames; i += s) b[(i + s) * ch + c] += b[i * ch + c];
    }
}

// n overlays of one source in call order (see the file comment).  Workgroup =
// OV_PER x 256 consecutive target samples (thread: OV_PER samples 256 apart,
// coalesced), so each scan of the start list serves 1024 samples.
constexpr int OV_PER = 4;
__global__ __launch_bounds__(AWG) void k_overlay_many(f64* __restrict__ tgt, i64 tgtFrames, const f64* __restrict__ src,
                                                      i64 srcFrames, i64 ch, const i64* __restrict__ starts, i64 n) {
    __shared__ i64 hit[AWG];
    __shared__ int wcnt[AWG / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const i64 total = tgtFrames * ch;
    constexpr i64 CH = (i64)AWG * OV_PER;
    for (i64 e0 = (i64)blockIdx.x * CH; e0 < total; e0 += (i64)gridDim.x * CH) {
        const i64 fa = e0 / ch, fb = ((e0 + CH < total ? e0 + CH : total) - 1) / ch;   // frames this chunk touches
        f64 acc[OV_PER];
        i64 fr[OV_PER], cc[OV_PER];
#pragma unroll
        for (int j = 0; j < OV_PER; ++j) {
            const i64 e = e0 + j * AWG + tid;
            fr[j] = e < total ? e / ch : -((i64)1 << 62);   // a dead slot matches no overlay
            cc[j] = e < total ? e - fr[j] * ch : 0;
            acc[j] = e < total ? tgt[e] : 0.0;
        }
        for (i64 k0 = 0; k0 < n; k0 += AWG) {
            const i64 k = k0 + tid;
            bool h = false;
            i64 s = 0;
            if (k < n) {
                s = starts[k];
                h = s <= fb && s > fa - srcFrames;
            }
            const u64 m = __ballot(h);
            if (lane == 0) wcnt[w] = __popcll(m);
            __syncthreads();
            int base = 0, cnt = 0;
#pragma unroll
            for (int q = 0; q < AWG / 64; ++q) {
                base += q < w ? wcnt[q] : 0;
                cnt += wcnt[q];
            }
            if (h) hit[base + __popcll(m & ((1ull << lane) - 1ull))] = s;
            __syncthreads();
            for (int q = 0; q < cnt; ++q) {
                const i64 hs = hit[q];
#pragma unroll
                for (int j = 0; j < OV_PER; ++j) {
                    const i64 i = fr[j] - hs;
                    if (i >= 0 && i < srcFrames) acc[j] += src[i * ch + cc[j]];
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < OV_PER; ++j) {
            const i64 e = e0 + j * AWG + tid;
            if (e < total) tgt[e] = acc[j];
        }
    }
}

// cpp:1265-1279 (see the file comment for frames outside the source)
__global__ void k_cut(const f64* __restrict__ src, i64 srcFrames, i64 ch, i64 start, f64* __restrict__ dst, i64 frames) {
    const i64 n = frames * ch;
    for (i64 e = (i64)blockIdx.x * AWG + threadIdx.x; e < n; e += (i64)gridDim.x * AWG) {
        const i64 i = e / ch, c = e - i * ch;
        const i64 sf = start + i;
        dst[e] = (sf >= 0 && sf < srcFrames) ? src[sf * ch + c] : 0.0;
    }
}

// cpp:1215-1222: (i16)(clamp(v, -1, 1) * 32767.0); the x86 conversion goes
// through int32, and a NaN (which passes the clamp) becomes 0x80000000 -> 0.
__global__ void k_to_i16(const f64* __restrict__ p, short* __restrict__ out, i64 n) {
    for (i64 i = (i64)blockIdx.x * AWG + threadIdx.x; i < n; i += (i64)gridDim.x * AWG) {
        const f64 v = p[i];
        const f64 x = (v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v)) * 32767.0;
        out[i] = x != x ? (short)0 : (short)(int)x;
    }
}

std::mutex g_cache_mu;
std::atomic<u64> g_clip_uid{0};

// Resample cache for OverlayAudioClip(..., autoResample): the reference
// clones and resamples the source on every call (cpp:1135-1143), so the demo's
// 876 calls with one source (Pybind.py:689-691) resample it 876 times.  Here
// the resampled copy is kept, keyed by (source uid, source version, target
// rate and channels); any change of the source bumps its version, so a cached
// copy always equals what a fresh clone + resample would give.
struct CacheEntry {
    u64 uid = 0, version = 0;
    i64 rate = 0, channels = 0;
    AudioClip* clip = nullptr;
};
constexpr int CACHE_N = 4;
CacheEntry g_cache[CACHE_N];
int g_cache_next = 0;

AudioClip* new_clip(i64 rate, i64 ch, i64 frames) {
    AudioClip* a = new AudioClip();
    a->sampleRate = rate; a->channels = ch; a->numFrames = frames;
    a->version = 0;
    a->external = false;
    NR_CHECK(hipGetDevice(&a->device));
    a->uid = ++g_clip_uid;
    a->buffer = alloc_samples(frames * ch, nr_stream_for(a->device));
    return a;
}

// frees a buffer the stream may still be using (stream-ordered when it came
// from hipMallocAsync; otherwise after the stream drains)
void free_after(hipStream_t s, void* p) {
    {
        std::lock_guard<std::mutex> lk(g_async_mu);
        auto it = g_async_ptrs.find(p);
        if (it != g_async_ptrs.end()) {
            g_async_ptrs.erase(it);
            NR_CHECK(hipFreeAsync(p, s));
            return;
        }
    }
    NR_CHECK(hipStreamSynchronize(s));
    NR_CHECK(hipFree(p));
}

hipStream_t clip_stream(AudioClip* a) {
    NR_CHECK(hipSetDevice(a->device));
    return nr_stream_for(a->device);
}

void destroy_clip(AudioClip* clip) {
    hipStream_t s = clip_stream(clip);
    free_after(s, clip->buffer);
    delete clip;
}

}  // namespace

extern "C" {

// cpp:990-996
i64 GetAudioClipBufferSizeFromData(i64 numFrames, i64 channels) { return numFrames * channels; }
i64 GetAudioClipBufferSize(AudioClip* clip) { return clip->numFrames * clip->channels; }

// cpp:998-1012 (the caller's samples are copied)
AudioClip* CreateAudioClipFromBuffer(i64 sampleRate, i64 channels, i64 numFrames, f64* buffer) {
    AudioClip* a = new_clip(sampleRate, channels, numFrames);
    hipStream_t s = nr_stream_for(a->device);
    const i64 n = numFrames * channels;
    if (n > 0) NR_CHECK(hipMemcpyAsync(a->buffer, buffer, (size_t)n * sizeof(f64), hipMemcpyHostToDevice, s));
    NR_CHECK(hipStreamSynchronize(s));   // caller owns `buffer`
    return a;
}

// cpp:1016-1034: i16 -> f64 on the GPU
AudioClip* CreateAudioClipFromInt16Buffer(i64 sampleRate, i64 channels, i64 numFrames, short* buffer) {
    AudioClip* a = new_clip(sampleRate, channels, numFrames);
    hipStream_t s = nr_stream_for(a->device);
    const i64 n = numFrames * channels;
    if (n > 0) {
        short* d = static_cast<short*>(alloc_bytes((size_t)n * sizeof(short), s));
        NR_CHECK(hipMemcpyAsync(d, buffer, (size_t)n * sizeof(short), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_i16_to_f64, dim3(grid_for(n)), dim3(AWG), 0, s, d, a->buffer, n);
        NR_CHECK(hipGetLastError());
        free_after(s, d);
    }
    NR_CHECK(hipStreamSynchronize(s));
    return a;
}

// cpp:1036-1046
AudioClip* CreateSilentAudioClip(i64 sampleRate, i64 channels, i64 numFrames) {
    AudioClip* a = new_clip(sampleRate, channels, numFrames);
    const i64 n = numFrames * channels;
    if (n > 0) NR_CHECK(hipMemsetAsync(a->buffer, 0, (size_t)n * sizeof(f64), nr_stream_for(a->device)));
    return a;
}

// cpp:1048-1052 is a no-op (the reference leaks); here the clip is freed
void DestroyAudioClip(AudioClip* clip) {
    if (!clip) return;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);   // the resampled copies of this clip go with it
        for (CacheEntry& e : g_cache)
            if (e.clip && e.uid == clip->uid) {
                destroy_clip(e.clip);
                e = CacheEntry();
            }
    }
    hipStream_t s = clip_stream(clip);
    free_after(s, clip->buffer);
    delete clip;
}

// cpp:1054-1061
AudioClip* CloneAudioClip(AudioClip* clip) {
    hipStream_t s = clip_stream(clip);
    AudioClip* a = new_clip(clip->sampleRate, clip->channels, clip->numFrames);
    const i64 n = clip->numFrames * clip->channels;
    if (n > 0) NR_CHECK(hipMemcpyAsync(a->buffer, clip->buffer, (size_t)n * sizeof(f64), hipMemcpyDeviceToDevice, s));
    return a;
}

// cpp:1242-1244
f64 GetAudioClipDuration(AudioClip* clip) { return (f64)clip->numFrames / (f64)clip->sampleRate; }

// cpp:1063-1120
void ApplyResampleAudioClip(AudioClip* clip, i64 sampleRate, i64 channels) {
    if (clip->sampleRate == sampleRate && clip->channels == channels) return;
    const f64 dur = GetAudioClipDuration(clip);
    i64 frames = nr_f2i64(dur * (f64)sampleRate);
    if (frames < 0) frames = 0;
    hipStream_t s = clip_stream(clip);
    f64* nb = alloc_samples(frames * channels, s);
    if (frames > 0 && channels > 0) {
        hipLaunchKernelGGL(k_resample, dim3(grid_for(frames)), dim3(AWG), 0, s, clip->buffer, clip->numFrames,
                           clip->channels, clip->sampleRate, nb, frames, channels, sampleRate);
        NR_CHECK(hipGetLastError());
    }
    free_after(s, clip->buffer);
    clip->buffer = nb;
    clip->sampleRate = sampleRate;
    clip->channels = channels;
    clip->numFrames = frames;
    ++clip->version;
}

// cpp:1122-1127
void ResampleAudioClipLike(AudioClip* clip, AudioClip* like) {
    ApplyResampleAudioClip(clip, like->sampleRate, like->channels);
}

// Shared front half of OverlayAudioClip(Many), cpp:1135-1143: the resampled
// copy of `source` when asked for and needed (from the resample cache; `tmp`
// = an uncached copy the caller releases, for clips whose device pointer was
// handed out; the reference leaks its copy), or an error code.
static i64 overlay_source(AudioClip* target, AudioClip*& source, bool autoResample, AudioClip*& tmp) {
    tmp = nullptr;
    if (target->device != source->device) {
        nr_set_error_msg("OverlayAudioClip: target and source live on different devices");
        return -3;
    }
    if (autoResample && (target->sampleRate != source->sampleRate || target->channels != source->channels)) {
        AudioClip* hit = nullptr;   // the caller holds g_cache_mu until its launch is queued
        for (CacheEntry& e : g_cache)
            if (e.clip && e.uid == source->uid && e.version == source->version && e.rate == target->sampleRate &&
                e.channels == target->channels && e.clip->device == target->device)
                hit = e.clip;
        if (!hit) {
            hit = CloneAudioClip(source);
            ResampleAudioClipLike(hit, target);
            if (source->external) {
                tmp = hit;   // released by the caller
            } else {
                CacheEntry& e = g_cache[g_cache_next];
                g_cache_next = (g_cache_next + 1) % CACHE_N;
                AudioClip* old = e.clip;
                e = {source->uid, source->version, target->sampleRate, target->channels, hit};
                if (old) destroy_clip(old);
            }
        }
        source = hit;
    }
    if (target->sampleRate != source->sampleRate) return -1;
    if (target->channels != source->channels) return -2;
    return 0;
}

// cpp:1129-1154
i64 OverlayAudioClip(AudioClip* target, AudioClip* source, i64 startFrame, bool autoResample) {
    AudioClip* tmp;
    std::unique_lock<std::mutex> lk(g_cache_mu, std::defer_lock);
    if (autoResample) lk.lock();   // a cached copy is not evicted before the launch below is queued
    const i64 rc = overlay_source(target, source, autoResample, tmp);
    if (rc == 0 && source == target && startFrame > 0 && startFrame < target->numFrames) {
        hipStream_t s = clip_stream(target);
        hipLaunchKernelGGL(k_overlay_self, dim3(grid_for(startFrame * target->channels)), dim3(AWG), 0, s,
                           target->buffer, target->numFrames, target->channels, startFrame);
        NR_CHECK(hipGetLastError());
    } else if (rc == 0 && source == target && startFrame == 0) {
        const i64 n = target->numFrames * target->channels;
        if (n > 0) {
            hipLaunchKernelGGL(k_overlay_same, dim3(grid_for(n)), dim3(AWG), 0, clip_stream(target), target->buffer, n);
            NR_CHECK(hipGetLastError());
        }
    } else if (rc == 0) {
        hipStream_t s = clip_stream(target);
        if (source == target && startFrame < 0 && !tmp) {
            // reads run ahead of the writes in the reference's loop (every
            // read sees the original sample): overlay from a copy
            tmp = CloneAudioClip(target);
            source = tmp;
        }
        const i64 n = source->numFrames * source->channels;
        if (n > 0 && startFrame < target->numFrames) {
            hipLaunchKernelGGL(k_overlay, dim3(grid_for(n)), dim3(AWG), 0, s, target->buffer, target->numFrames,
                               source->buffer, source->numFrames, source->channels, startFrame);
            NR_CHECK(hipGetLastError());
        }
    }
    if (rc == 0) ++target->version;
    if (lk.owns_lock()) lk.unlock();
    if (tmp) DestroyAudioClip(tmp);
    return rc;
}

// cpp:1156-1163
i64 OverlayAudioClipSecond(AudioClip* target, AudioClip* source, f64 startSecond, bool autoResample) {
    return OverlayAudioClip(target, source, nr_f2i64(startSecond * (f64)target->sampleRate), autoResample);
}

// NEW: n calls of OverlayAudioClip(target, source, startFrames[k], autoResample)
// in order, as one launch (the note loop of milrenderer.py:810-815).  Same
// return codes; the source is resampled at most once.
i64 OverlayAudioClipMany(AudioClip* target, AudioClip* source, const i64* startFrames, i64 n, bool autoResample) {
    AudioClip* tmp;
    std::unique_lock<std::mutex> lk(g_cache_mu, std::defer_lock);
    if (autoResample) lk.lock();   // a cached copy is not evicted before the launch below is queued
    const i64 rc = overlay_source(target, source, autoResample, tmp);
    const i64 total = target->numFrames * target->channels;
    if (rc == 0 && source == target) {   // self-overlays depend on each other: one call at a time
        if (lk.owns_lock()) lk.unlock();
        for (i64 k = 0; k < n; ++k) OverlayAudioClip(target, target, startFrames[k], false);
        return rc;
    }
    if (rc == 0 && n > 0 && total > 0 && source->numFrames > 0) {
        hipStream_t s = clip_stream(target);
        i64* d = static_cast<i64*>(alloc_bytes((size_t)n * sizeof(i64), s));
        NR_CHECK(hipMemcpyAsync(d, startFrames, (size_t)n * sizeof(i64), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_overlay_many, dim3(grid_for((total + OV_PER - 1) / OV_PER)), dim3(AWG), 0, s, target->buffer, target->numFrames,
                           source->buffer, source->numFrames, source->channels, d, n);
        NR_CHECK(hipGetLastError());
        free_after(s, d);
        NR_CHECK(hipStreamSynchronize(s));   // caller owns startFrames
    }
    if (rc == 0) ++target->version;
    if (lk.owns_lock()) lk.unlock();
    if (tmp) DestroyAudioClip(tmp);
    return rc;
}

// NEW: OverlayAudioClipMany with start times in seconds (cpp:1162 per time)
i64 OverlayAudioClipManySecond(AudioClip* target, AudioClip* source, const f64* startSeconds, i64 n,
                               bool autoResample) {
    std::vector<i64> f((size_t)(n > 0 ? n : 0));
    for (i64 k = 0; k < n; ++k) f[(size_t)k] = nr_f2i64(startSeconds[k] * (f64)target->sampleRate);
    return OverlayAudioClipMany(target, source, f.data(), n, autoResample);
}

// cpp:1165-1228: RIFF/WAVE PCM16 header built on the host, samples converted
// on the GPU and copied behind it
WapperedBytes* SaveAudioClipAsWav(AudioClip* clip) {
    const i64 n = clip->numFrames * clip->channels;
    const i64 size = 44 + n * 2;
    WapperedBytes* w = new WapperedBytes();
    w->size = size;
    w->data = new iu8[(size_t)size];
    iu8* d = w->data;
    auto put32 = [&](int off, int32_t v) { std::memcpy(d + off, &v, 4); };
    auto put16 = [&](int off, int16_t v) { std::memcpy(d + off, &v, 2); };
    std::memcpy(d + 0, "RIFF", 4);
    put32(4, (int32_t)(size - 8));
    std::memcpy(d + 8, "WAVEfmt ", 8);
    put32(16, 0x10);
    put16(20, 1);
    put16(22, (int16_t)clip->channels);
    put32(24, (int32_t)clip->sampleRate);
    put32(28, (int32_t)(clip->sampleRate * clip->channels * 2));
    put16(32, (int16_t)(clip->channels * 2));
    put16(34, 16);
    std::memcpy(d + 36, "data", 4);
    put32(40, (int32_t)(n * 2));
    hipStream_t s = clip_stream(clip);
    if (n > 0) {
        short* dv = static_cast<short*>(alloc_bytes((size_t)n * sizeof(short), s));
        hipLaunchKernelGGL(k_to_i16, dim3(grid_for(n)), dim3(AWG), 0, s, clip->buffer, dv, n);
        NR_CHECK(hipGetLastError());
        d2h_pinned(d + 44, dv, (size_t)n * sizeof(short), s);
        free_after(s, dv);
    }
    NR_CHECK(hipStreamSynchronize(s));
    return w;
}

i64 GetAudioClipSampleRate(AudioClip* clip) { return clip->sampleRate; }   // cpp:1230-1232
i64 GetAudioClipChannels(AudioClip* clip) { return clip->channels; }       // cpp:1234-1236
i64 GetAudioClipNumFrames(AudioClip* clip) { return clip->numFrames; }     // cpp:1238-1240
iu8* GetWapperedBytesDataPtr(WapperedBytes* bytes) { return bytes->data; } // cpp:1246-1248
i64 GetWapperedBytesDataSize(WapperedBytes* bytes) { return bytes->size; } // cpp:1250-1252

// NEW: the reference never frees WapperedBytes
void DestroyWapperedBytes(WapperedBytes* bytes) {
    if (!bytes) return;
    delete[] bytes->data;
    delete bytes;
}

// cpp:1254-1259
void ApplyVolumeGain(AudioClip* clip, f64 gain) {
    const i64 n = clip->numFrames * clip->channels;
    if (n <= 0) return;
    hipStream_t s = clip_stream(clip);
    hipLaunchKernelGGL(k_gain, dim3(grid_for(n)), dim3(AWG), 0, s, clip->buffer, n, gain);
    NR_CHECK(hipGetLastError());
    ++clip->version;
}

// cpp:1265-1279
void ApplyCutAudioClip(AudioClip* clip, i64 startFrame, i64 endFrame) {
    i64 frames = endFrame - startFrame;
    if (frames < 0) frames = 0;
    hipStream_t s = clip_stream(clip);
    const i64 n = frames * clip->channels;
    f64* nb = alloc_samples(n, s);
    if (n > 0) {
        hipLaunchKernelGGL(k_cut, dim3(grid_for(n)), dim3(AWG), 0, s, clip->buffer, clip->numFrames, clip->channels,
                           startFrame, nb, frames);
        NR_CHECK(hipGetLastError());
    }
    free_after(s, clip->buffer);
    clip->buffer = nb;
    clip->numFrames = frames;
    ++clip->version;
}

// cpp:1281-1283: i64 *= f64 -> (i64)((f64)rate * speed)
void ApplySpeedAudioClip(AudioClip* clip, f64 speed) {
    clip->sampleRate = nr_f2i64((f64)clip->sampleRate * speed);
    ++clip->version;
}

// NEW: the clip's interleaved samples into a host buffer of
// GetAudioClipBufferSize(clip) doubles
void GetAudioClipBuffer(AudioClip* clip, f64* out) {
    const i64 n = clip->numFrames * clip->channels;
    hipStream_t s = clip_stream(clip);
    if (n > 0) d2h_pinned(out, clip->buffer, (size_t)n * sizeof(f64), s);
    NR_CHECK(hipStreamSynchronize(s));
}

// NEW (testing): sample and scratch buffers from the stream-ordered allocator
// (hipMallocAsync / hipFreeAsync) instead of hipMalloc; see alloc_bytes.
void SetAudioStreamOrderedAlloc(bool on) { g_async_alloc.store(on); }

// NEW: the device pointer of the samples (interop)
void* GetAudioClipDevicePtr(AudioClip* clip) {
    clip->external = true;   // may change behind the library's back: its resampled copies are not cached
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (CacheEntry& e : g_cache)
        if (e.clip && e.uid == clip->uid) {
            destroy_clip(e.clip);
            e = CacheEntry();
        }
    return clip->buffer;
}

}  // extern "C"
