/*
 * libNativeCPURenderer.h — C ABI of the MI355X (gfx950) raster library.
 *
 * Drop-in for the render part of the reference's ABI
 * (/root/reference/src/libNativeCPURenderer.h:83-152): the same symbol names
 * and parameter types (LP64: i64 = long, f64 = double, bool = C/C++ bool,
 * handles are opaque pointers), so the reference's ctypes binding
 * (libNativeCPURendererPybind.py) can load this .so unchanged for every raster
 * call.  Each declaration cites the reference prototype it replaces as
 * h:<line> and the implementation it restates as cpp:<lines>.
 *
 * Differences in behaviour: pixel data lives in HBM and draws
 * are asynchronous kernel launches — readback calls (GetBuffer*, GetColor,
 * GetDepthBuffer) and Flush are the sync points; Destroy* really free;
 * CreateRenderContext returns NULL when no HIP device is usable (no CPU path).
 * New entry points are additive and marked NEW.
 */
#ifndef LIBNATIVECPURENDERER_AMD_H
#define LIBNATIVECPURENDERER_AMD_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef long i64;
typedef double f64;
typedef unsigned char iu8;

typedef struct RenderContext RenderContext;   /* h:32-42 (opaque here) */
typedef struct Texture Texture;               /* h:44-49 (opaque here) */
typedef struct TriangleBuffer TriangleBuffer; /* NEW: device-resident triangle soup */

/* ---- render context (cpp:3-45, 277-316) ---------------------------------- */
i64 GetBufferSize(RenderContext* ctx);                                   /* h:84  */
RenderContext* CreateRenderContext(i64 width, i64 height, bool enableAlpha); /* h:85 */
void DestroyRenderContext(RenderContext* ctx);                           /* h:86  */
void ResizeRenderContext(RenderContext* ctx, i64 width, i64 height);     /* h:149 */
void SaveContextState(RenderContext* ctx);                               /* h:92  */
bool RestoreContextState(RenderContext* ctx);                            /* h:93  */
void GetBuffer(RenderContext* ctx, f64* buffer);                         /* h:94  */
void GetBufferAsUInt8(RenderContext* ctx, iu8* buffer);                  /* h:95  */

/* ---- textures (cpp:318-384, 950-988) ------------------------------------- */
Texture* CreateTexture(i64 width, i64 height, bool enableAlpha, f64* buffer);      /* h:96  */
Texture* CreateTextureUInt8(i64 width, i64 height, bool enableAlpha, iu8* buffer); /* h:97  */
void DestroyTexture(Texture* tex);                                       /* h:98  */
Texture* CreateTextureFromRenderContext(RenderContext* ctx);             /* h:99  */
Texture* CreateTextureFromRenderContextShared(RenderContext* ctx);       /* h:148 */
Texture* ResampleTexture(Texture* tex, i64 width, i64 height);           /* h:119 */
i64 GetTextureWidth(Texture* tex);                                       /* h:120 */
i64 GetTextureHeight(Texture* tex);                                      /* h:121 */
bool GetTextureEnableAlpha(Texture* tex);                                /* h:122 */

/* ---- audio clips (cpp:990-1283): interleaved f64 samples in HBM, ops as kernels */
typedef struct AudioClip AudioClip;           /* h:70-75 (opaque here) */
typedef struct WapperedBytes WapperedBytes;   /* h:77-80 (opaque here) */
i64 GetAudioClipBufferSizeFromData(i64 numFrames, i64 channels);          /* h:123 */
i64 GetAudioClipBufferSize(AudioClip* clip);                              /* h:124 */
AudioClip* CreateAudioClipFromBuffer(i64 sampleRate, i64 channels, i64 numFrames, f64* buffer); /* h:125 */
AudioClip* CreateAudioClipFromInt16Buffer(i64 sampleRate, i64 channels, i64 numFrames, short* buffer); /* h:126 */
AudioClip* CreateSilentAudioClip(i64 sampleRate, i64 channels, i64 numFrames); /* h:127 */
void DestroyAudioClip(AudioClip* clip);                                   /* h:128 (frees; a no-op there) */
AudioClip* CloneAudioClip(AudioClip* clip);                               /* h:129 */
void ApplyResampleAudioClip(AudioClip* clip, i64 sampleRate, i64 channels); /* h:130 */
void ResampleAudioClipLike(AudioClip* clip, AudioClip* like);             /* h:131 */
i64 OverlayAudioClip(AudioClip* target, AudioClip* source, i64 startFrame, bool autoResample); /* h:132;
                                                   0, -1 rate mismatch, -2 channel mismatch, -3 devices differ */
i64 OverlayAudioClipSecond(AudioClip* target, AudioClip* source, f64 startSecond, bool autoResample); /* h:133 */
WapperedBytes* SaveAudioClipAsWav(AudioClip* clip);                       /* h:134 */
i64 GetAudioClipSampleRate(AudioClip* clip);                              /* h:135 */
i64 GetAudioClipChannels(AudioClip* clip);                                /* h:136 */
i64 GetAudioClipNumFrames(AudioClip* clip);                               /* h:137 */
f64 GetAudioClipDuration(AudioClip* clip);                                /* h:138 */
iu8* GetWapperedBytesDataPtr(WapperedBytes* bytes);                       /* h:139 */
i64 GetWapperedBytesDataSize(WapperedBytes* bytes);                       /* h:140 */
void ApplyVolumeGain(AudioClip* clip, f64 gain);                          /* h:141 */
void ApplyCutAudioClip(AudioClip* clip, i64 startFrame, i64 endFrame);    /* h:144 */
void ApplySpeedAudioClip(AudioClip* clip, f64 speed);                     /* h:145 */
i64 OverlayAudioClipMany(AudioClip* target, AudioClip* source, const i64* startFrames, i64 n,
                         bool autoResample);  /* NEW: n OverlayAudioClip calls in order, one launch
                                                 (the note loop of milrenderer.py:810-815) */
i64 OverlayAudioClipManySecond(AudioClip* target, AudioClip* source, const f64* startSeconds, i64 n,
                               bool autoResample);  /* NEW: the same with OverlayAudioClipSecond times */
void DestroyWapperedBytes(WapperedBytes* bytes); /* NEW (the reference never frees them) */
void GetAudioClipBuffer(AudioClip* clip, f64* out); /* NEW: samples to the host */
void* GetAudioClipDevicePtr(AudioClip* clip);    /* NEW: samples in HBM (interop) */
void SetAudioStreamOrderedAlloc(bool on);        /* NEW (tests): clip buffers from hipMallocAsync/hipFreeAsync */

/* ---- texture preparation: procedural hit-effect shader (cpp:1318-1440) */
Texture* CreateMilthmHitEffectTexture(Texture* mask, f64 seed, f64 t, f64 r, f64 g, f64 b); /* h:151; NULL
                                                                   when the mask has no alpha (cpp:1418) */
void GetMilthmHitEffectPixel(f64 seed, f64 t, f64 x, f64 y, f64* a);     /* h:150 (inline there: not exported) */
bool CreateMilthmHitEffectTextures(Texture* mask, f64 seed, const f64* ts, i64 n, f64 r, f64 g, f64 b,
                                   Texture** out);  /* NEW: n thresholds ts[k] -> out[k], one launch
                                                       (Helpers.create_milthm_hit_effect_textures, Pybind:34-48) */

/* ---- transform / colour-transform state, host side (cpp:386-492, 623-641) */
void SetTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f);   /* h:100 */
void ApplyTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f); /* h:101 */
void Scale(RenderContext* ctx, f64 sx, f64 sy);                          /* h:102 */
void Translate(RenderContext* ctx, f64 tx, f64 ty);                      /* h:103 */
void Rotate(RenderContext* ctx, f64 angle);                              /* h:104 */
void TransformPoint(RenderContext* ctx, f64 x, f64 y, f64* out_x, f64* out_y); /* h:105 (inline in cpp:455; exported here) */
void GetTransform(RenderContext* ctx, f64 out_matrix[6]);                /* h:106 */
void GetInverseTransform(RenderContext* ctx, f64 out_matrix[6]);         /* h:107 */
void SetColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);  /* h:110 */
void ApplyColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a); /* h:111 */

/* ---- pixel ops and primitives (cpp:494-948, 1285-1316) ------------------- */
bool SetPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a);   /* h:108 */
bool ApplyPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a); /* h:109 (inline in cpp:515; exported here) */
void SetColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);           /* h:112 */
void GetColor(RenderContext* ctx, f64 x, f64 y, f64* out_r, f64* out_g, f64* out_b, f64* out_a); /* h:113 */
void FillColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);          /* h:114 */
void DrawTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height); /* h:115 */
void DrawRect(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height, f64 r, f64 g, f64 b, f64 a); /* h:116 */
void DrawLine(RenderContext* ctx, f64 x1, f64 y1, f64 x2, f64 y2, f64 width,
              f64 r, f64 g, f64 b, f64 a);                               /* h:117 */
void DrawCircle(RenderContext* ctx, f64 x, f64 y, f64 radius, f64 r, f64 g, f64 b, f64 a); /* h:118 */
void DrawVerticalGrd(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height,
                     f64 top_r, f64 top_g, f64 top_b, f64 top_a,
                     f64 bottom_r, f64 bottom_g, f64 bottom_b, f64 bottom_a); /* h:146 */
void DrawSplittedTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height,
                         f64 uStart, f64 uEnd, f64 vStart, f64 vEnd);    /* h:147 */
i64 GetVersion(void);                                                     /* h:143, =1 (h:9) */

/* ---- NEW: triangles, depth, Gouraud (the north-star path) --
 * xy: n*6 f64 (x0,y0,x1,y1,x2,y2) in user space (the context transform is
 * applied); z: n*3 f64 depths in [0,1] or NULL; rgba: n*4 f64 flat colours,
 * or n*12 per-vertex colours when gouraud. */
void SetDepthState(RenderContext* ctx, bool test, bool write);           /* NEW: LESS test, write enable */
void ClearDepth(RenderContext* ctx, uint32_t value);                     /* NEW: deferred, on-chip */
void GetDepthBuffer(RenderContext* ctx, uint32_t* out);                  /* NEW: W*H u32, sync */
void DrawTriangles(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba,
                   i64 n, bool gouraud);                                  /* NEW: host arrays */
void DrawTrianglesDevice(RenderContext* ctx, const f64* xy, const f64* z, const f64* rgba,
                         i64 n, bool gouraud);                            /* NEW: device pointers; keep them valid
                                 and unchanged until the batch has executed (Flush / readback / device sync) */
TriangleBuffer* CreateTriangleBuffer(i64 n, const f64* xy, const f64* z, const f64* rgba,
                                     bool gouraud);                       /* NEW: one H2D upload */
void DestroyTriangleBuffer(TriangleBuffer* tb);                          /* NEW */
void DrawTriangleBuffer(RenderContext* ctx, TriangleBuffer* tb);         /* NEW */
i64 GetTriangleBufferCount(TriangleBuffer* tb);                          /* NEW */
void SetFragmentCounting(RenderContext* ctx, bool on);                   /* NEW: covered-fragment counter */
i64 GetFragmentCount(RenderContext* ctx);                                /* NEW */
i64 GetLastRasterPath(RenderContext* ctx);                               /* NEW: 1 order-free tiled, 2 ordered, 3 order-free frame */
void SetForceOrderedRaster(RenderContext* ctx, bool on);                 /* NEW: A/B and tests */
void SetPairCapacityOverride(RenderContext* ctx, i64 pairs);             /* NEW: tests (0 = automatic) */
void SetCoopRaster(RenderContext* ctx, i64 mode);                        /* NEW: k_vis variant 0 auto, 1 coop, 2 lane-only */
void SetWarmBinning(RenderContext* ctx, i64 mode);                       /* NEW: one-pass binning of a repeat draw 0 auto, 1 on, 2 off */
i64 GetWarmBatchCount(RenderContext* ctx);                               /* NEW (testing): batches binned warm */
i64 GetLooseBatchCount(RenderContext* ctx);                              /* NEW (testing): of those, binned into the loose
                                                                            ranges of a changed transform */
void SetWarmFaultInjection(RenderContext* ctx, i64 mode);                /* NEW (testing): fault in the next warm batch
                                 1 range overflow, 2 withheld token, 3 dropped pairs, 4 binning delayed past the
                                 raster's token wait (the frame must stay exact) */
i64 GetWarmFailureCount(RenderContext* ctx);                             /* NEW (testing): warm batches that failed a check */
void SetSplitLimits(RenderContext* ctx, i64 splitAt, i64 dslice);       /* NEW: dense-tile split limits (0: defaults) */

/* ---- NEW: multi-GPU frames (tile-row sharding + RCCL assembly) */
typedef struct NrComm NrComm;
bool GetCommUniqueId(iu8* out128);              /* rank 0: 128-byte RCCL id to distribute */
NrComm* CreateComm(i64 nranks, i64 rank, const iu8* id128); /* on the current device */
void DestroyComm(NrComm* comm);
void SetShard(RenderContext* ctx, i64 nshards, i64 shard);  /* own tile rows ty % nshards == shard */
void SetShardSlots(RenderContext* ctx, i64 nshards, i64 shard, const i64* slots); /* weighted: rank p owns slots[p]
                                                 of every sum(slots) <= 64 bands, interleaved (same call on all ranks) */
i64 GetShardPattern(RenderContext* ctx, iu8* out64);   /* band b -> rank out64[b % period]; returns the period */
bool GatherFrameU8(RenderContext* ctx, NrComm* comm, i64 root);  /* u8 frame (cpp:52-57) assembled on root */
bool GetFrameU8(RenderContext* ctx, iu8* out);
void* GetFrameU8DevicePtr(RenderContext* ctx);
i64 DeliverFrameU8(RenderContext* ctx, iu8* host);  /* async D2H of that frame into pinned `host` on the gather
                                                       stream, overlapped with the next frame; -> ticket (-1: none) */
bool WaitFrameDelivered(RenderContext* ctx, i64 ticket);
void* AllocHostBuffer(i64 bytes);                   /* pinned host memory (DeliverFrameU8 targets) */
void FreeHostBuffer(void* p);
i64 DeliverFrameBands(RenderContext* ctx, iu8* host); /* §8e: this rank's bands of its frame output straight into
                                                       their places in a host frame (every rank into the same one:
                                                       assembled by each GPU's own PCIe link, no GPU ingress);
                                                       async on the gather stream -> ticket for WaitFrameDelivered.
                                                       `host` should be pinned (AllocHostBuffer /
                                                       AllocSharedHostBuffer): small shares are then written by a
                                                       copy kernel through its device address; any other host
                                                       pointer takes the (slower) runtime copies */
void* AllocSharedHostBuffer(const char* name, i64 bytes); /* pinned POSIX shared memory "/name" (one host frame for
                                                       the processes of a sharded frame) */
void FreeSharedHostBuffer(void* p, i64 bytes);
bool UnlinkSharedHostBuffer(const char* name);
bool SetFrameFormat(RenderContext* ctx, i64 format); /* 0: u8 image (default), 1: YUV420P planes written by the
                                                       raster and gathered as such (W, H even; same on all ranks) */
i64 GetFrameFormat(RenderContext* ctx);
bool GetFrameYUV420P(RenderContext* ctx, iu8* out); /* §8f-2: YUV420P planes of that frame (W, H even), the
                                                       encoder input of PutRendererContextFrame (cpp:232-275) */
bool GatherFramebuffer(RenderContext* ctx, NrComm* comm, i64 root); /* f64 + depth bands to root (a rank without
                                                       a depth buffer sends its cleared one) */
bool GatherFramebufferEx(RenderContext* ctx, NrComm* comm, i64 root, bool withDepth); /* withDepth: the same on
                                                       every rank (it alone decides the posted send/recvs) */
bool GatherFrameU8Local(RenderContext** ctxs, i64 n, i64 root); /* tests: GatherFrameU8's packed assembly of n
                                                                    shards of one process, device copies for RCCL */
bool GatherFrameU8LocalRccl(RenderContext** ctxs, i64 n, i64 root, NrComm* self); /* tests: the same with the packs
                                              moved by RCCL send/recv pairs over a one-rank communicator `self` */

/* ---- NEW: deferred command list ---------------------------
 * Replaces the reference's recording proxy MultiThreadedVideoRenderContext-
 * Preparer (libNativeCPURendererPybind.py:302-367, whose replay is a stub).
 * While recording, DrawTexture / DrawSplittedTexture / DrawRect / DrawLine /
 * DrawCircle / DrawVerticalGrd / FillColor / ApplyPixel / SetPixel are queued
 * and then run together by ONE launch, per pixel in recording order, with the
 * exact results of the immediate calls (every pixel read and written once per
 * list instead of once per draw).  Any call that reads or otherwise touches
 * the framebuffer runs the queue first; SetColor discards it (overwritten). */
void BeginCommandList(RenderContext* ctx);       /* start queueing primitive draws */
void EndCommandList(RenderContext* ctx);         /* run the queue, stop queueing */
void FlushCommandList(RenderContext* ctx);       /* run the queue, keep queueing (end of a frame) */
i64 GetCommandListLength(RenderContext* ctx);    /* draws queued and not yet run */
bool IsRecordingCommands(RenderContext* ctx);
/* A frame's draw and state calls as ONE packed f64 array (replaces the reference's
 * per-call ctypes round trips, Pybind:74-300; its unfinished frame recorder is
 * Pybind:302-367).  Command = opcode word + fixed arguments, run in order through
 * the same entry points as the single calls (bit-identical):
 *   0 SaveContextState  1 RestoreContextState  2 SetTransform a..f  3 ApplyTransform a..f
 *   4 Scale sx sy  5 Translate tx ty  6 Rotate angle  7 SetColorTransform rgba
 *   8 ApplyColorTransform rgba  9 SetColor rgba  10 FillColor rgba
 *   11 DrawTexture tex x y w h  12 DrawSplittedTexture tex x y w h uS uE vS vE
 *   13 DrawRect x y w h rgba  14 DrawLine x1 y1 x2 y2 width rgba  15 DrawCircle x y radius rgba
 *   16 DrawVerticalGrd x y w h top-rgba bottom-rgba  17 SetPixel x y rgba  18 ApplyPixel x y rgba
 * (tex: index into `textures`).  Returns the commands run, -1 on a malformed array
 * (the commands before the bad one have run; error latched). */
i64 ExecuteCommands(RenderContext* ctx, const f64* words, i64 nwords, Texture* const* textures, i64 ntextures);

/* ---- NEW: device, sync, interop, errors, measurement --------------------- */
bool SetDevice(i64 device);                      /* device for objects created next on this thread */
i64 GetDeviceCount(void);
i64 GetContextDevice(RenderContext* ctx);
void Flush(RenderContext* ctx);                  /* wait for every queued draw */
void ResolvePending(RenderContext* ctx);         /* materialise deferred clears */
void* GetDeviceBufferPtr(RenderContext* ctx);    /* framebuffer in HBM (RCCL / interop); writes the pending
                                                    clears first -- the bytes are current after Flush */
void* GetStreamPtr(RenderContext* ctx);          /* hipStream_t the context launches on */
void GetBufferAsUInt8Device(RenderContext* ctx, iu8* dev_out); /* cpp:52-57 into HBM */
void GetTextureBuffer(Texture* tex, f64* out);
const char* GetLastErrorString(void);            /* "" when no HIP call failed */
void ClearLastError(void);
void EnableKernelTiming(RenderContext* ctx, bool on);
bool GetKernelTiming(RenderContext* ctx, const char* name, f64* total_ms, i64* count);
void ResetKernelTiming(RenderContext* ctx);
void SetKernelTimingFilter(RenderContext* ctx, const char* names); /* comma-separated kernel names, "" = all */

#ifdef __cplusplus
}
#endif
#endif
