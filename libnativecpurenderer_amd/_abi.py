"""ctypes signature table of the C ABI (include/libNativeCPURenderer.h).

The reference's binding re-declares argtypes/restype inside every method
(/root/reference/src/libNativeCPURendererPybind.py:51-300); here they are
declared once per library from this table.  The table is pure data so the
test-suite can apply the shared part of it to the CPU oracle as well.
"""
from __future__ import annotations

import ctypes

P = ctypes.c_void_p
L = ctypes.c_long
D = ctypes.c_double
B = ctypes.c_bool
U32 = ctypes.c_uint32

# name -> (restype, argtypes).  "ref" = entry point of the reference ABI
# (h:83-152); "new" = additive entry point of this library.
REFERENCE_ABI = {
    "GetBufferSize": (L, (P,)),
    "CreateRenderContext": (P, (L, L, B)),
    "DestroyRenderContext": (None, (P,)),
    "ResizeRenderContext": (None, (P, L, L)),
    "SaveContextState": (None, (P,)),
    "RestoreContextState": (B, (P,)),
    "GetBuffer": (None, (P, P)),
    "GetBufferAsUInt8": (None, (P, P)),
    "CreateTexture": (P, (L, L, B, P)),
    "CreateTextureUInt8": (P, (L, L, B, P)),
    "DestroyTexture": (None, (P,)),
    "CreateTextureFromRenderContext": (P, (P,)),
    "CreateTextureFromRenderContextShared": (P, (P,)),
    "SetTransform": (None, (P, D, D, D, D, D, D)),
    "ApplyTransform": (None, (P, D, D, D, D, D, D)),
    "Scale": (None, (P, D, D)),
    "Translate": (None, (P, D, D)),
    "Rotate": (None, (P, D)),
    "TransformPoint": (None, (P, D, D, P, P)),
    "GetTransform": (None, (P, P)),
    "GetInverseTransform": (None, (P, P)),
    "SetPixel": (B, (P, L, L, D, D, D, D)),
    "ApplyPixel": (B, (P, L, L, D, D, D, D)),
    "SetColorTransform": (None, (P, D, D, D, D)),
    "ApplyColorTransform": (None, (P, D, D, D, D)),
    "SetColor": (None, (P, D, D, D, D)),
    "GetColor": (None, (P, D, D, P, P, P, P)),
    "FillColor": (None, (P, D, D, D, D)),
    "DrawTexture": (None, (P, P, D, D, D, D)),
    "DrawSplittedTexture": (None, (P, P, D, D, D, D, D, D, D, D)),
    "DrawRect": (None, (P, D, D, D, D, D, D, D, D)),
    "DrawLine": (None, (P, D, D, D, D, D, D, D, D, D)),
    "DrawCircle": (None, (P, D, D, D, D, D, D, D)),
    "DrawVerticalGrd": (None, (P, D, D, D, D, D, D, D, D, D, D, D, D)),
    "ResampleTexture": (P, (P, L, L)),
    "GetTextureWidth": (L, (P,)),
    "GetTextureHeight": (L, (P,)),
    "GetTextureEnableAlpha": (B, (P,)),
    "GetVersion": (L, ()),
    "CreateMilthmHitEffectTexture": (P, (P, D, D, D, D, D)),
    "GetMilthmHitEffectPixel": (None, (D, D, D, D, P)),
}

# triangles / depth (also exported by the oracle)
TRIANGLE_ABI = {
    "SetDepthState": (None, (P, B, B)),
    "ClearDepth": (None, (P, U32)),
    "GetDepthBuffer": (None, (P, P)),
    "DrawTriangles": (None, (P, P, P, P, L, B)),
}

# HIP-library-only additions
DEVICE_ABI = {
    "DrawTrianglesDevice": (None, (P, P, P, P, L, B)),
    "CreateTriangleBuffer": (P, (L, P, P, P, B)),
    "DestroyTriangleBuffer": (None, (P,)),
    "DrawTriangleBuffer": (None, (P, P)),
    "GetTriangleBufferCount": (L, (P,)),
    "SetFragmentCounting": (None, (P, B)),
    "GetFragmentCount": (L, (P,)),
    "GetLastRasterPath": (L, (P,)),
    "SetForceOrderedRaster": (None, (P, B)),
    "SetPairCapacityOverride": (None, (P, L)),
    "SetCoopRaster": (None, (P, L)),
    "SetWarmBinning": (None, (P, L)),
    "GetWarmBatchCount": (L, (P,)),
    "GetLooseBatchCount": (L, (P,)),
    "ExecuteCommands": (L, (P, P, L, P, L)),
    "SetWarmFaultInjection": (None, (P, L)),
    "GetWarmFailureCount": (L, (P,)),
    "SetSplitLimits": (None, (P, L, L)),
    "GetLastErrorString": (ctypes.c_char_p, ()),
    "ClearLastError": (None, ()),
    "SetDevice": (B, (L,)),
    "GetDeviceCount": (L, ()),
    "GetContextDevice": (L, (P,)),
    "Flush": (None, (P,)),
    "ResolvePending": (None, (P,)),
    "GetDeviceBufferPtr": (P, (P,)),
    "GetStreamPtr": (P, (P,)),
    "GetBufferAsUInt8Device": (None, (P, P)),
    "GetTextureBuffer": (None, (P, P)),
    "GetCommUniqueId": (B, (P,)),
    "CreateComm": (P, (L, L, P)),
    "DestroyComm": (None, (P,)),
    "SetShard": (None, (P, L, L)),
    "SetShardSlots": (None, (P, L, L, P)),
    "GetShardPattern": (L, (P, P)),
    "GatherFrameU8": (B, (P, P, L)),
    "GetFrameU8": (B, (P, P)),
    "GetFrameU8DevicePtr": (P, (P,)),
    "DeliverFrameU8": (L, (P, P)),
    "WaitFrameDelivered": (B, (P, L)),
    "AllocHostBuffer": (P, (L,)),
    "FreeHostBuffer": (None, (P,)),
    "DeliverFrameBands": (L, (P, P)),
    "AllocSharedHostBuffer": (P, (ctypes.c_char_p, L)),
    "FreeSharedHostBuffer": (None, (P, L)),
    "UnlinkSharedHostBuffer": (B, (ctypes.c_char_p,)),
    "GetFrameYUV420P": (B, (P, P)),
    "SetFrameFormat": (B, (P, L)),
    "GetFrameFormat": (L, (P,)),
    "GatherFramebuffer": (B, (P, P, L)),
    "GatherFramebufferEx": (B, (P, P, L, B)),
    "GatherFrameU8Local": (B, (P, L, L)),
    "GatherFrameU8LocalRccl": (B, (P, L, L, P)),
    "CreateMilthmHitEffectTextures": (B, (P, D, P, L, D, D, D, P)),
    "EnableKernelTiming": (None, (P, B)),
    "GetKernelTiming": (B, (P, ctypes.c_char_p, P, P)),
    "ResetKernelTiming": (None, (P,)),
    "SetKernelTimingFilter": (None, (P, ctypes.c_char_p)),
    "BeginCommandList": (None, (P,)),
    "EndCommandList": (None, (P,)),
    "FlushCommandList": (None, (P,)),
    "GetCommandListLength": (L, (P,)),
    "IsRecordingCommands": (B, (P,)),
}

# Audio clips (h:123-145).  OverlayAudioClip's startFrame is an
# i64 here: the reference binding declares c_double for it (Pybind:580), which
# lands the bool in the i64 register (the frame-unit overlay is broken there).
AUDIO_ABI = {
    "GetAudioClipBufferSizeFromData": (L, (L, L)),
    "GetAudioClipBufferSize": (L, (P,)),
    "CreateAudioClipFromBuffer": (P, (L, L, L, P)),
    "CreateAudioClipFromInt16Buffer": (P, (L, L, L, P)),
    "CreateSilentAudioClip": (P, (L, L, L)),
    "DestroyAudioClip": (None, (P,)),
    "CloneAudioClip": (P, (P,)),
    "ApplyResampleAudioClip": (None, (P, L, L)),
    "ResampleAudioClipLike": (None, (P, P)),
    "OverlayAudioClip": (L, (P, P, L, B)),
    "OverlayAudioClipSecond": (L, (P, P, D, B)),
    "SaveAudioClipAsWav": (P, (P,)),
    "GetAudioClipSampleRate": (L, (P,)),
    "GetAudioClipChannels": (L, (P,)),
    "GetAudioClipNumFrames": (L, (P,)),
    "GetAudioClipDuration": (D, (P,)),
    "GetWapperedBytesDataPtr": (P, (P,)),
    "GetWapperedBytesDataSize": (L, (P,)),
    "DestroyWapperedBytes": (None, (P,)),
    "ApplyVolumeGain": (None, (P, D)),
    "ApplyCutAudioClip": (None, (P, L, L)),
    "ApplySpeedAudioClip": (None, (P, D)),
    "GetAudioClipBuffer": (None, (P, P)),
}
AUDIO_DEVICE_ABI = {
    "OverlayAudioClipMany": (L, (P, P, P, L, B)),
    "OverlayAudioClipManySecond": (L, (P, P, P, L, B)),
    "GetAudioClipDevicePtr": (P, (P,)),
    "SetAudioStreamOrderedAlloc": (None, (B,)),
}

HIP_LIBRARY_ABI = {**REFERENCE_ABI, **TRIANGLE_ABI, **DEVICE_ABI, **AUDIO_ABI, **AUDIO_DEVICE_ABI}
ORACLE_ABI = {**REFERENCE_ABI, **TRIANGLE_ABI, **AUDIO_ABI, "OracleLastFragmentCount": (L, ()),
              "OracleGetTextureBuffer": (None, (P, P))}


def bind(lib: ctypes.CDLL, table: dict) -> ctypes.CDLL:
    """Declares restype/argtypes of every entry of `table` on `lib`;
    raises AttributeError naming the first missing export."""
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
