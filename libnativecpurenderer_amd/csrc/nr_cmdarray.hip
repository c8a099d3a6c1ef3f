// nr_cmdarray.hip — a frame's draw and state calls submitted as one packed
// array (ExecuteCommands), so a caller that issues hundreds of small calls per
// frame (milrenderer.py:865-1038: a transform, a draw and a restore per note)
// crosses the Python -> C boundary once per frame instead of once per call.
// The reference's own attempt at batching a frame is the unfinished recorder
// MultiThreadedVideoRenderContextPreparer (Pybind:302-367).
//
// Each command runs the same entry point as the single call it stands for, in
// array order, so the result is the immediate sequence's bit for bit; inside
// a command list (BeginCommandList) the draws are queued and run as one
// launch at the flush, as single calls are.
//
// Array layout: f64 words, each command = opcode followed by its arguments
// (ExecOp below; arity fixed per opcode).  Textures are indices into the
// `textures` array of the call; SetPixel / ApplyPixel coordinates are whole
// numbers stored as f64.
#include "nr_common.h"

extern "C" {
void SaveContextState(RenderContext* ctx);
bool RestoreContextState(RenderContext* ctx);
void SetTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f);
void ApplyTransform(RenderContext* ctx, f64 a, f64 b, f64 c, f64 d, f64 e, f64 f);
void Scale(RenderContext* ctx, f64 sx, f64 sy);
void Translate(RenderContext* ctx, f64 tx, f64 ty);
void Rotate(RenderContext* ctx, f64 angle);
void SetColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);
void ApplyColorTransform(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);
void SetColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);
void FillColor(RenderContext* ctx, f64 r, f64 g, f64 b, f64 a);
void DrawTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height);
void DrawSplittedTexture(RenderContext* ctx, Texture* tex, f64 x, f64 y, f64 width, f64 height, f64 uStart,
                         f64 uEnd, f64 vStart, f64 vEnd);
void DrawRect(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height, f64 r, f64 g, f64 b, f64 a);
void DrawLine(RenderContext* ctx, f64 x1, f64 y1, f64 x2, f64 y2, f64 width, f64 r, f64 g, f64 b, f64 a);
void DrawCircle(RenderContext* ctx, f64 x, f64 y, f64 radius, f64 r, f64 g, f64 b, f64 a);
void DrawVerticalGrd(RenderContext* ctx, f64 x, f64 y, f64 width, f64 height, f64 top_r, f64 top_g, f64 top_b,
                     f64 top_a, f64 bottom_r, f64 bottom_g, f64 bottom_b, f64 bottom_a);
bool SetPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a);
bool ApplyPixel(RenderContext* ctx, i64 x, i64 y, f64 r, f64 g, f64 b, f64 a);
}

namespace {

enum ExecOp {
    OP_SAVE = 0, OP_RESTORE, OP_SET_TRANSFORM, OP_APPLY_TRANSFORM, OP_SCALE, OP_TRANSLATE, OP_ROTATE,
    OP_SET_CT, OP_APPLY_CT, OP_SET_COLOR, OP_FILL_COLOR, OP_TEXTURE, OP_SPLIT_TEXTURE, OP_RECT, OP_LINE,
    OP_CIRCLE, OP_VGRD, OP_SET_PIXEL, OP_APPLY_PIXEL, OP_COUNT_
};
// arguments per opcode (after the opcode word)
constexpr int kArity[OP_COUNT_] = {0, 0, 6, 6, 2, 2, 1, 4, 4, 4, 4, 5, 9, 8, 9, 7, 12, 6, 6};

// A whole number that fits i64 (pixel coordinates, texture indices).
bool as_i64(f64 v, i64* out) {
    if (!(v >= -9.2e18 && v <= 9.2e18) || v != (f64)(i64)v) return false;
    *out = (i64)v;
    return true;
}

}  // namespace

extern "C" {

// NEW: runs `nwords` f64 words of packed commands on ctx, in order.  Returns
// the number of commands run, or -1 when the array is malformed (unknown
// opcode, truncated command, texture index outside [0, ntextures), fractional
// index or pixel coordinate): the commands before the bad one have run, the
// rest have not, and the error is latched (GetLastErrorString).
i64 ExecuteCommands(RenderContext* ctx, const f64* words, i64 nwords, Texture* const* textures, i64 ntextures) {
    if (!ctx || (nwords > 0 && !words)) {
        nr_set_error_msg("ExecuteCommands: null context or array");
        return -1;
    }
    i64 pos = 0, ncmd = 0;
    auto fail = [&](const char* why) {
        char buf[160];
        snprintf(buf, sizeof buf, "ExecuteCommands: %s at word %ld (command %ld)", why, (long)pos, (long)ncmd);
        nr_set_error_msg(buf);
        return (i64)-1;
    };
    while (pos < nwords) {
        i64 op = -1;
        if (!as_i64(words[pos], &op) || op < 0 || op >= OP_COUNT_) return fail("unknown opcode");
        if (pos + 1 + kArity[op] > nwords) return fail("truncated command");
        const f64* a = words + pos + 1;
        Texture* tex = nullptr;
        if (op == OP_TEXTURE || op == OP_SPLIT_TEXTURE) {
            i64 ti = -1;
            if (!as_i64(a[0], &ti) || ti < 0 || ti >= ntextures || !textures || !textures[ti])
                return fail("bad texture index");
            tex = textures[ti];
        }
        i64 px = 0, py = 0;
        if ((op == OP_SET_PIXEL || op == OP_APPLY_PIXEL) && (!as_i64(a[0], &px) || !as_i64(a[1], &py)))
            return fail("fractional pixel coordinate");
        switch (op) {
            case OP_SAVE: SaveContextState(ctx); break;
            case OP_RESTORE: RestoreContextState(ctx); break;
            case OP_SET_TRANSFORM: SetTransform(ctx, a[0], a[1], a[2], a[3], a[4], a[5]); break;
            case OP_APPLY_TRANSFORM: ApplyTransform(ctx, a[0], a[1], a[2], a[3], a[4], a[5]); break;
            case OP_SCALE: Scale(ctx, a[0], a[1]); break;
            case OP_TRANSLATE: Translate(ctx, a[0], a[1]); break;
            case OP_ROTATE: Rotate(ctx, a[0]); break;
            case OP_SET_CT: SetColorTransform(ctx, a[0], a[1], a[2], a[3]); break;
            case OP_APPLY_CT: ApplyColorTransform(ctx, a[0], a[1], a[2], a[3]); break;
            case OP_SET_COLOR: SetColor(ctx, a[0], a[1], a[2], a[3]); break;
            case OP_FILL_COLOR: FillColor(ctx, a[0], a[1], a[2], a[3]); break;
            case OP_TEXTURE: DrawTexture(ctx, tex, a[1], a[2], a[3], a[4]); break;
            case OP_SPLIT_TEXTURE: DrawSplittedTexture(ctx, tex, a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8]); break;
            case OP_RECT: DrawRect(ctx, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]); break;
            case OP_LINE: DrawLine(ctx, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8]); break;
            case OP_CIRCLE: DrawCircle(ctx, a[0], a[1], a[2], a[3], a[4], a[5], a[6]); break;
            case OP_VGRD:
                DrawVerticalGrd(ctx, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11]);
                break;
            case OP_SET_PIXEL: SetPixel(ctx, px, py, a[2], a[3], a[4], a[5]); break;
            case OP_APPLY_PIXEL: ApplyPixel(ctx, px, py, a[2], a[3], a[4], a[5]); break;
        }
        pos += 1 + kArity[op];
        ++ncmd;
    }
    return ncmd;
}

}  // extern "C"
