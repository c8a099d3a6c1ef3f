// nr_shader.hip — texture preparation: the procedural hit-
// effect texture of milrenderer (cpp:1318-1440, ShaderUtils +
// GetMilthmHitEffectPixel + CreateMilthmHitEffectTexture), one thread per
// texel.
//
// Semantics kept from the reference:
//  * every expression in f64, in the reference's order, no FMA
//    (-ffp-contract=off, Appendix A.1);
//  * `abs(atan2(...))` (cpp:1388) is the double overload: the reference build
//    includes the FFmpeg headers, whose libavutil/common.h includes <math.h>,
//    and libstdc++'s <math.h> brings std::abs(double) into the global
//    namespace (without it, unqualified abs would be ::abs(int) and truncate);
//  * texel (i, j) is stored at (i * h + j) * 4 and the mask's alpha is read at
//    the same index (GetPixelChannel, cpp:1413-1415): column-major, so the
//    output is the transpose of the row-major image for square masks;
//  * a mask without alpha gives NULL (cpp:1418).
// The noise value n of a texel does not depend on the threshold t, so the
// batched entry point (the n textures Helpers.create_milthm_hit_effect_textures
// makes, Pybind:34-48) evaluates it once per texel and writes every texture.
//
// Parity: sin and atan2 are the device library's f64 versions (within an ULP
// of glibc's); the output alpha is binary (n < t ? 0 : 1), and an ULP of sin
// moves n by ~1e-11 (rand() scales sin by 43758.5453), so a texel can differ
// only when n lies within that distance of t.
#include "nr_common.h"

namespace {

struct v2 {
    f64 x, y;
};

__device__ __forceinline__ f64 sh_fract(f64 x) { return x - floor(x); }

// rand(n) = fract(sin(dot(n, (12.9898, 78.233))) * 43758.5453), cpp:1341-1343
__device__ __forceinline__ f64 sh_rand(v2 n) { return sh_fract(sin(n.x * 12.9898 + n.y * 78.233) * 43758.5453); }

__device__ __forceinline__ f64 sh_mix(f64 a, f64 b, f64 t) { return a + (b - a) * t; }

// value noise, cpp:1370-1381
__device__ __forceinline__ f64 sh_noise(v2 p) {
    const v2 ip = {floor(p.x), floor(p.y)};
    const v2 u = {sh_fract(p.x), sh_fract(p.y)};
    const f64 a = sh_rand(ip);
    const f64 b = sh_rand({ip.x + 1.0, ip.y + 0.0});
    const f64 c = sh_rand({ip.x + 0.0, ip.y + 1.0});
    const f64 d = sh_rand({ip.x + 1.0, ip.y + 1.0});
    // u * u * (vec2{3, 3} - 2.0 * u), component-wise, left to right
    const v2 s = {u.x * u.x * (3.0 - 2.0 * u.x), u.y * u.y * (3.0 - 2.0 * u.y)};
    return sh_mix(sh_mix(a, b, s.x), sh_mix(c, d, s.x), s.y);
}

// circularNoise(uv, density, seed), cpp:1384-1401
__device__ __forceinline__ f64 sh_circular_noise(v2 uv, f64 density, f64 seed) {
    const v2 center = {uv.x - 0.5, uv.y - 0.5};
    const f64 radius = sqrt(center.x * center.x + center.y * center.y) * density;
    f64 angle = fabs(atan2(center.y, center.x));
    if (uv.y > 0.5) angle += sin(angle) * 2.0;
    const v2 off = {seed * 100.0, seed * 100.0};
    const v2 polar = {radius + off.x, angle + off.y};
    f64 n = 0.0;
    n += sh_noise(polar) * 0.7;
    n += sh_noise({polar.x * 2.0, polar.y * 2.0}) * 0.3;
    n += sh_noise({polar.x * 4.0, polar.y * 4.0}) * 0.1;
    return n;
}

// One thread per texel (i, j) of every requested texture: the noise once,
// then texture k gets alpha (n < t_k ? 0 : 1) * mask_a.
__global__ void k_hit_effect(const f64* __restrict__ mask, i64 w, i64 h, f64 seed, const f64* __restrict__ ts,
                             f64* const* __restrict__ outs, int nt, f64 r, f64 g, f64 b) {
    const i64 n = w * h;
    for (i64 q = (i64)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (i64)gridDim.x * blockDim.x) {
        const i64 i = q / h, j = q - i * h;   // q = i * h + j: the reference's storage index
        const f64 nv = sh_circular_noise({(f64)i / w, (f64)j / h}, 50.0, seed);
        const f64 ma = mask[q * 4 + 3];
        for (int k = 0; k < nt; ++k) {
            const f64 a = nv < ts[k] ? 0.0 : 1.0;
            f64* o = outs[k] + q * 4;
            o[0] = r; o[1] = g; o[2] = b; o[3] = a * ma;
        }
    }
}

__global__ void k_hit_pixel(f64 seed, f64 t, f64 x, f64 y, f64* out) {
    *out = sh_circular_noise({x, y}, 50.0, seed) < t ? 0.0 : 1.0;
}

constexpr int MAX_BATCH = 4096;

}  // namespace

extern "C" {

// NEW: n hit-effect textures of one mask and seed, texture k at threshold
// ts[k], written to out[k] (one launch; the batched form of cpp:1416-1438).
// Returns false (out untouched) when the mask has no alpha.
bool CreateMilthmHitEffectTextures(Texture* mask, f64 seed, const f64* ts, i64 n, f64 r, f64 g, f64 b,
                                   Texture** out) {
    if (!mask || !mask->enableAlpha || n < 0 || n > MAX_BATCH) {
        if (n > MAX_BATCH) nr_set_error_msg("CreateMilthmHitEffectTextures: at most 4096 textures per call");
        return false;
    }
    NR_CHECK(hipSetDevice(mask->device));
    if (mask->aliasOf) nr_materialize_color(mask->aliasOf);
    hipStream_t s = nr_stream_for(mask->device);
    if (n == 0) return true;
    for (i64 k = 0; k < n; ++k) out[k] = nr_new_texture(mask->width, mask->height, true);
    const i64 texels = mask->width * mask->height;
    if (texels > 0) {
        // thresholds + output pointers: one small H2D copy (pinned staging)
        const size_t bytes = (size_t)n * (sizeof(f64) + sizeof(f64*));
        void* host = nullptr;
        void* dev = nullptr;
        NR_CHECK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
        NR_CHECK(hipMalloc(&dev, bytes));
        f64* hts = static_cast<f64*>(host);
        f64** hptr = reinterpret_cast<f64**>(hts + n);
        for (i64 k = 0; k < n; ++k) {
            hts[k] = ts[k];
            hptr[k] = out[k]->buffer;
        }
        NR_CHECK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
        const f64* dts = static_cast<const f64*>(dev);
        f64* const* dptr = reinterpret_cast<f64* const*>(dts + n);
        const int grid = (int)std::min<i64>((texels + 255) / 256, 8192);
        hipLaunchKernelGGL(k_hit_effect, dim3(grid), dim3(256), 0, s, mask->buffer, mask->width, mask->height, seed,
                           dts, dptr, (int)n, r, g, b);
        NR_CHECK(hipGetLastError());
        NR_CHECK(hipStreamSynchronize(s));   // the device and pinned staging are released below
        NR_CHECK(hipFree(dev));
        NR_CHECK(hipHostFree(host));
    }
    return true;
}

// cpp:1416-1438 (h:151)
Texture* CreateMilthmHitEffectTexture(Texture* mask, f64 seed, f64 t, f64 r, f64 g, f64 b) {
    Texture* out = nullptr;
    if (!CreateMilthmHitEffectTextures(mask, seed, &t, 1, r, g, b, &out)) return nullptr;
    return out;
}

// cpp:1405-1410 (h:150; inline in the reference, so not exported there)
void GetMilthmHitEffectPixel(f64 seed, f64 t, f64 x, f64 y, f64* a) {
    int dev = 0;
    NR_CHECK(hipGetDevice(&dev));
    hipStream_t s = nr_stream_for(dev);
    f64* d = nullptr;
    NR_CHECK(hipMalloc(&d, sizeof(f64)));
    hipLaunchKernelGGL(k_hit_pixel, dim3(1), dim3(1), 0, s, seed, t, x, y, d);
    NR_CHECK(hipGetLastError());
    NR_CHECK(hipMemcpyAsync(a, d, sizeof(f64), hipMemcpyDeviceToHost, s));
    NR_CHECK(hipStreamSynchronize(s));
    NR_CHECK(hipFree(d));
}

}  // extern "C"
