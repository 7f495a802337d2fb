// shs_post_internal.hpp -- launch interface of shs_post.hip (the passes after the raster path).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "shs_shard.hpp"

namespace shs_dev {

// PassTonemap + the present staging.  thr[k] (k = 1..255) is the smallest x = c / (1 + c) whose
// reference byte clamp(lround(pow(x, inv_gamma) * 255), 0, 255) is >= k (+inf when none is): the
// byte of any x is the number of thresholds <= x (the composite is monotone in x), so the GPU
// reproduces the host libm's pow / lround exactly without evaluating them.
struct TonemapParams {
    const float4 *hdr;      // W*H, rows y up (RT_ColorHDR)
    uint32_t *ldr;          // W*H RGBA8, rows y up (RT_ColorLDR), or null
    uint32_t *present;      // W*H RGBA8, rows top-down (upload_ldr_to_rgba8), or null
    int W, H;
    int rank, count;        // the camera pass's tile shard (count 1: the whole frame)
    ShardRegion reg;        // ... its region (reg.on) or interleaved tiles
    float exposure;         // max(0.0001, exposure)
    float inv_gamma;        // 1 / max(0.001, gamma): only steers the first guess
    float thr[256];         // thr[0] unused
};

// One channel: exposure, std::max(0, c) (NaN -> 0), Reinhard, then the byte by threshold count.
// The first guess comes from a fast pow; the two loops move it to the exact count.
__device__ __forceinline__ uint32_t tonemap_byte(float s, float exposure, float inv_gamma, const float *thr) {
    const float e = s * exposure;
    const float c = (0.0f < e) ? e : 0.0f;
    const float x = c / (1.0f + c);
    if (!(x >= 0.0f)) return 0u;   // c = inf: inf / inf = NaN, and the reference's lround(NaN) casts to 0
    const float g = x > 0.0f ? __builtin_amdgcn_exp2f(inv_gamma * __builtin_amdgcn_logf(x)) : 0.0f;
    int k = (int)fminf(fmaxf(g * 255.0f + 0.5f, 0.0f), 255.0f);
    while (k < 255 && thr[k + 1] <= x) ++k;
    while (k > 0 && thr[k] > x) --k;
    return (uint32_t)k;
}

// PassMotionBlur (passes/pass_motion_blur.hpp:38-170) with the pass's parameter clamps applied
// on the host (identical float expressions).
struct MotionBlurParams {
    const uint32_t *src;    // RT_ColorLDR RGBA8, rows y up
    const float *depth;     // RT_ColorDepthMotion depth, rows y up
    const float2 *motion;   // RT_ColorDepthMotion motion (px), rows y up
    uint32_t *dst;          // blurred RT_ColorLDR
    uint32_t *present;      // its upload_ldr_to_rgba8 staging (rows top-down), or null
    int W, H;
    int enable, samples;    // samples clamped to [4, 32]
    float strength, max_vel, min_vel, depth_eps, dt_scale;
};

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_tonemap(const shs_dev::TonemapParams &p, hipStream_t s);
hipError_t launch_motion_blur(const shs_dev::MotionBlurParams &p, hipStream_t s);
}  // namespace shs_internal
