// shs_post.hip -- gfx950 kernels for the step after the raster path:
//   PassTonemap::execute     shs-renderer-lib/include/shs/passes/pass_tonemap.hpp:36-83
//   upload_ldr_to_rgba8      exp-plumbing/hello_pass_basics.cpp:102-119 (the SDL texture staging)
//   PassMotionBlur::execute  shs-renderer-lib/include/shs/passes/pass_motion_blur.hpp:38-170
// (paths relative to /root/reference/cpp-folders/src/).  One launch reads the HDR target once and
// writes the LDR target and / or the present staging once: 16 B read + 4 or 8 B written per pixel,
// HBM-bound.
#include <float.h>

#include "shs_post_internal.hpp"

namespace shs_dev {

// tonemap_byte: shs_post_internal.hpp (shared with k_lib_resolve's fused tonemap)

__device__ __forceinline__ void tonemap_pixel(const TonemapParams &p, const float *thr, int x, int y) {
    const float4 s = p.hdr[(size_t)y * p.W + x];
    const uint32_t rgba = tonemap_byte(s.x, p.exposure, p.inv_gamma, thr) |
                          (tonemap_byte(s.y, p.exposure, p.inv_gamma, thr) << 8) |
                          (tonemap_byte(s.z, p.exposure, p.inv_gamma, thr) << 16) | (255u << 24);
    if (p.ldr) __builtin_nontemporal_store(rgba, &p.ldr[(size_t)y * p.W + x]);
    if (p.present) __builtin_nontemporal_store(rgba, &p.present[(size_t)(p.H - 1 - y) * p.W + x]);
}

// 64 x 4 pixels per workgroup: each wave reads 64 float4 of one row (1 KB) and writes 256 B rows.
__global__ __launch_bounds__(256) void k_tonemap(TonemapParams p) {
    __shared__ float thr[256];
    thr[threadIdx.x] = p.thr[threadIdx.x];
    __syncthreads();
    const int x = (int)blockIdx.x * 64 + (int)(threadIdx.x & 63u);
    const int y = (int)blockIdx.y * 4 + (int)(threadIdx.x >> 6);
    if (x >= p.W || y >= p.H) return;
    tonemap_pixel(p, thr, x, y);
}

// Tile-sharded camera pass: only the rank's 32x32 tiles (rows y up, tile % count == rank or its region) hold
// pixels, so one workgroup per owned tile maps them (32-px rows: 512-B reads, 128-B writes).
__global__ __launch_bounds__(256) void k_tonemap_tiles(TonemapParams p) {
    __shared__ float thr[256];
    thr[threadIdx.x] = p.thr[threadIdx.x];
    __syncthreads();
    const int tiles_x = (p.W + 31) / 32;
    const int t = shard_tile(p.rank, p.count, p.reg, (int)blockIdx.x, tiles_x);
    const int x = (t % tiles_x) * 32 + (int)(threadIdx.x & 31u);
    const int y0 = (t / tiles_x) * 32 + (int)(threadIdx.x >> 5);
    if (x >= p.W) return;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (y0 + 8 * k < p.H) tonemap_pixel(p, thr, x, y0 + 8 * k);
}

// std::lround then the (int) cast of the reference: half away from zero, 64-bit, then truncated.
// x86-64's lround returns LONG_MIN (cvtss2si's "integer indefinite") for NaN and |v| >= 2^63, and
// the (int) cast of LONG_MIN is 0; on AMDGPU that conversion would be poison, so it is explicit.
__device__ __forceinline__ int lround_int(float v) {
    const float r = roundf(v);
    if (!(fabsf(r) < 9.2233720e18f)) return 0;
    return (int)(long long)r;
}

__device__ __forceinline__ int clamp_i(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// One pixel of PassMotionBlur: the velocity (scaled, clamped), `samples` taps along it at
// lround(p + v * t), depth-rejected, averaged as floats and rounded back to bytes.
__global__ __launch_bounds__(256) void k_motion_blur(MotionBlurParams p) {
    const int x = (int)blockIdx.x * 64 + (int)(threadIdx.x & 63u);
    const int y = (int)blockIdx.y * 4 + (int)(threadIdx.x >> 6);
    if (x >= p.W || y >= p.H) return;
    const size_t o = (size_t)y * p.W + x;
    uint32_t out = p.src[o];
    if (p.enable) {
        const float2 mv = p.motion[o];
        float vx = mv.x * p.strength * p.dt_scale;
        float vy = mv.y * p.strength * p.dt_scale;
        const float len = sqrtf(vx * vx + vy * vy);
        if (!(len < p.min_vel)) {
            if (len > p.max_vel && len > 1e-6f) {
                const float s = p.max_vel / len;
                vx *= s;
                vy *= s;
            }
            const float cd = p.depth[o];
            float ar = 0.0f, ag = 0.0f, ab = 0.0f, aw = 0.0f;
            for (int i = 0; i < p.samples; ++i) {
                const float t = ((float)i / (float)(p.samples - 1) - 0.5f);
                const int sx = clamp_i(lround_int((float)x + vx * t), 0, p.W - 1);
                const int sy = clamp_i(lround_int((float)y + vy * t), 0, p.H - 1);
                const size_t so = (size_t)sy * p.W + sx;
                if (fabsf(p.depth[so] - cd) > p.depth_eps) continue;
                const uint32_t c = p.src[so];
                ar += (float)(c & 255u);
                ag += (float)((c >> 8) & 255u);
                ab += (float)((c >> 16) & 255u);
                aw += 1.0f;
            }
            if (!(aw < 1.0f)) {
                out = (uint32_t)clamp_i(lround_int(ar / aw), 0, 255) | ((uint32_t)clamp_i(lround_int(ag / aw), 0, 255) << 8) |
                      ((uint32_t)clamp_i(lround_int(ab / aw), 0, 255) << 16) | (255u << 24);
            }
        }
    }
    p.dst[o] = out;
    if (p.present) p.present[(size_t)(p.H - 1 - y) * p.W + x] = out;
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_motion_blur(const MotionBlurParams &p, hipStream_t s) {
    const dim3 grid((unsigned)((p.W + 63) / 64), (unsigned)((p.H + 3) / 4));
    hipLaunchKernelGGL(k_motion_blur, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_tonemap(const TonemapParams &p, hipStream_t s) {
    if (p.count > 1) {
        const int n_tiles = ((p.W + 31) / 32) * ((p.H + 31) / 32);
        const int n_owned = shard_n_owned(p.rank, p.count, p.reg, n_tiles);
        if (n_owned > 0) hipLaunchKernelGGL(k_tonemap_tiles, dim3((unsigned)n_owned), dim3(256), 0, s, p);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((p.W + 63) / 64), (unsigned)((p.H + 3) / 4));
    hipLaunchKernelGGL(k_tonemap, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace shs_internal
