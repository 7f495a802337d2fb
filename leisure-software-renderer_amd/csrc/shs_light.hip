// shs_light.hip -- gfx950 kernels for the Forward+ light-list binning:
//   k_light_project  one thread per light: resolve_cull_sphere + project_light_screen
//                    (shaders/vulkan/fp_stress_light_cull.comp:47-127) -- tile independent, so done
//                    once per light instead of once per (tile, light) as the GLSL does
//   k_depth_reduce   one wave per tile: min / max linear view depth of the tile's covered pixels
//                    (fp_stress_depth_reduce.comp:38-82) from the library depth buffer
//   k_light_cull     one wave per tile (or cluster): the projected lights staged in LDS, tested 64 at a
//                    time; a ballot + prefix keeps the reference's ascending light order and its
//                    `count < max_per_tile` truncation (fp_stress_light_cull.comp:148-266)
// Paths relative to /root/reference/cpp-folders/src/shs-renderer-lib/.
#include <algorithm>

#include "shs_lib_device.hpp"
#include "shs_light_internal.hpp"
#include "shs_wave.hpp"

namespace shs_dev {

__device__ __forceinline__ float gmax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float gmin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }

// mat4 * vec4 in GLM order
__device__ __forceinline__ void mv4(const float *m, const float (&v)[4], float (&o)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * v[0] + m[4 + r] * v[1]) + (m[8 + r] * v[2] + m[12 + r] * v[3]);
}

// Projected light record: cx, cy, radius_px, view_depth, cull radius, -, -, valid.
__global__ __launch_bounds__(256) void k_light_project(LightCullParams p, const CullLight *lights, float4 *proj) {
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i >= (int)p.n_lights) return;
    const CullLight L = lights[i];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (L.type_shape_flags[2] & 1u) {   // SHS_LIGHT_FLAG_ENABLED
        // resolve_cull_sphere (:47-96), point / spot branch + AABB fallback
        float s[4] = {L.cull_sphere[0], L.cull_sphere[1], L.cull_sphere[2], L.cull_sphere[3]};
        const uint32_t type = L.type_shape_flags[0];
        const float shading_range = gmax(L.position_range[3], 0.0f);
        if ((type == 2u || type == 1u) && (s[3] <= 0.0f || s[3] < shading_range)) {
            s[0] = L.position_range[0]; s[1] = L.position_range[1]; s[2] = L.position_range[2]; s[3] = shading_range;
        }
        if (!(s[3] > 0.0f)) {
            float e[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) e[k] = gmax((L.cull_aabb_max[k] - L.cull_aabb_min[k]) * 0.5f, 0.0f);
            const float r = sqrtf((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]);
            if (r > 0.0f) {
#pragma unroll
                for (int k = 0; k < 3; ++k) s[k] = (L.cull_aabb_min[k] + L.cull_aabb_max[k]) * 0.5f;
                s[3] = r;
            } else {
                s[0] = L.position_range[0]; s[1] = L.position_range[1]; s[2] = L.position_range[2];
                s[3] = gmax(L.position_range[3], 0.0f);
            }
        }
        // project_light_screen (:98-127)
        const float r = s[3];
        const float p4[4] = {s[0], s[1], s[2], 1.0f};
        float v4[4], c4[4];
        mv4(p.view, p4, v4);
        const float near_z = gmax(p.zn, 0.001f);
        if (!(v4[2] + r <= near_z)) {
            const float vd = gmax(near_z, v4[2]);
            mv4(p.proj, v4, c4);
            const float W = (float)max(p.W, 1), H = (float)max(p.H, 1);
            float cx, cy, rpx;
            if (c4[3] <= 1e-6f || (v4[2] - r) <= near_z) {
                cx = W * 0.5f; cy = H * 0.5f;
                rpx = (float)max(max(p.W, 1), max(p.H, 1));
            } else {
                const float nx = c4[0] / c4[3], ny = c4[1] / c4[3];
                cx = (nx * 0.5f + 0.5f) * W;
                cy = (0.5f - ny * 0.5f) * H;
                const float rp = fabsf(((r * p.proj[5]) * H) / vd);
                const float inflate = 1.0f + gclamp(r / gmax(vd, near_z), 0.0f, 2.5f) * 0.65f;
                rpx = rp * inflate + 4.0f;
            }
            a = make_float4(cx, cy, rpx, vd);
            b = make_float4(r, 0.0f, 0.0f, 1.0f);
        }
    }
    proj[2 * i] = a;
    proj[2 * i + 1] = b;
}

// fp_stress_depth_reduce.comp; the library depth is linear view depth (rasterizer.hpp:354-357),
// inverted as zn + d * (zf - zn); a perspective LH_NO depth uses the shader's own reconstruction.
__device__ __forceinline__ float depth_to_view(const LightCullParams &p, float d01) {
    const float near_z = gmax(p.zn, 0.001f);
    const float far_z = gmax(p.zf, near_z + 0.01f);
    const float d = gclamp(d01, 0.0f, 1.0f);
    if (p.depth_linear) return p.zn + d * (p.zf - p.zn);
    return (near_z * far_z) / gmax(far_z - d * (far_z - near_z), 1e-5f);
}

__device__ __forceinline__ bool list_owned(const LightCullParams &p, uint32_t tx, uint32_t ty) {
    if (p.count <= 1 || (32u % p.tile_size) != 0u) return true;
    const uint32_t px = tx * p.tile_size, py_down = ty * p.tile_size;
    // bin tiles are counted in library rows (y-up): the tile's rows are H-1-py_down .. downwards
    const int row_up = p.H - 1 - (int)py_down;
    const int bx = (int)px / 32, by = row_up / 32;
    const int tiles_x = (p.W + 31) / 32;
    return ((by * tiles_x + bx) % p.count) == p.rank;
}

__global__ __launch_bounds__(256) void k_depth_reduce(LightCullParams p, const float *depth, float2 *ranges) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t tile = blockIdx.x * 4 + wave;
    if (tile >= p.tiles_x * p.tiles_y) return;
    const uint32_t tx = tile % p.tiles_x, ty = tile / p.tiles_x;
    const uint32_t x0 = tx * p.tile_size, y0 = ty * p.tile_size;
    const uint32_t x1 = min(x0 + p.tile_size, (uint32_t)p.W), y1 = min(y0 + p.tile_size, (uint32_t)p.H);
    const uint32_t w = x1 - x0, n = w * (y1 - y0);
    float mn = 1e30f, mx = 0.0f;
    bool any = false;
    for (uint32_t k = lane; k < n; k += 64) {
        const uint32_t px = x0 + k % w, py = y0 + k / w;
        const float d = depth[(size_t)(p.H - 1 - (int)py) * p.W + px];
        if (d >= 1.0f) continue;
        const float vz = depth_to_view(p, d);
        mn = gmin(mn, vz);
        mx = gmax(mx, vz);
        any = true;
    }
    for (int o = 32; o > 0; o >>= 1) {
        mn = gmin(mn, __shfl_xor(mn, o));
        mx = gmax(mx, __shfl_xor(mx, o));
    }
    const bool a = __ballot(any) != 0;
    if (lane == 0) ranges[tile] = a ? make_float2(mn, mx) : make_float2(0.0f, 0.0f);
}

constexpr int CULL_LDS_LIGHTS = 1024;   // projected lights staged per pass (32 KB)

__global__ __launch_bounds__(256) void k_light_cull(LightCullParams p, const float4 *proj, const float2 *ranges,
                                                    uint32_t *counts, uint32_t *indices) {
    __shared__ float4 sl[CULL_LDS_LIGHTS * 2];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t list = blockIdx.x * 4 + wave;
    const uint32_t per_slice = p.tiles_x * p.tiles_y;
    const bool valid_list = list < p.n_lists;
    const uint32_t tz = valid_list ? list / per_slice : 0u, rem = valid_list ? list % per_slice : 0u;
    const uint32_t tx = rem % p.tiles_x, ty = rem / p.tiles_x;
    const bool work = valid_list && p.mode != 0u && list_owned(p, tx, ty);
    const uint32_t ts = p.tile_size, maxp = p.max_per_tile;
    const float tminx = (float)(tx * ts), tminy = (float)(ty * ts);
    const float tmaxx = (float)min((tx + 1) * ts, (uint32_t)p.W), tmaxy = (float)min((ty + 1) * ts, (uint32_t)p.H);
    const float near_z = gmax(p.zn, 0.001f), far_z = gmax(p.zf, near_z + 0.01f);
    float zlo = 0.0f, zhi = 0.0f;
    if (p.mode == 3u) {   // cluster_slice_depth_bounds (:138-146)
        const float s0 = (float)tz / (float)p.z_slices, s1 = (float)(tz + 1) / (float)p.z_slices;
        zlo = near_z * powf(far_z / near_z, s0);
        zhi = near_z * powf(far_z / near_z, s1);
    } else if (p.mode == 2u && work) {   // tile depth range (:187-209)
        const float2 rg = ranges[ty * p.tiles_x + tx];
        float r0 = rg.x, r1 = rg.y;
        if (r0 <= 0.0f && r1 <= 0.0f) { r0 = near_z; r1 = far_z; }
        r0 = gclamp(r0, near_z, far_z);
        r1 = gclamp(r1, near_z, far_z);
        const float expand = gmax(0.05f, r1 * 0.0015f);
        r0 = gclamp(r0 - expand, near_z, far_z);
        r1 = gclamp(r1 + expand, near_z, far_z);
        if (r1 < r0) r1 = r0;
        r1 = gmin(far_z, gmax(r1, r0 + gmax(0.02f, r0 * 0.0005f)));
        zlo = r0; zhi = r1;
    }
    uint32_t count = 0;
    for (uint32_t base = 0; base < p.n_lights; base += CULL_LDS_LIGHTS) {
        const uint32_t m = min((uint32_t)CULL_LDS_LIGHTS, p.n_lights - base);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 2 * m; i += 256) sl[i] = proj[2 * base + i];
        __syncthreads();
        if (!work) continue;
        for (uint32_t c = 0; c < m && count < maxp; c += 64) {
            const uint32_t li = c + lane;
            bool pass = false;
            if (li < m) {
                const float4 a = sl[2 * li], b = sl[2 * li + 1];
                const float cx = a.x, cy = a.y, rpx = a.z, vd = a.w, rad = b.x;
                pass = b.w != 0.0f && !(((cx + rpx) + 16.0f) < tminx) && !(((cy + rpx) + 16.0f) < tminy) &&
                       !(((cx - rpx) - 16.0f) > tmaxx) && !(((cy - rpx) - 16.0f) > tmaxy);
                if (pass && (p.mode == 2u || p.mode == 3u)) {
                    const float pad = p.mode == 2u ? gmax(1.0f, gmax(rad * 0.35f, vd * 0.03f)) : gmax(0.8f, gmax(rad * 0.25f, vd * 0.02f));
                    const float lmin = (vd - rad) - pad, lmax = (vd + rad) + pad;
                    if ((lmax < zlo || lmin > zhi) && rpx < (float)ts * 4.0f) pass = false;
                }
            }
            const uint64_t bal = __ballot(pass);
            const uint32_t slot = count + lanes_below(bal);
            if (pass && slot < maxp) indices[(size_t)list * maxp + slot] = base + li;
            count += (uint32_t)__popcll(bal);
        }
    }
    if (valid_list && lane == 0) counts[list] = work ? min(count, maxp) : 0u;
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_light_cull(const LightCullParams &p, const CullLight *lights, float4 *proj, const float *depth, float2 *ranges,
                             uint32_t *counts, uint32_t *indices, hipStream_t s) {
    if (p.n_lights > 0)
        hipLaunchKernelGGL(k_light_project, dim3((p.n_lights + 255) / 256), dim3(256), 0, s, p, lights, proj);
    if (p.mode == 2u)
        hipLaunchKernelGGL(k_depth_reduce, dim3((p.tiles_x * p.tiles_y + 3) / 4), dim3(256), 0, s, p, depth, ranges);
    hipLaunchKernelGGL(k_light_cull, dim3(std::max(1u, (p.n_lists + 3) / 4)), dim3(256), 0, s, p, proj, ranges, counts, indices);
    return hipGetLastError();
}

}  // namespace shs_internal
