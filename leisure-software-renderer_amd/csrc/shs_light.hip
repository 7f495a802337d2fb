// shs_light.hip -- gfx950 kernels for the Forward+ light-list binning:
//   k_depth_reduce   one wave per tile: min / max linear view depth of the tile's covered pixels
//                    (fp_stress_depth_reduce.comp:38-82) from the library depth buffer
//   k_light_cull     each workgroup projects the lights into LDS (resolve_cull_sphere +
//                    project_light_screen, fp_stress_light_cull.comp:47-127), then one wave per tile
//                    (or cluster) list -- up to 4 lists per wave -- tests them 64 at a time; a ballot +
//                    prefix keeps the reference's ascending light order and its `count < max_per_tile`
//                    truncation (:148-266).  Tile-sharded passes fill only this rank's lists.
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
__device__ __forceinline__ void project_light(const LightCullParams &p, const CullLight &L, float4 &a_out, float4 &b_out) {
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
    a_out = a;
    b_out = b;
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

// A workgroup projects the pass's lights into LDS (resolve_cull_sphere + project_light_screen,
// fp_stress_light_cull.comp:47-127: tile independent, so once per workgroup instead of once per
// (tile, light)), CULL_LDS_LIGHTS at a time, then each of its waves tests them against `lpw` lists.
// Lists come from `work` when the pass is tile-sharded (this rank's lists first, n_work of them;
// the rest get count 0), else list k is list k.
constexpr int CULL_LDS_LIGHTS = 1024;   // projected lights staged per round (2 float4 each)
constexpr int CULL_LPW = 4;             // lists per wave, at most

__device__ __forceinline__ bool light_in_list(const LightCullParams &p, float4 a, float4 b, float tminx, float tminy,
                                              float tmaxx, float tmaxy, float zlo, float zhi) {
    const float cx = a.x, cy = a.y, rpx = a.z, vd = a.w, rad = b.x;
    bool pass = b.w != 0.0f && !(((cx + rpx) + 16.0f) < tminx) && !(((cy + rpx) + 16.0f) < tminy) &&
                !(((cx - rpx) - 16.0f) > tmaxx) && !(((cy - rpx) - 16.0f) > tmaxy);
    if (pass && (p.mode == 2u || p.mode == 3u)) {
        const float pad = p.mode == 2u ? gmax(1.0f, gmax(rad * 0.35f, vd * 0.03f)) : gmax(0.8f, gmax(rad * 0.25f, vd * 0.02f));
        const float lmin = (vd - rad) - pad, lmax = (vd + rad) + pad;
        if ((lmax < zlo || lmin > zhi) && rpx < (float)p.tile_size * 4.0f) pass = false;
    }
    return pass;
}

struct ListBox {
    float tminx, tminy, tmaxx, tmaxy, zlo, zhi;
};

__device__ __forceinline__ ListBox list_box(const LightCullParams &p, const float2 *ranges, uint32_t list) {
    const uint32_t per_slice = p.tiles_x * p.tiles_y;
    const uint32_t tz = list / per_slice, rem = list % per_slice;
    const uint32_t tx = rem % p.tiles_x, ty = rem / p.tiles_x;
    const uint32_t ts = p.tile_size;
    ListBox o;
    o.tminx = (float)(tx * ts); o.tminy = (float)(ty * ts);
    o.tmaxx = (float)min((tx + 1) * ts, (uint32_t)p.W); o.tmaxy = (float)min((ty + 1) * ts, (uint32_t)p.H);
    const float near_z = gmax(p.zn, 0.001f), far_z = gmax(p.zf, near_z + 0.01f);
    o.zlo = 0.0f; o.zhi = 0.0f;
    if (p.mode == 3u) {   // cluster_slice_depth_bounds (:138-146)
        const float s0 = (float)tz / (float)p.z_slices, s1 = (float)(tz + 1) / (float)p.z_slices;
        o.zlo = near_z * powf(far_z / near_z, s0);
        o.zhi = near_z * powf(far_z / near_z, s1);
    } else if (p.mode == 2u) {   // tile depth range (:187-209)
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
        o.zlo = r0; o.zhi = r1;
    }
    return o;
}

__global__ __launch_bounds__(256) void k_light_cull(LightCullParams p, const CullLight *lights, const float2 *ranges,
                                                    const uint32_t *work, uint32_t n_work, uint32_t lpw, uint32_t *counts,
                                                    uint32_t *indices) {
    extern __shared__ float4 sl[];   // 2 * min(n_lights, CULL_LDS_LIGHTS)
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (work) {   // tile-sharded: the lists of other ranks' tiles read count 0
        for (uint32_t k = n_work + blockIdx.x * 256 + threadIdx.x; k < p.n_lists; k += gridDim.x * 256) counts[work[k]] = 0u;
    }
    const uint32_t k0 = (blockIdx.x * 4 + wave) * lpw;
    uint32_t list[CULL_LPW], count[CULL_LPW];
    ListBox box[CULL_LPW];
#pragma unroll
    for (int j = 0; j < CULL_LPW; ++j) {
        const uint32_t k = k0 + (uint32_t)j;
        list[j] = ((uint32_t)j < lpw && k < n_work) ? (work ? work[k] : k) : UINT32_MAX;
        count[j] = 0u;
        if (list[j] != UINT32_MAX) box[j] = list_box(p, ranges, list[j]);
    }
    const uint32_t maxp = p.max_per_tile;
    for (uint32_t base = 0; base < p.n_lights; base += CULL_LDS_LIGHTS) {
        const uint32_t m = min((uint32_t)CULL_LDS_LIGHTS, p.n_lights - base);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += 256) project_light(p, lights[base + i], sl[2 * i], sl[2 * i + 1]);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < CULL_LPW; ++j) {
            if (list[j] == UINT32_MAX) continue;   // wave-uniform
            const ListBox &bx = box[j];
            for (uint32_t c = 0; c < m && count[j] < maxp; c += 64) {
                const uint32_t li = c + lane;
                const bool pass = li < m && light_in_list(p, sl[2 * li], sl[2 * li + 1], bx.tminx, bx.tminy, bx.tmaxx,
                                                          bx.tmaxy, bx.zlo, bx.zhi);
                const uint64_t bal = __ballot(pass);
                const uint32_t slot = count[j] + lanes_below(bal);
                if (pass && slot < maxp) indices[(size_t)list[j] * maxp + slot] = base + li;
                count[j] += (uint32_t)__popcll(bal);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < CULL_LPW; ++j)
        if (list[j] != UINT32_MAX && lane == 0) counts[list[j]] = min(count[j], maxp);
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_light_cull(const LightCullParams &p, const CullLight *lights, const float *depth, float2 *ranges,
                             const uint32_t *work, uint32_t n_work, uint32_t *counts, uint32_t *indices, hipStream_t s) {
    if (p.mode == 0u || n_work == 0u) {   // no lists to fill: every count is 0
        return hipMemsetAsync(counts, 0, (size_t)p.n_lists * sizeof(uint32_t), s);
    }
    if (p.mode == 2u)
        hipLaunchKernelGGL(k_depth_reduce, dim3((p.tiles_x * p.tiles_y + 3) / 4), dim3(256), 0, s, p, depth, ranges);
    // lists per wave: enough waves to fill the chip (~8K), at most CULL_LPW
    const uint32_t lpw = std::max(1u, std::min((uint32_t)CULL_LPW, n_work / 8192u));
    const uint32_t waves = (n_work + lpw - 1) / lpw;
    const size_t lds = 2 * sizeof(float4) * std::min<size_t>(std::max(p.n_lights, 1u), CULL_LDS_LIGHTS);
    hipLaunchKernelGGL(k_light_cull, dim3(std::max(1u, (waves + 3) / 4)), dim3(256), lds, s, p, lights, ranges, work, n_work,
                       lpw, counts, indices);
    return hipGetLastError();
}

}  // namespace shs_internal
