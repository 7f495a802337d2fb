// shs_abi_lightbin.cpp -- C ABI of the software library's CPU light binning on the GPU (SURVEY.md 8a
// row a15): build_light_bin_culling (shs-renderer-lib/include/shs/lighting/light_culling_runtime.hpp
// :266-371) over the lights' SceneShape world AABBs.  The per-call host part -- inverse(view_proj),
// the camera-frustum pre-pass of every light (extract_frustum_planes + classify_vs_frustum), the
// lights' Jolt bounding spheres and the per-tile / per-slice cell depths -- runs here in the same
// float operations; the per-bin work runs in k_light_bin (shs_lightbin.hip).
#include <cmath>
#include <cstring>
#include <vector>

#include "shs_ctx.hpp"
#include "shs_glm.hpp"
#include "shs_lightbin_internal.hpp"

namespace {

struct HPlane { float nx, ny, nz, d; };

float smax(float a, float b) { return (a < b) ? b : a; }   // std::max

float hdot(float ax, float ay, float az, float bx, float by, float bz) {
    const float x = ax * bx, y = ay * by, z = az * bz;
    return (x + y) + z;
}

// make_plane_from_vec4 (geometry/frustum_culling.hpp:32-46)
HPlane plane_from_vec4(float x, float y, float z, float w) {
    const float len = std::sqrt(hdot(x, y, z, x, y, z));
    if (len <= 1e-8f) return {0.0f, 1.0f, 0.0f, w};
    return {x / len, y / len, z / len, w / len};
}

float sdist(const HPlane &p, float x, float y, float z) { return hdot(p.nx, p.ny, p.nz, x, y, z) + p.d; }

// classify_vs_frustum(SceneShape) != Outside (geometry/jolt_culling.hpp:187-229, 260-275): the Jolt
// bounding sphere of the world AABB, then the AABB's p-vertices
bool frustum_visible(const HPlane (&fr)[6], const shs_dev::BinLight &L) {
    const float r = smax(L.r, 0.0f);
    bool inside_all = true;
    for (const HPlane &p : fr) {
        const float dist = sdist(p, L.cx, L.cy, L.cz);
        if (dist < -(r + 1e-5f)) return false;
        if (dist < (r + 1e-5f)) inside_all = false;
    }
    if (inside_all) return true;
    for (const HPlane &p : fr) {
        const float px = p.nx >= 0.0f ? L.mxx : L.mnx, py = p.ny >= 0.0f ? L.mxy : L.mny, pz = p.nz >= 0.0f ? L.mxz : L.mnz;
        if (sdist(p, px, py, pz) < -1e-5f) return false;
    }
    return true;
}

// ndc_from_view_depth_lh_no (lighting/jolt_light_culling.hpp:84-92)
float ndc_from_view_depth(float view_depth, float z_near, float z_far) {
    const float n = smax(z_near, 1e-4f);
    const float f = smax(z_far, n + 1e-3f);
    const float z = view_depth < n ? n : (f < view_depth ? f : view_depth);
    const float denom = smax(f - n, 1e-6f);
    return ((f + n) / denom) - ((2.0f * f * n) / (denom * z));
}

}  // namespace

extern "C" int shs_light_bin_culling(shs_ctx *ctx, const shs_light_bin_desc *desc, const float *light_aabbs, int32_t n_lights,
                                     uint32_t bins_xyz[3], uint32_t *counts, uint32_t *indices) {
    if (!ctx || !desc || !bins_xyz || n_lights < 0 || (n_lights > 0 && !light_aabbs)) return SHS_ERR_INVALID;
    const shs_light_bin_desc &d = *desc;
    if (d.width <= 0 || d.height <= 0 || d.width > 16384 || d.height > 16384 || d.mode > SHS_LIGHT_CULL_CLUSTERED ||
        d.z_slices > 4096) {
        ctx->err = "bad light bin description";
        return SHS_ERR_INVALID;
    }
    bins_xyz[0] = bins_xyz[1] = bins_xyz[2] = 0u;   // LightBinCullingData defaults: mode None / no lights
    if (d.mode == SHS_LIGHT_CULL_NONE || n_lights == 0) return SHS_OK;
    const uint32_t ts = d.tile_size > 1u ? d.tile_size : 1u;
    const float zn = smax(d.z_near, 1e-4f), zf = smax(d.z_far, zn + 1e-3f);   // :283-284
    const uint32_t bx = ((uint32_t)d.width + ts - 1u) / ts, by = ((uint32_t)d.height + ts - 1u) / ts;
    const uint32_t slices = d.mode == SHS_LIGHT_CULL_CLUSTERED ? (d.z_slices > 1u ? d.z_slices : 1u) : 1u;
    const size_t n_bins = (size_t)bx * by * slices;
    if (!counts || (d.max_per_bin > 0 && !indices)) { ctx->err = "light bin outputs"; return SHS_ERR_INVALID; }

    shs_dev::LightBinParams p{};
    p.W = d.width; p.H = d.height;
    p.ts = ts; p.bx = bx; p.by = by; p.slices = slices; p.cap = d.max_per_bin;
    shs_host::inverse(d.view_proj, p.inv_vp);
    // extract_frustum_planes (frustum_culling.hpp:48-65): left/right, bottom/top, near/far from rows
    HPlane fr[6];
    {
        float r[4][4];
        for (int row = 0; row < 4; ++row)
            for (int c = 0; c < 4; ++c) r[row][c] = d.view_proj[4 * c + row];
        for (int k = 0; k < 3; ++k) {
            fr[2 * k] = plane_from_vec4(r[3][0] + r[k][0], r[3][1] + r[k][1], r[3][2] + r[k][2], r[3][3] + r[k][3]);
            fr[2 * k + 1] = plane_from_vec4(r[3][0] - r[k][0], r[3][1] - r[k][1], r[3][2] - r[k][2], r[3][3] - r[k][3]);
        }
    }
    // the lights: Jolt AABox centre 0.5 * (min + max), radius |0.5 * (max - min)| (scene_shape.hpp:56-68)
    std::vector<shs_dev::BinLight> vis;
    vis.reserve((size_t)n_lights);
    for (int li = 0; li < n_lights; ++li) {
        const float *a = light_aabbs + 6 * (size_t)li;
        shs_dev::BinLight L{};
        L.mnx = a[0]; L.mny = a[1]; L.mnz = a[2];
        L.mxx = a[3]; L.mxy = a[4]; L.mxz = a[5];
        L.cx = (a[0] + a[3]) * 0.5f; L.cy = (a[1] + a[4]) * 0.5f; L.cz = (a[2] + a[5]) * 0.5f;
        const float ex = (a[3] - a[0]) * 0.5f, ey = (a[4] - a[1]) * 0.5f, ez = (a[5] - a[2]) * 0.5f;
        L.r = std::sqrt(hdot(ex, ey, ez, ex, ey, ez));
        uint32_t idx = (uint32_t)li;
        std::memcpy(&L.index_f, &idx, 4);
        if (frustum_visible(fr, L)) vis.push_back(L);
    }
    // cell depths: clustered log slices (cull_lights_clustered, :372-380) or per-tile view-depth ranges
    // (cull_lights_tiled_view_depth_range, :300-307; other sizes fall back to plain tiles, :341-352)
    std::vector<float2> ndc;
    const bool depth_ok = d.mode == SHS_LIGHT_CULL_TILED_DEPTH && d.tile_min_view_depth && d.tile_max_view_depth &&
                          d.n_depth_tiles == (int32_t)(bx * by);
    if (d.mode == SHS_LIGHT_CULL_CLUSTERED) {
        const float log_ratio = std::log(zf / zn);
        for (uint32_t cz = 0; cz < slices; ++cz) {
            const float s_near = zn * std::exp(log_ratio * static_cast<float>(cz) / static_cast<float>(slices));
            const float s_far = zn * std::exp(log_ratio * static_cast<float>(cz + 1) / static_cast<float>(slices));
            ndc.push_back(make_float2(ndc_from_view_depth(s_near, zn, zf), ndc_from_view_depth(s_far, zn, zf)));
        }
    } else if (depth_ok) {
        for (uint32_t t = 0; t < bx * by; ++t)
            ndc.push_back(make_float2(ndc_from_view_depth(d.tile_min_view_depth[t], zn, zf),
                                      ndc_from_view_depth(d.tile_max_view_depth[t], zn, zf)));
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (ensure(ctx, ctx->lb_lights, std::max<size_t>(vis.size(), 1)) || ensure(ctx, ctx->lb_counts, n_bins) ||
        ensure(ctx, ctx->lb_ndc, std::max<size_t>(ndc.size(), 1)) ||
        ensure(ctx, ctx->lb_indices, std::max<size_t>(n_bins * d.max_per_bin, 1)))
        return SHS_ERR_HIP;
    hipStream_t st = ctx->stream;
    if (!vis.empty())
        HIP_TRY(ctx, hipMemcpyAsync(ctx->lb_lights.p, vis.data(), vis.size() * sizeof(shs_dev::BinLight), hipMemcpyHostToDevice, st));
    if (!ndc.empty()) HIP_TRY(ctx, hipMemcpyAsync(ctx->lb_ndc.p, ndc.data(), ndc.size() * sizeof(float2), hipMemcpyHostToDevice, st));
    p.n_vis = (uint32_t)vis.size();
    p.lights = ctx->lb_lights.p;
    p.ndc_range = ndc.empty() ? nullptr : ctx->lb_ndc.p;
    p.ndc_per_tile = depth_ok ? 1 : 0;
    p.counts = ctx->lb_counts.p;
    p.indices = ctx->lb_indices.p;
    HIP_TRY(ctx, shs_internal::launch_light_bin(p, st));
    HIP_TRY(ctx, hipMemcpyAsync(counts, ctx->lb_counts.p, n_bins * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (d.max_per_bin > 0)
        HIP_TRY(ctx, hipMemcpyAsync(indices, ctx->lb_indices.p, n_bins * d.max_per_bin * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(ctx, hipStreamSynchronize(st));
    bins_xyz[0] = bx; bins_xyz[1] = by; bins_xyz[2] = slices;
    return SHS_OK;
}
