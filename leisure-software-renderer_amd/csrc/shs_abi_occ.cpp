// shs_abi_occ.cpp -- C ABI of the software occlusion pass (include/shs_gpu.h):
// culling_sw::run_software_occlusion_pass (shs-renderer-lib/include/shs/geometry/culling_software.hpp
// :229-331) as SceneCullingContext::run_software_occlusion drives it (scene/scene_culling.hpp:187-219).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "shs_ctx.hpp"
#include "shs_occlusion_internal.hpp"

namespace {

// view_depth_of_aabb_center (culling_software.hpp:220-227): (view * vec4(0.5 (min + max), 1)).z
float aabb_center_view_z(const shs_occluder &o, const float *view) {
    const float c[4] = {0.5f * (o.aabb_min[0] + o.aabb_max[0]), 0.5f * (o.aabb_min[1] + o.aabb_max[1]),
                        0.5f * (o.aabb_min[2] + o.aabb_max[2]), 1.0f};
    return (view[2] * c[0] + view[6] * c[1]) + (view[10] * c[2] + view[14] * c[3]);
}

}  // namespace

extern "C" int shs_occlusion_pass(shs_ctx *ctx, const shs_occlusion_desc *desc, const shs_occluder *objects,
                                  int32_t n_objects, const uint32_t *frustum_visible, int32_t n_frustum_visible,
                                  uint8_t *occluded, uint32_t *visible, int32_t *n_visible, float *depth) {
    if (!ctx || !desc || (n_objects > 0 && !objects) || (n_frustum_visible > 0 && !frustum_visible) || !occluded ||
        !visible || !n_visible || n_objects < 0 || n_frustum_visible < 0)
        return SHS_ERR_INVALID;
    if (desc->width <= 0 || desc->height <= 0 || desc->width > 65535 || desc->height > 65535) {
        ctx->err = "occlusion buffer size: 1 .. 65535 per side";
        return SHS_ERR_INVALID;
    }
    std::memset(occluded, 0, (size_t)n_objects);
    // the frustum-visible objects, sorted by view depth (std::sort's strict '<'; equal keys keep the
    // input order here), out-of-range indices dropped as the reference's comparator pushes them last
    std::vector<uint32_t> order;
    order.reserve((size_t)n_frustum_visible);
    for (int32_t k = 0; k < n_frustum_visible; ++k)
        if (frustum_visible[k] < (uint32_t)n_objects) order.push_back(frustum_visible[k]);
    if (!desc->enable) {   // every frustum-visible object is visible, the depth is untouched
        std::copy(order.begin(), order.end(), visible);
        *n_visible = (int32_t)order.size();
        return SHS_OK;
    }
    std::vector<float> key((size_t)n_objects, 0.0f);
    for (uint32_t idx : order) key[idx] = aabb_center_view_z(objects[idx], desc->view);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    std::vector<shs_dev::OccObject> objs(order.size());
    size_t n_tris_total = 0;
    for (size_t s = 0; s < order.size(); ++s) {
        const shs_occluder &o = objects[order[s]];
        if (o.mesh_id < 0 || o.mesh_id >= (int)ctx->meshes.size() || !ctx->meshes[o.mesh_id].live ||
            !ctx->meshes[o.mesh_id].lib || !ctx->meshes[o.mesh_id].idx) {
            ctx->err = "occluder mesh must be an indexed shs_mesh_upload mesh";
            return SHS_ERR_INVALID;
        }
        const auto &m = ctx->meshes[o.mesh_id];
        shs_dev::OccObject &d = objs[s];
        d.pos = m.pos;
        d.idx = m.idx;
        d.n_verts = m.n_verts;
        d.n_idx = m.n_tris * 3;
        d.index = order[s];
        d.tri_base = (uint32_t)n_tris_total;
        n_tris_total += (size_t)m.n_tris;
        std::memcpy(d.model, o.model, sizeof d.model);
        std::memcpy(d.aabb_min, o.aabb_min, sizeof d.aabb_min);
        std::memcpy(d.aabb_max, o.aabb_max, sizeof d.aabb_max);
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const size_t npx = (size_t)desc->width * desc->height;
    if (ensure(ctx, ctx->occ_depth, npx) || ensure(ctx, ctx->occ_objs, std::max<size_t>(objs.size(), 1)) ||
        ensure(ctx, ctx->occ_flags, std::max<size_t>((size_t)n_objects, 1)) ||
        ensure(ctx, ctx->occ_visible, std::max<size_t>(order.size(), 1) + 1) ||
        ensure(ctx, ctx->occ_rects, objs.size() + 2) || ensure(ctx, ctx->occ_tris, std::max<size_t>(n_tris_total, 1)))
        return SHS_ERR_HIP;
    if (!objs.empty())
        HIP_TRY(ctx, hipMemcpyAsync(ctx->occ_objs.p, objs.data(), objs.size() * sizeof(shs_dev::OccObject),
                                    hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->occ_rects.p + objs.size(), 0, 2 * sizeof(shs_dev::OccRect), ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->occ_flags.p, 0, std::max<size_t>((size_t)n_objects, 1), ctx->stream));
    shs_dev::OccParams p{};
    p.objs = ctx->occ_objs.p;
    p.rects = ctx->occ_rects.p;
    p.tris = ctx->occ_tris.p;
    p.n = (int32_t)objs.size();
    p.W = desc->width;
    p.H = desc->height;
    std::memcpy(p.vp, desc->view_proj, sizeof p.vp);
    p.eps = desc->depth_epsilon;
    p.chunk = (int32_t)std::min<uint64_t>(1024, 0xffffffffull / npx);
    p.depth = ctx->occ_depth.p;
    p.occluded = ctx->occ_flags.p;
    p.visible = ctx->occ_visible.p + 1;
    p.n_visible = ctx->occ_visible.p;
    p.prof = shs_exp_env("SHS_OCC_PROF") != nullptr;
    HIP_TRY(ctx, shs_internal::launch_occlusion(p, ctx->stream));
    std::vector<uint32_t> vis(order.size() + 1);
    HIP_TRY(ctx, hipMemcpyAsync(vis.data(), ctx->occ_visible.p, vis.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    if (n_objects > 0)
        HIP_TRY(ctx, hipMemcpyAsync(occluded, ctx->occ_flags.p, (size_t)n_objects, hipMemcpyDeviceToHost, ctx->stream));
    if (depth) HIP_TRY(ctx, hipMemcpyAsync(depth, ctx->occ_depth.p, npx * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_visible = (int32_t)vis[0];
    std::copy(vis.begin() + 1, vis.begin() + 1 + vis[0], visible);
    return SHS_OK;
}
