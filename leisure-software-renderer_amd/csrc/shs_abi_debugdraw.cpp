// shs_abi_debugdraw.cpp -- C ABI of the software library's debug_draw colour + depth raster
// (include/shs_gpu.h): draw_mesh_blinn_phong_transformed
// (shs-renderer-lib/include/shs/sw_render/debug_draw.hpp:147-203) as hello_occlusion_culling_sw.cpp
// :387-407 and hello_culling_sw.cpp:315 drive it over the visible instances, and draw_filled_triangle
// (:60-109) for callers that shade triangles themselves (hello_light_types_culling_sw.cpp:379-421).
// The canvas and depth buffer cross the boundary as host buffers (the demos hold them in host memory
// and present them right after); one call draws every triangle of the list in submission order.
#include <cmath>
#include <cstring>
#include <vector>

#include "shs_ctx.hpp"

namespace {

int dd_targets(shs_ctx *ctx, int W, int H, size_t n_tris, const uint8_t *rgba, const float *depth) {
    const size_t npx = (size_t)W * H;
    if (ensure(ctx, ctx->dd_tris, std::max<size_t>(n_tris, 1)) || ensure(ctx, ctx->dd_big, n_tris + 1) || ensure(ctx, ctx->dd_depth0, npx) ||
        ensure(ctx, ctx->dd_depth, npx) || ensure(ctx, ctx->dd_rgba, npx) || ensure(ctx, ctx->dd_keys, npx))
        return SHS_ERR_HIP;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->dd_depth0.p, depth, npx * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->dd_depth.p, ctx->dd_depth0.p, npx * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->dd_rgba.p, rgba, npx * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->dd_big.p, 0, sizeof(uint32_t), ctx->stream));
    return SHS_OK;
}

int dd_finish(shs_ctx *ctx, shs_dev::DDParams &p, uint8_t *rgba, float *depth) {
    const size_t npx = (size_t)p.W * p.H;
    p.depth0 = ctx->dd_depth0.p;
    p.keys = ctx->dd_keys.p;
    p.rgba = ctx->dd_rgba.p;
    p.depth = ctx->dd_depth.p;
    p.big_count = ctx->dd_big.p;
    p.big_list = ctx->dd_big.p + 1;
    HIP_TRY(ctx, shs_internal::launch_dd_fill(p, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(rgba, ctx->dd_rgba.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(depth, ctx->dd_depth.p, npx * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return SHS_OK;
}

bool canvas_ok(shs_ctx *ctx, int W, int H) {
    if (W > 0 && H > 0 && W <= 32767 && H <= 32767) return true;
    ctx->err = "debug_draw canvas size: 1 .. 32767 per side";
    return false;
}

}  // namespace

extern "C" {

int shs_debug_draw_meshes(shs_ctx *ctx, const shs_debug_draw_desc *desc, const shs_debug_mesh *meshes, int32_t n_meshes,
                          uint8_t *rgba, float *depth, float *tri_lit) {
    if (!ctx || !desc || (n_meshes > 0 && !meshes) || n_meshes < 0 || !rgba || !depth) return SHS_ERR_INVALID;
    if (!canvas_ok(ctx, desc->width, desc->height)) return SHS_ERR_INVALID;
    std::vector<shs_dev::DDObject> objs;
    objs.reserve((size_t)n_meshes);
    size_t n_tris = 0;
    for (int32_t i = 0; i < n_meshes; ++i) {
        const shs_debug_mesh &m = meshes[i];
        if (m.mesh_id < 0 || m.mesh_id >= (int)ctx->meshes.size() || !ctx->meshes[m.mesh_id].live ||
            !ctx->meshes[m.mesh_id].lib || (!ctx->meshes[m.mesh_id].idx && ctx->meshes[m.mesh_id].n_tris > 0)) {
            ctx->err = "debug_draw mesh must be an indexed shs_mesh_upload mesh";
            return SHS_ERR_INVALID;
        }
        const auto &mesh = ctx->meshes[m.mesh_id];
        if (mesh.n_tris == 0) continue;   // fewer than 3 indices: nothing to draw
        shs_dev::DDObject o{};
        o.pos = mesh.pos;
        o.idx = mesh.idx;
        o.n_verts = mesh.n_verts;
        o.n_tris = mesh.n_tris;
        o.tri_base = (uint32_t)n_tris;
        std::memcpy(o.model, m.model, sizeof o.model);
        std::memcpy(o.base, m.base_color, sizeof o.base);
        objs.push_back(o);
        n_tris += (size_t)mesh.n_tris;
    }
    if (n_tris >= (size_t)0x7fffffff) { ctx->err = "debug_draw: too many triangles"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (dd_targets(ctx, desc->width, desc->height, n_tris, rgba, depth)) return SHS_ERR_HIP;
    if (ensure(ctx, ctx->dd_objs, std::max<size_t>(objs.size(), 1)) || (tri_lit && ensure(ctx, ctx->dd_lit_b, std::max<size_t>(n_tris, 1))))
        return SHS_ERR_HIP;
    if (!objs.empty())
        HIP_TRY(ctx, hipMemcpyAsync(ctx->dd_objs.p, objs.data(), objs.size() * sizeof(shs_dev::DDObject), hipMemcpyHostToDevice, ctx->stream));
    shs_dev::DDParams p{};
    p.W = desc->width;
    p.H = desc->height;
    p.n_tris = (int32_t)n_tris;
    p.n_objects = (int32_t)objs.size();
    std::memcpy(p.vp, desc->view_proj, sizeof p.vp);
    std::memcpy(p.cam, desc->camera_pos, sizeof p.cam);
    // L = glm::normalize(-light_dir_ws) (debug_draw.hpp:159): v * (1 / sqrt(dot)), dot = (x x + y y) + z z
    const float lx = -desc->light_dir_ws[0], ly = -desc->light_dir_ws[1], lz = -desc->light_dir_ws[2];
    const float xx = lx * lx, yy = ly * ly, zz = lz * lz;
    const float inv = 1.0f / std::sqrt((xx + yy) + zz);
    p.L[0] = lx * inv;
    p.L[1] = ly * inv;
    p.L[2] = lz * inv;
    p.objects = ctx->dd_objs.p;
    p.tris = ctx->dd_tris.p;
    p.lit_b = tri_lit ? ctx->dd_lit_b.p : nullptr;
    p.big_count = ctx->dd_big.p;
    p.big_list = ctx->dd_big.p + 1;
    HIP_TRY(ctx, shs_internal::launch_dd_mesh_setup(p, ctx->stream));
    const int rc = dd_finish(ctx, p, rgba, depth);
    if (rc || !tri_lit || n_tris == 0) return rc;
    std::vector<shs_dev::DDTri> t(n_tris);
    std::vector<float> b(n_tris);
    HIP_TRY(ctx, hipMemcpy(t.data(), ctx->dd_tris.p, n_tris * sizeof(shs_dev::DDTri), hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(b.data(), ctx->dd_lit_b.p, n_tris * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n_tris; ++i) {
        tri_lit[4 * i + 0] = t[i].lit[0];
        tri_lit[4 * i + 1] = t[i].lit[1];
        tri_lit[4 * i + 2] = b[i];
        tri_lit[4 * i + 3] = (t[i].flags & 2u) ? 1.0f : 0.0f;   // passes the area test
    }
    return SHS_OK;
}

int shs_debug_fill_triangles(shs_ctx *ctx, int32_t width, int32_t height, const shs_debug_triangle *tris, int32_t n_tris,
                             uint8_t *rgba, float *depth) {
    if (!ctx || (n_tris > 0 && !tris) || n_tris < 0 || !rgba || !depth) return SHS_ERR_INVALID;
    if (!canvas_ok(ctx, width, height)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (dd_targets(ctx, width, height, (size_t)n_tris, rgba, depth)) return SHS_ERR_HIP;
    std::vector<shs_dev::DDTri> t((size_t)n_tris);
    for (int32_t i = 0; i < n_tris; ++i) {
        const shs_debug_triangle &s = tris[i];
        shs_dev::DDTri &d = t[(size_t)i];
        d.x0 = s.p0[0]; d.y0 = s.p0[1]; d.x1 = s.p1[0]; d.y1 = s.p1[1]; d.x2 = s.p2[0]; d.y2 = s.p2[1];
        d.z0 = s.z[0]; d.z1 = s.z[1]; d.z2 = s.z[2];
        std::memcpy(&d.rgba, s.rgba, 4);
    }
    if (n_tris > 0)
        HIP_TRY(ctx, hipMemcpyAsync(ctx->dd_tris.p, t.data(), t.size() * sizeof(shs_dev::DDTri), hipMemcpyHostToDevice, ctx->stream));
    shs_dev::DDParams p{};
    p.W = width;
    p.H = height;
    p.n_tris = n_tris;
    p.tris = ctx->dd_tris.p;
    return dd_finish(ctx, p, rgba, depth);
}

}  // extern "C"
