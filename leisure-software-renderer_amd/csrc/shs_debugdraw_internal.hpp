// shs_debugdraw_internal.hpp -- launch interface of shs_debugdraw.hip: the software library's
// debug_draw filled-triangle raster (sw_render/debug_draw.hpp:60-109) and its
// Blinn-Phong mesh caller (:158-205).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace shs_dev {

// One mesh of draw_mesh_blinn_phong_transformed: DebugMesh vertices / indices, the model matrix, the
// base colour, and its first triangle in the batch's submission order.
struct DDObject {
    const float *pos;
    const uint32_t *idx;
    int32_t n_verts, n_tris;
    uint32_t tri_base;
    float model[16];
    float base[3];
};

// A filled triangle ready for draw_filled_triangle: screen points, depths, edge_fn area, colour,
// integer bbox (min_x | min_y << 16, max_x | max_y << 16); area == 0: skipped.
struct alignas(16) DDTri {
    float x0, y0, x1, y1;
    float x2, y2, z0, z1;
    float z2, area;
    uint32_t rgba;
    uint32_t flags;     // bit 0: drawn (bbox on the canvas); bit 1: |area| > 1e-6
    uint32_t bmin, bmax;
    float lit[2];       // lit.r / lit.g before the byte conversion (lit.b in the slot below)
};

constexpr int DD_BIG = 4096;         // bbox pixels above which a triangle is rastered by every workgroup

struct DDParams {
    int32_t W, H;
    int32_t n_tris, n_objects;
    float vp[16];
    float cam[3], L[3];              // camera position, normalize(-light_dir_ws)
    const DDObject *objects;         // mesh mode (nullptr: triangles given directly)
    DDTri *tris;
    float *lit_b;                    // per triangle lit.b (tests)
    const float *depth0;             // the depth buffer before the draw (W*H)
    unsigned long long *keys;        // per pixel (depth, triangle) minimum
    uint32_t *big_count;             // [0]: triangles with a bbox above DD_BIG pixels, listed in big_list
    uint32_t *big_list;
    uint32_t *rgba;                  // RT_ColorLDR (W*H, rows as given)
    float *depth;                    // depth buffer out
};

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_dd_mesh_setup(const shs_dev::DDParams &p, hipStream_t s);
hipError_t launch_dd_fill(const shs_dev::DDParams &p, hipStream_t s);
}  // namespace shs_internal
