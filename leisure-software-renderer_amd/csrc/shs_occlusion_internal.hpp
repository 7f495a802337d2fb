// shs_occlusion_internal.hpp -- launch interface of shs_occlusion.hip (software occlusion pass).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace shs_dev {

// One frustum-visible object in visit order (sorted by the view z of its AABB centre).
struct OccObject {
    const float *pos;        // DebugMesh vertices (xyz)
    const uint32_t *idx;     // DebugMesh indices
    int32_t n_verts, n_idx;
    uint32_t index;          // the caller's object index
    uint32_t tri_base;       // first OccTri of the object
    float model[16];
    float aabb_min[3], aabb_max[3];
};

// k_occ_setup's per-object record (visit order): project_aabb_to_screen_rect and the object's
// triangle range in the OccTri array.
struct OccRect {
    int32_t x0, y0, x1, y1;
    float z_near;            // clamped to [0, 1]
    int32_t valid;           // the rect is non-empty (an invalid rect is never occluded)
    uint32_t tri_base, n_tris;
    uint32_t index;          // the caller's object index
    uint32_t pad[3];
};

// One triangle's rasterize_depth_triangle setup, 3 x 16 bytes: corners (sx, sy, sz) x 3, the
// signed area and the clamped bbox (x0 | y0 << 16, w | h << 16; w = h = 0 when the reference skips
// the triangle).  Buffer sides are < 2^16 (checked by the ABI).
struct OccTri {
    float4 a;                // sx0 sy0 sz0 sx1
    float4 b;                // sy1 sz1 sx2 sy2
    float4 c;                // sz2 area (x0 | y0 << 16) (w | h << 16), the last two as uint bits
};

struct OccParams {
    const OccObject *objs;   // n in visit order
    OccRect *rects;          // n (+ 2 padding records)
    OccTri *tris;            // sum of n_tris
    int32_t n;
    int32_t W, H;
    float vp[16];
    float eps;
    uint32_t *depth;         // W*H occlusion depth (float bits; all values are in [0, 1])
    uint8_t *occluded;       // per caller object index
    uint32_t *visible;       // visible object indices in visit order
    uint32_t *n_visible;     // [1]
    int32_t chunk;           // triangles per raster chunk: <= 1024 with chunk * W * H < 2^32
    int prof;                // SHS_OCC_PROF: print per-phase wall-clock totals
};

}  // namespace shs_dev

namespace shs_internal {
// k_occ_setup (one block per object, parallel) then k_occlusion (the sequential walk, one block)
hipError_t launch_occlusion(const shs_dev::OccParams &p, hipStream_t s);
}  // namespace shs_internal
