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
    float model[16];
    float aabb_min[3], aabb_max[3];
};

struct OccParams {
    const OccObject *objs;   // n in visit order
    int32_t n;
    int32_t W, H;
    float vp[16];
    float eps;
    uint32_t *depth;         // W*H occlusion depth (float bits; all values are in [0, 1])
    uint8_t *occluded;       // per caller object index
    uint32_t *visible;       // visible object indices in visit order
    uint32_t *n_visible;     // [1]
};

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_occlusion(const shs_dev::OccParams &p, hipStream_t s);
}  // namespace shs_internal
