// shs_canvas_post_internal.hpp -- launch interface of shs_canvas_post.hip: the Canvas-API multi-pass
// extras that consume the motion / depth buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace shs_dev {

// combined_motion_blur_pass (hello-render-target/hello_pbr.cpp:1128-1252) with the camera-velocity
// reconstruction it calls (:1051-1122).  Buffers indexed y * W + x, as the pass indexes raw().
struct CanvasMBParams {
    const uint32_t *src;      // shs::Canvas colours
    const float *depth;       // ZBuffer (view z; FLT_MAX = empty)
    const float2 *velocity;   // Buffer<glm::vec2> (canvas px)
    uint32_t *dst;
    int32_t W, H;
    float prev_vp[16], inv_curr_vp[16], curr_proj[16];
    int32_t samples, soft_knee;
    float strength, w_obj, w_cam, knee, max_px;
};

// hello-render-target/hello_depth_of_field.cpp: gaussian_blur_pass (:175-251),
// autofocus_depth_median_center (:257-285), dof_composite_pass (:287-343).
struct CanvasDofParams {
    const uint32_t *sharp;
    const uint32_t *blur;
    const float *depth;       // ZBuffer (view z)
    uint32_t *out;
    float *focus;             // device: the autofocus result
    int32_t W, H;
    int32_t cx, cy, radius;
    float range, max_blur;
};

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_canvas_motion_blur(const shs_dev::CanvasMBParams &p, hipStream_t s);
hipError_t launch_canvas_gaussian(const uint32_t *src, uint32_t *dst, int W, int H, bool horizontal, hipStream_t s);
hipError_t launch_canvas_autofocus(const shs_dev::CanvasDofParams &p, hipStream_t s);
hipError_t launch_canvas_dof_composite(const shs_dev::CanvasDofParams &p, hipStream_t s);
}  // namespace shs_internal
