// shs_lib_internal.hpp -- launch wrappers of the library-path kernels (shs_lib.hip) for shs_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "shs_lib_device.hpp"

namespace shs_internal {
// shadow = true: PassShadowMap's depth pass; false: rasterize_mesh + builtin programs.
// listed (tile-sharded camera pass): each setup workgroup culls CULL_PER x 256 triangles to the rank's
// and sets up those (lib_setup_grid); otherwise one workgroup per 256 triangles.
hipError_t launch_lib_setup(const shs_dev::LibFrameParams &fp, const shs_dev::LibBuffers &fb, bool shadow, bool listed,
                            hipStream_t s);
int lib_setup_grid(int n_tris, bool listed);
// shallow: the 256-candidate-round k_lib_raster (every bin tile's list fits one gather round)
int lib_raster_resident_blocks(int device, bool shadow, bool shallow);   // CUs x occupancy of k_lib_raster
hipError_t launch_lib_raster(const shs_dev::LibFrameParams &fp, const shs_dev::LibBuffers &fb, bool shadow, bool shallow,
                             int grid, hipStream_t s);
// The camera pass's shading: every owned pixel's winner (fb.keys) shaded into hdr / depth / motion.
// prog: the program every draw of the pass runs (5 Forward+, 0 PBR: specialised kernels) or -1.
// CUs x occupancy of k_lib_resolve<prog> (wide: the whole frame's build, else a sharded rank's)
int lib_resolve_resident_blocks(int device, int prog, bool wide);
hipError_t launch_lib_resolve(const shs_dev::LibFrameParams &fp, const shs_dev::LibBuffers &fb, int prog, bool wide,
                              int grid, hipStream_t s);
}  // namespace shs_internal
