// shs_internal.hpp -- kernel launch wrappers shared between shs_legacy.hip and shs_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "shs_device.hpp"

namespace shs_internal {
hipError_t launch_setup(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, const shs_dev::KArgDraws &ka,
                        hipStream_t s);
hipError_t launch_ghost(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, hipStream_t s);
hipError_t launch_raster(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, const shs_dev::KArgDraws &ka,
                         int grid, hipStream_t s);
// k_pipe: batch k - 1's raster (fpR / fbR, grid = its persistent raster grid) and batch k's setup in one launch
hipError_t launch_pipe(const shs_dev::FrameParams &fpR, const shs_dev::FrameBuffers &fbR, int grid, const shs_dev::FrameParams &fpS,
                       const shs_dev::FrameBuffers &fbS, hipStream_t s);
}  // namespace shs_internal
