// shs_light_internal.hpp -- launch wrapper of the light-list binning kernels (shs_light.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "shs_lib_device.hpp"

namespace shs_internal {
// Does list tile (tx, ty) (cull tiles, rows down) cover a pixel of one of this rank's 32x32 bin tiles
// (rows up, tile % count == rank)?  Columns align (the tile size divides 32); rows are counted from
// opposite edges, so when H is not a multiple of the tile size a list tile straddles two bin rows and
// both owners build it (the same list).  Tile sizes that do not divide 32 keep every list.
__host__ __device__ inline bool light_list_owned(const shs_dev::LightCullParams &p, uint32_t tx, uint32_t ty) {
    if (p.count <= 1 || (32u % p.tile_size) != 0u) return true;
    const uint32_t px = tx * p.tile_size, py_down = ty * p.tile_size;
    const int top_up = p.H - 1 - (int)py_down;
    const int bot_up = top_up - (int)p.tile_size + 1 < 0 ? 0 : top_up - (int)p.tile_size + 1;
    const int bx = (int)px / 32, by0 = top_up / 32, by1 = bot_up / 32;
    const int tiles_x = (p.W + 31) / 32;
    return shs_dev::shard_owned(p.rank, p.count, p.reg, bx, by0, tiles_x) || shs_dev::shard_owned(p.rank, p.count, p.reg, bx, by1, tiles_x);
}

// (mode 2) k_depth_reduce over `depth`, then k_light_cull over lists work[0 .. n_work) (work == nullptr:
// lists 0 .. n_work) -- work[n_work ..] (the other ranks' lists) get count 0; mode 0 or no work lists:
// every count 0.  ranges: one float2 per tile, counts: p.n_lists, indices: p.n_lists * p.max_per_tile.
hipError_t launch_light_cull(const shs_dev::LightCullParams &p, const shs_dev::CullLight *lights, const float *depth,
                             float2 *ranges, const uint32_t *work, uint32_t n_work, uint32_t *counts, uint32_t *indices,
                             hipStream_t s);
}  // namespace shs_internal
