// shs_shard.hpp -- which 32x32 bin tiles of a frame a tile shard owns, shared by the
// library kernels, the light cull, the tonemap, the tile gather and their host code.
//
// Two layouts:
//   interleaved  tile t = by * tiles_x + bx belongs to rank t % count (the default: screen-centre
//                geometry spreads over every rank without any knowledge of the scene);
//   regions      rank r owns one rectangle of bin tiles (ShardRegion, inclusive; empty when x1 < x0),
//                the rectangles tiling the grid.  A rank then needs only the geometry whose screen
//                bounds reach its rectangle, so whole 256-triangle setup blocks whose chunk bounds miss
//                it are skipped (k_lib_setup), and the rectangles come from a cost-balanced split of the
//                previous camera pass's block bounds (shs_abi_shard.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shs_dev {

struct ShardRegion {
    int32_t on;                 // 0: interleaved ownership (tile % count == rank); 1: the rectangle below
    int32_t x0, y0, x1, y1;     // bin tiles, inclusive (x1 < x0 or y1 < y0: nothing owned)
};

__host__ __device__ inline bool region_empty(const ShardRegion &g) { return g.x1 < g.x0 || g.y1 < g.y0; }

__host__ __device__ inline bool shard_owned(int rank, int count, const ShardRegion &g, int bx, int by, int tiles_x) {
    if (count <= 1) return true;
    if (g.on) return bx >= g.x0 && bx <= g.x1 && by >= g.y0 && by <= g.y1;
    return ((by * tiles_x + bx) % count) == rank;
}

// Does the tile rectangle [tx0, tx1] x [ty0, ty1] hold an owned tile?
__host__ __device__ inline bool shard_owns_any(int rank, int count, const ShardRegion &g, int tx0, int tx1, int ty0, int ty1,
                                               int tiles_x) {
    if (count <= 1) return true;
    if (tx1 < tx0 || ty1 < ty0) return false;
    if (g.on) return !(tx1 < g.x0 || tx0 > g.x1 || ty1 < g.y0 || ty0 > g.y1);
    if (tx1 - tx0 + 1 >= count) return true;   // a row of count consecutive tiles holds every rank's
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx)
            if (((ty * tiles_x + tx) % count) == rank) return true;
    return false;
}

__host__ __device__ inline int shard_n_owned(int rank, int count, const ShardRegion &g, int n_tiles) {
    if (count <= 1) return n_tiles;
    if (g.on) return region_empty(g) ? 0 : (g.x1 - g.x0 + 1) * (g.y1 - g.y0 + 1);
    return n_tiles > rank ? (n_tiles - rank + count - 1) / count : 0;
}

// The i-th owned tile (row-major inside a region).
__host__ __device__ inline int shard_tile(int rank, int count, const ShardRegion &g, int i, int tiles_x) {
    if (count <= 1) return i;
    if (g.on) {
        const int w = g.x1 - g.x0 + 1;
        return (g.y0 + i / w) * tiles_x + g.x0 + i % w;
    }
    return rank + i * count;
}

}  // namespace shs_dev
