// shs_tiles.hip -- device-side packing of a tile shard's framebuffer pixels for the multi-GPU
// final-image gather: rank r owns the 32x32 tiles t = r, r + N, ... (or its region's
// tiles, row-major: shs_shard.hpp); its pixels are
// packed tile after tile into a contiguous device buffer (each tile padded to 32x32), exchanged with
// RCCL, and unpacked on rank 0 into the full frame.  One workgroup per owned tile, coalesced 32-px
// row segments.  Word layout per tile: colour words (legacy RGBA8: 1, library HDR: 4), then depth
// (1), then library motion (2), each pixel-major in screen rows (legacy colour: canvas row H-1-y).
#include <algorithm>

#include "shs_device.hpp"
#include "shs_tiles_internal.hpp"

namespace shs_dev {

// Owned tile i of p's rank: its pixels <-> the i-th 32x32-padded block of `packed`.
template <bool PACK>
__device__ __forceinline__ void tile_copy(const TileCopyParams &p, int i, uint32_t *packed) {
    const int tiles_x = (p.W + TILE - 1) / TILE;
    const int t = shard_tile(p.rank, p.count, p.reg, i, tiles_x);
    const int x0 = (t % tiles_x) * TILE, y0 = (t / tiles_x) * TILE;
    uint32_t *base = packed + (size_t)i * TILE * TILE * p.words;
    for (int k = threadIdx.x; k < TILE * TILE; k += 256) {
        const int x = x0 + (k & (TILE - 1)), y = y0 + k / TILE;
        if (x >= p.W || y >= p.H) continue;
        const size_t row = (size_t)y * p.W + x;
        const size_t crow = p.color_flip ? (size_t)(p.H - 1 - y) * p.W + x : row;
        uint32_t *w = base + (size_t)k;
        int c = 0;
        for (int j = 0; j < p.color_words; ++j, ++c) {
            if (PACK) w[(size_t)c * TILE * TILE] = p.color[crow * p.color_words + j];
            else p.color[crow * p.color_words + j] = w[(size_t)c * TILE * TILE];
        }
        if (p.depth) {
            if (PACK) w[(size_t)c * TILE * TILE] = p.depth[row];
            else p.depth[row] = w[(size_t)c * TILE * TILE];
            ++c;
        }
        for (int j = 0; p.motion && j < 2; ++j, ++c) {
            if (PACK) w[(size_t)c * TILE * TILE] = p.motion[row * 2 + j];
            else p.motion[row * 2 + j] = w[(size_t)c * TILE * TILE];
        }
    }
}

template <bool PACK>
__global__ __launch_bounds__(256) void k_tiles_copy(TileCopyParams p, uint32_t *packed) {
    tile_copy<PACK>(p, (int)blockIdx.x, packed);
}

// Rank 0's unpack of several peers' packed tiles in one launch (the gather's receive side): block b is
// owned tile b - first[k] of peer k (ranks rank[k], buffers src[k]; a uniform search over <= 16 peers).
__global__ __launch_bounds__(256) void k_tiles_unpack_multi(TileUnpackMulti m) {
    const int b = (int)blockIdx.x;
    int k = 0;
    while (k + 1 < m.n && m.first[k + 1] <= b) ++k;
    TileCopyParams p = m.p;
    p.rank = m.rank[k];
    p.reg = m.reg[k];
    tile_copy<false>(p, b - m.first[k], const_cast<uint32_t *>(m.src[k]));
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_tiles_copy(const TileCopyParams &p, bool pack, void *packed, hipStream_t s) {
    const int n_tiles = ((p.W + TILE - 1) / TILE) * ((p.H + TILE - 1) / TILE);
    const int n_owned = shard_n_owned(p.rank, p.count, p.reg, n_tiles);
    if (n_owned <= 0) return hipSuccess;
    if (pack) hipLaunchKernelGGL(k_tiles_copy<true>, dim3(n_owned), dim3(256), 0, s, p, static_cast<uint32_t *>(packed));
    else hipLaunchKernelGGL(k_tiles_copy<false>, dim3(n_owned), dim3(256), 0, s, p, static_cast<uint32_t *>(packed));
    return hipGetLastError();
}

hipError_t launch_tiles_unpack_multi(const TileUnpackMulti &m, hipStream_t s) {
    if (m.n <= 0 || m.first[m.n] <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tiles_unpack_multi, dim3(m.first[m.n]), dim3(256), 0, s, m);
    return hipGetLastError();
}

}  // namespace shs_internal
