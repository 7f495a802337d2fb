// shs_tiles_internal.hpp -- tile-shard pack / unpack of framebuffers (shs_tiles.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "shs_shard.hpp"

namespace shs_dev {
struct TileCopyParams {
    int32_t W, H, rank, count;
    int32_t words;          // words per pixel in the packed layout
    int32_t color_words;    // 1 (RGBA8) or 4 (RGBA32F)
    int32_t color_flip;     // colour rows are canvas rows (H-1-y)
    uint32_t *color;        // framebuffer words
    uint32_t *depth;        // nullptr if absent
    uint32_t *motion;       // nullptr if absent (2 words per pixel)
    ShardRegion reg;        // reg.on: rank's rectangle of bin tiles (else tile % count == rank)
};

// Up to UNPACK_PEERS peers' packed buffers unpacked by one launch: p is rank-independent (the target's
// planes), peer k is rank[k] with rectangle reg[k], its owned tiles are blocks first[k] .. first[k+1]-1.
constexpr int UNPACK_PEERS = 16;
struct TileUnpackMulti {
    TileCopyParams p;
    int32_t n;
    int32_t first[UNPACK_PEERS + 1];
    int32_t rank[UNPACK_PEERS];
    ShardRegion reg[UNPACK_PEERS];
    const uint32_t *src[UNPACK_PEERS];
};
}  // namespace shs_dev

namespace shs_internal {
// pack: framebuffers -> packed (one 32x32-padded block of `words` planes per owned tile);
// unpack: packed -> framebuffers.
hipError_t launch_tiles_copy(const shs_dev::TileCopyParams &p, bool pack, void *packed, hipStream_t s);
hipError_t launch_tiles_unpack_multi(const shs_dev::TileUnpackMulti &m, hipStream_t s);
}  // namespace shs_internal
