// shs_abi_shard.cpp -- the region layout of a tile-sharded frame (shs_shard.hpp).
//
// With SHS_OPT_SHARD_LAYOUT = SHS_SHARD_REGIONS every rank of a sharded library frame owns one rectangle
// of 32x32 bin tiles.  The rectangles come from a recursive bisection of the bin grid at equal predicted
// cost.  The prediction is made from the previous camera pass of the context: k_lib_setup writes, per
// 256-triangle setup block, the bin-tile bounds of its chunks' projected model-space boxes (LibBuffers::
// blkrect, mapped host memory).  Every rank computes the same bounds from the same draws, so every rank
// derives the same rectangles without any exchange -- and the host knows them when it enqueues the frame,
// so the raster order, the light-list table and the gather sizes are plain host data.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/shs_gpu.h"
#include "shs_ctx.hpp"

using shs_dev::ShardRegion;

namespace {

// Predicted cost of a bin tile, in units of (triangle x covering bound): every pixel is written
// (REGION_PX), a pixel some bounded block covers is also shaded (REGION_COVERED_PX), and every setup block
// whose bounds cover the tile adds its triangle count (the raster's (primitive, pixel) pair tests grow
// with the triangles' screen size, which grows with the bounds they spread over, so a block costs about
// its triangles on each tile of its bounds).  Fitted to the measured per-rank times of the 8-way C4 frame
// (tools/region_model.py): covered pixels about 19x a (triangle, tile) pair.
#ifndef SHS_REGION_PX
#define SHS_REGION_PX 5.0
#endif
#ifndef SHS_REGION_COVERED_PX
#define SHS_REGION_COVERED_PX 15.0
#endif
constexpr double REGION_PX = SHS_REGION_PX, REGION_COVERED_PX = SHS_REGION_COVERED_PX;

struct Sat {   // summed-area table over the bin grid
    int tx, ty;
    std::vector<double> s;   // (tx + 1) * (ty + 1)
    double at(int x, int y) const { return s[(size_t)y * (tx + 1) + x]; }
    double sum(int x0, int y0, int x1, int y1) const {   // inclusive tile rect
        return at(x1 + 1, y1 + 1) - at(x0, y1 + 1) - at(x1 + 1, y0) + at(x0, y0);
    }
};

// Ranks r0 .. r0 + n - 1 share [x0, x1] x [y0, y1] in proportion to their capacities (cap[r]: 1, rank 0
// root_share): the cut goes where the lower ranks' part reaches their capacity's share of the cost.
void bisect(const Sat &sat, const std::vector<double> &cap, int x0, int y0, int x1, int y1, int r0, int n,
            std::vector<ShardRegion> &out) {
    if (n == 1) {
        out[r0] = ShardRegion{1, x0, y0, x1, y1};
        return;
    }
    const int w = x1 - x0 + 1, h = y1 - y0 + 1;
    if (w <= 0 || h <= 0 || (w == 1 && h == 1)) {   // nothing left to split: rank r0 takes it, the rest none
        out[r0] = ShardRegion{1, x0, y0, x1, y1};
        for (int r = 1; r < n; ++r) out[r0 + r] = ShardRegion{1, 1, 1, 0, 0};
        return;
    }
    const int n1 = n / 2, n2 = n - n1;
    const bool along_x = h == 1 || (w > 1 && w >= h);   // cut the longer side: squarish regions
    double c1 = 0.0, c_all = 0.0;
    for (int r = 0; r < n; ++r) (r < n1 ? c1 : c_all) += cap[(size_t)(r0 + r)];
    c_all += c1;
    const double total = sat.sum(x0, y0, x1, y1), want = c_all > 0.0 ? total * c1 / c_all : total * 0.5;
    const int lo = along_x ? x0 : y0, hi = along_x ? x1 : y1;
    // first cut c (the left / lower part is [lo, c - 1]) whose left part reaches `want`, or the one before
    int best = lo + 1;
    double best_err = -1.0;
    for (int c = lo + 1; c <= hi; ++c) {
        const double left = along_x ? sat.sum(x0, y0, c - 1, y1) : sat.sum(x0, y0, x1, c - 1);
        const double err = left > want ? left - want : want - left;
        if (best_err < 0.0 || err < best_err) { best = c; best_err = err; }
        if (left >= want) break;
    }
    if (along_x) {
        bisect(sat, cap, x0, y0, best - 1, y1, r0, n1, out);
        bisect(sat, cap, best, y0, x1, y1, r0 + n1, n2, out);
    } else {
        bisect(sat, cap, x0, y0, x1, best - 1, r0, n1, out);
        bisect(sat, cap, x0, best, x1, y1, r0 + n1, n2, out);
    }
}

}  // namespace

void shs_shard_balance(const uint4 *blk, int n_blk, int tiles_x, int tiles_y, int W, int H, int count,
                       std::vector<ShardRegion> &out, double root_share) {
    out.assign((size_t)std::max(count, 0), ShardRegion{1, 1, 1, 0, 0});
    if (count <= 0 || tiles_x <= 0 || tiles_y <= 0) return;
    // 2D difference arrays of the covering blocks' triangles and of the bounded-block coverage
    std::vector<double> tri((size_t)(tiles_x + 1) * (tiles_y + 1), 0.0);
    std::vector<int32_t> cov((size_t)(tiles_x + 1) * (tiles_y + 1), 0);
    auto at = [&](int x, int y) { return (size_t)y * (tiles_x + 1) + x; };
    for (int i = 0; blk && i < n_blk; ++i) {
        const uint4 e = blk[i];
        if (e.z == 0u || e.w == 0u) continue;   // empty, or no bounds (a block straddling draws)
        const int x0 = (int)(e.x & 0xffffu), x1 = (int)(e.x >> 16), y0 = (int)(e.y & 0xffffu), y1 = (int)(e.y >> 16);
        if (x1 < x0 || y1 < y0 || x1 >= tiles_x || y1 >= tiles_y) continue;   // off screen (or stale)
        const double v = (double)e.z;
        tri[at(x0, y0)] += v; tri[at(x1 + 1, y0)] -= v; tri[at(x0, y1 + 1)] -= v; tri[at(x1 + 1, y1 + 1)] += v;
        cov[at(x0, y0)] += 1; cov[at(x1 + 1, y0)] -= 1; cov[at(x0, y1 + 1)] -= 1; cov[at(x1 + 1, y1 + 1)] += 1;
    }
    for (int y = 0; y <= tiles_y; ++y)
        for (int x = 0; x <= tiles_x; ++x) {
            if (x > 0) { tri[at(x, y)] += tri[at(x - 1, y)]; cov[at(x, y)] += cov[at(x - 1, y)]; }
            if (y > 0) { tri[at(x, y)] += tri[at(x, y - 1)]; cov[at(x, y)] += cov[at(x, y - 1)]; }
            if (x > 0 && y > 0) { tri[at(x, y)] -= tri[at(x - 1, y - 1)]; cov[at(x, y)] -= cov[at(x - 1, y - 1)]; }
        }
    Sat sat{tiles_x, tiles_y, std::vector<double>((size_t)(tiles_x + 1) * (tiles_y + 1), 0.0)};
    for (int y = 0; y < tiles_y; ++y)
        for (int x = 0; x < tiles_x; ++x) {
            const double px = (double)(std::min(32, W - 32 * x) * std::min(32, H - 32 * y));
            const double c = px * (REGION_PX + (cov[at(x, y)] > 0 ? REGION_COVERED_PX : 0.0)) + tri[at(x, y)];
            sat.s[(size_t)(y + 1) * (tiles_x + 1) + (x + 1)] =
                c + sat.at(x, y + 1) + sat.at(x + 1, y) - sat.at(x, y);
        }
    std::vector<double> cap((size_t)count, 1.0);
    cap[0] = std::min(1.0, std::max(0.0, root_share));
    bisect(sat, cap, 0, 0, tiles_x - 1, tiles_y - 1, 0, count, out);
}

int shs_regions_next(shs_ctx *ctx, int count, int w, int h) {
    if (ctx->reg_next_fresh && ctx->reg_next_count == count && ctx->reg_next_w == w && ctx->reg_next_h == h) return SHS_OK;
    const int tiles_x = (w + shs_dev::TILE - 1) / shs_dev::TILE, tiles_y = (h + shs_dev::TILE - 1) / shs_dev::TILE;
    auto &wk = ctx->lib_cam;
    const bool have = wk.blkrect_valid && wk.blkrect_w == w && wk.blkrect_h == h && wk.h_blkrect;
    if (have && wk.ov_valid) HIP_TRY(ctx, hipEventSynchronize(wk.ov_after));   // that pass's setup wrote them
    // the same bounds as last time (a static camera, or every rank's first frames): the same layout
    const int n_in = have ? wk.blkrect_n : 0;
    const bool same = ctx->reg_in_count == count && ctx->reg_in_w == w && ctx->reg_in_h == h &&
                      ctx->reg_in_root == ctx->shard_root_permille && (int)ctx->reg_in.size() == n_in &&
                      (n_in == 0 || std::memcmp(ctx->reg_in.data(), wk.h_blkrect, (size_t)n_in * sizeof(uint4)) == 0) &&
                      (int)ctx->reg_next.size() == count;
    if (!same) {
        ctx->reg_in.assign(have ? wk.h_blkrect : nullptr, have ? wk.h_blkrect + n_in : nullptr);
        shs_shard_balance(ctx->reg_in.data(), n_in, tiles_x, tiles_y, w, h, count, ctx->reg_next,
                          ctx->shard_root_permille / 1000.0);
        ctx->reg_in_count = count;
        ctx->reg_in_w = w;
        ctx->reg_in_h = h;
        ctx->reg_in_root = ctx->shard_root_permille;
    }
    ctx->reg_next_count = count;
    ctx->reg_next_w = w;
    ctx->reg_next_h = h;
    ctx->reg_next_fresh = true;
    return SHS_OK;
}

extern "C" {

int shs_shard_balance_rects(const uint32_t *blocks, int32_t n_blocks, int32_t width, int32_t height, int32_t count,
                            int32_t root_permille, int32_t *rects) {
    if (width <= 0 || height <= 0 || count <= 0 || n_blocks < 0 || (n_blocks > 0 && !blocks) || !rects || root_permille < 0 ||
        root_permille > 1000)
        return SHS_ERR_INVALID;
    const int tiles_x = (width + shs_dev::TILE - 1) / shs_dev::TILE, tiles_y = (height + shs_dev::TILE - 1) / shs_dev::TILE;
    std::vector<ShardRegion> out;
    shs_shard_balance(reinterpret_cast<const uint4 *>(blocks), n_blocks, tiles_x, tiles_y, width, height, count, out,
                      root_permille / 1000.0);
    for (int r = 0; r < count; ++r) {
        rects[4 * r] = out[(size_t)r].x0; rects[4 * r + 1] = out[(size_t)r].y0;
        rects[4 * r + 2] = out[(size_t)r].x1; rects[4 * r + 3] = out[(size_t)r].y1;
    }
    return SHS_OK;
}

int shs_get_shard_regions(shs_ctx *ctx, int32_t count, int32_t *rects) {
    if (!ctx || !rects || count <= 0) return SHS_ERR_INVALID;
    if (ctx->reg_last_count != count || (int)ctx->reg_last.size() != count) {
        ctx->err = "no region-sharded camera pass with this shard count";
        return SHS_ERR_INVALID;
    }
    for (int r = 0; r < count; ++r) {
        const ShardRegion &g = ctx->reg_last[(size_t)r];
        rects[4 * r] = g.x0; rects[4 * r + 1] = g.y0; rects[4 * r + 2] = g.x1; rects[4 * r + 3] = g.y1;
    }
    return SHS_OK;
}

}  // extern "C"
