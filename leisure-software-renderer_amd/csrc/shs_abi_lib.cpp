// shs_abi_lib.cpp -- host side of the library raster path of libshs_gpu.so (include/shs_gpu.h,
// "Library path"): MeshData upload, PassShadowMap, PassPBRForward (rasterize_mesh per item) and
// the resolves.  Paths are relative to /root/reference/cpp-folders/src/shs-renderer-lib/include/shs/.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/shs_gpu.h"
#include "shs_ctx.hpp"
#include "shs_footprint.hpp"
#include "shs_glm.hpp"
#include "shs_lib_device.hpp"
#include "shs_lib_internal.hpp"
#include "shs_light_internal.hpp"
#include "shs_tiles_internal.hpp"

using shs_dev::LibBuffers;
using shs_dev::LibDrawGPU;
using shs_dev::LibFrameParams;
using Work = shs_ctx::LibWork;

namespace {

// Smaller passes scan every primitive's box per busy tile (no bins); above this the per-tile bins win
// even for ~1.5K primitives (C5: raster 0.51 -> 0.44 ms, the gather was a 1.5K-box scan per tile).
constexpr int SCAN_MAX_PRIMS = 512;

int harvest(shs_ctx *ctx, Work &w, int k) {
    if (!w.ring_pending[k]) return SHS_OK;
    HIP_TRY(ctx, hipEventSynchronize(w.ring_ev[k][2]));
    float a = 0.0f, b = 0.0f;
    HIP_TRY(ctx, hipEventElapsedTime(&a, w.ring_ev[k][0], w.ring_ev[k][1]));
    HIP_TRY(ctx, hipEventElapsedTime(&b, w.ring_ev[k][1], w.ring_ev[k][2]));
    w.acc_ms[0] += a;
    w.acc_ms[1] += b;
    w.acc_n++;
    w.ring_pending[k] = false;
    return SHS_OK;
}

int harvest_all(shs_ctx *ctx, Work &w) {
    for (int j = 0; j < Work::RING; ++j)
        if (harvest(ctx, w, (w.ring_next + j) % Work::RING)) return SHS_ERR_HIP;
    return SHS_OK;
}

void release_work(Work &w) {
    for (auto &ev : w.ring_ev)
        for (auto &e : ev)
            if (e) { (void)hipEventDestroy(e); e = nullptr; }
    release(w.draws); release(w.recs); release(w.shade); release(w.boxes); release(w.xbase); release(w.zord); release(w.s2s); release(w.blist);
    w.dev_table.clear();
    w.dev_table_at = nullptr;
    w.dev_table_cap = 0;
    release(w.tile_count); release(w.bins); release(w.counters); release(w.busy);
    release(w.spill); release(w.blk_stat); release(w.rstat); release(w.uvw); release(w.items); release(w.pkeys); release(w.pcount); release(w.dynq); release(w.hsq); release(w.hsr); release(w.clipq); release(w.bigq); release(w.bigpre); release(w.rqueue);
    if (w.raster_ev) (void)hipEventDestroy(w.raster_ev);
    if (w.resolve_ev) (void)hipEventDestroy(w.resolve_ev);
    w.raster_ev = w.resolve_ev = nullptr;
    if (w.ov_after) (void)hipEventDestroy(w.ov_after);
    if (w.h_ov) (void)hipHostFree(const_cast<uint32_t *>(w.h_ov));
    if (w.h_blkrect) (void)hipHostFree(w.h_blkrect);
    w.h_blkrect = nullptr;
    w.blkrect_cap = 0;
    w.blkrect_valid = false;
    w.ov_after = nullptr;
    w.h_ov = nullptr;
    w.ov_valid = false;
    w.resolve_ev_valid = false;
    for (int i = 0; i < 2; ++i) {
        if (w.h_draws[i]) (void)hipHostFree(w.h_draws[i]);
        if (w.slot_ev[i]) (void)hipEventDestroy(w.slot_ev[i]);
        w.h_draws[i] = nullptr;
        w.slot_ev[i] = nullptr;
    }
}

// Per-draw block: the uniform-only products of the reference's per-vertex / per-fragment code,
// computed once with the same float operations (shs_glm.hpp restates GLM's op order).
void build_lib_draw(const shs_lib_draw &in, const Mesh &m, int32_t base, LibDrawGPU &o) {
    using namespace shs_host;
    std::memset(&o, 0, sizeof o);
    o.pos = m.pos; o.nrm = m.nrm; o.uv = m.uv; o.idx = m.idx;
    o.cbox = m.cbox;
    o.orig = m.orig;
    o.n_verts = m.n_verts;
    o.tri_base = base;
    o.n_tris = m.n_tris;
    o.program = in.program;
    o.cull_mode = in.cull_mode;
    o.front_ccw = in.front_face_ccw != 0;
    o.shadow = in.shadow != 0;
    o.motion = in.enable_motion_vectors != 0;
    std::memcpy(o.model, in.model, sizeof o.model);
    std::memcpy(o.viewproj, in.viewproj, sizeof o.viewproj);
    lib_normal_matrix(in.model, o.nmat);                       // builtin_shaders.hpp:93-95
    if (std::fabs(det4(in.model)) > 1e-10f) {                  // rasterizer.hpp:296-308
        float inv[16];
        inverse(in.model, inv);
        mul(in.prev_model, inv, o.c2p);
    } else {
        identity(o.c2p);
    }
    std::memcpy(o.prev_vp, in.prev_viewproj, sizeof o.prev_vp);
    std::memcpy(o.light_vp, in.light_viewproj, sizeof o.light_vp);
    const vec3 L = gnormalize(gneg(vec3{in.light_dir_ws[0], in.light_dir_ws[1], in.light_dir_ws[2]}));
    o.L[0] = L.x; o.L[1] = L.y; o.L[2] = L.z;
    for (int i = 0; i < 3; ++i) {
        o.cam[i] = in.camera_pos[i];
        o.lcol[i] = in.light_color[i];
        o.base[i] = in.base_color[i];
    }
    o.lcol[3] = in.light_intensity;
    o.base[3] = in.metallic;
    o.mat[0] = in.roughness;
    o.mat[1] = in.ao;
    o.mat[2] = in.shadow_strength;
    // ShadowParams as the builtin FS builds them: pcf_radius = max(0, r), pcf_step = max(1, step)
    o.shp[0] = in.shadow_bias_const;
    o.shp[1] = in.shadow_bias_slope;
    const int32_t rad = std::max(0, in.shadow_pcf_radius);
    std::memcpy(&o.shp[2], &rad, sizeof rad);
    o.shp[3] = (1.0f < in.shadow_pcf_step) ? in.shadow_pcf_step : 1.0f;
}

// u.base_color_tex (pass_pbr_forward.hpp:173-176): texture id k >= 1, 0 = none.
void bind_texture(const shs_ctx *ctx, int32_t id, LibDrawGPU &o) {
    if (id <= 0) return;
    const Texture &t = ctx->textures[(size_t)id - 1];
    o.tex = t.texels;
    o.tex_w = t.w;
    o.tex_h = t.h;
}

// Upload the draw table through the work's pinned 2-slot staging.  A table equal to the one the
// device buffer already holds (a prepared pass re-rendered) is not sent again: the stream-ordered copy
// is a DMA between two kernels, ~20 us of idle GPU per frame.
int upload_draws(shs_ctx *ctx, Work &w, const std::vector<LibDrawGPU> &d, hipStream_t st) {
    const size_t n = std::max<size_t>(d.size(), 1);
    if (ensure(ctx, w.draws, n)) return SHS_ERR_HIP;
    if (w.dev_table_at == w.draws.p && w.dev_table_cap == w.draws.cap && w.dev_table.size() == d.size() &&
        (d.empty() || std::memcmp(w.dev_table.data(), d.data(), d.size() * sizeof(LibDrawGPU)) == 0))
        return SHS_OK;
    const int s = w.slot;
    w.slot ^= 1;
    if (!w.slot_ev[0])
        for (int i = 0; i < 2; ++i) HIP_TRY(ctx, hipEventCreateWithFlags(&w.slot_ev[i], hipEventDisableTiming));
    if (w.slot_used[s]) HIP_TRY(ctx, hipEventSynchronize(w.slot_ev[s]));
    if (n > w.h_cap) {
        for (int i = 0; i < 2; ++i) {
            if (i != s && w.slot_used[i]) HIP_TRY(ctx, hipEventSynchronize(w.slot_ev[i]));
            if (w.h_draws[i]) HIP_TRY(ctx, hipHostFree(w.h_draws[i]));
            w.h_draws[i] = nullptr;
        }
        const size_t cap = std::max<size_t>(n, 16);
        for (int i = 0; i < 2; ++i) HIP_TRY(ctx, hipHostMalloc(reinterpret_cast<void **>(&w.h_draws[i]), cap * sizeof(LibDrawGPU)));
        w.h_cap = cap;
    }
    if (!d.empty()) {
        std::memcpy(w.h_draws[s], d.data(), d.size() * sizeof(LibDrawGPU));
        HIP_TRY(ctx, hipMemcpyAsync(w.draws.p, w.h_draws[s], d.size() * sizeof(LibDrawGPU), hipMemcpyHostToDevice, st));
    }
    HIP_TRY(ctx, hipEventRecord(w.slot_ev[s], st));
    w.slot_used[s] = true;
    w.dev_table = d;
    w.dev_table_at = w.draws.p;
    w.dev_table_cap = w.draws.cap;
    return SHS_OK;
}


// k_lib_raster's tile order.  Workgroups b and b + 8 share an XCD (and its L2), and workgroup b
// takes positions b, b + G, ... then tickets of queue b & 7 (positions = q mod 8), so position j
// runs on the XCD j % 8.  Owned bin tiles are grouped into supertiles of st x st bin tiles, the
// supertiles dealt over the 8 XCDs; an XCD's positions walk its supertiles in order, the 4 raster
// rows of a bin tile together.  A primitive's tiles, and a bin tile's 4 rows sharing one bin list,
// then mostly land in one L2 instead of up to eight.  st = 0: the plain order (bin tile, row).
std::vector<int32_t> build_rt_order(int tiles_x, int tiles_y, int rtiles_y, int rank, int count, const shs_dev::ShardRegion &reg,
                                    int st) {
    auto owned = [&](int t) { return shs_dev::shard_owned(rank, count, reg, t % tiles_x, t / tiles_x, tiles_x); };
    constexpr int RPB = shs_dev::TILE / 8;   // raster rows per bin tile
    std::vector<int32_t> out;
    auto push_bt = [&](std::vector<int32_t> &v, int t) {
        const int col = t % tiles_x, brow = t / tiles_x;
        for (int r = 0; r < RPB; ++r) {
            const int row = brow * RPB + r;
            if (row < rtiles_y) v.push_back(row * tiles_x + col);
        }
    };
    if (st <= 0) {
        for (int t = 0; t < tiles_x * tiles_y; ++t)
            if (owned(t)) push_bt(out, t);
        return out;
    }
    const int nsx = (tiles_x + st - 1) / st, nsy = (tiles_y + st - 1) / st;
    std::vector<std::vector<int32_t>> lists(8);
    for (int sy = 0; sy < nsy; ++sy)
        for (int sx = 0; sx < nsx; ++sx) {
            std::vector<int32_t> &v = lists[(size_t)((sy * nsx + sx) + 3 * sy) & 7u];
            for (int by = sy * st; by < std::min(tiles_y, (sy + 1) * st); ++by)
                for (int bx = sx * st; bx < std::min(tiles_x, (sx + 1) * st); ++bx) {
                    const int t = by * tiles_x + bx;
                    if (owned(t)) push_bt(v, t);
                }
        }
    size_t longest = 0;
    for (const auto &v : lists) longest = std::max(longest, v.size());
    for (size_t m = 0; m < longest; ++m)
        for (int x = 0; x < 8; ++x)
            if (m < lists[x].size()) out.push_back(lists[x][m]);
    return out;
}

// A device table (raster tile order, owned light lists) for a 4-word key, built and uploaded once into
// its own buffer: a synchronous copy into fresh memory waits for no stream, so a changed shard layout
// costs no pipeline drain.  Past ORDER_CACHE entries the cache is dropped (after the streams drain).
constexpr size_t ORDER_CACHE = 48;

template <typename Build>
int order_lookup(shs_ctx *ctx, std::vector<shs_ctx::OrderEntry> &cache, const uint64_t (&key)[4], Build build,
                 const shs_ctx::OrderEntry *&out) {
    for (const auto &e : cache)
        if (std::memcmp(e.key, key, sizeof key) == 0) { out = &e; return SHS_OK; }
    if (cache.size() >= ORDER_CACHE) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
        for (auto &e : cache) (void)hipFree(e.dev);
        cache.clear();
    }
    std::vector<int32_t> v;
    int n_owned = 0;
    build(v, n_owned);
    shs_ctx::OrderEntry e;
    std::memcpy(e.key, key, sizeof key);
    e.n = (int)v.size();
    e.n_owned = n_owned;
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&e.dev), std::max<size_t>(v.size(), 1) * sizeof(int32_t)));
    if (!v.empty()) HIP_TRY(ctx, hipMemcpy(e.dev, v.data(), v.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    cache.push_back(e);
    out = &cache.back();
    return SHS_OK;
}

uint64_t region_key(const shs_dev::ShardRegion &g) {
    return (uint64_t)(uint16_t)g.x0 | ((uint64_t)(uint16_t)g.y0 << 16) | ((uint64_t)(uint16_t)g.x1 << 32) |
           ((uint64_t)(uint16_t)g.y1 << 48);
}

// Enqueue one pass (w.last_fp / w.last_draws describe it): workspace sizing, draw upload, the two
// kernels.  shadow: PassShadowMap's depth pass into ctx->shadow_map.
int enqueue_pass(shs_ctx *ctx, Work &w, bool shadow) {
    LibFrameParams fp = w.last_fp;
    // With ctx->cam_after_shadow (timing experiments only since round 6, SHS_EXP_CAM_SIDE_STREAM) the camera
    // pass's setup and raster run on the side stream (ctx->setup_stream) beside the shadow pass on the main
    // stream; they read only the meshes and the draw table, and wait for the previous camera resolve (it
    // reads the records, the draw table and the keys this pass rewrites); the resolve waits for the raster.
    hipStream_t ps = (shadow || !ctx->cam_after_shadow) ? ctx->stream : ctx->setup_stream;
    if (!shadow) {
        if (!w.raster_ev) {
            HIP_TRY(ctx, hipEventCreateWithFlags(&w.raster_ev, hipEventDisableTiming));
            HIP_TRY(ctx, hipEventCreateWithFlags(&w.resolve_ev, hipEventDisableTiming));
        }
        if (w.resolve_ev_valid && ps != ctx->stream) HIP_TRY(ctx, hipStreamWaitEvent(ps, w.resolve_ev, 0));
    }
    const int W = fp.W, H = fp.H;
    const int tiles_x = (W + shs_dev::TILE - 1) / shs_dev::TILE, tiles_y = (H + shs_dev::TILE - 1) / shs_dev::TILE;
    const int n_tiles = tiles_x * tiles_y;
    const int rtiles_y = (H + 7) / 8;
    const int n_rt = tiles_x * rtiles_y;
    int64_t total = 0;
    for (const auto &d : w.last_draws) total += d.n_tris;
    if (total > (1 << 27)) { ctx->err = "too many triangles in one pass"; return SHS_ERR_INVALID; }
    const int n_tris = (int)total;
    if (w.extra_cap == 0) w.extra_cap = (uint32_t)std::max(4096, n_tris / 4);
    const size_t n_slots = (size_t)std::max(n_tris, 1) + (shadow ? 0 : w.extra_cap);
    if (ensure(ctx, w.recs, n_slots) || ensure(ctx, w.boxes, n_slots) || ensure(ctx, w.zord, n_slots)) return SHS_ERR_HIP;
    if (!shadow && (ensure(ctx, w.shade, n_slots) || ensure(ctx, w.xbase, (size_t)std::max(n_tris, 1)) ||
                    ensure(ctx, w.clipq, (size_t)std::max(n_tris, 1))))
        return SHS_ERR_HIP;
    bool permuted = false;   // a spatially ordered mesh: the resolve maps winners to slots through s2s
    for (const auto &d : w.last_draws) permuted = permuted || d.orig != nullptr;
    if (!shadow && permuted) {
        if (ensure(ctx, w.s2s, (size_t)std::max(n_tris, 1))) return SHS_ERR_HIP;
        fp.flags |= shs_dev::LF_PERM;
    } else {
        fp.flags &= ~shs_dev::LF_PERM;
    }
    bool textured = false;
    for (const auto &d : w.last_draws) textured = textured || d.tex != nullptr;
    if (textured && !shadow) {
        if (ensure(ctx, w.uvw, 2 * n_slots)) return SHS_ERR_HIP;
        if (!ctx->srgb_lut.p) {   // srgb_to_linear_rgb (builtin_shaders.hpp:25-31) with the host's std::pow
            float lut[256];
            for (int i = 0; i < 256; ++i) lut[i] = std::pow((float)i / 255.0f, 2.2f);
            if (ensure(ctx, ctx->srgb_lut, 256)) return SHS_ERR_HIP;
            HIP_TRY(ctx, hipMemcpy(ctx->srgb_lut.p, lut, sizeof lut, hipMemcpyHostToDevice));
        }
    }
    // every slot enters the large-primitive queue at most once
    if (ensure(ctx, w.bigq, n_slots) || ensure(ctx, w.bigpre, n_slots)) return SHS_ERR_HIP;
    int st = 2;   // supertile edge in bin tiles (SHS_LIB_XCD_ST: timing experiments; 0 = plain order)
    if (const char *e = shs_exp_env("SHS_LIB_XCD_ST")) st = (int)std::strtol(e, nullptr, 0);
    const uint64_t gkey = ((uint64_t)tiles_x << 48) ^ ((uint64_t)tiles_y << 32);
    // rtiles_y too: a height change inside the same bin-tile rows changes the raster-tile rows
    bool reset = gkey != w.geom_key || rtiles_y != w.geom_rtiles_y;
    if (w.tile_count.cap < 2 * (size_t)n_tiles || !w.tile_count.p) {
        if (ensure(ctx, w.tile_count, 2 * (size_t)n_tiles)) return SHS_ERR_HIP;
        reset = true;
    }
    if (w.busy.cap < (size_t)n_rt || !w.busy.p) {
        if (ensure(ctx, w.busy, n_rt)) return SHS_ERR_HIP;
        reset = true;
    }
    if (!w.counters.p) {
        if (ensure(ctx, w.counters, 2 * shs_dev::LC_N) || ensure(ctx, w.rqueue, 2 * shs_dev::LIB_NQW * shs_dev::LIB_QSTRIDE))
            return SHS_ERR_HIP;
        reset = true;
    }
    if (reset) {
        HIP_TRY(ctx, hipMemsetAsync(w.tile_count.p, 0, w.tile_count.cap * sizeof(uint32_t), ps));
        HIP_TRY(ctx, hipMemsetAsync(w.busy.p, 0, w.busy.cap * sizeof(uint32_t), ps));
        HIP_TRY(ctx, hipMemsetAsync(w.counters.p, 0, w.counters.cap * sizeof(uint32_t), ps));
        HIP_TRY(ctx, hipMemsetAsync(w.rqueue.p, 0, w.rqueue.cap * sizeof(uint32_t), ps));
        w.geom_key = gkey;
        w.geom_rtiles_y = rtiles_y;
    }
    const shs_ctx::OrderEntry *order = nullptr;
    {   // the raster tile order of this geometry and ownership
        const shs_dev::ShardRegion reg = fp.count > 1 ? fp.reg : shs_dev::ShardRegion{0, 0, 0, 0, 0};
        const int rank = fp.count > 1 ? fp.rank : 0, count = std::max(fp.count, 1);
        const uint64_t key[4] = {(uint64_t)tiles_x | ((uint64_t)tiles_y << 16) | ((uint64_t)rtiles_y << 32) | ((uint64_t)(st & 0xff) << 56),
                                 (uint64_t)(uint32_t)rank | ((uint64_t)(uint32_t)count << 32), region_key(reg), (uint64_t)reg.on};
        if (order_lookup(ctx, ctx->rt_orders, key,
                         [&](std::vector<int32_t> &v, int &n_owned) {
                             v = build_rt_order(tiles_x, tiles_y, rtiles_y, rank, count, reg, st);
                             n_owned = (int)v.size();
                         },
                         order))
            return SHS_ERR_HIP;
    }
    if (ensure(ctx, w.bins, (size_t)n_tiles * w.bin_cap)) return SHS_ERR_HIP;
    if (!w.spill.p && ensure(ctx, w.spill, 1 << 16)) return SHS_ERR_HIP;
    const int setup_blocks = std::max(1, (n_tris + 255) / 256);
    if (ensure(ctx, w.blk_stat, (size_t)setup_blocks)) return SHS_ERR_HIP;
    // The draw table travels with two int32 arrays appended (as whole 16-B-aligned pseudo records): the
    // compact tri_base per draw (+ sentinel) and the draw of each setup block's first triangle, so the
    // kernels' triangle -> draw lookups start from one load instead of a search over the records.
    const size_t nd = w.last_draws.size();
    const size_t n_int = (nd + 1) + (size_t)setup_blocks;
    const size_t n_extra = (n_int * sizeof(int32_t) + sizeof(LibDrawGPU) - 1) / sizeof(LibDrawGPU);
    std::vector<LibDrawGPU> table(w.last_draws);
    table.resize(nd + n_extra);
    int32_t *ints = reinterpret_cast<int32_t *>(table.data() + nd);
    for (size_t i = 0; i < nd; ++i) ints[i] = w.last_draws[i].tri_base;
    ints[nd] = n_tris;
    for (int b = 0, d = 0; b < setup_blocks; ++b) {
        while (d + 1 < (int)nd && w.last_draws[d + 1].tri_base <= b * 256) ++d;
        ints[nd + 1 + b] = d;
    }
    if (upload_draws(ctx, w, table, ps)) return SHS_ERR_HIP;

    fp.tiles_x = tiles_x; fp.tiles_y = tiles_y; fp.rtiles_y = rtiles_y;
    fp.n_tris = n_tris;
    fp.n_draws = (int)w.last_draws.size();
    fp.bin_cap = w.bin_cap;
    fp.spill_cap = (uint32_t)std::min<size_t>(w.spill.cap, 0xffffffffu);
    fp.extra_cap = shadow ? 0u : w.extra_cap;
    fp.parity = w.frame_index & 1u;
    // scan mode (every busy tile tests every primitive's box) for small passes, per-tile bins above
    {
        const char *e = shs_exp_env("SHS_LIB_SCAN_MAX");   // timing experiments: the scan / bin threshold
        const long scan_max = e ? std::strtol(e, nullptr, 0) : SCAN_MAX_PRIMS;
        fp.scan_mode = n_tris <= scan_max ? 1u : 0u;
    }
    fp.setup_blocks = setup_blocks;
    {
        const char *e = shs_exp_env("SHS_LIB_EXP");   // timing experiments only: parts of the setup skipped
        fp.exp_flags = e ? (uint32_t)std::strtoul(e, nullptr, 0) : 0u;
    }
    fp.n_owned_rt = order->n;
    // Camera pass, tile-sharded: k_lib_plan splits the busy tiles whose bin list is longer than `part`
    // entries into parts rendered by several workgroups (SHS_OPT_LIB_PART: -1 auto = 512 when sharded,
    // 0 = off, else the part size for every camera pass).
    fp.part = 0u;
    if (!shadow && !fp.scan_mode) {
        if (ctx->lib_part > 0) fp.part = (uint32_t)ctx->lib_part;
        else if (ctx->lib_part < 0 && fp.count > 1) fp.part = 512u;
    }
    if (fp.part && ensure(ctx, w.items, (size_t)std::max(fp.n_owned_rt, 1) * shs_dev::LIB_MAXK)) return SHS_ERR_HIP;
    if (fp.part) {   // split tiles' key slots: KEY_EMPTY / 0 once, then reset by each tile's last part
        fp.split_cap = (uint32_t)std::min(std::max(fp.n_owned_rt, 1), 8192);
        const size_t nk = (size_t)fp.split_cap * shs_dev::LIB_RTH_PX;
        if (w.pkeys.cap < nk || w.pcount.cap < fp.split_cap) {
            if (ensure(ctx, w.pkeys, nk) || ensure(ctx, w.pcount, fp.split_cap)) return SHS_ERR_HIP;
            HIP_TRY(ctx, hipMemsetAsync(w.pkeys.p, 0xff, w.pkeys.cap * sizeof(unsigned long long), ps));
            HIP_TRY(ctx, hipMemsetAsync(w.pcount.p, 0, w.pcount.cap * sizeof(uint32_t), ps));
        }
    }
    // the shallow raster (256-candidate rounds, twice the workgroups per CU) when the previous frame's
    // fullest bin tile fit one such round (scan mode: every primitive is a candidate)
    const uint64_t fullest = fp.scan_mode ? (uint64_t)n_tris + (shadow ? 0u : w.st_extra) : w.st_maxbin;
    static const int force_deep = [] {   // SHS_LIB_DEEP=1 (timing experiments): the deep raster for every camera pass
        const char *e = shs_exp_env("SHS_LIB_DEEP");
        return e ? std::atoi(e) : 0;
    }();
    const bool shallow = w.st_checked && fullest <= 256u && !(force_deep && !shadow);
    int &resident = ctx->lib_resident[shadow ? 1 : 0][shallow ? 1 : 0];
    if (resident <= 0) resident = shs_internal::lib_raster_resident_blocks(ctx->device, shadow, shallow);
    const int raster_grid = std::max(1, std::min(fp.n_owned_rt, resident));
    if (ensure(ctx, w.rstat, (size_t)raster_grid)) return SHS_ERR_HIP;
    fp.raster_grid = raster_grid;
    {   // static share of the raster items (SHS_LIB_STATIC_DIV: timing experiments)
        static const int div = [] { const char *e = shs_exp_env("SHS_LIB_STATIC_DIV"); return e ? std::atoi(e) : 2; }();
        fp.static_div = div;
    }
    if (!shadow) {   // k_lib_dyn's per-queue lists: every work position could be dynamic
        const size_t n_max = (size_t)std::max(fp.n_owned_rt, 1) * (fp.part ? 1 + shs_dev::LIB_MAXK : 1);
        fp.dyn_cap = (uint32_t)((n_max + shs_dev::LIB_NQ - 1) / shs_dev::LIB_NQ + 1);
        if (ensure(ctx, w.dynq, (size_t)2 * shs_dev::LIB_NQ * fp.dyn_cap)) return SHS_ERR_HIP;
        // heavy tiles (bin list entries; SHS_LIB_HEAVY: timing experiments, 0 = none)
        static const int heavy = [] { const char *e = shs_exp_env("SHS_LIB_HEAVY"); return e ? std::atoi(e) : 2048; }();
        fp.heavy_min = (uint32_t)std::max(heavy, 0);
    }
    // Camera pass, deep raster: bin lists longer than one candidate round are depth-sorted whole
    // (k_lib_hsort) when the previous pass had such lists (the raster trusts fp.hsort, never the
    // statistics).  Not with k_lib_plan's parts (a part takes a range of list positions).
    fp.hsort = 0u;
    fp.hsort_min = shs_dev::LIB_HSORT_MIN;
#ifndef SHS_EXP_NO_HSORT
    if (!shadow && !fp.scan_mode && !fp.part && !shallow && (!w.st_checked || w.st_maxbin > fp.hsort_min)) {
        if (ensure(ctx, w.hsq, (size_t)n_tiles) || ensure(ctx, w.hsr, (size_t)n_tiles)) return SHS_ERR_HIP;
        fp.hsort = 1u;
    }
#endif

    LibBuffers fb;
    std::memset(&fb, 0, sizeof fb);
    fb.draws = w.draws.p; fb.recs = w.recs.p; fb.shade = w.shade.p; fb.boxes = w.boxes.p; fb.xbase = w.xbase.p; fb.zord = w.zord.p;
    fb.tile_count = w.tile_count.p; fb.bins = w.bins.p; fb.spill = w.spill.p; fb.counters = w.counters.p;
    fb.busy = w.busy.p; fb.blk_stat = w.blk_stat.p; fb.rstat = w.rstat.p;
    fb.clipq = w.clipq.p; fb.bigq = w.bigq.p; fb.bigpre = w.bigpre.p;
    fb.s2s = (fp.flags & shs_dev::LF_PERM) ? w.s2s.p : nullptr;
    fb.dbase = reinterpret_cast<int32_t *>(w.draws.p + nd);
    fb.bdraw = fb.dbase + nd + 1;
    fb.rqueue = w.rqueue.p;
    fb.dynq = shadow ? nullptr : w.dynq.p;
    fb.items = fp.part ? w.items.p : nullptr;
    fb.pkeys = fp.part ? w.pkeys.p : nullptr;
    fb.pcount = fp.part ? w.pcount.p : nullptr;
    fb.hsq = fp.hsort ? w.hsq.p : nullptr;
    fb.hsr = fp.hsort ? w.hsr.p : nullptr;
    // Tile-sharded camera pass in bin mode: each setup workgroup first keeps the rank's triangles of its
    // inputs, positions only (SHS_OPT_SHARD_CULL 0: off).
    const bool listed = !shadow && !fp.scan_mode && fp.count > 1 && !fp.reg.on && ctx->shard_cull;
    const int setup_grid = shs_internal::lib_setup_grid(n_tris, listed);
    fb.rt_order = order->dev;
    if (!shadow && fp.count > 1 && fp.reg.on) {
        // region-sharded camera pass: per setup block its chunk bounds, into mapped host memory (the
        // next pass's region balance reads them once this pass's setup is done)
        if ((size_t)setup_blocks > w.blkrect_cap) {
            if (w.h_blkrect) {
                if (w.ov_valid) HIP_TRY(ctx, hipEventSynchronize(w.ov_after));
                HIP_TRY(ctx, hipHostFree(w.h_blkrect));
                w.h_blkrect = nullptr;
            }
            const size_t cap = std::max<size_t>((size_t)setup_blocks, 1024);
            HIP_TRY(ctx, hipHostMalloc(reinterpret_cast<void **>(&w.h_blkrect), cap * sizeof(uint4),
                                       hipHostMallocMapped | hipHostMallocCoherent));
            w.blkrect_cap = cap;
        }
        fb.blkrect = w.h_blkrect;
        if (ensure(ctx, w.blist, (size_t)setup_blocks)) return SHS_ERR_HIP;
        fb.blist = w.blist.p;
        w.blkrect_n = setup_blocks;
        w.blkrect_w = W;
        w.blkrect_h = H;
        w.blkrect_valid = true;
    }
    if (shadow) {
        fb.depth = ctx->shadow_map.p;
        if (ctx->want_timeline && ctx->timeline_shadow) {   // (profiling: the shadow raster's workgroups)
            const size_t n = (size_t)raster_grid * shs_dev::LTL_STRIDE;
            if (ensure(ctx, ctx->lib_timeline, n)) return SHS_ERR_HIP;
            HIP_TRY(ctx, hipMemsetAsync(ctx->lib_timeline.p, 0, n * sizeof(uint64_t), ps));
            fb.timeline = ctx->lib_timeline.p;
        }
    } else {
        fb.hdr = ctx->lib_hdr.p; fb.depth = ctx->lib_depth.p; fb.motion = ctx->lib_motion.p;
        fb.keys = ctx->lib_keys.p;
        fb.uvw = textured ? w.uvw.p : nullptr;
        fb.srgb_lut = ctx->srgb_lut.p;
        fb.blkcov = ctx->lib_blkcov.p;
        if (w.tm_fused) {   // PassTonemap in k_lib_resolve (shs_lib_fuse_tonemap)
            const shs_tonemap_desc &d = w.tm_desc;
            const size_t npx = (size_t)W * H;
            if ((d.flags & SHS_TONEMAP_LDR) && ensure(ctx, ctx->lib_ldr, npx)) return SHS_ERR_HIP;
            if ((d.flags & SHS_TONEMAP_PRESENT) && ensure(ctx, ctx->lib_present, npx)) return SHS_ERR_HIP;
            const float g = std::max(0.001f, d.gamma);
            if (ensure(ctx, ctx->tm_thr_dev, 256)) return SHS_ERR_HIP;
            if (ctx->tm_thr_dev_gamma != g) {   // rare (a new gamma): a synchronous upload
                float thr[256];
                shs_tonemap_thresholds(g, thr);
                HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
                HIP_TRY(ctx, hipMemcpy(ctx->tm_thr_dev.p, thr, sizeof thr, hipMemcpyHostToDevice));
                ctx->tm_thr_dev_gamma = g;
            }
            fb.tm_thr = ctx->tm_thr_dev.p;
            fb.tm_ldr = (d.flags & SHS_TONEMAP_LDR) ? ctx->lib_ldr.p : nullptr;
            fb.tm_present = (d.flags & SHS_TONEMAP_PRESENT) ? ctx->lib_present.p : nullptr;
            fp.tm_exposure = std::max(0.0001f, d.exposure);
            fp.tm_inv_gamma = 1.0f / g;
        }
        fb.shadow_map = ctx->have_shadow ? ctx->shadow_map.p : nullptr;
        fb.lights = ctx->lights.p;
        fb.tile_counts = ctx->list_counts.p;
        fb.tile_indices = ctx->list_indices.p;
        if (ctx->want_timeline && !ctx->timeline_shadow) {
            const size_t n = (size_t)raster_grid * shs_dev::LTL_STRIDE;
            if (ensure(ctx, ctx->lib_timeline, n)) return SHS_ERR_HIP;
            HIP_TRY(ctx, hipMemsetAsync(ctx->lib_timeline.p, 0, n * sizeof(uint64_t), ps));
            fb.timeline = ctx->lib_timeline.p;
            const size_t ns = (size_t)std::max(setup_blocks, 1) * shs_dev::STL_STRIDE;
            if (ensure(ctx, ctx->lib_stimeline, ns)) return SHS_ERR_HIP;
            HIP_TRY(ctx, hipMemsetAsync(ctx->lib_stimeline.p, 0, ns * sizeof(uint64_t), ps));
            fb.stimeline = ctx->lib_stimeline.p;
        }
    }
    hipEvent_t *ev = nullptr;
    if (ctx->timing) {
        const int k = w.ring_next;
        w.ring_next = (k + 1) % Work::RING;
        if (harvest(ctx, w, k)) return SHS_ERR_HIP;
        if (!w.ring_ev[k][0])
            for (int i = 0; i < 3; ++i) HIP_TRY(ctx, hipEventCreateWithFlags(&w.ring_ev[k][i], hipEventDisableSystemFence));
        ev = w.ring_ev[k];
        w.ring_pending[k] = true;
    }
    if (!w.ov_after) {
        HIP_TRY(ctx, hipEventCreateWithFlags(&w.ov_after, hipEventDisableTiming));
        HIP_TRY(ctx, shs_host_ov_alloc(&w.h_ov));
    }
    // the previous pass's setup (the only other writer of the word) is done before it is zeroed
    if (w.ov_valid) HIP_TRY(ctx, hipEventSynchronize(w.ov_after));
    *w.h_ov = 0u;
    fb.ov_host = const_cast<uint32_t *>(w.h_ov);
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[0], ps));
    HIP_TRY(ctx, shs_internal::launch_lib_setup(fp, fb, shadow, listed, ps));
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[1], ps));
    // the pass's overflow word is final after its setup kernels (setup, clip, large-primitive marks), so
    // superseding the pass checks it at ov_after, without waiting for the raster
    HIP_TRY(ctx, hipEventRecord(w.ov_after, ps));
    w.ov_valid = true;
    HIP_TRY(ctx, shs_internal::launch_lib_raster(fp, fb, shadow, shallow, raster_grid, ps));
    if (!shadow) {   // the camera pass's shading runs in its own kernel (event [2] closes both)
        if (ps != ctx->stream) {
            HIP_TRY(ctx, hipEventRecord(w.raster_ev, ps));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, w.raster_ev, 0));
        }
        int prog = w.last_draws.empty() ? -1 : w.last_draws[0].program;
        for (const auto &d : w.last_draws)
            if (d.program != prog) prog = -1;
        if (prog != 5 && prog != 0) prog = -1;
        const bool wide = fp.count <= 1;   // the whole frame's build (PBR: 5 waves) or a sharded rank's
        int &res = ctx->lib_resolve_resident[(prog == 5 ? 0 : prog == 0 ? 1 : 2) * 2 + wide];
        if (res <= 0) res = shs_internal::lib_resolve_resident_blocks(ctx->device, prog, wide);
        const int rgrid = std::max(1, std::min(fp.n_owned_rt, res));
        HIP_TRY(ctx, shs_internal::launch_lib_resolve(fp, fb, prog, wide, rgrid, ctx->stream));
        HIP_TRY(ctx, hipEventRecord(w.resolve_ev, ctx->stream));
        w.resolve_ev_valid = true;
    }
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[2], ctx->stream));
    w.last_parity = fp.parity;
    w.frame_index++;
    w.last_setup_blocks = setup_grid;
    w.last_raster_grid = raster_grid;
    w.last_n_tris = n_tris;
    w.need_check = true;
    w.done = true;
    return SHS_OK;
}

// A pass about to be superseded (its workspace and targets rewritten) whose overflow word is set is
// finished first -- re-issued with grown capacities -- so no stream-ordered consumer of it (a tonemap,
// a copy, a gather queued behind it) sees an incomplete pass.
int lib_finish(shs_ctx *ctx);
int check_superseded(shs_ctx *ctx, Work &w) {
    if (!w.need_check || !w.ov_valid) return SHS_OK;
    HIP_TRY(ctx, hipEventSynchronize(w.ov_after));
    return *w.h_ov ? lib_finish(ctx) : SHS_OK;
}

uint32_t next_pow2(uint64_t v) {
    uint32_t p = 1;
    while (p < v && p < (1u << 30)) p <<= 1;
    return p;
}

// Read one pass's counters and statistics; grows what overflowed and returns true then.
int check_pass(shs_ctx *ctx, Work &w, bool &grew) {
    grew = false;
    if (!w.need_check) return SHS_OK;
    uint32_t *c = ctx->h_lib_counters;
    HIP_TRY(ctx, hipMemcpy(c, w.counters.p + w.last_parity * shs_dev::LC_N, shs_dev::LC_N * sizeof(uint32_t),
                           hipMemcpyDeviceToHost));
    std::vector<uint2> bs(w.last_setup_blocks), rs(w.last_raster_grid);
    HIP_TRY(ctx, hipMemcpy(bs.data(), w.blk_stat.p, bs.size() * sizeof(uint2), hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(rs.data(), w.rstat.p, rs.size() * sizeof(uint2), hipMemcpyDeviceToHost));
    w.st_clip = w.st_raster = w.st_covered = w.st_maxbin = 0;
    for (const uint2 &b : bs) { w.st_clip += b.x; w.st_raster += b.y; }
    for (const uint2 &r : rs) { w.st_covered += r.x; w.st_maxbin = std::max<uint64_t>(w.st_maxbin, r.y); }
    if (&w == &ctx->lib_cam) w.st_covered = c[shs_dev::LC_COVERED];   // counted by k_lib_resolve
    w.st_spill = c[shs_dev::LC_SPILL];
    w.st_extra = c[shs_dev::LC_EXTRA];
    if (w.st_maxbin > w.bin_cap) w.bin_cap = next_pow2(std::min<uint64_t>(w.st_maxbin, 1u << 24));
    w.st_checked = true;
    const uint32_t ov = c[shs_dev::LC_OVERFLOW];
    if (ov & shs_dev::LOV_SPILL) {
        const size_t need = c[shs_dev::LC_SPILL];
        release(w.spill);
        if (ensure(ctx, w.spill, need + need / 4 + 1024)) return SHS_ERR_HIP;
        grew = true;
    }
    if (ov & shs_dev::LOV_EXTRA) {
        w.extra_cap = (uint32_t)std::min<uint64_t>((uint64_t)c[shs_dev::LC_EXTRA] + c[shs_dev::LC_EXTRA] / 4 + 4096, 1u << 28);
        grew = true;
    }
    w.need_check = false;
    return SHS_OK;
}

// Wait for the enqueued passes; a pass that overflowed a capacity is re-issued (and a camera pass
// that sampled a re-issued shadow map with it).
int lib_finish(shs_ctx *ctx) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (int attempt = 0; attempt < 6; ++attempt) {
        bool g_sh = false, g_cam = false;
        if (check_pass(ctx, ctx->lib_shadow, g_sh) || check_pass(ctx, ctx->lib_cam, g_cam)) return SHS_ERR_HIP;
        if (!g_sh && !g_cam) return SHS_OK;
        if (g_sh && enqueue_pass(ctx, ctx->lib_shadow, true)) return SHS_ERR_HIP;
        if ((g_cam || (g_sh && ctx->cam_after_shadow)) && ctx->lib_cam.done) {
            if (enqueue_pass(ctx, ctx->lib_cam, false)) return SHS_ERR_HIP;
            if (ctx->have_ldr && shs_tonemap_reissue(ctx)) return SHS_ERR_HIP;
        }
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->err = "capacity overflow persisted";
    return SHS_ERR_OVERFLOW;
}

int check_lib_mesh(shs_ctx *ctx, int32_t id) {
    if (id < 0 || id >= (int)ctx->meshes.size() || !ctx->meshes[id].live || !ctx->meshes[id].lib) {
        ctx->err = "bad mesh id (not a library mesh)";
        return SHS_ERR_INVALID;
    }
    return SHS_OK;
}

}  // namespace

int shs_lib_ensure_final(shs_ctx *ctx) {
    const int rc = check_superseded(ctx, ctx->lib_shadow);
    return rc ? rc : check_superseded(ctx, ctx->lib_cam);
}

void shs_lib_release(shs_ctx *ctx) {
    release_work(ctx->lib_cam);
    release_work(ctx->lib_shadow);
    for (auto *cache : {&ctx->rt_orders, &ctx->cull_orders}) {
        for (auto &e : *cache) (void)hipFree(e.dev);
        cache->clear();
    }
    for (auto &t : ctx->textures)
        if (t.texels) (void)hipFree(t.texels);
    ctx->textures.clear();
    release(ctx->srgb_lut);
    release(ctx->lib_hdr); release(ctx->lib_keys); release(ctx->lib_blkcov); ctx->blkcov_zero_at = nullptr; release(ctx->tm_thr_dev); ctx->tm_thr_dev_gamma = -1.0f; release(ctx->lib_depth); release(ctx->lib_motion); release(ctx->shadow_map);
    release(ctx->lights); release(ctx->depth_ranges);
    release(ctx->list_counts); release(ctx->list_indices); release(ctx->lib_timeline); release(ctx->lib_stimeline);
    release(ctx->lib_ldr); release(ctx->lib_present); release(ctx->lib_mb); release(ctx->lib_mb_present);
    release(ctx->lb_lights); release(ctx->lb_ndc); release(ctx->lb_counts); release(ctx->lb_indices);
    release(ctx->occ_depth); release(ctx->occ_visible); release(ctx->occ_flags); release(ctx->occ_objs); release(ctx->occ_rects); release(ctx->occ_tris);
    release(ctx->dd_objs); release(ctx->dd_tris); release(ctx->dd_depth0); release(ctx->dd_depth); release(ctx->dd_lit_b);
    release(ctx->dd_rgba); release(ctx->dd_keys); release(ctx->dd_big);
    release(ctx->cp_a); release(ctx->cp_b); release(ctx->cp_src); release(ctx->cp_depth); release(ctx->cp_vel); release(ctx->cp_focus);
    if (ctx->h_lib_counters) (void)hipHostFree(ctx->h_lib_counters);
    ctx->h_lib_counters = nullptr;
}

// The stored order of a library mesh's triangles: MeshData indices sorted by the 30-bit Morton code of
// the centroid in the mesh's bounds (stable; triangles with an out-of-range index or a non-finite
// centroid last).  Empty when the mesh fits one chunk or the order is the identity.
static std::vector<uint32_t> spatial_order(const float *pos, int32_t n_verts, const uint32_t *idx, int32_t n_tris) {
    std::vector<uint32_t> order;
    if (n_tris <= 256) return order;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    std::vector<float> cen((size_t)n_tris * 3);
    std::vector<uint8_t> ok((size_t)n_tris);
    for (int32_t t = 0; t < n_tris; ++t) {
        bool good = true;
        float c[3] = {0.0f, 0.0f, 0.0f};
        for (int k = 0; k < 3; ++k) {
            const uint32_t v = idx ? idx[3 * (size_t)t + k] : (uint32_t)(3 * t + k);
            if (v >= (uint32_t)n_verts) { good = false; break; }
            for (int q = 0; q < 3; ++q) c[q] += pos[3 * (size_t)v + q];
        }
        for (int q = 0; q < 3 && good; ++q) good = std::isfinite(c[q]);
        ok[t] = good;
        for (int q = 0; q < 3; ++q) {
            cen[3 * (size_t)t + q] = c[q];
            if (good) { lo[q] = std::min(lo[q], c[q]); hi[q] = std::max(hi[q], c[q]); }
        }
    }
    auto spread = [](uint32_t x) {   // 10 bits -> every third bit
        x &= 0x3ffu;
        x = (x | (x << 16)) & 0x030000ffu;
        x = (x | (x << 8)) & 0x0300f00fu;
        x = (x | (x << 4)) & 0x030c30c3u;
        x = (x | (x << 2)) & 0x09249249u;
        return x;
    };
    std::vector<uint64_t> key((size_t)n_tris);
    for (int32_t t = 0; t < n_tris; ++t) {
        uint32_t code = 0xffffffffu;
        if (ok[t]) {
            code = 0u;
            for (int q = 0; q < 3; ++q) {
                const float ext = hi[q] - lo[q];
                const float u = ext > 0.0f ? (cen[3 * (size_t)t + q] - lo[q]) / ext : 0.0f;
                const uint32_t b = (uint32_t)std::min(1023.0f, std::max(0.0f, u * 1024.0f));
                code |= spread(b) << q;
            }
        }
        key[t] = ((uint64_t)code << 32) | (uint32_t)t;   // ties keep the MeshData order
    }
    std::sort(key.begin(), key.end());
    order.resize((size_t)n_tris);
    bool identity = true;
    for (int32_t p = 0; p < n_tris; ++p) {
        order[p] = (uint32_t)key[p];
        identity = identity && order[p] == (uint32_t)p;
    }
    if (identity) order.clear();
    return order;
}

extern "C" {

int shs_mesh_upload(shs_ctx *ctx, const float *positions, int32_t n_verts, const float *normals, int32_t n_normals,
                    const float *uvs, int32_t n_uvs, const uint32_t *indices, int64_t n_indices, int32_t *mesh_id) {
    if (!ctx || !positions || n_verts <= 0 || !mesh_id || n_normals < 0 || n_uvs < 0 || n_indices < 0 ||
        (n_normals > 0 && !normals) || (n_uvs > 0 && !uvs) || (n_indices > 0 && !indices))
        return SHS_ERR_INVALID;
    const int64_t n_tris = indices ? n_indices / 3 : n_verts / 3;
    if (n_tris > (1 << 27)) { ctx->err = "mesh too large"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    // read_v's defaults (rasterizer.hpp:196-202) materialised: normal (0,1,0), uv (0,0)
    std::vector<float> nrm((size_t)n_verts * 3), uv((size_t)n_verts * 2, 0.0f);
    for (int32_t i = 0; i < n_verts; ++i) {
        const bool hn = i < n_normals;
        nrm[3 * (size_t)i] = hn ? normals[3 * (size_t)i] : 0.0f;
        nrm[3 * (size_t)i + 1] = hn ? normals[3 * (size_t)i + 1] : 1.0f;
        nrm[3 * (size_t)i + 2] = hn ? normals[3 * (size_t)i + 2] : 0.0f;
        if (i < n_uvs) { uv[2 * (size_t)i] = uvs[2 * (size_t)i]; uv[2 * (size_t)i + 1] = uvs[2 * (size_t)i + 1]; }
    }
    Mesh m;
    m.lib = true;
    m.n_verts = n_verts;
    m.n_tris = (int32_t)n_tris;
    if (indices && n_indices < 3) m.n_tris = 0;
    // a HIP_TRY that returns early frees what this upload already allocated (the mesh is not registered)
    struct Guard {
        Mesh &m;
        bool keep = false;
        ~Guard() {
            if (keep) return;
            for (void *p : {(void *)m.orig, (void *)m.pos, (void *)m.nrm, (void *)m.uv, (void *)m.idx, (void *)m.cbox})
                if (p) (void)hipFree(p);
        }
    } guard{m};
    // Spatial order (meshes over one 256-triangle chunk): the triangles are stored sorted by the Morton
    // code of their centroid, so a setup block's chunk box is tight and a region-sharded rank skips the
    // blocks that miss its rectangle.  The submission order stays the MeshData order:
    // `orig` gives every stored triangle its MeshData index, the sequence the z ties and the clipped
    // fans are ordered by (rasterizer.hpp:181-442 draws in index order).  A soup's vertices move with
    // their triangle; an indexed mesh keeps its vertices and reorders its index triples.
    const std::vector<uint32_t> order = spatial_order(positions, n_verts, indices, m.n_tris);
    std::vector<float> pos_s, nrm_s, uv_s;
    std::vector<uint32_t> idx_s;
    if (!order.empty()) {
        if (indices) {
            idx_s.resize((size_t)m.n_tris * 3);
            for (size_t p = 0; p < order.size(); ++p)
                for (int k = 0; k < 3; ++k) idx_s[3 * p + k] = indices[3 * (size_t)order[p] + k];
            indices = idx_s.data();
        } else {
            pos_s.assign(positions, positions + (size_t)n_verts * 3);
            nrm_s = nrm;
            uv_s = uv;
            for (size_t p = 0; p < order.size(); ++p)
                for (int k = 0; k < 3; ++k) {
                    const size_t dv = 3 * p + k, sv = 3 * (size_t)order[p] + k;
                    for (int q = 0; q < 3; ++q) { pos_s[3 * dv + q] = positions[3 * sv + q]; nrm_s[3 * dv + q] = nrm[3 * sv + q]; }
                    uv_s[2 * dv] = uv[2 * sv]; uv_s[2 * dv + 1] = uv[2 * sv + 1];
                }
            positions = pos_s.data();
            nrm.swap(nrm_s);
            uv.swap(uv_s);
        }
        HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.orig), order.size() * sizeof(uint32_t)));
        HIP_TRY(ctx, hipMemcpy(m.orig, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    // model-space bounds (PassShadowMap's mesh_bounds_cache, pass_shadow_map.hpp:90-102)
    for (int k = 0; k < 3; ++k) { m.bmin[k] = 3.402823466e38f; m.bmax[k] = -3.402823466e38f; }
    for (int32_t i = 0; i < n_verts; ++i)
        for (int k = 0; k < 3; ++k) {
            const float p = positions[3 * (size_t)i + k];
            m.bmin[k] = (p < m.bmin[k]) ? p : m.bmin[k];   // glm::min(bmin, p)
            m.bmax[k] = (m.bmax[k] < p) ? p : m.bmax[k];   // glm::max(bmax, p)
        }
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.pos), (size_t)n_verts * 3 * sizeof(float)));
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.nrm), (size_t)n_verts * 3 * sizeof(float)));
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.uv), (size_t)n_verts * 2 * sizeof(float)));
    HIP_TRY(ctx, hipMemcpy(m.pos, positions, (size_t)n_verts * 3 * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(m.nrm, nrm.data(), nrm.size() * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(m.uv, uv.data(), uv.size() * sizeof(float), hipMemcpyHostToDevice));
    if (indices && n_indices >= 3) {
        HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.idx), (size_t)n_tris * 3 * sizeof(uint32_t)));
        HIP_TRY(ctx, hipMemcpy(m.idx, indices, (size_t)n_tris * 3 * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (m.n_tris > 0) {   // chunk boxes (k_lib_setup's block bounds): out-of-range indices are skipped there
        const int64_t n_chunks = ((int64_t)m.n_tris + 255) / 256;
        std::vector<float4> cb((size_t)n_chunks * 2);
        for (int64_t c = 0; c < n_chunks; ++c) {
            float mn[3] = {3.402823466e38f, 3.402823466e38f, 3.402823466e38f}, mx[3] = {-3.402823466e38f, -3.402823466e38f, -3.402823466e38f};
            const int64_t t1 = std::min<int64_t>(m.n_tris, (c + 1) * 256);
            for (int64_t t = c * 256; t < t1; ++t)
                for (int k = 0; k < 3; ++k) {
                    const uint32_t v = indices ? indices[3 * t + k] : (uint32_t)(3 * t + k);
                    if (v >= (uint32_t)n_verts) continue;
                    for (int q = 0; q < 3; ++q) {
                        const float p = positions[3 * (size_t)v + q];
                        mn[q] = std::min(mn[q], p);
                        mx[q] = std::max(mx[q], p);
                    }
                }
            cb[2 * c] = make_float4(mn[0], mn[1], mn[2], 0.0f);
            cb[2 * c + 1] = make_float4(mx[0], mx[1], mx[2], 0.0f);
        }
        HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.cbox), cb.size() * sizeof(float4)));
        HIP_TRY(ctx, hipMemcpy(m.cbox, cb.data(), cb.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    m.live = true;
    ctx->meshes.push_back(m);
    guard.keep = true;
    *mesh_id = (int32_t)ctx->meshes.size() - 1;
    return SHS_OK;
}

int shs_texture_upload(shs_ctx *ctx, const uint8_t *rgba, int32_t w, int32_t h, int32_t *tex_id) {
    if (!ctx || !rgba || !tex_id || w <= 0 || h <= 0 || (int64_t)w * h > (1ll << 28)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    Texture t;
    const size_t bytes = (size_t)w * h * 4;
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&t.texels), bytes));
    const hipError_t e = hipMemcpy(t.texels, rgba, bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(t.texels);
        ctx->err = hipGetErrorString(e);
        return SHS_ERR_HIP;
    }
    t.w = w;
    t.h = h;
    t.live = true;
    // a released slot is reused (ids stay small); TextureAssetHandle convention: 1-based, 0 = none
    size_t slot = 0;
    while (slot < ctx->textures.size() && ctx->textures[slot].live) ++slot;
    if (slot == ctx->textures.size()) ctx->textures.push_back(t);
    else ctx->textures[slot] = t;
    *tex_id = (int32_t)slot + 1;
    return SHS_OK;
}

int shs_texture_release(shs_ctx *ctx, int32_t tex_id) {
    if (!ctx || tex_id <= 0 || tex_id > (int32_t)ctx->textures.size() || !ctx->textures[(size_t)tex_id - 1].live)
        return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
    Texture &t = ctx->textures[(size_t)tex_id - 1];
    HIP_TRY(ctx, hipFree(t.texels));
    t = Texture{};
    return SHS_OK;
}

int shs_render_shadow_map(shs_ctx *ctx, int32_t w, int32_t h, const float sun_dir[3], const shs_shadow_caster *casters,
                          int32_t n_casters, float light_viewproj_out[16]) {
    if (!ctx || !sun_dir || w <= 0 || h <= 0 || w > 16384 || h > 16384 || n_casters < 0 || (n_casters > 0 && !casters))
        return SHS_ERR_INVALID;
    for (int i = 0; i < n_casters; ++i)
        if (check_lib_mesh(ctx, casters[i].mesh_id)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (!ctx->h_lib_counters && hipHostMalloc(reinterpret_cast<void **>(&ctx->h_lib_counters), shs_dev::LC_N * sizeof(uint32_t)) != hipSuccess)
        return SHS_ERR_HIP;
    {   // the pending passes are checked before this one rewrites the shadow map they read / wrote
        const int rc = check_superseded(ctx, ctx->lib_shadow);
        if (rc) return rc;
        const int rc2 = check_superseded(ctx, ctx->lib_cam);
        if (rc2) return rc2;
    }
    using namespace shs_host;
    // scene AABB of the casters (pass_shadow_map.hpp:80-131)
    vec3 mn = {1e30f, 1e30f, 1e30f}, mx = {-1e30f, -1e30f, -1e30f};
    auto expand = [&](vec3 p) {
        mn = {(p.x < mn.x) ? p.x : mn.x, (p.y < mn.y) ? p.y : mn.y, (p.z < mn.z) ? p.z : mn.z};
        mx = {(mx.x < p.x) ? p.x : mx.x, (mx.y < p.y) ? p.y : mx.y, (mx.z < p.z) ? p.z : mx.z};
    };
    bool any = false;
    for (int i = 0; i < n_casters; ++i) {
        const Mesh &m = ctx->meshes[casters[i].mesh_id];
        const float *b0 = m.bmin, *b1 = m.bmax, *M = casters[i].model;
        const vec3 c[8] = {{b0[0], b0[1], b0[2]}, {b1[0], b0[1], b0[2]}, {b0[0], b1[1], b0[2]}, {b1[0], b1[1], b0[2]},
                           {b0[0], b0[1], b1[2]}, {b1[0], b0[1], b1[2]}, {b0[0], b1[1], b1[2]}, {b1[0], b1[1], b1[2]}};
        for (const vec3 &p : c)
            expand(vec3{(M[0] * p.x + M[4] * p.y) + (M[8] * p.z + M[12] * 1.0f), (M[1] * p.x + M[5] * p.y) + (M[9] * p.z + M[13] * 1.0f),
                        (M[2] * p.x + M[6] * p.y) + (M[10] * p.z + M[14] * 1.0f)});
        any = true;
    }
    if (!any) { expand(vec3{-1.0f, -1.0f, -1.0f}); expand(vec3{1.0f, 1.0f, 1.0f}); }
    float view[16], proj[16];
    dir_light_camera_aabb(vec3{sun_dir[0], sun_dir[1], sun_dir[2]}, mn, mx, 10.0f, (uint32_t)std::max(w, 1), view, proj,
                          ctx->shadow_vp);
    if (light_viewproj_out) std::memcpy(light_viewproj_out, ctx->shadow_vp, sizeof ctx->shadow_vp);

    if (ensure(ctx, ctx->shadow_map, (size_t)w * h)) return SHS_ERR_HIP;
    Work &wk = ctx->lib_shadow;
    wk.last_draws.clear();
    int32_t base = 0;
    for (int i = 0; i < n_casters; ++i) {
        const Mesh &m = ctx->meshes[casters[i].mesh_id];
        LibDrawGPU d;
        std::memset(&d, 0, sizeof d);
        d.pos = m.pos; d.nrm = m.nrm; d.uv = m.uv; d.idx = m.idx;
        d.n_verts = m.n_verts; d.tri_base = base; d.n_tris = m.n_tris;
        std::memcpy(d.model, casters[i].model, sizeof d.model);
        std::memcpy(d.viewproj, ctx->shadow_vp, sizeof d.viewproj);
        wk.last_draws.push_back(d);
        base += m.n_tris;
    }
    LibFrameParams fp;
    std::memset(&fp, 0, sizeof fp);
    fp.W = w; fp.H = h;
    fp.rank = 0; fp.count = 1;   // the whole shadow map (SHS_OPT_SHADOW_FOOTPRINT: the next camera pass narrows it)
    wk.last_fp = fp;
    ctx->shadow_w = w;
    ctx->shadow_h = h;
    ctx->cam_after_shadow = false;
    ctx->have_shadow = true;
    if (ctx->shadow_footprint) {   // recorded; shs_render_pbr_forward enqueues it for the texels it reads
        ctx->shadow_pending = true;
        return SHS_OK;
    }
    ctx->shadow_pending = false;
    ctx->shadow_reg = shs_dev::ShardRegion{0, 0, 0, 0, 0};
    ctx->shadow_span.clear();
    return enqueue_pass(ctx, wk, true);
}

// Enqueue the recorded shadow pass over the bin tiles of `reg` (reg.on = 0: the whole map), within it
// only the row spans `span` (per bin-tile row, x0 | x1 << 16; empty: the whole rectangle).
static int enqueue_shadow(shs_ctx *ctx, const shs_dev::ShardRegion &reg, const std::vector<uint32_t> &span = {}) {
    Work &wk = ctx->lib_shadow;
    wk.last_fp.reg = reg;
    wk.last_fp.rank = 0;
    wk.last_fp.count = reg.on ? 2 : 1;   // a region pass: only the rectangle's tiles are owned
    const bool spans = reg.on && !span.empty() && span.size() <= (size_t)shs_dev::LIB_SPAN_ROWS;
    wk.last_fp.span_rows = spans ? (int32_t)span.size() : 0;
    for (size_t r = 0; spans && r < span.size(); ++r) wk.last_fp.span[r] = span[r];
    ctx->shadow_pending = false;
    ctx->shadow_reg = reg;
    ctx->shadow_span = spans ? span : std::vector<uint32_t>{};
    return enqueue_pass(ctx, wk, true);
}

}  // extern "C"

int shs_lib_flush_shadow(shs_ctx *ctx) {
    if (!ctx->shadow_pending) return SHS_OK;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    return enqueue_shadow(ctx, shs_dev::ShardRegion{0, 0, 0, 0, 0});
}

// A footprint-restricted shadow map whose casters include `pos` (a mesh about to be released) is
// rendered whole first: a later camera pass that reads beyond the footprint could not re-render it.
int shs_lib_widen_shadow(shs_ctx *ctx, const float *pos) {
    if (ctx->shadow_pending || !ctx->have_shadow || !ctx->shadow_reg.on) return SHS_OK;
    bool reads = false;
    for (const LibDrawGPU &d : ctx->lib_shadow.last_draws) reads = reads || d.pos == pos;
    if (!reads) return SHS_OK;
    const int rc = check_superseded(ctx, ctx->lib_shadow);
    return rc ? rc : enqueue_shadow(ctx, shs_dev::ShardRegion{0, 0, 0, 0, 0});
}

extern "C" {

// SHS_OPT_SHADOW_FOOTPRINT: the shadow-map bin tiles the camera pass about to be enqueued can read
// (shs_footprint.hpp): the union over its shadowed draws of the light-space bounds of (the draw's world
// box) ∩ (the camera frustum slice of the pixels this rank shades), widened by the PCF reach.
// Also the rows' spans (shs_footprint.hpp footprint_rows, in bin tiles): empty when the map is taller
// than LIB_SPAN_ROWS bin tiles or some draw has no bound.  (-DSHS_SHADOW_SPANS=0: rectangles only,
// a timing comparison.)
#ifndef SHS_SHADOW_SPANS
#define SHS_SHADOW_SPANS 1
#endif
static shs_dev::ShardRegion shadow_region_for(const shs_ctx *ctx, const shs_lib_frame &f, const shs_lib_draw *draws,
                                              int32_t n_draws, const shs_dev::ShardRegion &cam_reg,
                                              std::vector<uint32_t> &span) {
    const int W = f.width, H = f.height;
    int px[4] = {0, 0, W - 1, H - 1};
    if (f.shard_count > 1 && cam_reg.on) {
        px[0] = cam_reg.x0 * shs_dev::TILE;
        px[1] = cam_reg.y0 * shs_dev::TILE;
        px[2] = std::min(W, (cam_reg.x1 + 1) * shs_dev::TILE) - 1;
        px[3] = std::min(H, (cam_reg.y1 + 1) * shs_dev::TILE) - 1;
    }
    const int T = shs_dev::TILE;
    const int rows = (ctx->shadow_h + T - 1) / T;
    bool spans = SHS_SHADOW_SPANS && rows <= shs_dev::LIB_SPAN_ROWS;
    std::vector<int> sx0((size_t)rows, 1), sx1((size_t)rows, 0);   // texel columns per row (x1 < x0: none)
    double pts[220][2];
    shs_fp::TexelRect t;
    for (int i = 0; i < n_draws; ++i) {
        const shs_lib_draw &d = draws[i];
        if (!d.shadow) continue;
        const Mesh &m = ctx->meshes[d.mesh_id];
        double bmin[3], bmax[3];
        shs_fp::world_box(d.model, m.bmin, m.bmax, bmin, bmax);
        const int rad = std::max(0, d.shadow_pcf_radius);
        const int step = std::max(1, (int)std::round((1.0f < d.shadow_pcf_step) ? d.shadow_pcf_step : 1.0f));
        int n_pts = 0;
        t = shs_fp::unite(t, shs_fp::shadow_footprint(d.light_viewproj, ctx->shadow_w, ctx->shadow_h, d.viewproj, W, H, px,
                                                      bmin, bmax, rad * step, pts, &n_pts));
        if (n_pts < 0) spans = false;   // no bound: the whole map
        else if (spans) shs_fp::footprint_rows(pts, n_pts, ctx->shadow_w, ctx->shadow_h, rad * step, T, rows, sx0.data(), sx1.data());
    }
    span.clear();
    if (t.empty()) return shs_dev::ShardRegion{1, 0, 0, -1, -1};
    const shs_dev::ShardRegion reg{1, t.x0 / T, t.y0 / T, t.x1 / T, t.y1 / T};
    if (spans) {
        span.resize((size_t)rows);
        for (int r = 0; r < rows; ++r)
            span[(size_t)r] = sx1[(size_t)r] < sx0[(size_t)r] ? 1u
                              : (uint32_t)(sx0[(size_t)r] / T) | ((uint32_t)(sx1[(size_t)r] / T) << 16);
    }
    return reg;
}

// Is every tile of (need, need_span) rendered by (have, have_span)?  Spans as in enqueue_shadow.
static bool shadow_covers(const shs_dev::ShardRegion &have, const std::vector<uint32_t> &have_span,
                          const shs_dev::ShardRegion &need, const std::vector<uint32_t> &need_span) {
    auto empty = [](const shs_dev::ShardRegion &r) { return r.x1 < r.x0 || r.y1 < r.y0; };
    if (empty(need)) return true;
    if (empty(have) || need.x0 < have.x0 || need.y0 < have.y0 || need.x1 > have.x1 || need.y1 > have.y1) return false;
    if (have_span.empty()) return true;
    for (int y = need.y0; y <= need.y1; ++y) {
        int a = need.x0, b = need.x1;   // the row's needed columns
        if (!need_span.empty()) {
            if ((size_t)y >= need_span.size()) return false;
            a = std::max(a, (int)(need_span[(size_t)y] & 0xffffu));
            b = std::min(b, (int)(need_span[(size_t)y] >> 16));
        }
        if (a > b) continue;
        if ((size_t)y >= have_span.size()) return false;
        if (a < (int)(have_span[(size_t)y] & 0xffffu) || b > (int)(have_span[(size_t)y] >> 16)) return false;
    }
    return true;
}

int shs_render_pbr_forward(shs_ctx *ctx, const shs_lib_frame *frame, const shs_lib_draw *draws, int32_t n_draws) {
    if (!ctx || !frame || n_draws < 0 || (n_draws > 0 && !draws)) return SHS_ERR_INVALID;
    const shs_lib_frame &f = *frame;
    if (f.width <= 0 || f.height <= 0 || f.width > 16384 || f.height > 16384) { ctx->err = "bad frame size"; return SHS_ERR_INVALID; }
    if (f.shard_count <= 0 || f.shard_rank < 0 || f.shard_rank >= f.shard_count) { ctx->err = "bad shard"; return SHS_ERR_INVALID; }
    for (int i = 0; i < n_draws; ++i) {
        if (check_lib_mesh(ctx, draws[i].mesh_id)) return SHS_ERR_INVALID;
        if (draws[i].program < SHS_PROGRAM_PBR_MR || draws[i].program > SHS_PROGRAM_FORWARD_PLUS) { ctx->err = "bad program"; return SHS_ERR_INVALID; }
        if (draws[i].program == SHS_PROGRAM_FORWARD_PLUS &&
            (!ctx->have_cull || ctx->cull.W != f.width || ctx->cull.H != f.height)) {
            ctx->err = "Forward+ draw needs shs_light_cull for this frame size";
            return SHS_ERR_INVALID;
        }
        if (draws[i].cull_mode < SHS_CULL_NONE || draws[i].cull_mode > SHS_CULL_FRONT) { ctx->err = "bad cull mode"; return SHS_ERR_INVALID; }
        if (draws[i].shadow && !ctx->have_shadow) { ctx->err = "draw samples a shadow map but none was rendered"; return SHS_ERR_INVALID; }
        const int32_t tx = draws[i].base_color_tex;
        if (tx < 0 || tx > (int32_t)ctx->textures.size() || (tx > 0 && !ctx->textures[(size_t)tx - 1].live)) {
            ctx->err = "bad base_color_tex (not a live texture id)";
            return SHS_ERR_INVALID;
        }
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (!ctx->h_lib_counters && hipHostMalloc(reinterpret_cast<void **>(&ctx->h_lib_counters), shs_dev::LC_N * sizeof(uint32_t)) != hipSuccess)
        return SHS_ERR_HIP;
    {   // the pending camera pass is checked before this one rewrites its targets
        const int rc = check_superseded(ctx, ctx->lib_cam);
        if (rc) return rc;
    }
    const size_t npx = (size_t)f.width * f.height;
    if (ensure(ctx, ctx->lib_hdr, npx) || ensure(ctx, ctx->lib_keys, npx)) return SHS_ERR_HIP;
    const size_t n_blk = (size_t)((f.width + 31) / 32) * ((f.height + 7) / 8) * 4;   // 16x4 blocks
    if (ensure(ctx, ctx->lib_blkcov, n_blk)) return SHS_ERR_HIP;
    {   // the block flags start at zero (then every resolve leaves them so); rare: a sync memset
        const uint64_t bk = (uint64_t)(uint32_t)f.width | ((uint64_t)(uint32_t)f.height << 32);
        if (ctx->blkcov_zero_at != ctx->lib_blkcov.p || ctx->blkcov_zero_cap != ctx->lib_blkcov.cap || ctx->blkcov_zero_key != bk) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->setup_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
            HIP_TRY(ctx, hipMemset(ctx->lib_blkcov.p, 0, ctx->lib_blkcov.cap * sizeof(uint32_t)));
            ctx->blkcov_zero_at = ctx->lib_blkcov.p;
            ctx->blkcov_zero_cap = ctx->lib_blkcov.cap;
            ctx->blkcov_zero_key = bk;
        }
    }
    const bool dm = (f.flags & SHS_LIB_DEPTH_MOTION) != 0;
    if (dm && (ensure(ctx, ctx->lib_depth, npx) || ensure(ctx, ctx->lib_motion, npx))) return SHS_ERR_HIP;

    Work &wk = ctx->lib_cam;
    wk.last_draws.resize(n_draws);
    int32_t base = 0;
    for (int i = 0; i < n_draws; ++i) {
        const Mesh &m = ctx->meshes[draws[i].mesh_id];
        build_lib_draw(draws[i], m, base, wk.last_draws[i]);
        bind_texture(ctx, draws[i].base_color_tex, wk.last_draws[i]);
        base += m.n_tris;
    }
    LibFrameParams fp;
    std::memset(&fp, 0, sizeof fp);
    fp.W = f.width; fp.H = f.height;
    fp.rank = f.shard_rank; fp.count = f.shard_count;
    const bool regions = f.shard_count > 1 && ctx->shard_layout == SHS_SHARD_REGIONS;
    if (regions) {   // this rank's rectangle of the balanced layout (the pass's light cull used the same)
        if (shs_regions_next(ctx, f.shard_count, f.width, f.height)) return SHS_ERR_HIP;
        fp.reg = ctx->reg_next[(size_t)f.shard_rank];
    }
    fp.flags = (f.flags & SHS_LIB_BG_GRADIENT) ? shs_dev::LF_GRADIENT : 0u;
    if (dm) {
        fp.flags |= shs_dev::LF_DEPTH | shs_dev::LF_MOTION;
        if (f.zf > f.zn + 1e-6f) fp.flags |= shs_dev::LF_LINZ;   // rasterizer.hpp:354
    }
    fp.zn = f.zn; fp.zf = f.zf; fp.zspan = f.zf - f.zn;
    for (int i = 0; i < 4; ++i) fp.clear[i] = f.clear_hdr[i];
    fp.sm_w = ctx->shadow_w; fp.sm_h = ctx->shadow_h;
    if (ctx->have_cull) {
        const shs_dev::LightCullParams &c = ctx->cull;
        fp.lt_size = c.tile_size; fp.lt_tx = c.tiles_x; fp.lt_ty = c.tiles_y; fp.lt_maxp = c.max_per_tile;
        fp.lt_mode = c.mode; fp.lt_zs = c.z_slices; fp.n_lights = c.n_lights;
        fp.lt_view_z[0] = c.view[2]; fp.lt_view_z[1] = c.view[6]; fp.lt_view_z[2] = c.view[10]; fp.lt_view_z[3] = c.view[14];
        fp.lt_zn = c.zn; fp.lt_zf = c.zf;
    }
    wk.last_fp = fp;
    if (ctx->shadow_pending) {   // the recorded shadow pass, narrowed to what this pass reads
        std::vector<uint32_t> span;
        const shs_dev::ShardRegion need = shadow_region_for(ctx, f, draws, n_draws, fp.reg, span);
        const int rc = enqueue_shadow(ctx, need, span);
        if (rc) return rc;
    } else if (ctx->have_shadow && ctx->shadow_reg.on) {
        // A map rendered for an earlier camera pass's footprint, sampled again (a static sun reused over
        // frames, another view or region): the texels this pass reads must lie inside what was
        // rendered, or the pass is enqueued again over the union (stream-ordered after the earlier
        // camera passes; re-rendered texels get the same values).
        bool shadowed = false;
        for (int i = 0; i < n_draws; ++i) shadowed = shadowed || draws[i].shadow;
        if (shadowed) {
            std::vector<uint32_t> span;
            const shs_dev::ShardRegion need = shadow_region_for(ctx, f, draws, n_draws, fp.reg, span);
            const shs_dev::ShardRegion have = ctx->shadow_reg;
            const std::vector<uint32_t> have_span = ctx->shadow_span;
            if (!shadow_covers(have, have_span, need, span)) {
                // re-rendered over the union: the rectangles' bounding rectangle, the rows' spans united
                // (either side without spans: the whole rectangle)
                auto empty = [](const shs_dev::ShardRegion &r) { return r.x1 < r.x0 || r.y1 < r.y0; };
                const shs_dev::ShardRegion u = empty(have) ? need
                    : shs_dev::ShardRegion{1, std::min(need.x0, have.x0), std::min(need.y0, have.y0),
                                           std::max(need.x1, have.x1), std::max(need.y1, have.y1)};
                std::vector<uint32_t> us;
                if (empty(have)) us = span;
                else if (!span.empty() && !have_span.empty() && span.size() == have_span.size()) {
                    us.resize(span.size());
                    for (size_t r = 0; r < span.size(); ++r) {
                        const int a0 = (int)(span[r] & 0xffffu), a1 = (int)(span[r] >> 16);
                        const int b0 = (int)(have_span[r] & 0xffffu), b1 = (int)(have_span[r] >> 16);
                        const bool ea = a1 < a0 || (int)r < need.y0 || (int)r > need.y1;
                        const bool eb = b1 < b0 || (int)r < have.y0 || (int)r > have.y1;
                        us[r] = ea && eb ? 1u : ea ? have_span[r] : eb ? span[r]
                              : (uint32_t)std::min(a0, b0) | ((uint32_t)std::max(a1, b1) << 16);
                    }
                }
                int rc = check_superseded(ctx, ctx->lib_shadow);
                if (!rc) rc = enqueue_shadow(ctx, u, us);
                if (rc) return rc;
            }
        }
    }
    ctx->lib_frame = f;
    // The camera pass runs on the context's stream after its shadow pass (round 6): with three frames in
    // flight the frames overlap each other, and a context with one busy stream keeps the process's 4
    // hardware queues to one stream per frame -- on the side stream beside the shadow pass, C5's strong
    // leg after the C4 leg read 0.394-0.405 against 0.370-0.371 ms per frame, --config c5 unchanged
    // (profiles/r06_c5_one_stream_ab.txt).  (SHS_EXP_CAM_SIDE_STREAM: the side stream, timing only.)
#ifdef SHS_EXP_CAM_SIDE_STREAM
    ctx->cam_after_shadow = ctx->have_shadow;
#else
    ctx->cam_after_shadow = false;
#endif
    wk.tm_fused = ctx->tm_fuse;
    wk.tm_desc = ctx->tm_fuse_desc;
    const int rc = enqueue_pass(ctx, wk, false);
    if (rc) return rc;
    if (regions) {   // the layout of this pass (tonemap, gather); the next pass balances anew
        ctx->reg_last = ctx->reg_next;
        ctx->reg_last_count = f.shard_count;
        ctx->reg_next_fresh = false;
    } else {
        ctx->reg_last.clear();
        ctx->reg_last_count = 0;
    }
    ctx->have_lib_frame = true;
    // a new camera pass: a tonemap (and motion blur) must follow it again, unless it ran fused
    ctx->have_ldr = wk.tm_fused;
    if (wk.tm_fused) ctx->tm_desc = wk.tm_desc;
    ctx->have_mb = false;
    return SHS_OK;
}

int shs_resolve_lib(shs_ctx *ctx, float *hdr, float *depth, float *motion) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_lib_frame) { ctx->err = "no library frame rendered"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = lib_finish(ctx);
    if (rc) return rc;
    const size_t npx = (size_t)ctx->lib_frame.width * ctx->lib_frame.height;
    const bool dm = (ctx->lib_frame.flags & SHS_LIB_DEPTH_MOTION) != 0;
    if ((depth || motion) && !dm) { ctx->err = "frame has no depth_motion target"; return SHS_ERR_INVALID; }
    if (hdr) HIP_TRY(ctx, hipMemcpy(hdr, ctx->lib_hdr.p, npx * sizeof(float4), hipMemcpyDeviceToHost));
    if (depth) HIP_TRY(ctx, hipMemcpy(depth, ctx->lib_depth.p, npx * sizeof(float), hipMemcpyDeviceToHost));
    if (motion) HIP_TRY(ctx, hipMemcpy(motion, ctx->lib_motion.p, npx * sizeof(float2), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_get_shadow_region(shs_ctx *ctx, int32_t rect[4]) {
    if (!ctx || !rect) return SHS_ERR_INVALID;
    if (!ctx->have_shadow) { ctx->err = "no shadow map rendered"; return SHS_ERR_INVALID; }
    const shs_dev::ShardRegion &g = ctx->shadow_reg;
    const int tx = (ctx->shadow_w + shs_dev::TILE - 1) / shs_dev::TILE, ty = (ctx->shadow_h + shs_dev::TILE - 1) / shs_dev::TILE;
    if (ctx->shadow_pending) { rect[0] = 1; rect[1] = 1; rect[2] = 0; rect[3] = 0; return SHS_OK; }
    rect[0] = g.on ? g.x0 : 0; rect[1] = g.on ? g.y0 : 0;
    rect[2] = g.on ? g.x1 : tx - 1; rect[3] = g.on ? g.y1 : ty - 1;
    return SHS_OK;
}

int shs_shadow_footprint(const float light_viewproj[16], int32_t sm_w, int32_t sm_h, const float camera_viewproj[16],
                         int32_t width, int32_t height, const int32_t px_rect[4], const float world_min[3],
                         const float world_max[3], int32_t reach, int32_t texel_rect[4]) {
    if (!light_viewproj || !camera_viewproj || !px_rect || !world_min || !world_max || !texel_rect || reach < 0)
        return SHS_ERR_INVALID;
    const int px[4] = {px_rect[0], px_rect[1], px_rect[2], px_rect[3]};
    const double b0[3] = {world_min[0], world_min[1], world_min[2]}, b1[3] = {world_max[0], world_max[1], world_max[2]};
    const shs_fp::TexelRect t = shs_fp::shadow_footprint(light_viewproj, sm_w, sm_h, camera_viewproj, width, height, px, b0, b1, reach);
    texel_rect[0] = t.x0; texel_rect[1] = t.y0; texel_rect[2] = t.x1; texel_rect[3] = t.y1;
    return SHS_OK;
}

int shs_shadow_footprint_rows(const float light_viewproj[16], int32_t sm_w, int32_t sm_h, const float camera_viewproj[16],
                              int32_t width, int32_t height, const int32_t px_rect[4], const float world_min[3],
                              const float world_max[3], int32_t reach, int32_t row_h, int32_t n_rows, int32_t *x0,
                              int32_t *x1) {
    if (!light_viewproj || !camera_viewproj || !px_rect || !world_min || !world_max || !x0 || !x1 || reach < 0 ||
        row_h <= 0 || n_rows < 0)
        return SHS_ERR_INVALID;
    const int px[4] = {px_rect[0], px_rect[1], px_rect[2], px_rect[3]};
    const double b0[3] = {world_min[0], world_min[1], world_min[2]}, b1[3] = {world_max[0], world_max[1], world_max[2]};
    double pts[220][2];
    int n_pts = 0;
    shs_fp::shadow_footprint(light_viewproj, sm_w, sm_h, camera_viewproj, width, height, px, b0, b1, reach, pts, &n_pts);
    for (int r = 0; r < n_rows; ++r) {
        x0[r] = n_pts < 0 ? 0 : 1;
        x1[r] = n_pts < 0 ? sm_w - 1 : 0;
    }
    if (n_pts > 0) shs_fp::footprint_rows(pts, n_pts, sm_w, sm_h, reach, row_h, n_rows, x0, x1);
    return SHS_OK;
}

int shs_resolve_shadow_map(shs_ctx *ctx, float *depth) {
    if (!ctx || !depth) return SHS_ERR_INVALID;
    if (!ctx->have_shadow) { ctx->err = "no shadow map rendered"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = shs_lib_flush_shadow(ctx);   // a recorded footprint pass is rendered whole for a readback
    if (rc) return rc;
    rc = lib_finish(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(depth, ctx->shadow_map.p, (size_t)ctx->shadow_w * ctx->shadow_h * sizeof(float), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_lib_debug_setup_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out) {
    if (!ctx || !n_out) return SHS_ERR_INVALID;
    if (!ctx->want_timeline || !ctx->lib_stimeline.p || ctx->lib_cam.last_setup_blocks <= 0) {
        ctx->err = "timeline not enabled or no camera pass yet";
        return SHS_ERR_INVALID;
    }
    const int64_t n = (int64_t)ctx->lib_cam.last_setup_blocks * shs_dev::STL_STRIDE;
    *n_out = n;
    if (!out) return SHS_OK;
    if (capacity < n) { ctx->err = "capacity too small"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipMemcpy(out, ctx->lib_stimeline.p, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_lib_debug_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out) {
    if (!ctx || !n_out) return SHS_ERR_INVALID;
    const Work &tw = ctx->timeline_shadow ? ctx->lib_shadow : ctx->lib_cam;
    if (!ctx->want_timeline || !ctx->lib_timeline.p || tw.last_raster_grid <= 0) {
        ctx->err = "timeline not enabled or no such pass yet";
        return SHS_ERR_INVALID;
    }
    const int64_t n = (int64_t)tw.last_raster_grid * shs_dev::LTL_STRIDE;
    *n_out = n;
    if (!out) return SHS_OK;
    if (capacity < n) { ctx->err = "capacity too small"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipMemcpy(out, ctx->lib_timeline.p, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_get_lib_stats(shs_ctx *ctx, shs_lib_stats *st) {
    if (!ctx || !st || !ctx->have_lib_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = lib_finish(ctx);
    if (rc) return rc;
    const Work &w = ctx->lib_cam;
    st->tri_input = (uint64_t)w.last_n_tris;
    st->tri_after_clip = w.st_clip;
    st->tri_raster = w.st_raster;
    st->covered_pixels = w.st_covered;
    st->max_tile_bin = w.st_maxbin;
    st->spilled = w.st_spill;
    st->clipped_extra = w.st_extra;
    return SHS_OK;
}

int shs_lib_device_targets(shs_ctx *ctx, void **hdr_dev, void **depth_dev, void **motion_dev) {
    if (!ctx || !ctx->have_lib_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int rc = lib_finish(ctx);   // the pass is final (re-issued on overflow) before it is handed out
    if (rc) return rc;
    if (hdr_dev) *hdr_dev = ctx->lib_hdr.p;
    if (depth_dev) *depth_dev = ctx->lib_depth.p;
    if (motion_dev) *motion_dev = ctx->lib_motion.p;
    return SHS_OK;
}

int shs_lights_upload(shs_ctx *ctx, const shs_culling_light *lights, int32_t n) {
    static_assert(sizeof(shs_culling_light) == sizeof(shs_dev::CullLight), "CullingLightGPU layout");
    if (!ctx || n < 0 || (n > 0 && !lights)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (ensure(ctx, ctx->lights, (size_t)std::max(n, 1))) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));   // the previous set may still be read
    if (n > 0) HIP_TRY(ctx, hipMemcpy(ctx->lights.p, lights, (size_t)n * sizeof(shs_dev::CullLight), hipMemcpyHostToDevice));
    ctx->n_lights = n;
    return SHS_OK;
}

int shs_light_cull(shs_ctx *ctx, const shs_light_cull_desc *d) {
    if (!ctx || !d) return SHS_ERR_INVALID;
    if (d->width <= 0 || d->height <= 0 || d->tile_size == 0 || d->max_per_tile == 0 || d->mode > 3u ||
        (d->mode == 3u && d->z_slices == 0) || d->shard_count <= 0 || d->shard_rank < 0 || d->shard_rank >= d->shard_count) {
        ctx->err = "bad light cull description";
        return SHS_ERR_INVALID;
    }
    if (d->mode == 2u && (!ctx->have_lib_frame || !(ctx->lib_frame.flags & SHS_LIB_DEPTH_MOTION) ||
                          ctx->lib_frame.width != d->width || ctx->lib_frame.height != d->height)) {
        ctx->err = "tiled-depth culling needs a library frame with a depth target of the same size";
        return SHS_ERR_INVALID;
    }
    if (d->mode == 2u && d->shard_count > 1 && ctx->shard_layout == SHS_SHARD_REGIONS) {
        // the depth ranges come from the previous camera pass's depth, which a region rank holds only for
        // its previous rectangle; rectangles move between passes, so a newly owned tile would read stale
        // depth.  Interleaved ownership is static and keeps the depth of every owned tile.
        ctx->err = "tiled-depth culling needs the interleaved shard layout (region rectangles move between passes)";
        return SHS_ERR_INVALID;
    }
    if (d->mode == 2u && d->shard_count > 1 && (32u % d->tile_size) == 0u && ((uint32_t)d->height % 32u) % d->tile_size != 0u) {
        // light tiles count rows top-down, bin tiles bottom-up: at this height a light tile straddles two
        // bin rows, i.e. two ranks' pixels, and its depth range would read the other rank's stale depth
        ctx->err = "sharded tiled-depth culling needs height % 32 to be a multiple of the light tile size";
        return SHS_ERR_INVALID;
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (d->mode == 2u) {   // the depth it reduces must be final: an overflowed camera pass is re-issued first
        const int rc = check_superseded(ctx, ctx->lib_cam);
        if (rc) return rc;
    }
    shs_dev::LightCullParams p;
    std::memset(&p, 0, sizeof p);
    p.W = d->width; p.H = d->height;
    p.tile_size = d->tile_size; p.max_per_tile = d->max_per_tile; p.mode = d->mode;
    p.z_slices = std::max(d->z_slices, 1u);
    p.tiles_x = (d->width + d->tile_size - 1) / d->tile_size;
    p.tiles_y = (d->height + d->tile_size - 1) / d->tile_size;
    p.n_lists = p.tiles_x * p.tiles_y * (d->mode == 3u ? p.z_slices : 1u);
    p.n_lights = (uint32_t)ctx->n_lights;
    p.zn = d->zn; p.zf = d->zf;
    p.depth_linear = d->depth_linear;
    p.rank = d->shard_rank; p.count = d->shard_count;
    if (p.count > 1 && ctx->shard_layout == SHS_SHARD_REGIONS) {   // the upcoming camera pass's rectangle
        if (shs_regions_next(ctx, p.count, p.W, p.H)) return SHS_ERR_HIP;
        p.reg = ctx->reg_next[(size_t)p.rank];
    }
    std::memcpy(p.view, d->view, sizeof p.view);
    std::memcpy(p.proj, d->proj, sizeof p.proj);
    if (ensure(ctx, ctx->depth_ranges, (size_t)p.tiles_x * p.tiles_y) || ensure(ctx, ctx->list_counts, p.n_lists) ||
        ensure(ctx, ctx->list_indices, (size_t)p.n_lists * p.max_per_tile) || ensure(ctx, ctx->lights, 1))
        return SHS_ERR_HIP;
    const uint32_t *work = nullptr;
    uint32_t n_work = p.n_lists;
    if (p.count > 1 && (32u % p.tile_size) == 0u) {   // tile-sharded: this rank's lists first (cached table)
        const shs_ctx::OrderEntry *e = nullptr;
        const uint64_t key[4] = {(uint64_t)(uint32_t)p.W | ((uint64_t)(uint32_t)p.H << 32),
                                 (uint64_t)p.tile_size | ((uint64_t)p.n_lists << 32),
                                 (uint64_t)(uint32_t)p.rank | ((uint64_t)(uint32_t)p.count << 32),
                                 p.reg.on ? region_key(p.reg) ^ (1ull << 63) : 0ull};
        if (order_lookup(ctx, ctx->cull_orders, key,
                         [&](std::vector<int32_t> &v, int &n_owned) {
                             std::vector<int32_t> rest;
                             const uint32_t per_slice = p.tiles_x * p.tiles_y;
                             for (uint32_t l = 0; l < p.n_lists; ++l) {
                                 const uint32_t rem = l % per_slice;
                                 (shs_internal::light_list_owned(p, rem % p.tiles_x, rem / p.tiles_x) ? v : rest).push_back((int32_t)l);
                             }
                             n_owned = (int)v.size();
                             v.insert(v.end(), rest.begin(), rest.end());
                         },
                         e))
            return SHS_ERR_HIP;
        work = reinterpret_cast<const uint32_t *>(e->dev);
        n_work = (uint32_t)e->n_owned;
    }
    HIP_TRY(ctx, shs_internal::launch_light_cull(p, ctx->lights.p, ctx->lib_depth.p, ctx->depth_ranges.p, work, n_work,
                                                 ctx->list_counts.p, ctx->list_indices.p, ctx->stream));
    ctx->cull = p;
    ctx->have_cull = true;
    return SHS_OK;
}

int shs_resolve_light_lists(shs_ctx *ctx, uint32_t *counts, uint32_t *indices, float *ranges) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_cull) { ctx->err = "no light cull run"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const shs_dev::LightCullParams &p = ctx->cull;
    if (counts) HIP_TRY(ctx, hipMemcpy(counts, ctx->list_counts.p, p.n_lists * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (indices)
        HIP_TRY(ctx, hipMemcpy(indices, ctx->list_indices.p, (size_t)p.n_lists * p.max_per_tile * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (ranges)
        HIP_TRY(ctx, hipMemcpy(ranges, ctx->depth_ranges.p, (size_t)p.tiles_x * p.tiles_y * sizeof(float2), hipMemcpyDeviceToHost));
    return SHS_OK;
}

static int tile_params(shs_ctx *ctx, int target, int32_t rank, int32_t count, shs_dev::TileCopyParams &p) {
    std::memset(&p, 0, sizeof p);
    if (count <= 0 || rank < 0 || rank >= count) { ctx->err = "bad shard"; return SHS_ERR_INVALID; }
    p.rank = rank;
    p.count = count;
    // a region-sharded library frame: rank's rectangle of the last camera pass's layout
    if ((target == SHS_TARGET_LIB || target == SHS_TARGET_LIB_PRESENT) && count > 1 && ctx->reg_last_count == count)
        p.reg = ctx->reg_last[(size_t)rank];
    if (target == SHS_TARGET_LEGACY) {
        if (!ctx->have_frame) { ctx->err = "no legacy frame rendered"; return SHS_ERR_INVALID; }
        p.W = ctx->frame.width; p.H = ctx->frame.height;
        p.color_words = 1; p.color_flip = 1;
        p.color = reinterpret_cast<uint32_t *>(ctx->color.p);
        p.depth = reinterpret_cast<uint32_t *>(ctx->depth.p);
    } else if (target == SHS_TARGET_PRESENT) {
        // the legacy frame's SDL staging: screen rows, the legacy tiles' own row order
        if (!ctx->have_frame || !(ctx->frame.flags & SHS_FRAME_PRESENT)) { ctx->err = "no legacy present staging"; return SHS_ERR_INVALID; }
        p.W = ctx->frame.width; p.H = ctx->frame.height;
        p.color_words = 1; p.color_flip = 0;
        p.color = ctx->present.p;
    } else if (target == SHS_TARGET_LIB_PRESENT) {
        // the last tonemap's present staging: rows top-down, library tiles count rows y up
        if (!ctx->have_ldr || !(ctx->tm_desc.flags & SHS_TONEMAP_PRESENT)) { ctx->err = "no tonemap present staging"; return SHS_ERR_INVALID; }
        p.W = ctx->lib_frame.width; p.H = ctx->lib_frame.height;
        p.color_words = 1; p.color_flip = 1;
        p.color = ctx->lib_present.p;
    } else if (target == SHS_TARGET_LIB) {
        if (!ctx->have_lib_frame) { ctx->err = "no library frame rendered"; return SHS_ERR_INVALID; }
        p.W = ctx->lib_frame.width; p.H = ctx->lib_frame.height;
        p.color_words = 4; p.color_flip = 0;
        p.color = reinterpret_cast<uint32_t *>(ctx->lib_hdr.p);
        if (ctx->lib_frame.flags & SHS_LIB_DEPTH_MOTION) {
            p.depth = reinterpret_cast<uint32_t *>(ctx->lib_depth.p);
            p.motion = reinterpret_cast<uint32_t *>(ctx->lib_motion.p);
        }
    } else {
        ctx->err = "bad target";
        return SHS_ERR_INVALID;
    }
    p.words = p.color_words + (p.depth ? 1 : 0) + (p.motion ? 2 : 0);
    return SHS_OK;
}

int shs_tiles_rank_words(shs_ctx *ctx, int target, int32_t rank, int32_t count, int64_t *words_out) {
    if (!ctx || !words_out) return SHS_ERR_INVALID;
    shs_dev::TileCopyParams p;
    if (tile_params(ctx, target, rank, count, p)) return SHS_ERR_INVALID;
    const int n_tiles = ((p.W + 31) / 32) * ((p.H + 31) / 32);
    *words_out = (int64_t)shs_dev::shard_n_owned(rank, count, p.reg, n_tiles) * 32 * 32 * p.words;
    return SHS_OK;
}

int shs_tiles_packed_words(shs_ctx *ctx, int target, int32_t count, int64_t *words_out) {
    if (!ctx || !words_out) return SHS_ERR_INVALID;
    int64_t most = 0;
    for (int32_t r = 0; r < std::max(count, 1); ++r) {
        int64_t w = 0;
        if (shs_tiles_rank_words(ctx, target, r, count, &w)) return SHS_ERR_INVALID;
        most = std::max(most, w);
    }
    *words_out = most;
    return SHS_OK;
}

// A frame whose capacity overflowed is re-issued before its tiles leave the rank or peers' tiles land in
// it (legacy: the batch, a pipelined batch's pending raster included -- it clears the whole frame;
// library: the pass chain, tonemap included).  Only its setup is waited for: the overflow word is final
// then, and the copy is stream-ordered after the (possibly re-issued) frame.
static int final_before_copy(shs_ctx *ctx, int target) {
    return (target == SHS_TARGET_LEGACY || target == SHS_TARGET_PRESENT) ? shs_legacy_ensure_final(ctx)
                                                                        : shs_lib_ensure_final(ctx);
}

int shs_tiles_pack(shs_ctx *ctx, int target, int32_t rank, int32_t count, void *dst_dev) {
    if (!ctx || !dst_dev) return SHS_ERR_INVALID;
    shs_dev::TileCopyParams p;
    if (tile_params(ctx, target, rank, count, p)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int rc = final_before_copy(ctx, target);
    if (rc) return rc;
    HIP_TRY(ctx, shs_internal::launch_tiles_copy(p, true, dst_dev, ctx->stream));
    return SHS_OK;
}

int shs_tiles_unpack(shs_ctx *ctx, int target, int32_t rank, int32_t count, const void *src_dev) {
    if (!ctx || !src_dev) return SHS_ERR_INVALID;
    shs_dev::TileCopyParams p;
    if (tile_params(ctx, target, rank, count, p)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int rc = final_before_copy(ctx, target);
    if (rc) return rc;
    HIP_TRY(ctx, shs_internal::launch_tiles_copy(p, false, const_cast<void *>(src_dev), ctx->stream));
    return SHS_OK;
}

int shs_tiles_unpack_ranks(shs_ctx *ctx, int target, int32_t count, const void *const *src_dev) {
    if (!ctx || !src_dev || count <= 0) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    {
        const int rc = final_before_copy(ctx, target);
        if (rc) return rc;
    }
    shs_dev::TileUnpackMulti m;
    std::memset(&m, 0, sizeof m);
    for (int32_t r = 0; r < count; ++r) {
        if (!src_dev[r]) continue;
        shs_dev::TileCopyParams p;
        if (tile_params(ctx, target, r, count, p)) return SHS_ERR_INVALID;
        const int n_tiles = ((p.W + shs_dev::TILE - 1) / shs_dev::TILE) * ((p.H + shs_dev::TILE - 1) / shs_dev::TILE);
        const int owned = shs_dev::shard_n_owned(p.rank, p.count, p.reg, n_tiles);
        if (owned <= 0) continue;
        if (m.n == shs_dev::UNPACK_PEERS) {   // a launch per UNPACK_PEERS peers
            HIP_TRY(ctx, shs_internal::launch_tiles_unpack_multi(m, ctx->stream));
            std::memset(&m, 0, sizeof m);
        }
        m.p = p;
        m.rank[m.n] = r;
        m.reg[m.n] = p.reg;
        m.src[m.n] = static_cast<const uint32_t *>(src_dev[r]);
        m.first[m.n + 1] = m.first[m.n] + owned;
        ++m.n;
    }
    HIP_TRY(ctx, shs_internal::launch_tiles_unpack_multi(m, ctx->stream));
    return SHS_OK;
}

int shs_lib_timing_reset(shs_ctx *ctx) {
    if (!ctx) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (Work *w : {&ctx->lib_shadow, &ctx->lib_cam}) {
        if (harvest_all(ctx, *w)) return SHS_ERR_HIP;
        w->acc_ms[0] = w->acc_ms[1] = 0.0;
        w->acc_n = 0;
    }
    return SHS_OK;
}

int shs_lib_timing_read(shs_ctx *ctx, double sum_ms4[4], int64_t n_passes2[2]) {
    if (!ctx || !sum_ms4 || !n_passes2) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (harvest_all(ctx, ctx->lib_shadow) || harvest_all(ctx, ctx->lib_cam)) return SHS_ERR_HIP;
    sum_ms4[0] = ctx->lib_shadow.acc_ms[0]; sum_ms4[1] = ctx->lib_shadow.acc_ms[1];
    sum_ms4[2] = ctx->lib_cam.acc_ms[0]; sum_ms4[3] = ctx->lib_cam.acc_ms[1];
    n_passes2[0] = ctx->lib_shadow.acc_n;
    n_passes2[1] = ctx->lib_cam.acc_n;
    return SHS_OK;
}

int shs_look_at_lh(const float eye[3], const float center[3], const float up[3], float out16[16]) {
    if (!eye || !center || !up || !out16) return SHS_ERR_INVALID;
    shs_host::look_at_lh({eye[0], eye[1], eye[2]}, {center[0], center[1], center[2]}, {up[0], up[1], up[2]}, out16);
    return SHS_OK;
}

int shs_perspective_lh_no(float fovy, float aspect, float zn, float zf, float out16[16]) {
    if (!out16) return SHS_ERR_INVALID;
    shs_host::perspective_lh_no(fovy, aspect, zn, zf, out16);
    return SHS_OK;
}

int shs_model_euler(const float pos[3], const float rot[3], const float scl[3], float out16[16]) {
    if (!pos || !rot || !scl || !out16) return SHS_ERR_INVALID;
    shs_host::model_euler({pos[0], pos[1], pos[2]}, {rot[0], rot[1], rot[2]}, {scl[0], scl[1], scl[2]}, out16);
    return SHS_OK;
}

int shs_dir_light_camera_aabb(const float sun_dir[3], const float mn[3], const float mx[3], float margin, uint32_t res,
                              float view16[16], float proj16[16], float viewproj16[16]) {
    if (!sun_dir || !mn || !mx || !view16 || !proj16 || !viewproj16) return SHS_ERR_INVALID;
    shs_host::dir_light_camera_aabb({sun_dir[0], sun_dir[1], sun_dir[2]}, {mn[0], mn[1], mn[2]}, {mx[0], mx[1], mx[2]}, margin,
                                    res, view16, proj16, viewproj16);
    return SHS_OK;
}

}  // extern "C"
