// shs_abi.cpp -- host side of libshs_gpu.so: the C ABI declared in include/shs_gpu.h.
//
// Owns device-resident meshes, the per-frame workspace (triangle records, tile bins, framebuffers)
// and the HIP stream the four kernels of shs_legacy.hip are enqueued on.  Replaces the tile-job
// submission loop of RendererSystem::process (hello_pipeline_blinn_phong_shading.cpp:244-313).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/shs_gpu.h"
#include "shs_ctx.hpp"
#include "shs_device.hpp"
#include "shs_glm.hpp"
#include "shs_internal.hpp"

using shs_dev::DrawGPU;
using shs_dev::FrameBuffers;
using shs_dev::FrameParams;

extern "C" {

static int flush_pending(shs_ctx *ctx);   // SHS_OPT_LEGACY_PIPELINE (below enqueue_frame's helpers)

int shs_abi_version(void) { return 1; }

int shs_gpu_tile_size(void) { return shs_dev::TILE; }

int shs_create(int device, shs_ctx **out) {
    if (!out) return SHS_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SHS_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SHS_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::fprintf(stderr, "shs_gpu: device %d is %s, this build targets gfx950 only\n", device, prop.gcnArchName);
        return SHS_ERR_NO_DEVICE;
    }
    shs_ctx *ctx = new shs_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SHS_ERR_HIP;
    }
    ctx->stream = ctx->own_stream;
    if (hipStreamCreateWithFlags(&ctx->setup_stream, hipStreamNonBlocking) != hipSuccess) { shs_destroy(ctx); return SHS_ERR_HIP; }
    for (auto &w : ctx->lslot)
        if (hipEventCreateWithFlags(&w.setup_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&w.raster_done, hipEventDisableTiming) != hipSuccess ||
            shs_host_ov_alloc(&w.h_ov) != hipSuccess) {
            shs_destroy(ctx);
            return SHS_ERR_HIP;
        }
    for (int i = 0; i < 5; ++i)
        if (hipEventCreateWithFlags(&ctx->tev[i], hipEventDisableSystemFence) != hipSuccess) { shs_destroy(ctx); return SHS_ERR_HIP; }
    if (hipHostMalloc(reinterpret_cast<void **>(&ctx->h_counters), shs_dev::C_NCOUNTERS * sizeof(uint32_t)) != hipSuccess) {
        shs_destroy(ctx);
        return SHS_ERR_HIP;
    }
    std::memset(ctx->h_counters, 0, shs_dev::C_NCOUNTERS * sizeof(uint32_t));
    if (ensure(ctx, ctx->counters, shs_dev::N_CSETS * shs_dev::CSET) != SHS_OK ||
        hipMemset(ctx->counters.p, 0, shs_dev::N_CSETS * shs_dev::CSET * sizeof(uint32_t)) != hipSuccess) {
        shs_destroy(ctx);
        return SHS_ERR_HIP;
    }
    *out = ctx;
    return SHS_OK;
}

int shs_destroy(shs_ctx *ctx) {
    if (!ctx) return SHS_ERR_INVALID;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->setup_stream) (void)hipStreamSynchronize(ctx->setup_stream);
    for (auto &m : ctx->meshes) {
        if (m.borrowed) continue;   // the owning context frees them
        if (m.pos) (void)hipFree(m.pos);
        if (m.nrm) (void)hipFree(m.nrm);
        if (m.uv) (void)hipFree(m.uv);
        if (m.idx) (void)hipFree(m.idx);
        if (m.orig) (void)hipFree(m.orig);
        if (m.cbox) (void)hipFree(m.cbox);
    }
    shs_lib_release(ctx);
    for (auto &w : ctx->lslot) {
        release(w.draws); release(w.recs); release(w.rext); release(w.shade); release(w.tile_count); release(w.bins);
        release(w.spill); release(w.frags); release(w.busy); release(w.boxes); release(w.slivers); release(w.busy_list);
        release(w.blk_stat); release(w.rstat);
        if (w.h_draws) (void)hipHostFree(w.h_draws);
        if (w.setup_done) (void)hipEventDestroy(w.setup_done);
        if (w.raster_done) (void)hipEventDestroy(w.raster_done);
        if (w.h_ov) (void)hipHostFree(const_cast<uint32_t *>(w.h_ov));
    }
    release(ctx->counters); release(ctx->timeline);
    release(ctx->color); release(ctx->depth); release(ctx->prequant); release(ctx->present);
    for (int i = 0; i < 5; ++i)
        if (ctx->tev[i]) (void)hipEventDestroy(ctx->tev[i]);
    for (int k = 0; k < shs_ctx::RING; ++k)
        for (int i = 0; i < 5; ++i)
            if (ctx->ring_ev[k][i]) (void)hipEventDestroy(ctx->ring_ev[k][i]);
    if (ctx->h_counters) (void)hipHostFree(ctx->h_counters);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    if (ctx->setup_stream) (void)hipStreamDestroy(ctx->setup_stream);
    delete ctx;
    return SHS_OK;
}

const char *shs_last_error(shs_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int shs_set_stream(shs_ctx *ctx, void *s) {
    if (!ctx) return SHS_ERR_INVALID;
    if (flush_pending(ctx)) return SHS_ERR_HIP;   // on the stream its setup ran on
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
    ctx->stream = s ? reinterpret_cast<hipStream_t>(s) : ctx->own_stream;
    return SHS_OK;
}

void *shs_get_stream(shs_ctx *ctx) { return ctx ? reinterpret_cast<void *>(ctx->stream) : nullptr; }

int shs_mesh_upload_soup(shs_ctx *ctx, const float *positions, const float *normals, int32_t n_tris, int32_t *mesh_id) {
    if (!ctx || !positions || !normals || n_tris <= 0 || !mesh_id) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    Mesh m;
    const size_t bytes = (size_t)n_tris * 9 * sizeof(float);
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.pos), bytes));
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&m.nrm), bytes));
    HIP_TRY(ctx, hipMemcpy(m.pos, positions, bytes, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(m.nrm, normals, bytes, hipMemcpyHostToDevice));
    m.n_tris = n_tris;
    m.live = true;
    ctx->meshes.push_back(m);
    *mesh_id = (int32_t)ctx->meshes.size() - 1;
    return SHS_OK;
}

int shs_mesh_release(shs_ctx *ctx, int32_t id) {
    if (!ctx || id < 0 || id >= (int32_t)ctx->meshes.size() || !ctx->meshes[id].live) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    if (ctx->shadow_pending) {   // a recorded footprint shadow pass may read the mesh: render it first
        const int rc = shs_lib_flush_shadow(ctx);
        if (rc) return rc;
    } else if (ctx->meshes[id].lib) {   // a footprint-restricted map that reads it is rendered whole
        const int rc = shs_lib_widen_shadow(ctx, ctx->meshes[id].pos);
        if (rc) return rc;
    }
    if (flush_pending(ctx)) return SHS_ERR_HIP;   // a pending legacy raster may read it too
    HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    Mesh &m = ctx->meshes[id];
    if (m.borrowed) {   // shs_mesh_share: this context's reads are done; the owner keeps the buffers
        m = Mesh{};
        return SHS_OK;
    }
    HIP_TRY(ctx, hipFree(m.pos));
    HIP_TRY(ctx, hipFree(m.nrm));
    if (m.uv) HIP_TRY(ctx, hipFree(m.uv));
    if (m.idx) HIP_TRY(ctx, hipFree(m.idx));
    if (m.orig) HIP_TRY(ctx, hipFree(m.orig));
    if (m.cbox) HIP_TRY(ctx, hipFree(m.cbox));
    m = Mesh{};
    return SHS_OK;
}

int shs_mesh_share(shs_ctx *dst, shs_ctx *src, int32_t src_mesh_id, int32_t *mesh_id) {
    if (!dst || !src || !mesh_id || dst == src || dst->device != src->device) return SHS_ERR_INVALID;
    if (src_mesh_id < 0 || src_mesh_id >= (int32_t)src->meshes.size() || !src->meshes[src_mesh_id].live) return SHS_ERR_INVALID;
    Mesh m = src->meshes[src_mesh_id];   // (its upload copied synchronously: the buffers are complete)
    m.borrowed = true;
    dst->meshes.push_back(m);
    *mesh_id = (int32_t)dst->meshes.size() - 1;
    return SHS_OK;
}

static void build_draw(const shs_legacy_draw &in, const Mesh &m, int32_t base, DrawGPU &o) {
    std::memset(&o, 0, sizeof o);
    o.pos = m.pos;
    o.nrm = m.nrm;
    o.tri_base = base;
    o.n_tris = m.n_tris;
    o.shading = in.shading;
    std::memcpy(o.mvp, in.mvp, sizeof o.mvp);
    std::memcpy(o.model, in.model, sizeof o.model);
    using namespace shs_host;
    if (in.shading == SHS_SHADING_FLAT) {
        // flat_shading.cpp:54 normal = mat3(u.mv) * n ; FS :76 l = normalize(u.light_dir_view)
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) o.nmat[c * 3 + r] = in.model[c * 4 + r];
        const vec3 l = gnormalize(vec3{in.light_dir[0], in.light_dir[1], in.light_dir[2]});
        o.light[0] = l.x; o.light[1] = l.y; o.light[2] = l.z;
    } else {
        // mat3(transpose(inverse(model))) and normalize(-light_dir): per-vertex / per-fragment in the
        // reference, uniform across the draw, hence computed once here with the same operations
        normal_matrix(in.model, o.nmat);
        const vec3 l = gnormalize(gneg(vec3{in.light_dir[0], in.light_dir[1], in.light_dir[2]}));
        o.light[0] = l.x; o.light[1] = l.y; o.light[2] = l.z;
    }
    o.cam[0] = in.camera_pos[0]; o.cam[1] = in.camera_pos[1]; o.cam[2] = in.camera_pos[2];
    for (int i = 0; i < 3; ++i) {
        o.ocol[i] = (float)in.color[i] / 255.0f;   // glm::vec3(r,g,b) / 255.0f
        o.colf[i] = (float)in.color[i];            // int colour promoted in u.color.r * intensity
    }
}

static int harvest_slot(shs_ctx *ctx, int k) {
    if (!ctx->ring_pending[k]) return SHS_OK;
    HIP_TRY(ctx, hipEventSynchronize(ctx->ring_ev[k][2]));
    float ms[4];
    // [0] k_setup (ev0..ev1, setup_stream), [3] k_raster (ev3..ev2, stream: ev3 is recorded after the
    // wait for the setup, so it marks the raster's start)
    ms[1] = ms[2] = 0.0f;
    HIP_TRY(ctx, hipEventElapsedTime(&ms[0], ctx->ring_ev[k][0], ctx->ring_ev[k][1]));
    HIP_TRY(ctx, hipEventElapsedTime(&ms[3], ctx->ring_ev[k][3], ctx->ring_ev[k][2]));
    for (int i = 0; i < 4; ++i) { ctx->acc_ms[i] += ms[i]; ctx->last_ms[i] = ms[i]; }
    if (ctx->ring_counts[k]) ctx->acc_frames++;
    ctx->ring_pending[k] = false;
    return SHS_OK;
}

static int harvest_all(shs_ctx *ctx) {
    // oldest first
    for (int j = 0; j < shs_ctx::RING; ++j) {
        int rc = harvest_slot(ctx, (ctx->ring_next + j) % shs_ctx::RING);
        if (rc) return rc;
    }
    return SHS_OK;
}

// The next ring entry's events (timing on), or nullptr; counts: the entry is a batch's enqueue.
static int ring_take(shs_ctx *ctx, bool counts, hipEvent_t *&ev) {
    ev = nullptr;
    if (!ctx->timing) return SHS_OK;
    const int k = ctx->ring_next;
    ctx->ring_next = (k + 1) % shs_ctx::RING;
    if (harvest_slot(ctx, k)) return SHS_ERR_HIP;
    if (!ctx->ring_ev[k][0])
        for (int i = 0; i < 5; ++i) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ring_ev[k][i], hipEventDisableSystemFence));
    ev = ctx->ring_ev[k];
    ctx->ring_pending[k] = true;
    ctx->ring_counts[k] = counts;
    return SHS_OK;
}

// SHS_OPT_LEGACY_PIPELINE: launch the pending batch's raster on its own (k_raster), stream-ordered after
// its setup.  Everything that reads a batch's frames, or enqueues work that is not pipelined, calls this.
static int flush_pending(shs_ctx *ctx) {
    if (!ctx->pend.on) return SHS_OK;
    ctx->pend.on = false;
    static const shs_dev::KArgDraws no_karg = {};   // pipelined batches use the device draw table
    hipEvent_t *ev = nullptr;
    if (ring_take(ctx, false, ev)) return SHS_ERR_HIP;
    hipStream_t st = ctx->stream;
    if (ev) {   // the raster's time joins the batch sums (no batch of its own)
        HIP_TRY(ctx, hipEventRecord(ev[0], st));
        HIP_TRY(ctx, hipEventRecord(ev[1], st));
        HIP_TRY(ctx, hipEventRecord(ev[3], st));
    }
    HIP_TRY(ctx, shs_internal::launch_raster(ctx->pend.fp, ctx->pend.fb, no_karg, ctx->pend.grid, st));
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[2], st));
    HIP_TRY(ctx, hipEventRecord(ctx->lslot[ctx->pend.slot].raster_done, st));
    return SHS_OK;
}

static int enqueue_frame(shs_ctx *ctx) {
    const shs_frame_desc &f = ctx->frame;
    const int n_frames = ctx->last_n_frames;
    const int n_draws = ctx->frame_draws;                 // per frame
    const int n_draws_all = (int)ctx->last_draws.size();  // n_frames * n_draws
    const int tiles_x = (f.width + shs_dev::TILE - 1) / shs_dev::TILE;
    const int tiles_y = (f.height + shs_dev::TILE - 1) / shs_dev::TILE;
    const int n_tiles = tiles_x * tiles_y;
    const int rtiles_y = (f.height + shs_dev::RTH - 1) / shs_dev::RTH;
    const int n_rt = tiles_x * rtiles_y;
    const size_t npx = (size_t)f.width * f.height;

    int64_t total = 0;
    for (int i = 0; i < n_draws; ++i) total += ctx->meshes[ctx->last_draws[i].mesh_id].n_tris;
    if (total * n_frames > 0x3fffffff) { ctx->err = "too many triangles in one batch"; return SHS_ERR_INVALID; }
    const int n_tris = (int)total;   // per frame (every frame of a batch has the same count)
    const size_t nt_all = (size_t)std::max(n_tris, 1) * n_frames;
    static const bool ghost_list_env = shs_exp_env("SHS_GHOST_LIST") && std::atoi(shs_exp_env("SHS_GHOST_LIST")) != 0;
    const bool scan = ctx->force_mode == 1 || (ctx->force_mode == 0 && n_tris <= shs_dev::SCAN_MAX_TRIS);
    // pipelined (SHS_OPT_LEGACY_PIPELINE): scan-mode batches (their ghost waves live in k_setup) with a
    // device draw table; the frame buffers the pending raster writes must not be reallocated under it
    const size_t npx0 = (size_t)f.width * f.height;
    const bool pipe = ctx->legacy_pipeline && scan && !ghost_list_env && n_draws_all > shs_dev::KARG_DRAWS && !ctx->want_timeline;
    const bool grows = ctx->color.cap < npx0 * 4 * n_frames || ctx->depth.cap < npx0 * n_frames ||
                       ((f.flags & SHS_FRAME_PREQUANT) && ctx->prequant.cap < npx0 * n_frames) ||
                       ((f.flags & SHS_FRAME_PRESENT) && ctx->present.cap < npx0 * n_frames);
    if ((!pipe || grows) && flush_pending(ctx)) return SHS_ERR_HIP;

    // This batch's workspace slot.  Its previous user (batch n - 2) is complete on the host side once
    // its k_setup is (the pinned draw table is rewritten below), and on the device side once its
    // k_raster is (setup_stream waits for raster_done before reusing the slot's buffers).
    const int slot = (int)(ctx->frame_index & 1u);
    shs_ctx::LegacySlot &ws = ctx->lslot[slot];
    // pipelined batches run everything on the context stream (one launch per batch)
    // SHS_LEGACY_ONE_STREAM=1 (timing experiments): the setup on the raster's stream, in order
    static const bool one_stream_env = shs_exp_env("SHS_LEGACY_ONE_STREAM") && std::atoi(shs_exp_env("SHS_LEGACY_ONE_STREAM")) != 0;
    hipStream_t sst = (pipe || one_stream_env) ? ctx->stream : ctx->setup_stream, st = ctx->stream;
    if (ws.used) HIP_TRY(ctx, hipEventSynchronize(ws.setup_done));
    *ws.h_ov = 0u;   // the slot's previous setup (the only other writer) is done

    if (ensure(ctx, ws.recs, nt_all) || ensure(ctx, ws.rext, nt_all) || ensure(ctx, ws.shade, nt_all) || ensure(ctx, ws.boxes, nt_all) ||
        ensure(ctx, ws.slivers, nt_all))
        return SHS_ERR_HIP;
    const size_t n_bt_all = (size_t)n_tiles * n_frames;
    if (ensure(ctx, ws.tile_count, n_bt_all) || ensure(ctx, ws.busy_list, std::max((size_t)n_rt, (size_t)n_tiles * (shs_dev::TILE / shs_dev::RTH)) * n_frames)) return SHS_ERR_HIP;
    // busy flags hold the epoch of the batch that marked them: reset only when the buffer is new or the
    // tile geometry / shard / batch size changes
    const uint64_t gkey = ((uint64_t)tiles_x << 48) ^ ((uint64_t)tiles_y << 32) ^ ((uint64_t)f.shard_rank << 16) ^
                          (uint64_t)f.shard_count ^ ((uint64_t)n_frames << 24);
    bool reset = gkey != ctx->geom_key[slot];
    if (ws.busy.cap < (size_t)n_rt * n_frames || !ws.busy.p) {
        if (ensure(ctx, ws.busy, (size_t)n_rt * n_frames)) return SHS_ERR_HIP;
        reset = true;
    }
    if (ensure(ctx, ws.bins, (size_t)n_tiles * ctx->bin_cap * n_frames)) return SHS_ERR_HIP;
    const int setup_blocks = (n_tris + 63) / 64;   // a quad of lanes per triangle, per frame
    if (ensure(ctx, ws.blk_stat, (size_t)std::max(setup_blocks, 1) * n_frames)) return SHS_ERR_HIP;
    if (!ws.spill.p && ensure(ctx, ws.spill, 1 << 16)) return SHS_ERR_HIP;
    if (!ws.frags.p && ensure(ctx, ws.frags, 1 << 12)) return SHS_ERR_HIP;
    if (ensure(ctx, ctx->color, npx * 4 * n_frames) || ensure(ctx, ctx->depth, npx * n_frames)) return SHS_ERR_HIP;
    const bool want_pq = (f.flags & SHS_FRAME_PREQUANT) != 0;
    if (want_pq && ensure(ctx, ctx->prequant, npx * n_frames)) return SHS_ERR_HIP;
    const bool want_present = (f.flags & SHS_FRAME_PRESENT) != 0;
    if (want_present && ensure(ctx, ctx->present, npx * n_frames)) return SHS_ERR_HIP;

    // ---- setup_stream: wait for the slot's last k_raster, reset, upload, set up ----
    if (ws.used) HIP_TRY(ctx, hipStreamWaitEvent(sst, ws.raster_done, 0));
    if (pipe && ws.used) HIP_TRY(ctx, hipStreamWaitEvent(sst, ws.setup_done, 0));   // (a non-pipelined setup)
    if (reset) {
        HIP_TRY(ctx, hipMemsetAsync(ws.busy.p, 0, ws.busy.cap * sizeof(uint32_t), sst));
        ctx->geom_key[slot] = gkey;
    }

    // per-draw uniform blocks: kernel arguments for small batches, the slot's device table otherwise.
    // tri_base restarts at 0 in every frame (submission order is per frame)
    shs_dev::KArgDraws ka;
    std::memset(&ka, 0, sizeof ka);
    int32_t base = 0;
    const int32_t *bdraw = nullptr;   // FrameBuffers::bdraw
    if (n_draws_all <= shs_dev::KARG_DRAWS) {
        for (int i = 0; i < n_draws_all; ++i) {
            if (i % std::max(n_draws, 1) == 0) base = 0;
            const shs_legacy_draw &d = ctx->last_draws[i];
            build_draw(d, ctx->meshes[d.mesh_id], base, ka.d[i]);
            base += ctx->meshes[d.mesh_id].n_tris;
        }
    } else {
        // Every frame with frame 0's draw layout (the same mesh per draw index): the table travels with
        // one int per setup block appended, the frame-local draw of the block's first triangle
        // (FrameBuffers::bdraw), so k_setup finds a triangle's draw with one tri_base load.
        bool same_layout = n_draws > 1;
        for (int i = n_draws; i < n_draws_all && same_layout; ++i)
            same_layout = ctx->last_draws[i].mesh_id == ctx->last_draws[i % n_draws].mesh_id;
        const size_t n_extra = same_layout ? ((size_t)setup_blocks * sizeof(int32_t) + sizeof(DrawGPU) - 1) / sizeof(DrawGPU) : 0;
        const size_t n_tab = (size_t)n_draws_all + n_extra;
        if (ensure(ctx, ws.draws, n_tab)) return SHS_ERR_HIP;
        if (n_tab > ws.h_cap) {
            if (ws.h_draws) HIP_TRY(ctx, hipHostFree(ws.h_draws));
            ws.h_draws = nullptr;
            const size_t cap = std::max<size_t>(n_tab, 64);
            HIP_TRY(ctx, hipHostMalloc(reinterpret_cast<void **>(&ws.h_draws), cap * sizeof(DrawGPU)));
            ws.h_cap = cap;
        }
        for (int i = 0; i < n_draws_all; ++i) {
            if (i % std::max(n_draws, 1) == 0) base = 0;
            const shs_legacy_draw &d = ctx->last_draws[i];
            build_draw(d, ctx->meshes[d.mesh_id], base, ws.h_draws[i]);
            base += ctx->meshes[d.mesh_id].n_tris;
        }
        if (same_layout) {
            int32_t *bd = reinterpret_cast<int32_t *>(ws.h_draws + n_draws_all);
            for (int b = 0, d = 0; b < setup_blocks; ++b) {
                while (d + 1 < n_draws && ws.h_draws[d + 1].tri_base <= b * 64) ++d;
                bd[b] = d;
            }
            bdraw = reinterpret_cast<const int32_t *>(ws.draws.p + n_draws_all);
        }
        HIP_TRY(ctx, hipMemcpyAsync(ws.draws.p, ws.h_draws, n_tab * sizeof(DrawGPU), hipMemcpyHostToDevice, sst));
    }

    FrameParams fp;
    std::memset(&fp, 0, sizeof fp);
    fp.W = f.width; fp.H = f.height;
    fp.rtw = f.ref_tile_w; fp.rth = f.ref_tile_h;
    fp.rank = f.shard_rank; fp.count = f.shard_count;
    fp.tiles_x = tiles_x; fp.tiles_y = tiles_y;
    fp.rtiles_y = rtiles_y;
    fp.rt_x = (f.width + f.ref_tile_w - 1) / f.ref_tile_w;
    fp.rt_y = (f.height + f.ref_tile_h - 1) / f.ref_tile_h;
    fp.n_tris = n_tris; fp.n_draws = n_draws;
    fp.clear_rgba = (uint32_t)f.clear_color[0] | ((uint32_t)f.clear_color[1] << 8) | ((uint32_t)f.clear_color[2] << 16) |
                    ((uint32_t)f.clear_color[3] << 24);
    fp.flags = (f.flags & (SHS_EXPERIMENTS ? ~0u : ~shs_dev::DBG_MASK) & ~(shs_dev::RF_PER_PIXEL | shs_dev::RF_NO_RECS | shs_dev::RF_SHARED_VARY | shs_dev::RF_GHOST_INLINE | shs_dev::RF_XCD_ROWS)) | (ctx->pair_loop ? 0u : shs_dev::RF_PER_PIXEL);
    fp.bin_cap = ctx->bin_cap;
    fp.spill_cap = (uint32_t)std::min<size_t>(ws.spill.cap, 0xffffffffu);
    fp.frag_cap = (uint32_t)std::min<size_t>(ws.frags.cap, 0xffffffffu);
    {   // ~1K ghost waves per launch: small scenes split each sliver group over a few waves.  Measured
        // at C2 (61 groups, ~17 unbounded slivers): 4K waves 8.9 us setup, 2K 7.7, 1K 7.3, 512 8.1,
        // 256 9.3 -- past ~1K the extra workgroup launches cost more than the shorter enumerations save.
        // A batch of frames already brings n_frames x the groups.
        const int n_groups = std::max(1, (n_tris + 15) / 16) * n_frames;
        fp.ghost_slices = (uint32_t)std::min(16, std::max(1, 1024 / n_groups));
    }
    fp.parity = (uint32_t)(ctx->frame_index % shs_dev::N_CSETS);   // counter sets round-robin (zeroed by the
    fp.zero_set = (uint32_t)((ctx->frame_index + 1) % shs_dev::N_CSETS);   // previous batch's k_setup)
    if (++ctx->busy_epoch == 0u) ctx->busy_epoch = 1u;   // busy[] is zeroed on reset; 0 is never an epoch
    fp.epoch = ctx->busy_epoch;
    fp.scan_mode = scan ? 1u : 0u;
    if (!fp.scan_mode) HIP_TRY(ctx, hipMemsetAsync(ws.tile_count.p, 0, n_bt_all * sizeof(uint32_t), sst));
    // SHS_LEGACY_NORECS=1: binned frames keep no per-triangle records, k_raster recomputes them from the
    // resident mesh (RF_NO_RECS).  Off by default: measured C3 0.670 -> 0.699 ms per 16-frame step (the
    // staged candidates' draw -> matrix -> position chain costs more raster latency than the 184 B of
    // record traffic it removes).
    static const bool no_recs_env = shs_exp_env("SHS_LEGACY_NORECS") && std::atoi(shs_exp_env("SHS_LEGACY_NORECS")) != 0;
    const bool no_recs = !fp.scan_mode && no_recs_env;
    if (no_recs) {
        fp.flags |= shs_dev::RF_NO_RECS;
        if (ensure(ctx, ws.tdraw, nt_all)) return SHS_ERR_HIP;
    }
    // Shared varyings (RF_SHARED_VARY): every frame of the batch draws frame 0's meshes with Phong /
    // Blinn-Phong shading and bitwise the same model matrices -- a static scene under a batch of camera
    // poses -- so the corners' world positions and normals are computed and stored once for the batch.
    // SHS_LEGACY_SHARE_VARY=0 turns it off (timing experiments).
    static const bool share_env = [] { const char *e = shs_exp_env("SHS_LEGACY_SHARE_VARY"); return !e || std::atoi(e) != 0; }();
    if (share_env && !no_recs && n_frames > 1) {
        bool share = true;
        for (int i = 0; i < n_draws && share; ++i) {
            const shs_legacy_draw &d0 = ctx->last_draws[i];
            share = d0.shading == SHS_SHADING_PHONG || d0.shading == SHS_SHADING_BLINN_PHONG;
            for (int fr = 1; fr < n_frames && share; ++fr) {
                const shs_legacy_draw &d = ctx->last_draws[(size_t)fr * n_draws + i];
                share = d.mesh_id == d0.mesh_id && d.shading == d0.shading && std::memcmp(d.model, d0.model, sizeof d.model) == 0;
            }
        }
        if (share) fp.flags |= shs_dev::RF_SHARED_VARY;
    }
    // Bin-mode row groups dealt to one XCD (RF_XCD_ROWS): SHS_LEGACY_XCD_ROWS=0 turns it off (timing
    // experiments).
    static const bool xcd_rows_env = [] { const char *e = shs_exp_env("SHS_LEGACY_XCD_ROWS"); return !e || std::atoi(e) != 0; }();
    if (!fp.scan_mode && xcd_rows_env) fp.flags |= shs_dev::RF_XCD_ROWS;
    const int owned_bt = (n_tiles - f.shard_rank + f.shard_count - 1) / f.shard_count;
    const int n_groups = (n_tris + 15) / 16;
    fp.setup_blocks = setup_blocks;
    // Binned (large) scenes list their unbounded slivers in k_setup and enumerate them in k_ghost: ghost
    // waves would recompute every triangle's record (C3: ~1/3 of k_setup's time).  (Not inline as below:
    // a bin-mode tile's first appender marks its rows busy with plain stores, which a sliver fragment's
    // busy mark in the same kernel would race.)  Scan-mode setup waves enumerate their own unbounded
    // slivers (RF_GHOST_INLINE) instead of ghost blocks recomputing every triangle's record (C2: 976
    // ghost blocks per batch for ~17 slivers per frame).  SHS_GHOST_INLINE=0 restores the ghost blocks,
    // SHS_GHOST_LIST=1 lists scan-mode slivers for k_ghost (timing experiments).
    static const bool ghost_inline_env = [] { const char *e = shs_exp_env("SHS_GHOST_INLINE"); return !e || std::atoi(e) != 0; }();
    fp.ghost_list = (fp.scan_mode && !ghost_list_env) ? 0u : 1u;
    // (only when the ghost waves would take one slice per group anyway: a single frame's few slivers,
    // cut into up to 16 slices over the ghost blocks, finish sooner than walked by their setup waves --
    // C2 single frame 34 vs 51 us)
    if (!fp.ghost_list && ghost_inline_env && fp.ghost_slices == 1u) fp.flags |= shs_dev::RF_GHOST_INLINE;
    fp.ghost_blocks = (fp.ghost_list || (fp.flags & shs_dev::RF_GHOST_INLINE)) ? 0 : (n_groups * (int)fp.ghost_slices + 3) / 4;
    fp.clear_blocks = 0;
    fp.n_owned_rt = owned_bt * (shs_dev::TILE / shs_dev::RTH);
    fp.n_frames = n_frames;
    fp.frame_blocks = std::max(1, fp.setup_blocks + fp.ghost_blocks + fp.clear_blocks);
    // persistent raster grid: one resident wave of workgroups (k_raster runs 4 per CU)
    // Resident k_raster workgroups per CU: 4 fill every CU; bin-mode scenes leave one slot so the next
    // batch's k_setup / k_ghost (setup stream) run beside this raster instead of after it (measured,
    // C3: 0.76 -> 0.68 ms per 16-frame step; scan-mode C2 is best at 4).  SHS_RASTER_PER_CU overrides
    // (timing experiments).
    static const int rbpc_env = [] {
        const char *e = shs_exp_env("SHS_RASTER_PER_CU");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 && v <= 8 ? v : 0;
    }();
    const int rbpc = rbpc_env ? rbpc_env : (fp.scan_mode ? 4 : 3);
    const int raster_grid = std::max(1, std::min(fp.n_owned_rt * n_frames, 256 * rbpc));
    if (ensure(ctx, ws.rstat, (size_t)raster_grid)) return SHS_ERR_HIP;
    fp.setup_grid = fp.frame_blocks * n_frames;
    if (ctx->want_timeline) {
        const size_t n = (size_t)shs_dev::TL_STRIDE * (fp.setup_grid + raster_grid);
        if (ensure(ctx, ctx->timeline, n)) return SHS_ERR_HIP;
        HIP_TRY(ctx, hipMemsetAsync(ctx->timeline.p, 0, n * sizeof(uint64_t), sst));
    }

    FrameBuffers fb;
    fb.draws = ws.draws.p; fb.bdraw = bdraw; fb.recs = ws.recs.p; fb.rext = ws.rext.p; fb.shade = ws.shade.p; fb.tile_count = ws.tile_count.p; fb.bins = ws.bins.p;
    fb.spill = ws.spill.p; fb.frags = ws.frags.p; fb.counters = ctx->counters.p;
    fb.slivers = ws.slivers.p;
    fb.busy = ws.busy.p;
    fb.busy_list = ws.busy_list.p;
    fb.blk_stat = ws.blk_stat.p;
    fb.rstat = ws.rstat.p;
    fb.timeline = ctx->want_timeline ? ctx->timeline.p : nullptr;
    fb.boxes = ws.boxes.p;
    fb.tdraw = no_recs ? ws.tdraw.p : nullptr;
    fb.color = ctx->color.p; fb.depth = ctx->depth.p; fb.prequant = want_pq ? ctx->prequant.p : nullptr;
    fb.present = want_present ? ctx->present.p : nullptr;
    fb.ov_host = const_cast<uint32_t *>(ws.h_ov);

    hipEvent_t *ev = nullptr;
    if (ring_take(ctx, true, ev)) return SHS_ERR_HIP;
    if (pipe) {
        // one launch: the pending batch's raster with this batch's setup (k_pipe), or this setup alone;
        // this batch's raster is pending until the next batch or a flush.  Timing: the launch counts as
        // this batch's "raster" (setup 0): the sums over a run are then the device time per batch.
        if (ev) {
            HIP_TRY(ctx, hipEventRecord(ev[0], st));
            HIP_TRY(ctx, hipEventRecord(ev[1], st));
            HIP_TRY(ctx, hipEventRecord(ev[3], st));
        }
        if (ctx->pend.on) {
            HIP_TRY(ctx, shs_internal::launch_pipe(ctx->pend.fp, ctx->pend.fb, ctx->pend.grid, fp, fb, st));
            HIP_TRY(ctx, hipEventRecord(ctx->lslot[ctx->pend.slot].raster_done, st));
        } else {
            HIP_TRY(ctx, shs_internal::launch_setup(fp, fb, ka, st));
        }
        if (ev) HIP_TRY(ctx, hipEventRecord(ev[2], st));
        HIP_TRY(ctx, hipEventRecord(ws.setup_done, st));
        ctx->pend.on = true;
        ctx->pend.fp = fp;
        ctx->pend.fb = fb;
        ctx->pend.grid = raster_grid;
        ctx->pend.slot = slot;
    } else {
    // kernel durations: [0]..[1] k_setup (+ k_ghost in ghost_list mode) on setup_stream,
    // [3]..[2] k_raster on stream
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[0], sst));
    HIP_TRY(ctx, shs_internal::launch_setup(fp, fb, ka, sst));
    if (fp.ghost_list && !(fp.flags & shs_dev::DBG_SKIP_GHOST)) HIP_TRY(ctx, shs_internal::launch_ghost(fp, fb, sst));
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[1], sst));
    HIP_TRY(ctx, hipEventRecord(ws.setup_done, sst));
    // ---- stream: after the previous batch's raster (stream order) and this batch's setup ----
    HIP_TRY(ctx, hipStreamWaitEvent(st, ws.setup_done, 0));
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[3], st));
    HIP_TRY(ctx, shs_internal::launch_raster(fp, fb, ka, raster_grid, st));
    if (ev) HIP_TRY(ctx, hipEventRecord(ev[2], st));
    HIP_TRY(ctx, hipEventRecord(ws.raster_done, st));
    }
    ws.used = true;
    ctx->last_parity = fp.parity;
    ctx->last_slot = slot;
    ctx->last_no_recs = no_recs;
    ctx->frame_index++;
    ctx->have_frame = true;
    ctx->need_check = true;
    ctx->last_n_tris = n_tris;
    ctx->last_n_tiles = n_tiles;
    ctx->last_setup_blocks = setup_blocks * n_frames;
    ctx->last_raster_grid = raster_grid;
    ctx->last_setup_grid = fp.setup_grid;
    ctx->last_ghost_blocks = fp.ghost_blocks;
    ctx->last_clear_blocks = fp.clear_blocks;
    return SHS_OK;
}

static uint32_t next_pow2(uint32_t v) {
    uint32_t p = 1;
    while (p < v && p < (1u << 30)) p <<= 1;
    return p;
}

// Wait for the frame and read its counters; if a capacity overflowed, grow it and re-issue the frame.
static int finish_frame(shs_ctx *ctx) {
    if (flush_pending(ctx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));   // k_raster waited for its k_setup
    if (!ctx->need_check) return SHS_OK;
    for (int attempt = 0; attempt < 6; ++attempt) {
        HIP_TRY(ctx, hipMemcpy(ctx->h_counters, ctx->counters.p + ctx->last_parity * shs_dev::CSET,
                               shs_dev::C_NCOUNTERS * sizeof(uint32_t), hipMemcpyDeviceToHost));
        const uint32_t *c = ctx->h_counters;
        // per-block statistics: setup blocks (triangle classes, bin entries), raster blocks
        // (covered pixels, fullest bin tile)
        ctx->h_blk_stat.resize(ctx->last_setup_blocks);
        ctx->h_rstat.resize(ctx->last_raster_grid);
        if (ctx->last_setup_blocks)
            HIP_TRY(ctx, hipMemcpy(ctx->h_blk_stat.data(), ctx->lslot[ctx->last_slot].blk_stat.p, ctx->last_setup_blocks * sizeof(uint4),
                                   hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(ctx->h_rstat.data(), ctx->lslot[ctx->last_slot].rstat.p, ctx->last_raster_grid * sizeof(uint2),
                               hipMemcpyDeviceToHost));
        ctx->last_covered = ctx->last_bins = ctx->last_maxbin = ctx->last_setup = ctx->last_ghost = ctx->last_unb = 0;
        for (const uint4 &b : ctx->h_blk_stat) {
            ctx->last_setup += b.x; ctx->last_ghost += b.y; ctx->last_unb += b.z; ctx->last_bins += b.w;
        }
        for (const uint2 &r : ctx->h_rstat) {
            ctx->last_covered += r.x;
            ctx->last_maxbin = std::max<uint64_t>(ctx->last_maxbin, r.y);
        }
        // adapt the per-tile bin capacity to the fullest tile (spilled entries stay exact)
        if (ctx->last_maxbin > ctx->bin_cap) ctx->bin_cap = next_pow2((uint32_t)std::min<uint64_t>(ctx->last_maxbin, 1u << 30));
        const uint32_t ov = c[shs_dev::C_OVERFLOW];
        if (!ov) break;
        if (ov & shs_dev::OV_SPILL) {
            const size_t need = c[shs_dev::C_SPILL];
            for (auto &w : ctx->lslot) {
                release(w.spill);
                if (ensure(ctx, w.spill, need + need / 4 + 1024)) return SHS_ERR_HIP;
            }
        }
        if (ov & shs_dev::OV_FRAG) {
            const size_t need = c[shs_dev::C_FRAG];
            for (auto &w : ctx->lslot) {
                release(w.frags);
                if (ensure(ctx, w.frags, need + need / 4 + 1024)) return SHS_ERR_HIP;
            }
        }
        int rc = enqueue_frame(ctx);
        if (rc) return rc;
        if (flush_pending(ctx)) return SHS_ERR_HIP;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (ctx->h_counters[shs_dev::C_OVERFLOW]) { ctx->err = "capacity overflow persisted"; return SHS_ERR_OVERFLOW; }
    if (ctx->timing && harvest_all(ctx)) return SHS_ERR_HIP;
    ctx->need_check = false;
    return SHS_OK;
}

}  // extern "C"

int shs_legacy_ensure_final(shs_ctx *ctx) {
    if (flush_pending(ctx)) return SHS_ERR_HIP;
    if (!ctx->have_frame || !ctx->need_check) return SHS_OK;
    const shs_ctx::LegacySlot &p = ctx->lslot[ctx->last_slot];
    HIP_TRY(ctx, hipEventSynchronize(p.setup_done));
    return *p.h_ov ? finish_frame(ctx) : SHS_OK;
}

extern "C" {

int shs_render_legacy_batch(shs_ctx *ctx, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws,
                            int32_t n_frames) {
    if (!ctx || !frame || n_draws < 0 || (n_draws > 0 && !draws) || n_frames < 1 || n_frames > SHS_MAX_BATCH_FRAMES)
        return SHS_ERR_INVALID;
    const shs_frame_desc &f = *frame;
    if (f.width <= 0 || f.height <= 0 || f.width > 16384 || f.height > 16384) { ctx->err = "bad frame size"; return SHS_ERR_INVALID; }
    if (f.ref_tile_w <= 0 || f.ref_tile_h <= 0) { ctx->err = "bad reference tile size"; return SHS_ERR_INVALID; }
    if (f.shard_count <= 0 || f.shard_rank < 0 || f.shard_rank >= f.shard_count) { ctx->err = "bad shard"; return SHS_ERR_INVALID; }
    const int n_all = n_draws * n_frames;
    int64_t tris0 = 0;
    for (int i = 0; i < n_all; ++i) {
        const int id = draws[i].mesh_id;
        if (id < 0 || id >= (int)ctx->meshes.size() || !ctx->meshes[id].live || ctx->meshes[id].lib) {
            ctx->err = "bad mesh id (not a legacy soup mesh)";
            return SHS_ERR_INVALID;
        }
        if (draws[i].shading < SHS_SHADING_FLAT || draws[i].shading > SHS_SHADING_BLINN_PHONG) {
            ctx->err = "bad shading model";
            return SHS_ERR_INVALID;
        }
    }
    // every frame of a batch submits the same number of triangles (one submission-order layout)
    for (int fr = 0; fr < n_frames; ++fr) {
        int64_t t = 0;
        for (int i = 0; i < n_draws; ++i) t += ctx->meshes[draws[fr * n_draws + i].mesh_id].n_tris;
        if (fr == 0) tris0 = t;
        else if (t != tris0) { ctx->err = "frames of a batch must submit equal triangle counts"; return SHS_ERR_INVALID; }
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    // A still-pending previous batch is superseded by this one, but never unchecked: a stream-ordered
    // consumer of its frames (a copy queued behind it) must not see a batch that overflowed a
    // capacity.  Its overflow word is final once its setup is (long before its raster ends); if it is
    // set, the batch is finished -- re-issued with grown capacities -- before this one is enqueued.
    // (A pending pipelined batch is superseded without the check: its raster still runs -- in this
    // batch's launch or at the flush enqueue_frame does -- but its frames are overwritten by this batch
    // before any call can read them.)
    if (!ctx->pend.on) {
        const int rc = shs_legacy_ensure_final(ctx);
        if (rc) return rc;
    }
    ctx->frame = f;
    ctx->last_draws.assign(draws, draws + n_all);
    ctx->last_n_frames = n_frames;
    ctx->frame_draws = n_draws;
    return enqueue_frame(ctx);
}

int shs_render_legacy(shs_ctx *ctx, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws) {
    return shs_render_legacy_batch(ctx, frame, draws, n_draws, 1);
}

int shs_synchronize(shs_ctx *ctx) {
    if (!ctx) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    return finish_frame(ctx);
}

int shs_resolve_frame(shs_ctx *ctx, int32_t frame_index, uint8_t *color, float *depth) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_frame) { ctx->err = "no frame rendered"; return SHS_ERR_INVALID; }
    if (frame_index < 0 || frame_index >= ctx->last_n_frames) { ctx->err = "frame index outside the batch"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    const size_t npx = (size_t)ctx->frame.width * ctx->frame.height;
    if (color) HIP_TRY(ctx, hipMemcpy(color, ctx->color.p + npx * 4 * frame_index, npx * 4, hipMemcpyDeviceToHost));
    if (depth) HIP_TRY(ctx, hipMemcpy(depth, ctx->depth.p + npx * frame_index, npx * sizeof(float), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_resolve(shs_ctx *ctx, uint8_t *color, float *depth) { return shs_resolve_frame(ctx, 0, color, depth); }

int shs_resolve_present(shs_ctx *ctx, int32_t frame_index, uint8_t *pixels, int32_t pitch) {
    if (!ctx || !pixels) return SHS_ERR_INVALID;
    if (!ctx->have_frame || !(ctx->frame.flags & SHS_FRAME_PRESENT)) { ctx->err = "frame has no present staging (SHS_FRAME_PRESENT)"; return SHS_ERR_INVALID; }
    if (frame_index < 0 || frame_index >= ctx->last_n_frames) { ctx->err = "frame index outside the batch"; return SHS_ERR_INVALID; }
    const int W = ctx->frame.width, H = ctx->frame.height;
    if (pitch < W * 4) { ctx->err = "pitch below width * 4"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    const uint32_t *src = ctx->present.p + (size_t)W * H * frame_index;
    HIP_TRY(ctx, hipMemcpy2D(pixels, (size_t)pitch, src, (size_t)W * 4, (size_t)W * 4, (size_t)H, hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_present_device(shs_ctx *ctx, int32_t frame_index, void **present_dev) {
    if (!ctx || !present_dev) return SHS_ERR_INVALID;
    if (!ctx->have_frame || !(ctx->frame.flags & SHS_FRAME_PRESENT)) { ctx->err = "frame has no present staging (SHS_FRAME_PRESENT)"; return SHS_ERR_INVALID; }
    if (frame_index < 0 || frame_index >= ctx->last_n_frames) { ctx->err = "frame index outside the batch"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    // the batch is final (overflow checked, re-issued if needed) before its staging is handed out
    int rc = finish_frame(ctx);
    if (rc) return rc;
    *present_dev = ctx->present.p + (size_t)ctx->frame.width * ctx->frame.height * frame_index;
    return SHS_OK;
}

int shs_resolve_prequant_frame(shs_ctx *ctx, int32_t frame_index, float *pq) {
    if (!ctx || !pq) return SHS_ERR_INVALID;
    if (!ctx->have_frame || !(ctx->frame.flags & SHS_FRAME_PREQUANT)) { ctx->err = "frame has no prequant buffer"; return SHS_ERR_INVALID; }
    if (frame_index < 0 || frame_index >= ctx->last_n_frames) { ctx->err = "frame index outside the batch"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    const size_t npx = (size_t)ctx->frame.width * ctx->frame.height;
    HIP_TRY(ctx, hipMemcpy(pq, ctx->prequant.p + npx * frame_index, npx * sizeof(float4), hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_resolve_prequant(shs_ctx *ctx, float *pq) { return shs_resolve_prequant_frame(ctx, 0, pq); }

int shs_device_framebuffers(shs_ctx *ctx, void **color_dev, void **depth_dev) {
    if (!ctx || !ctx->have_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    if (color_dev) *color_dev = ctx->color.p;
    if (depth_dev) *depth_dev = ctx->depth.p;
    return SHS_OK;
}

int shs_get_stats(shs_ctx *ctx, shs_raster_stats *st) {
    if (!ctx || !st || !ctx->have_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    st->tri_input = (uint64_t)ctx->last_n_tris * ctx->last_n_frames;
    st->tri_setup = ctx->last_setup;
    st->tri_ghost = ctx->last_ghost;
    st->bin_entries = ctx->last_bins;
    st->tri_ghost_unbounded = ctx->last_unb;
    st->spilled = ctx->h_counters[shs_dev::C_SPILL];
    st->max_tile_bin = ctx->last_maxbin;
    st->ghost_fragments = ctx->h_counters[shs_dev::C_FRAG];
    st->covered_pixels = ctx->last_covered;
    return SHS_OK;
}

int shs_enable_timing(shs_ctx *ctx, int enable) {
    if (!ctx) return SHS_ERR_INVALID;
    ctx->timing = enable != 0;
    return SHS_OK;
}

int shs_timing_reset(shs_ctx *ctx) {
    if (!ctx) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    if (harvest_all(ctx)) return SHS_ERR_HIP;
    for (int i = 0; i < 4; ++i) ctx->acc_ms[i] = 0.0;
    ctx->acc_frames = 0;
    return SHS_OK;
}

int shs_timing_read(shs_ctx *ctx, double *sum_ms4, int64_t *n_frames) {
    if (!ctx || !sum_ms4 || !n_frames) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    if (harvest_all(ctx)) return SHS_ERR_HIP;
    for (int i = 0; i < 4; ++i) sum_ms4[i] = ctx->acc_ms[i];
    *n_frames = ctx->acc_frames;
    return SHS_OK;
}

int shs_last_kernel_ms(shs_ctx *ctx, float *ms4) {
    if (!ctx || !ms4) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    std::memcpy(ms4, ctx->last_ms, sizeof ctx->last_ms);
    return SHS_OK;
}

int shs_debug_records(shs_ctx *ctx, void *out, int64_t capacity, int64_t *n_out) {
    if (!ctx || !n_out || !ctx->have_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    if (ctx->last_no_recs) { ctx->err = "SHS_LEGACY_NORECS frames keep no triangle records"; return SHS_ERR_INVALID; }
    *n_out = ctx->last_n_tris;
    if (out && capacity > 0) {
        const size_t n = (size_t)std::min<int64_t>(capacity, ctx->last_n_tris);
        HIP_TRY(ctx, hipMemcpy(out, ctx->lslot[ctx->last_slot].recs.p, n * sizeof(shs_dev::TriHot), hipMemcpyDeviceToHost));
    }
    return SHS_OK;
}

int shs_debug_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out) {
    if (!ctx || !n_out || !ctx->have_frame) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    int rc = finish_frame(ctx);
    if (rc) return rc;
    if (!ctx->want_timeline || !ctx->timeline.p) { ctx->err = "timeline not enabled"; return SHS_ERR_INVALID; }
    const size_t pairs = (size_t)ctx->last_setup_grid + ctx->last_raster_grid;
    *n_out = (int64_t)(8 + shs_dev::TL_STRIDE * pairs);
    if (out && capacity >= *n_out) {
        const uint64_t head[8] = {(uint64_t)ctx->last_setup_grid, (uint64_t)ctx->last_raster_grid,
                                  (uint64_t)ctx->last_setup_blocks, (uint64_t)ctx->last_ghost_blocks,
                                  (uint64_t)ctx->last_clear_blocks, (uint64_t)shs_dev::TL_STRIDE, 0, 0};
        std::memcpy(out, head, sizeof head);
        HIP_TRY(ctx, hipMemcpy(out + 8, ctx->timeline.p, shs_dev::TL_STRIDE * pairs * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    return SHS_OK;
}

int shs_set_option(shs_ctx *ctx, int option, int64_t value) {
    if (!ctx) return SHS_ERR_INVALID;
    if (option == SHS_OPT_RASTER_MODE) {
        if (value < 0 || value > 2) return SHS_ERR_INVALID;
        ctx->force_mode = (int)value;
        return SHS_OK;
    }
    if (option == SHS_OPT_RASTER_LOOP) {
        if (value < 0 || value > 1) return SHS_ERR_INVALID;
        ctx->pair_loop = value == 1;
        return SHS_OK;
    }
    if (option == SHS_OPT_TIMELINE) {
        if (value < 0 || value > 2) return SHS_ERR_INVALID;
        ctx->want_timeline = value != 0;
        ctx->timeline_shadow = value == 2;
        return SHS_OK;
    }
    if (option == SHS_OPT_SHARD_CULL) {
        if (value < 0 || value > 1) return SHS_ERR_INVALID;
        ctx->shard_cull = value != 0;
        return SHS_OK;
    }
    if (option == SHS_OPT_SHARD_LAYOUT) {
        if (value != SHS_SHARD_INTERLEAVED && value != SHS_SHARD_REGIONS) return SHS_ERR_INVALID;
        ctx->shard_layout = (int)value;
        ctx->reg_next_fresh = false;
        return SHS_OK;
    }
    if (option == SHS_OPT_SHARD_ROOT_SHARE) {
        if (value < 0 || value > 1000) return SHS_ERR_INVALID;
        ctx->shard_root_permille = (int)value;
        ctx->reg_next_fresh = false;
        return SHS_OK;
    }
    if (option == SHS_OPT_LEGACY_PIPELINE) {
        if (value < 0 || value > 1) return SHS_ERR_INVALID;
        if (value == 0) {
            if (set_dev(ctx)) return SHS_ERR_HIP;
            if (flush_pending(ctx)) return SHS_ERR_HIP;
        }
        ctx->legacy_pipeline = value != 0;
        return SHS_OK;
    }
    if (option == SHS_OPT_SHADOW_FOOTPRINT) {
        if (value < 0 || value > 1) return SHS_ERR_INVALID;
        if (value == 0 && ctx->shadow_pending) {   // a recorded pass is rendered whole now
            const int rc = shs_lib_flush_shadow(ctx);
            if (rc) return rc;
        }
        ctx->shadow_footprint = value != 0;
        return SHS_OK;
    }
    if (option == SHS_OPT_LIB_PART) {
        if (value < -1 || value > (1 << 20)) return SHS_ERR_INVALID;
        ctx->lib_part = value;
        return SHS_OK;
    }
    if (option == SHS_OPT_SPILL_CAPACITY || option == SHS_OPT_FRAG_CAPACITY) {
        if (value < 1 || value > (1 << 28)) return SHS_ERR_INVALID;
        if (set_dev(ctx)) return SHS_ERR_HIP;
        int rc = finish_frame(ctx);
        if (rc) return rc;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
        for (auto &w : ctx->lslot) {
            if (option == SHS_OPT_SPILL_CAPACITY) {
                release(w.spill);
                if (ensure(ctx, w.spill, (size_t)value)) return SHS_ERR_HIP;
                w.spill.cap = (size_t)value;   // ensure() allocates at least 16
            } else {
                release(w.frags);
                if (ensure(ctx, w.frags, (size_t)value)) return SHS_ERR_HIP;
                w.frags.cap = (size_t)value;
            }
        }
        return SHS_OK;
    }
    if (option == SHS_OPT_BIN_CAPACITY) {
        if (value < 1 || value > (1 << 24)) return SHS_ERR_INVALID;
        if (set_dev(ctx)) return SHS_ERR_HIP;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        ctx->bin_cap = (uint32_t)value;
        return SHS_OK;
    }
    return SHS_ERR_INVALID;
}

int shs_camera3d(const float position[3], float ha, float va, float fov, float zn, float zf, float view16[16], float proj16[16]) {
    if (!position || !view16 || !proj16) return SHS_ERR_INVALID;
    shs_host::camera3d(shs_host::vec3{position[0], position[1], position[2]}, ha, va, fov, zn, zf, view16, proj16);
    return SHS_OK;
}

int shs_model_trs(const float position[3], float rot_deg_y, const float scl[3], float out16[16]) {
    if (!position || !scl || !out16) return SHS_ERR_INVALID;
    shs_host::model_trs(shs_host::vec3{position[0], position[1], position[2]}, rot_deg_y,
                        shs_host::vec3{scl[0], scl[1], scl[2]}, out16);
    return SHS_OK;
}

int shs_mat4_mul(const float a[16], const float b[16], float out[16]) {
    if (!a || !b || !out) return SHS_ERR_INVALID;
    shs_host::mul(a, b, out);
    return SHS_OK;
}

int shs_mat4_inverse(const float m[16], float out[16]) {
    if (!m || !out) return SHS_ERR_INVALID;
    shs_host::inverse(m, out);
    return SHS_OK;
}

}  // extern "C"
