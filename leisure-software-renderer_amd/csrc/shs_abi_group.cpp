// shs_abi_group.cpp -- multi-GPU from one host process (include/shs_gpu.h, "multi-GPU from one host
// process"): n contexts, one per rank, each rendering its interleaved 32x32 tiles (tile % n == r), and
// the final-image gather into rank 0 over peer copies (xGMI between MI355X devices).
//
// The reference host is a single C++ process (hello_pipeline_blinn_phong_shading.cpp:369-455;
// PluggablePipeline::execute, pipeline/pluggable_pipeline.hpp:980) -- this is what lets such a host use
// the node's GPUs without a second process or torch.distributed.  Every rank has a persistent host
// worker thread, so the per-rank enqueue work of a call runs concurrently over the ranks.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/shs_gpu.h"
#include "shs_ctx.hpp"

namespace {

// One host thread per rank: run() hands the same job to every worker and waits for all of them.
class RankPool {
public:
    explicit RankPool(int n) : n_(n), rc_(n, SHS_OK) {
        for (int r = 1; r < n; ++r) threads_.emplace_back([this, r] { loop(r); });
    }
    ~RankPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : threads_) t.join();
    }
    // job(rank) on every rank (rank 0 on the calling thread); -> the first failing rank or -1
    int run(const std::function<int(int)> &job, std::vector<int> &rcs) {
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &job;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        rc_[0] = job(0);
        {
            std::unique_lock<std::mutex> lk(m_);
            done_cv_.wait(lk, [this] { return pending_ == 0; });
            job_ = nullptr;
        }
        rcs = rc_;
        for (int r = 0; r < n_; ++r)
            if (rc_[r] != SHS_OK) return r;
        return -1;
    }

private:
    void loop(int r) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<int(int)> *job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            const int rc = (*job)(r);
            {
                std::lock_guard<std::mutex> lk(m_);
                rc_[r] = rc;
                if (--pending_ == 0) done_cv_.notify_one();
            }
        }
    }

    int n_;
    std::vector<int> rc_;
    std::vector<std::thread> threads_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<int(int)> *job_ = nullptr;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

}  // namespace

struct shs_group {
    std::vector<shs_ctx *> ctx;
    std::vector<int> dev;
    RankPool *pool = nullptr;
    std::string err;
    // gather staging, per rank r >= 1: its packed tiles on its device, two receive buffers on rank 0's
    // device (frame parity), and the events ordering send -> unpack -> next send into the same buffer
    struct Link {
        void *send = nullptr;
        void *recv[2] = {nullptr, nullptr};
        size_t bytes = 0;
        hipEvent_t sent[2] = {nullptr, nullptr};       // on the rank's device
        hipEvent_t consumed[2] = {nullptr, nullptr};   // on rank 0's device
        bool consumed_valid[2] = {false, false};
    };
    std::vector<Link> links;
    int parity = 0;
};

namespace {

int group_fail(shs_group *g, int rank, const std::vector<int> &rcs) {
    g->err = "rank " + std::to_string(rank) + ": " + shs_last_error(g->ctx[rank]);
    return rcs[rank];
}

// job(rank, ctx) on every rank, concurrently.
int for_ranks(shs_group *g, const std::function<int(int, shs_ctx *)> &job) {
    std::vector<int> rcs;
    const std::function<int(int)> j = [&](int r) { return job(r, g->ctx[r]); };
    const int bad = g->pool->run(j, rcs);
    return bad < 0 ? SHS_OK : group_fail(g, bad, rcs);
}

void free_links(shs_group *g) {
    for (size_t r = 1; r < g->links.size(); ++r) {
        shs_group::Link &l = g->links[r];
        if (l.send) { (void)hipSetDevice(g->dev[r]); (void)hipFree(l.send); }
        for (int p = 0; p < 2; ++p) {
            if (l.sent[p]) { (void)hipSetDevice(g->dev[r]); (void)hipEventDestroy(l.sent[p]); }
            if (l.recv[p]) { (void)hipSetDevice(g->dev[0]); (void)hipFree(l.recv[p]); }
            if (l.consumed[p]) { (void)hipSetDevice(g->dev[0]); (void)hipEventDestroy(l.consumed[p]); }
        }
        l = shs_group::Link{};
    }
}

#define G_TRY(g, expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (g)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                  \
            return SHS_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

// (Re)allocate the staging for `bytes` per rank.
int ensure_links(shs_group *g, size_t bytes) {
    const int n = (int)g->ctx.size();
    if ((int)g->links.size() == n && g->links.size() > 1 && g->links[1].bytes >= bytes) return SHS_OK;
    if (shs_group_synchronize(g)) return SHS_ERR_HIP;
    free_links(g);
    g->links.assign(n, shs_group::Link{});
    for (int r = 1; r < n; ++r) {
        shs_group::Link &l = g->links[r];
        G_TRY(g, hipSetDevice(g->dev[r]));
        G_TRY(g, hipMalloc(&l.send, bytes));
        for (int p = 0; p < 2; ++p) G_TRY(g, hipEventCreateWithFlags(&l.sent[p], hipEventDisableTiming));
        G_TRY(g, hipSetDevice(g->dev[0]));
        for (int p = 0; p < 2; ++p) {
            G_TRY(g, hipMalloc(&l.recv[p], bytes));
            G_TRY(g, hipEventCreateWithFlags(&l.consumed[p], hipEventDisableTiming));
        }
        l.bytes = bytes;
    }
    return SHS_OK;
}

}  // namespace

extern "C" {

int shs_group_create(const int32_t *devices, int32_t n, shs_group **out) {
    if (!devices || n < 1 || n > 64 || !out) return SHS_ERR_INVALID;
    *out = nullptr;
    shs_group *g = new shs_group();
    for (int r = 0; r < n; ++r) {
        shs_ctx *c = nullptr;
        const int rc = shs_create(devices[r], &c);
        if (rc) {
            for (shs_ctx *x : g->ctx) shs_destroy(x);
            delete g;
            return rc;
        }
        g->ctx.push_back(c);
        g->dev.push_back(devices[r]);
    }
    // peer access between rank 0's device and every other device (xGMI copies, cross-device waits)
    for (int r = 1; r < n; ++r) {
        if (g->dev[r] == g->dev[0]) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, g->dev[r], g->dev[0]) == hipSuccess && can) {
            (void)hipSetDevice(g->dev[r]);
            const hipError_t e = hipDeviceEnablePeerAccess(g->dev[0], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
    }
    g->pool = new RankPool(n);
    *out = g;
    return SHS_OK;
}

int shs_group_destroy(shs_group *g) {
    if (!g) return SHS_ERR_INVALID;
    (void)shs_group_synchronize(g);
    free_links(g);
    delete g->pool;
    for (shs_ctx *c : g->ctx) shs_destroy(c);
    delete g;
    return SHS_OK;
}

const char *shs_group_last_error(shs_group *g) { return g ? g->err.c_str() : "null group"; }

int shs_group_size(shs_group *g) { return g ? (int)g->ctx.size() : 0; }

int shs_group_context(shs_group *g, int32_t rank, shs_ctx **ctx) {
    if (!g || !ctx || rank < 0 || rank >= (int32_t)g->ctx.size()) return SHS_ERR_INVALID;
    *ctx = g->ctx[rank];
    return SHS_OK;
}

int shs_group_mesh_upload(shs_group *g, const float *positions, int32_t n_verts, const float *normals, int32_t n_normals,
                          const float *uvs, int32_t n_uvs, const uint32_t *indices, int64_t n_indices, int32_t *mesh_id) {
    if (!g || !mesh_id) return SHS_ERR_INVALID;
    std::vector<int32_t> ids(g->ctx.size(), -1);
    const int rc = for_ranks(g, [&](int r, shs_ctx *c) {
        return shs_mesh_upload(c, positions, n_verts, normals, n_normals, uvs, n_uvs, indices, n_indices, &ids[r]);
    });
    if (rc) return rc;
    for (int32_t id : ids)
        if (id != ids[0]) { g->err = "mesh ids differ across ranks (upload every mesh through the group)"; return SHS_ERR_INVALID; }
    *mesh_id = ids[0];
    return SHS_OK;
}

int shs_group_mesh_upload_soup(shs_group *g, const float *positions, const float *normals, int32_t n_tris, int32_t *mesh_id) {
    if (!g || !mesh_id) return SHS_ERR_INVALID;
    std::vector<int32_t> ids(g->ctx.size(), -1);
    const int rc = for_ranks(g, [&](int r, shs_ctx *c) { return shs_mesh_upload_soup(c, positions, normals, n_tris, &ids[r]); });
    if (rc) return rc;
    for (int32_t id : ids)
        if (id != ids[0]) { g->err = "mesh ids differ across ranks (upload every mesh through the group)"; return SHS_ERR_INVALID; }
    *mesh_id = ids[0];
    return SHS_OK;
}

int shs_group_texture_upload(shs_group *g, const uint8_t *rgba, int32_t w, int32_t h, int32_t *tex_id) {
    if (!g || !tex_id) return SHS_ERR_INVALID;
    std::vector<int32_t> ids(g->ctx.size(), 0);
    const int rc = for_ranks(g, [&](int r, shs_ctx *c) { return shs_texture_upload(c, rgba, w, h, &ids[r]); });
    if (rc) return rc;
    for (int32_t id : ids)
        if (id != ids[0]) { g->err = "texture ids differ across ranks (upload every texture through the group)"; return SHS_ERR_INVALID; }
    *tex_id = ids[0];
    return SHS_OK;
}

int shs_group_set_option(shs_group *g, int option, int64_t value) {
    if (!g) return SHS_ERR_INVALID;
    return for_ranks(g, [&](int, shs_ctx *c) { return shs_set_option(c, option, value); });
}

int shs_group_lights_upload(shs_group *g, const shs_culling_light *lights, int32_t n_lights) {
    if (!g) return SHS_ERR_INVALID;
    return for_ranks(g, [&](int, shs_ctx *c) { return shs_lights_upload(c, lights, n_lights); });
}

int shs_group_lib_fuse_tonemap(shs_group *g, const shs_tonemap_desc *desc) {
    if (!g) return SHS_ERR_INVALID;
    return for_ranks(g, [&](int, shs_ctx *c) { return shs_lib_fuse_tonemap(c, desc); });
}

int shs_group_light_cull(shs_group *g, const shs_light_cull_desc *desc) {
    if (!g || !desc) return SHS_ERR_INVALID;
    const int n = (int)g->ctx.size();
    return for_ranks(g, [&](int r, shs_ctx *c) {
        shs_light_cull_desc d = *desc;
        d.shard_rank = r;
        d.shard_count = n;
        return shs_light_cull(c, &d);
    });
}

int shs_group_render_shadow_map(shs_group *g, int32_t w, int32_t h, const float sun_dir[3], const shs_shadow_caster *casters,
                                int32_t n_casters, float light_viewproj_out[16]) {
    if (!g) return SHS_ERR_INVALID;
    return for_ranks(g, [&](int r, shs_ctx *c) {
        return shs_render_shadow_map(c, w, h, sun_dir, casters, n_casters, r == 0 ? light_viewproj_out : nullptr);
    });
}

int shs_group_render_pbr_forward(shs_group *g, const shs_lib_frame *frame, const shs_lib_draw *draws, int32_t n_draws) {
    if (!g || !frame) return SHS_ERR_INVALID;
    const int n = (int)g->ctx.size();
    return for_ranks(g, [&](int r, shs_ctx *c) {
        shs_lib_frame f = *frame;
        f.shard_rank = r;
        f.shard_count = n;
        return shs_render_pbr_forward(c, &f, draws, n_draws);
    });
}

int shs_group_render_legacy(shs_group *g, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws) {
    if (!g || !frame) return SHS_ERR_INVALID;
    const int n = (int)g->ctx.size();
    return for_ranks(g, [&](int r, shs_ctx *c) {
        shs_frame_desc f = *frame;
        f.shard_rank = r;
        f.shard_count = n;
        return shs_render_legacy(c, &f, draws, n_draws);
    });
}

int shs_group_gather(shs_group *g, int target) {
    if (!g) return SHS_ERR_INVALID;
    const int n = (int)g->ctx.size();
    if (n == 1) return SHS_OK;   // rank 0 rendered every tile
    int64_t words = 0;
    if (shs_tiles_packed_words(g->ctx[0], target, n, &words)) {
        g->err = std::string("rank 0: ") + shs_last_error(g->ctx[0]);
        return SHS_ERR_INVALID;
    }
    const size_t bytes = (size_t)std::max<int64_t>(words, 1) * 4;
    if (ensure_links(g, bytes)) return SHS_ERR_HIP;
    const int p = g->parity;
    g->parity ^= 1;
    // ranks >= 1: pack on their own stream, push to rank 0's device once rank 0 has unpacked what the
    // buffer held two gathers ago; rank 0: make its own frame final (its tiles are already in place)
    int rc = for_ranks(g, [&](int r, shs_ctx *c) {
        if (r == 0) return target == SHS_TARGET_LEGACY || target == SHS_TARGET_PRESENT ? shs_legacy_ensure_final(c)
                                                                                       : shs_lib_ensure_final(c);
        shs_group::Link &l = g->links[r];
        int e = shs_tiles_pack(c, target, r, n, l.send);
        if (e) return e;
        int64_t mine = 0;   // this rank's packed size (regions differ)
        e = shs_tiles_rank_words(c, target, r, n, &mine);
        if (e) return e;
        HIP_TRY(c, hipSetDevice(g->dev[r]));
        if (l.consumed_valid[p]) HIP_TRY(c, hipStreamWaitEvent(c->stream, l.consumed[p], 0));
        if (mine > 0) HIP_TRY(c, hipMemcpyPeerAsync(l.recv[p], g->dev[0], l.send, g->dev[r], (size_t)mine * 4, c->stream));
        HIP_TRY(c, hipEventRecord(l.sent[p], c->stream));
        return SHS_OK;
    });
    if (rc) return rc;
    shs_ctx *c0 = g->ctx[0];
    if (set_dev(c0)) { g->err = c0->err; return SHS_ERR_HIP; }
    for (int r = 1; r < n; ++r) {
        shs_group::Link &l = g->links[r];
        G_TRY(g, hipStreamWaitEvent(c0->stream, l.sent[p], 0));
        rc = shs_tiles_unpack(c0, target, r, n, l.recv[p]);
        if (rc) { g->err = std::string("rank 0: ") + shs_last_error(c0); return rc; }
        G_TRY(g, hipEventRecord(l.consumed[p], c0->stream));
        l.consumed_valid[p] = true;
    }
    return SHS_OK;
}

int shs_group_synchronize(shs_group *g) {
    if (!g) return SHS_ERR_INVALID;
    return for_ranks(g, [&](int, shs_ctx *c) {
        if (set_dev(c)) return SHS_ERR_HIP;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->setup_stream));
        return SHS_OK;
    });
}

}  // extern "C"
