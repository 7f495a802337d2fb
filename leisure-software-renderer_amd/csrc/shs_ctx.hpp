// shs_ctx.hpp -- the libshs_gpu context (struct shs_ctx) shared by the ABI translation units
// (shs_abi.cpp: legacy path; shs_abi_lib.cpp: library path).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/shs_gpu.h"
#include "shs_device.hpp"
#include "shs_lib_device.hpp"
#include "shs_canvas_post_internal.hpp"
#include "shs_debugdraw_internal.hpp"
#include "shs_lightbin_internal.hpp"
#include "shs_occlusion_internal.hpp"

// Timing-experiment switches (SHS_* environment variables and the frame's DBG_* debug bits; several give
// wrong images).  Only the -DSHS_TIMING_EXPERIMENTS build (`make exp` -> shs_gpu/libshs_gpu_exp.so,
// loaded by tools/ through SHS_GPU_LIB) reads them; the product library ignores the environment.
#ifdef SHS_TIMING_EXPERIMENTS
#include <cstdlib>
inline const char *shs_exp_env(const char *name) { return std::getenv(name); }
constexpr bool SHS_EXPERIMENTS = true;
#else
inline const char *shs_exp_env(const char *) { return nullptr; }
constexpr bool SHS_EXPERIMENTS = false;
#endif

namespace shs_host_detail {
struct Mesh {
    float *pos = nullptr;            // legacy soup: 9 floats per triangle; library mesh: 3 per vertex
    float *nrm = nullptr;
    int32_t n_tris = 0;
    bool live = false;
    // library MeshData (resources/mesh.hpp:23-43): uvs, indices (nullptr: soup), model-space bounds
    bool lib = false;
    float *uv = nullptr;
    uint32_t *idx = nullptr;
    int32_t n_verts = 0;
    float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
    float4 *cbox = nullptr;          // library mesh: per 256-triangle chunk its model-space box (min, max)
    uint32_t *orig = nullptr;        // library mesh stored in spatial order: per stored triangle its MeshData index
    bool borrowed = false;           // shs_mesh_share: another context's buffers (never freed here)
};

// A Texture2DData (resources/texture.hpp:23-49) on the device: w * h Color texels, y * w + x.
struct Texture {
    uint32_t *texels = nullptr;
    int32_t w = 0, h = 0;
    bool live = false;
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
};
}  // namespace shs_host_detail
using shs_host_detail::Mesh;
using shs_host_detail::Texture;
using shs_host_detail::DevBuf;

struct shs_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<Mesh> meshes;
    std::vector<Texture> textures;   // texture id k (>= 1, the TextureAssetHandle convention) at k - 1

    // Legacy-path workspace, double-buffered: batch n uses slot n & 1.  Its k_setup (plus the draw-table
    // copy and the counter resets) runs on setup_stream while batch n-1's k_raster still runs on
    // stream; setup of slot s waits for the k_raster that last used slot s (raster_done).
    struct LegacySlot {
        DevBuf<shs_dev::DrawGPU> draws;      // device draw table (> KARG_DRAWS draws)
        shs_dev::DrawGPU *h_draws = nullptr; // pinned staging of that table
        size_t h_cap = 0;
        DevBuf<shs_dev::TriHot> recs;        // per frame: 64-B stored records
        DevBuf<float4> rext;                 // per frame: float bboxes of ghosts
        DevBuf<shs_dev::ShadeRec> shade;
        DevBuf<uint32_t> tile_count;         // per frame: per-bin-tile counts (zeroed per batch)
        DevBuf<uint32_t> bins;               // per frame: n_tiles * bin_cap
        DevBuf<uint2> spill;
        DevBuf<shs_dev::GhostFrag> frags;    // ghost fragments
        DevBuf<uint32_t> slivers;            // unbounded sliver ids (ghost_list mode)
        DevBuf<uint2> boxes;                 // per-triangle bin boxes
        DevBuf<int32_t> tdraw;               // per-triangle draw (binned frames: no records kept)
        DevBuf<uint32_t> busy;               // per raster tile: the epoch of the last batch that marked it
        DevBuf<uint32_t> busy_list;          // busy tiles of the batch (k_raster's work items)
        DevBuf<uint4> blk_stat;              // per setup block
        DevBuf<uint2> rstat;                 // per raster block
        hipEvent_t setup_done = nullptr, raster_done = nullptr;
        // the batch's overflow word in mapped, coherent host memory: the setup kernels store 1 into it
        // with every overflow bit, so once setup_done has fired the host reads it without a copy and
        // without waiting for the raster (checked before the batch is superseded)
        volatile uint32_t *h_ov = nullptr;
        bool used = false;
    };
    LegacySlot lslot[2];
    hipStream_t setup_stream = nullptr;
    DevBuf<uint32_t> counters;       // 2 sets (one per slot) of CSET words
    uint32_t busy_epoch = 0;         // FrameParams::epoch of the last launch (never 0)
    int last_slot = 0;
    bool last_no_recs = false;       // the last legacy batch was binned without stored records (RF_NO_RECS)
    DevBuf<uint64_t> timeline;       // SHS_OPT_TIMELINE
    bool want_timeline = false;
    bool timeline_shadow = false;    // SHS_OPT_TIMELINE 2: the library's shadow raster records it instead
    int last_setup_grid = 0, last_ghost_blocks = 0, last_clear_blocks = 0;
    std::vector<uint4> h_blk_stat;
    std::vector<uint2> h_rstat;
    uint64_t geom_key[2] = {~0ull, ~0ull};   // (tiles, shard, frames) per slot: a change resets its busy flags
    int last_setup_blocks = 0, last_raster_grid = 0;
    uint64_t last_covered = 0, last_bins = 0, last_maxbin = 0, last_setup = 0, last_ghost = 0, last_unb = 0;
    uint32_t bin_cap = 256;
    int force_mode = 0;              // 0 auto, 1 scan, 2 bin (SHS_OPT_RASTER_MODE)
    bool pair_loop = true;           // SHS_OPT_RASTER_LOOP: (candidate, pixel) pair tasks (default)
    uint32_t frame_index = 0;        // parity of the counter set
    uint32_t last_parity = 0;
    DevBuf<uint8_t> color;
    DevBuf<float> depth;
    DevBuf<float4> prequant;
    DevBuf<uint32_t> present;        // SHS_FRAME_PRESENT staging (per frame of the batch)

    uint32_t *h_counters = nullptr;  // pinned, C_NCOUNTERS

    // last frame (re-issued if a bin capacity overflowed)
    shs_frame_desc frame{};
    std::vector<shs_legacy_draw> last_draws;
    bool have_frame = false;
    bool need_check = false;
    int last_n_frames = 1;           // frames of the last batch (last_draws holds n_frames x frame_draws)
    int frame_draws = 0;             // draws per frame of the last batch
    int last_n_tris = 0;             // triangles per frame
    int last_n_tiles = 0;

    bool timing = false;
    hipEvent_t tev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    float last_ms[4] = {0, 0, 0, 0};
    // ring of per-frame kernel events, harvested lazily: sums of kernel durations over many frames.
    // [0] [1] around k_setup (+ k_ghost) on setup_stream, [3] [2] around k_raster on stream.
    static constexpr int RING = 64;
    hipEvent_t ring_ev[RING][5] = {};
    bool ring_pending[RING] = {};
    bool ring_counts[RING] = {};     // the entry is a batch's enqueue (a pipeline flush adds time, no batch)
    int ring_next = 0;
    double acc_ms[4] = {0, 0, 0, 0};
    int64_t acc_frames = 0;

    // SHS_OPT_LEGACY_PIPELINE: batch k's raster runs inside batch k + 1's launch (k_pipe) or at the next
    // flush (anything that reads the frames, a non-pipelined batch, a stream change); `pend` is that
    // not yet launched raster.
    bool legacy_pipeline = false;
    struct PendingRaster {
        bool on = false;
        shs_dev::FrameParams fp;
        shs_dev::FrameBuffers fb;
        int grid = 0, slot = 0;
    } pend;

    // ---- library path (shs_abi_lib.cpp): one workspace per pass ----
    struct LibWork {
        DevBuf<shs_dev::LibDrawGPU> draws;
        DevBuf<shs_dev::LibRec> recs;
        DevBuf<shs_dev::LibShade> shade;
        DevBuf<uint2> boxes;
        DevBuf<uint32_t> xbase, zord, tile_count, counters, busy, clipq, bigpre;
        DevBuf<unsigned long long> pkeys;                 // split tiles' merged keys (k_lib_plan parts)
        DevBuf<uint32_t> pcount;                          // ... and finished parts
        DevBuf<uint32_t> blist;                            // region-sharded camera pass: listed setup blocks
        DevBuf<uint32_t> s2s;                              // LF_PERM: per input triangle (submission order) its slot
        DevBuf<uint4> bins;                                // per bin tile, bin_cap entries (slot, box, depth bound)
        DevBuf<uint4> bigq;
        DevBuf<uint32_t> rqueue;
        bool tm_fused = false;                             // camera pass: the fused tonemap of tm_desc
        hipEvent_t raster_ev = nullptr, resolve_ev = nullptr;   // camera pass: side-stream raster done, resolve done
        bool resolve_ev_valid = false;
        shs_tonemap_desc tm_desc{};
        DevBuf<uint2> spill, blk_stat, rstat;
        DevBuf<float4> uvw;                                // UV0 varyings of textured draws' slots
        DevBuf<uint2> items;                               // k_lib_plan's raster work items
        DevBuf<uint32_t> dynq;                             // k_lib_dyn's per-queue dynamic work items (camera pass)
        DevBuf<uint32_t> hsq;                              // k_lib_dyn's bin tiles for k_lib_hsort (camera pass)
        DevBuf<uint2> hsr;                                 // per bin tile: the range its sorted list was bucketed over
        shs_dev::LibDrawGPU *h_draws[2] = {nullptr, nullptr};   // pinned staging, 2 slots
        size_t h_cap = 0;
        hipEvent_t slot_ev[2] = {nullptr, nullptr};
        bool slot_used[2] = {false, false};
        // the pass's overflow word in mapped host memory (raise_overflow), final at ov_after (recorded
        // after its setup kernels): checked before the pass is superseded
        volatile uint32_t *h_ov = nullptr;
        hipEvent_t ov_after = nullptr;
        bool ov_valid = false;
        int slot = 0;
        uint64_t geom_key = ~0ull;
        int geom_rtiles_y = -1;
        uint32_t bin_cap = 256, extra_cap = 0, frame_index = 0, last_parity = 0;
        int last_setup_blocks = 0, last_raster_grid = 0, last_n_tris = 0;
        bool need_check = false, done = false;
        bool st_checked = false;                           // st_* hold a finished pass's statistics
        uint64_t st_clip = 0, st_raster = 0, st_covered = 0, st_maxbin = 0, st_spill = 0, st_extra = 0;
        std::vector<shs_dev::LibDrawGPU> last_draws;   // host copies (re-issue on overflow)
        std::vector<shs_dev::LibDrawGPU> dev_table;    // what w.draws holds (upload skipped when equal)
        const shs_dev::LibDrawGPU *dev_table_at = nullptr;   // ... at this allocation (pointer, capacity)
        size_t dev_table_cap = 0;
        shs_dev::LibFrameParams last_fp{};
        // camera pass: per setup block its chunk bounds (k_lib_setup, mapped host memory), final at ov_after
        uint4 *h_blkrect = nullptr;
        size_t blkrect_cap = 0;
        int blkrect_n = 0, blkrect_w = 0, blkrect_h = 0;
        bool blkrect_valid = false;
        // kernel timing (ctx->timing): events before k_lib_setup, between, after k_lib_raster
        static constexpr int RING = 64;
        hipEvent_t ring_ev[RING][3] = {};
        bool ring_pending[RING] = {};
        int ring_next = 0;
        double acc_ms[2] = {0, 0};
        int64_t acc_n = 0;
    };
    LibWork lib_cam, lib_shadow;
    int64_t lib_part = 0;                 // SHS_OPT_LIB_PART (off by default: measured)
    bool shard_cull = false;              // SHS_OPT_SHARD_CULL (off by default: measured)
    int shard_layout = 0;                 // SHS_OPT_SHARD_LAYOUT: 0 interleaved tiles, 1 cost-balanced regions
    // Region layout (shs_abi_shard.cpp): every rank's rectangle for the upcoming camera pass (computed
    // once per pass from the previous camera pass's block bounds; its light cull uses the same) and for
    // the last one (its tonemap and tile gather).
    std::vector<shs_dev::ShardRegion> reg_next, reg_last;
    int reg_next_count = 0, reg_next_w = 0, reg_next_h = 0, reg_last_count = 0;
    bool reg_next_fresh = false;
    int shard_root_permille = 1000;       // SHS_OPT_SHARD_ROOT_SHARE: rank 0's share of a region layout (it also unpacks)
    bool shadow_footprint = false;        // SHS_OPT_SHADOW_FOOTPRINT: shadow passes render only what the next camera pass reads
    bool shadow_pending = false;          // a footprint shadow pass recorded, not enqueued yet (the camera pass does it)
    shs_dev::ShardRegion shadow_reg{0, 0, 0, 0, 0};   // the bin tiles the last enqueued shadow pass rendered (on = 0: all)
    std::vector<uint32_t> shadow_span;   // ... and within that rectangle the row spans (empty: all of it; round 6)
    std::vector<uint4> reg_in;            // the block bounds reg_next was last balanced from (identical: reused)
    int reg_in_count = -1, reg_in_w = 0, reg_in_h = 0, reg_in_root = 0;
    // Tile orders / owned-list tables by geometry + ownership, uploaded once into their own buffers (a
    // changed region layout costs no stream synchronisation)
    struct OrderEntry {
        uint64_t key[4];
        int32_t *dev;
        int n, n_owned;
    };
    std::vector<OrderEntry> rt_orders, cull_orders;
    int lib_resident[2][2] = {{0, 0}, {0, 0}};   // resident k_lib_raster workgroups [camera, shadow][deep, shallow]
    DevBuf<uint64_t> lib_timeline;        // SHS_OPT_TIMELINE, camera pass raster
    DevBuf<uint64_t> lib_stimeline;       // SHS_OPT_TIMELINE, camera pass setup
    DevBuf<float4> lib_hdr;
    DevBuf<uint32_t> lib_keys;            // camera pass winners (k_lib_raster -> k_lib_resolve, LibBuffers::keys)
    DevBuf<uint32_t> lib_blkcov;          // ... and per 16x4 block whether it holds any
    // lib_blkcov is all zero between camera passes (k_lib_resolve resets the flags it read; the raster sets
    // only its busy tiles'): zeroed once per allocation and frame size
    const uint32_t *blkcov_zero_at = nullptr;
    size_t blkcov_zero_cap = 0;
    uint64_t blkcov_zero_key = 0;
    int lib_resolve_resident[6] = {};   // resident k_lib_resolve workgroups ((Forward+, PBR, mixed) x (sharded
                                        // rank's build, whole frame's build))
    DevBuf<float> srgb_lut;               // srgb_to_linear_rgb table (texture sampling)
    DevBuf<float> lib_depth;
    DevBuf<float2> lib_motion;
    DevBuf<float> shadow_map;
    int shadow_w = 0, shadow_h = 0;
    float shadow_vp[16] = {};
    shs_lib_frame lib_frame{};
    bool have_lib_frame = false, have_shadow = false, cam_after_shadow = false;
    uint32_t *h_lib_counters = nullptr;   // pinned, LC_N
    // Forward+ light lists (shs_light.hip)
    DevBuf<shs_dev::CullLight> lights;
    int32_t n_lights = 0;
    DevBuf<float2> depth_ranges;
    DevBuf<uint32_t> list_counts, list_indices;
    shs_dev::LightCullParams cull{};
    bool have_cull = false;
    // PassTonemap + present staging (shs_abi_post.cpp)
    DevBuf<uint32_t> lib_ldr, lib_present;
    shs_tonemap_desc tm_desc{};
    float tm_gamma = 0.0f;                // clamped gamma (max(0.001, gamma)) of tm_thr
    bool tm_thr_valid = false;            // tm_thr holds the thresholds of tm_gamma
    float tm_thr[256] = {};
    bool have_ldr = false;                // a tonemap follows the current camera pass
    bool tm_fuse = false;                 // shs_lib_fuse_tonemap: camera passes write tm_fuse_desc's targets
    shs_tonemap_desc tm_fuse_desc{};
    DevBuf<float> tm_thr_dev;             // the fused tonemap's thresholds (of tm_thr_dev_gamma)
    float tm_thr_dev_gamma = -1.0f;
    DevBuf<uint32_t> lib_mb, lib_mb_present;
    shs_motion_blur_desc mb_desc{};
    bool have_mb = false;                 // a motion blur follows that tonemap
    // CPU light binning on the GPU (shs_abi_lightbin.cpp)
    DevBuf<shs_dev::BinLight> lb_lights;
    DevBuf<float2> lb_ndc;
    DevBuf<uint32_t> lb_counts, lb_indices;
    // software occlusion pass (shs_abi_occ.cpp)
    DevBuf<uint32_t> occ_depth, occ_visible;
    DevBuf<uint8_t> occ_flags;
    DevBuf<shs_dev::OccObject> occ_objs;
    DevBuf<shs_dev::OccRect> occ_rects;
    DevBuf<shs_dev::OccTri> occ_tris;

    // debug_draw (shs_abi_debugdraw.cpp)
    DevBuf<shs_dev::DDObject> dd_objs;
    DevBuf<shs_dev::DDTri> dd_tris;
    DevBuf<float> dd_depth0, dd_depth, dd_lit_b;
    DevBuf<uint32_t> dd_rgba, dd_big;
    DevBuf<unsigned long long> dd_keys;

    // Canvas-API multi-pass extras (shs_abi_canvas_post.cpp)
    DevBuf<uint32_t> cp_a, cp_b, cp_src;
    DevBuf<float> cp_depth, cp_vel, cp_focus;
};

// Re-enqueues the tonemap after lib_finish re-issued the camera pass (shs_abi_post.cpp).
int shs_tonemap_reissue(shs_ctx *ctx);
// Make the pending frame final in stream order without waiting for its raster: wait for its setup
// (the overflow word is final then) and re-issue it only if a capacity overflowed.  Work queued on
// the context stream afterwards sees the final frame (shs_abi.cpp: legacy; shs_abi_lib.cpp: library).
int shs_legacy_ensure_final(shs_ctx *ctx);
int shs_lib_ensure_final(shs_ctx *ctx);
// A shadow pass recorded under SHS_OPT_SHADOW_FOOTPRINT and not yet enqueued: enqueue it for the whole map.
int shs_lib_flush_shadow(shs_ctx *ctx);
int shs_lib_widen_shadow(shs_ctx *ctx, const float *pos);
// Region layout (shs_abi_shard.cpp).  shs_shard_balance: `count` rectangles of the tiles_x x tiles_y bin
// grid of a W x H frame with equal predicted cost, from n_blk setup-block bounds (null: pixels only).
void shs_shard_balance(const uint4 *blk, int n_blk, int tiles_x, int tiles_y, int W, int H, int count,
                       std::vector<shs_dev::ShardRegion> &out, double root_share = 1.0);
// The regions of the next camera pass of a W x H frame over `count` ranks (ctx->reg_next), from the
// last camera pass's block bounds when it had the same frame size (waits for its setup).
int shs_regions_next(shs_ctx *ctx, int count, int w, int h);

#define HIP_TRY(ctx, expr)                                                                       \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                      \
            return SHS_ERR_HIP;                                                                  \
        }                                                                                        \
    } while (0)

template <typename T>
inline int ensure(shs_ctx *ctx, DevBuf<T> &b, size_t n) {
    if (n <= b.cap && b.p) return SHS_OK;
    size_t want = std::max<size_t>(n, 16);
    if (b.p) {
        // the old buffer may still be read by queued work on the streams
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->setup_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->setup_stream));
        HIP_TRY(ctx, hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
    }
    HIP_TRY(ctx, hipMalloc(reinterpret_cast<void **>(&b.p), want * sizeof(T)));
    b.cap = want;
    return SHS_OK;
}

template <typename T>
inline void release(DevBuf<T> &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

// One overflow word in mapped, coherent (fine-grained) host memory, zeroed: kernels store into it
// through its device alias (the same address under unified addressing), the host reads it directly.
inline hipError_t shs_host_ov_alloc(volatile uint32_t **out) {
    void *p = nullptr;
    const hipError_t e = hipHostMalloc(&p, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    *static_cast<volatile uint32_t *>(p) = 0u;
    *out = static_cast<volatile uint32_t *>(p);
    return hipSuccess;
}

inline int set_dev(shs_ctx *ctx) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return SHS_OK;
}

// Frees the library-path workspaces (shs_abi_lib.cpp); called by shs_destroy.
void shs_lib_release(shs_ctx *ctx);
