// shs_lib_device.hpp -- HBM layouts of the shs-renderer-lib software raster path on gfx950
// (rasterize_mesh + builtin programs, PassShadowMap), shared by shs_lib.hip and shs_abi.cpp.
// Paths are relative to /root/reference/cpp-folders/src/shs-renderer-lib/include/shs/.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "shs_shard.hpp"

namespace shs_dev {

// SHS_LIB_EXP bits (timing experiments, wrong images) are read only in the experiments build: the
// product kernels carry none of their branches.
#define SHS_LIB_EXP(fp, bit) (::shs_dev::DBG_BUILD && ((fp).exp_flags & (bit)))

// Per-draw block of one rasterize_mesh call (ShaderUniforms, shader/types.hpp:87-116, reduced to
// what the builtin programs read; uniform-only products are computed once on the host with the
// same float operations the reference runs per vertex / per fragment).
struct alignas(16) LibDrawGPU {
    const float *pos;        // MeshData positions, 3 floats per vertex
    const float *nrm;        // normals (missing entries filled with (0,1,0) at upload)
    const float *uv;         // uvs (missing entries (0,0))
    const uint32_t *idx;     // indices, nullptr for a non-indexed soup
    int32_t n_verts, tri_base, n_tris, program;
    int32_t cull_mode, front_ccw, shadow, motion;   // motion: u.enable_motion_vectors
    float model[16];         // u.model
    float viewproj[16];      // u.viewproj
    float nmat[12];          // transpose(inverse(mat3(model))) if |det| > 1e-8 else mat3(model) (9 used)
    float c2p[16];           // curr_to_prev_model (rasterizer.hpp:296-308)
    float prev_vp[16];       // u.prev_viewproj
    float light_vp[16];      // u.light_viewproj
    float L[4];              // normalize(-u.light_dir_ws)
    float cam[4];            // u.camera_pos
    float lcol[4];           // u.light_color, u.light_intensity
    float base[4];           // u.base_color, u.metallic
    float mat[4];            // u.roughness, u.ao, u.shadow_strength, 0
    float shp[4];            // bias_const, bias_slope, pcf radius (int bits), pcf_step
    const uint32_t *tex;     // u.base_color_tex: Texture2DData texels (Color RGBA8, y * w + x), or null
    int32_t tex_w, tex_h;
    const float4 *cbox;      // model-space bounds of the mesh's 256-triangle chunks (min, max per chunk)
    const uint32_t *orig;    // spatially ordered mesh: per stored triangle its submission (MeshData) index, or null
};

// Raster record of one primitive (a fan triangle of a clipped input triangle, or a shadow-pass
// triangle), 64 B: the per-triangle part of barycentric_2d (rasterizer.hpp:167-179), the 1/w
// terms and the corner depths.
struct alignas(16) LibRec {
    float ax, ay, v0x, v0y;      // s0, v0 = s1 - s0
    float v1x, v1y, inv_den, z0; // v1 = s2 - s0, 1/den; z_k = clip.z * (1/w) (shadow pass: NDC z)
    float z1, z2, iw0, iw1;      // 1/clip.w per corner
    float iw2;
    uint32_t seq;                // submission order: input triangle * 16 + fan index
    uint32_t bx, by;             // pixel bbox [min, max], packed int16 (lo | hi << 16)
};
static_assert(sizeof(LibRec) == 64, "LibRec must stay 64 B");

// Perspective-premultiplied varyings of the primitive's corners (varw, rasterizer.hpp:309-328) that
// the builtin programs read.  The UV0 varying lives in its own per-slot plane (LibBuffers::uvw), written
// and read only for draws with a base_color_tex: untextured passes move no UV bytes.
struct alignas(16) LibShade {
    float wp[9];                 // WorldPos varying * 1/w
    float n[9];                  // NormalWS varying * 1/w
    int32_t draw;
    int32_t pad;
};
static_assert(sizeof(LibShade) == 80, "LibShade must stay 80 B");

// CullingLightGPU (lighting/light_types.hpp:141-166), 160 B, as the caller uploads it.
struct alignas(16) CullLight {
    float position_range[4], color_intensity[4], direction_spot[4], axis_spot_outer[4], up_shape_x[4];
    float shape_attenuation[4];
    uint32_t type_shape_flags[4];
    float cull_sphere[4], cull_aabb_min[4], cull_aabb_max[4];
};
static_assert(sizeof(CullLight) == 160, "CullingLightGPU is 160 B");

// The light-list binning's view of the frame (CameraUBO fields of fp_stress_light_cull.comp).
struct LightCullParams {
    int32_t W, H;
    uint32_t tile_size, max_per_tile, mode, z_slices;   // mode 0 none, 1 tiled, 2 tiled depth range, 3 clustered
    uint32_t tiles_x, tiles_y, n_lists, n_lights;
    float zn, zf;
    int32_t depth_linear;                               // depth input: library linear view depth
    int32_t rank, count;                                // lists of owned 32x32 bin tiles only (tile sharding)
    int32_t pad;
    float view[16], proj[16];
    ShardRegion reg;                                    // count > 1: region ownership (shs_shard.hpp)
};

constexpr uint32_t LF_DEPTH = 1u;       // target.depth_motion present: strict-less z test, depth written
constexpr uint32_t LF_LINZ = 2u;        // ... with zf > zn + 1e-6: linear view depth
constexpr uint32_t LF_MOTION = 4u;      // motion buffer written (per draw: enable_motion_vectors)
constexpr uint32_t LF_GRADIENT = 8u;    // PassPBRForward's no-sky background gradient, else clear[]
constexpr uint32_t LF_PERM = 16u;       // a draw's mesh is stored in spatial order: winners map to slots via s2s

// counters[] (two parity sets, frame f uses set f & 1, k_lib_setup zeroes the other)
// LC_CLIPQ: input triangles queued for k_lib_clip; LC_BIGT / LC_BIGQ: the large-primitive queue's
// (primitive, tile) task total and length, one 64-bit word (tasks low, entries high) so that one
// atomicAdd hands an appender both bases and the queue's task prefix stays monotone; LC_N even keeps
// the second parity set's word 8-B aligned.
// LC_ITEMS: k_lib_plan's raster work items; LC_COVERED: camera-pass covered pixels (k_lib_resolve);
// LC_SPLITS: k_lib_plan's split tiles (their pkeys slots); LC_BLOCKS: k_lib_blocks' listed setup blocks;
// LC_HSORT: k_lib_dyn's bin tiles for k_lib_hsort.
constexpr int LC_OVERFLOW = 0, LC_SPILL = 1, LC_EXTRA = 2, LC_CLIPQ = 3, LC_BIGT = 4, LC_BIGQ = 5, LC_ITEMS = 6, LC_COVERED = 7,
              LC_SPLITS = 8, LC_BLOCKS = 9, LC_HSORT = 10, LC_N = 12;
static_assert(LC_BIGQ == LC_BIGT + 1 && LC_BIGT % 2 == 0 && LC_N % 2 == 0, "64-bit big-queue word");
constexpr uint32_t LOV_SPILL = 1u, LOV_EXTRA = 2u;

// Row spans of a footprint shadow pass (LibFrameParams::span): maps up to 64 bin tiles (2,048 texels) high.
constexpr int LIB_SPAN_ROWS = 64;

struct LibFrameParams {
    int32_t W, H;
    int32_t rank, count;             // shard ownership of 32x32 bin tiles (tile % count == rank, or reg)
    int32_t tiles_x, tiles_y, rtiles_y;
    int32_t n_tris, n_draws;
    uint32_t flags;                  // LF_*
    float zn, zf, zspan;             // RT_ColorDepthMotion zn / zf, zspan = zf - zn
    float clear[4];
    uint32_t bin_cap, spill_cap, extra_cap;
    uint32_t parity, scan_mode;
    int32_t setup_blocks, n_owned_rt;
    uint32_t exp_flags;              // timing experiments only (SHS_LIB_EXP; wrong images): 1 no shade, 2 no marks, 4 no recs,
                                     // 8 tile-sharded setup: cull front end only
    int32_t sm_w, sm_h;              // shadow map sampled by the programs
    // Forward+ program: the light lists of the last shs_light_cull
    uint32_t lt_size, lt_tx, lt_ty, lt_maxp, lt_mode, lt_zs, n_lights;
    float lt_view_z[4];              // view matrix row 2 (view-space z, cluster slice)
    float lt_zn, lt_zf;              // the light cull's depth_params
    float tm_exposure, tm_inv_gamma; // fused PassTonemap (LibBuffers::tm_thr)
    uint32_t part;                   // camera pass: k_lib_plan splits a tile's list into parts of about this
                                     // many entries (0: one work item per owned raster tile, no plan)
    uint32_t split_cap;              // ... at most this many split tiles per pass (LibBuffers::pkeys slots)
    int32_t raster_grid;             // k_lib_raster's workgroups (k_lib_dyn derives the same static share)
    int32_t static_div;              // k_lib_raster: n_work / (static_div * workgroups) static items per workgroup
    uint32_t heavy_min;              // camera pass: a busy tile whose bin list holds >= this many entries is
                                     // rendered from k_lib_dyn's heavy lists, first (0: no heavy lists)
    uint32_t dyn_cap;                // camera pass: entries per queue of LibBuffers::dynq
    uint32_t hsort;                  // camera pass: bin lists of more than hsort_min entries (and at most
    uint32_t hsort_min;              //   min(bin_cap, LIB_HSORT_MAX)) are depth-sorted whole by k_lib_hsort
    ShardRegion reg;                 // count > 1 with reg.on: this rank's rectangle of bin tiles
    int32_t span_rows;               // shadow pass of a footprint (round 6): > 0 -- per bin-tile row y < span_rows
    uint32_t span[LIB_SPAN_ROWS];    //   the bin columns x0 | x1 << 16 it renders (x1 < x0: none); 0 -- all of reg
};

struct LibBuffers {
    const LibDrawGPU *draws;
    LibRec *recs;                    // n_tris primaries (fan 0) then extra_cap extras (fans 1..6)
    LibShade *shade;
    uint2 *boxes;                    // per slot: packed pixel bbox, empty (0,-1) when not rasterised
    uint32_t *zord;                  // per slot: orderable bits of a lower bound of its depth (front-to-back sort key)
    uint32_t *xbase;                 // per input triangle: slot of its fan triangle 1
    uint32_t *tile_count;
    uint4 *bins;                     // per bin tile: bin_cap entries (slot, box x, box y, depth bound zord)
    uint2 *spill;
    uint32_t *counters;
    uint32_t *busy;                  // per 32x8 raster tile
    uint2 *blk_stat;                 // per setup block: (tri_after_clip, tri_raster)
    uint2 *rstat;                    // per raster block: (covered pixels, fullest bin)
    float4 *hdr;                     // W*H, rows y-up (RT_ColorHDR)
    float *depth;                    // W*H (RT_ColorDepthMotion depth / RT_ShadowDepth)
    float2 *motion;                  // W*H
    const float *shadow_map;         // sampled by the camera pass (sm_w * sm_h)
    const CullLight *lights;         // Forward+ program
    const uint32_t *tile_counts, *tile_indices;
    uint64_t *timeline;              // SHS_OPT_TIMELINE (camera pass): LTL_STRIDE per raster workgroup
    uint64_t *stimeline;             // SHS_OPT_TIMELINE (camera pass): STL_STRIDE per setup workgroup
    uint32_t *clipq;                 // input triangles that need clipping (camera pass), n_tris capacity
    uint4 *bigq;                     // primitives over SMALL_MARK raster tiles: (slot, bx, by, 0), one per slot
    uint32_t *bigpre;                // exclusive task prefix of bigq (written with the entries)
    const int32_t *dbase;            // draws[i].tri_base, compact (+ n_tris): the triangle -> draw search
    const int32_t *bdraw;            // per setup block: the draw of its first triangle
    uint32_t *rqueue;                // k_lib_raster ticket queues: 2 parities x LIB_NQW x LIB_QSTRIDE words
    uint32_t *dynq;                  // camera pass: k_lib_dyn's work item words, per queue q a heavy (2q) and a
                                     // light (2q + 1) list of dyn_cap entries
    const int32_t *rt_order;         // the owned raster tiles in processing order (n_owned_rt; XCD-coherent)
    uint32_t *keys;                  // camera pass: W*H winners, k_lib_raster -> k_lib_resolve: the winning key's
                                     // submission sequence + 1 (0: no winner; the resolve recomputes z)
    uint32_t *blkcov;                // camera pass: per 16x4 block (4 per raster tile, rt * 4 + sub): keys written
    // fused PassTonemap (shs_lib_fuse_tonemap): k_lib_resolve also writes the tonemapped bytes
    const float *tm_thr;             // the 256 byte thresholds (shs_post_internal.hpp), null: not fused
    uint32_t *tm_ldr, *tm_present;   // RT_ColorLDR (rows y up) / present staging (rows top-down), or null
    uint32_t *ov_host;               // the pass's overflow word in mapped host memory (raise_overflow)
    float4 *uvw;                     // per slot, 2 float4: UV0 varying * 1/w of the 3 corners (textured draws)
    const float *srgb_lut;           // srgb_to_linear_rgb's 256 values, std::pow(c / 255.0f, 2.2f) on the host
    uint2 *items;                    // k_lib_plan: raster work items (raster tile, part | parts << 8 | split id << 16)
    unsigned long long *pkeys;       // per split tile (split id): its 32x8 keys, merged by the parts (atomicMin),
                                     // KEY_EMPTY between passes (the last part resets them)
    uint32_t *pcount;                // per split tile: parts finished (the last part resets it)
    uint32_t *blist;                 // region-sharded camera pass: the setup blocks that can reach the rank (k_lib_blocks)
    uint32_t *s2s;                   // camera pass with LF_PERM: per input triangle in submission order, its slot
    uint4 *blkrect;                  // camera pass: per setup block (bx0 | bx1 << 16, by0 | by1 << 16, triangles,
                                     // bounded) of its chunk bounds, mapped host memory (the region balancer's input)
    uint32_t *hsq;                   // camera pass with fp.hsort: the bin tiles k_lib_hsort sorts (k_lib_dyn)
    uint2 *hsr;                      // ... per bin tile: the depth-bound range (lo, hi) its list was bucketed over
};

// k_lib_hsort: one 512-thread workgroup per listed bin tile, LIB_HSORT_PER entries per thread in registers (a
// 1024-thread workgroup waited for a whole free CU beside the other frames in flight: 8.5 -> 30 us at 8 ranks).
// Lists of more than LIB_HSORT_MIN entries (one deep candidate round, LIB_CAND_DEEP) are sorted.
constexpr int LIB_HSORT_T = 512, LIB_HSORT_PER = 16, LIB_HSORT_MAX = LIB_HSORT_T * LIB_HSORT_PER;
constexpr uint32_t LIB_HSORT_MIN = 1024;

// k_lib_plan: at most this many parts per raster tile (capacity: LIB_MAXK * owned raster tiles).
constexpr int LIB_MAXK = 16;
constexpr int LIB_RTH_PX = 32 * 8;   // pixels of a 32x8 raster tile (a split tile's pkeys slot)

// k_lib_raster's work distribution: owned raster tile b to workgroup b, the rest from LIB_NQ ticket
// counters a cache line apart (k_lib_setup zeroes the next frame's set).
constexpr int LIB_NQ = 8, LIB_QSTRIDE = 32;
// per parity: LIB_NQ ticket counters, then (camera pass) LIB_NQ light and LIB_NQ heavy k_lib_dyn list lengths
constexpr int LIB_NQW = 3 * LIB_NQ;

// Library setup timeline slots: start, after the per-triangle work, after the deferred marks,
// after the large-primitive marks (= end), large primitives, deferred-union width x height, after the
// tile-sharded cull front end (0 without it), kept triangles.
constexpr int STL_STRIDE = 8;

// Library raster timeline slots (s_memrealtime, 100 MHz ticks): per workgroup start, end, summed
// phase ticks over its busy tiles (gather, stage + pairs, resolve + shade), clear ticks, counts.
// Slots 16..23: the workgroup's longest busy tile -- its raster tile, list entries, candidate rounds,
// staging passes, staged candidates, pairs, gather ticks, passes that ended their round early.
constexpr int LTL_STRIDE = 24;
enum : int { LTL_START = 0, LTL_END, LTL_GATHER, LTL_PAIRS, LTL_SHADE, LTL_CLEAR, LTL_NBUSY, LTL_NCLEAR, LTL_CHUNKS,
             LTL_NPAIRS, LTL_NCAND, LTL_MAXTILE, LTL_STAGE, LTL_SEG, LTL_TILES, LTL_LAST,
             LTL_MT_RT, LTL_MT_ITEMS, LTL_MT_ROUNDS, LTL_MT_PASSES, LTL_MT_STAGED, LTL_MT_PAIRS, LTL_MT_GATHER,
             LTL_MT_BREAKS };

}  // namespace shs_dev
