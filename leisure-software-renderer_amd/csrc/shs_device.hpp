// shs_device.hpp -- device data layout and the bit-exact per-pixel arithmetic of the legacy
// shs_renderer path, shared by the setup / raster kernels (shs_legacy.hip).
//
// Every floating-point expression here restates a reference line operation for operation; the
// kernels are compiled with -ffp-contract=off and correctly rounded f32 divide/sqrt, so each
// operation rounds exactly as the reference's x86-64 SSE build (-O3, no FMA) does.
// Paths are relative to /root/reference/cpp-folders/src/.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace shs_dev {

// ---- HBM layouts -------------------------------------------------------------------------
// Per-draw uniform block (one entry per object of the scene loop, blinn_phong_shading.cpp:272-282).
struct alignas(16) DrawGPU {
    const float *pos;        // mesh soup positions, 9 floats per triangle
    const float *nrm;        // mesh soup normals
    int32_t tri_base;        // global index of this draw's first triangle (submission order)
    int32_t n_tris;
    int32_t shading;         // SHS_SHADING_*
    int32_t pad0;
    float mvp[16];           // Uniforms::mvp
    float model[16];         // Uniforms::model (Flat: Uniforms::mv)
    float nmat[12];          // mat3(transpose(inverse(model))) (Flat: mat3(mv)), col-major, 9 used
    float light[4];          // normalize(-light_dir) (Flat: normalize(light_dir_view))
    float cam[4];            // Uniforms::camera_pos
    float ocol[4];           // vec3(color.rgb) / 255.0f
    float colf[4];           // (float)color.rgb (Flat FS multiplies the int colour)
};

static_assert(offsetof(DrawGPU, light) % 16 == 0 && offsetof(DrawGPU, cam) == offsetof(DrawGPU, light) + 16 &&
                  offsetof(DrawGPU, ocol) == offsetof(DrawGPU, light) + 32 &&
                  offsetof(DrawGPU, colf) == offsetof(DrawGPU, light) + 48,
              "shading uniforms are read as 4 consecutive float4s");

// Per-triangle raster record written by k_setup, 96 B (6 x float4), read by k_raster through LDS.
// Holds exactly the per-triangle quantities of Canvas::barycentric_coordinate
// (shs_renderer.hpp:802-821) that do not depend on the pixel, plus the NDC z of the corners.
struct alignas(16) TriRec {
    float ax, ay, v0x, v0y;          // A, v0 = B - A
    float v1x, v1y, d00, d01;        // v1 = C - A, d00 = v0.v0, d01 = v0.v1
    float d11, denom, z0, z1;        // d11 = v1.v1, denom = d00*d11 - d01*d01, screen z
    float z2;
    uint32_t flags;                  // TRI_CULLED | TRI_GHOST | TRI_UNBOUNDED
    int32_t draw;                    // index into the draw table
    int32_t local;                   // triangle index inside the draw's mesh
    uint32_t ibx, iby;               // integer bbox [floor(min), floor(max)] clamped to the screen,
                                     // packed int16 (lo | hi << 16)
    uint32_t gbx, gby;               // cull/bin box: the ibox, or for a ghost the danger box
    float fminx, fmaxx, fminy, fmaxy;// float bbox of the screen-space corners
};
static_assert(sizeof(TriRec) == 96, "TriRec must stay 96 B");

// The record as k_setup stores it in HBM (round 6): TriRec's pixel-independent terms, the draw | flags
// word (draw | flags << 29) and the bin box, 64 B = four float4s, sector-aligned -- everything a staged
// candidate's pair tests, row spans and resolve read.  The float bbox (and the integer bbox derived from
// it) is needed only by ghosts (TRI_GHOST: the tile-clamp test) and k_ghost: it goes to a 16-B side
// array (FrameBuffers::rext, fminx fmaxx fminy fmaxy), stored for ghosts only.  local is not stored.
// (Was the whole 96-B TriRec per triangle: C3's raster staged 96 B per candidate and tile.)
struct alignas(16) TriHot {
    float ax, ay, v0x, v0y;
    float v1x, v1y, d00, d01;
    float d11, denom, z0, z1;
    float z2;
    uint32_t word;                   // draw | flags << 29
    uint32_t gbx, gby;               // bin box
};
static_assert(sizeof(TriHot) == 64, "TriHot must stay 64 B");

// Per-triangle shading varyings written by k_setup (the legacy VS outputs of the three corners the
// winning pixels interpolate), 80 B: Blinn-Phong/Phong: world_pos[3] then normalize(N*n)[3];
// Gouraud: the clamped per-vertex colour[3] (carried in world_pos, gouraud_shading.cpp:71);
// Flat: mat3(mv)*n[3] (flat_shading.cpp:54).
struct alignas(16) ShadeRec {
    float v[18];
    int32_t shading;
    int32_t draw;
};
static_assert(sizeof(ShadeRec) == 80, "ShadeRec must stay 80 B");

constexpr uint32_t TRI_CULLED = 1u;
constexpr uint32_t TRI_GHOST = 2u;       // tile-clamp pixels near the bbox may pass: test them
constexpr uint32_t TRI_UNBOUNDED = 4u;   // ... anywhere on screen, or too far out to bin: every visited
                                         // pixel outside the ibox is tested by k_setup's ghost waves

__device__ __forceinline__ uint32_t pack16(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }
__device__ __forceinline__ int lo16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ int hi16(uint32_t v) { return (int)(int16_t)(v >> 16); }

constexpr int TILE = 32;             // bin tile and shard unit (32x32 px)
constexpr int RTW = 32, RTH = 8;     // raster tile: one 256-thread workgroup, a wave per 8x8 block,
                                     // one pixel per lane; four raster tiles per bin tile
constexpr int CHUNK = 256;           // triangle records staged in LDS per pass
constexpr int CAND = 1024;           // candidate ids gathered per round (4 per thread)
constexpr int SCAN_MAX_TRIS = 4096;  // scenes up to this size skip binning (scan mode)
constexpr double GHOST_MAX_EXPAND = 48.0;  // larger danger boxes are handled as TRI_UNBOUNDED

// counters[] slots (three sets used round-robin by consecutive batches; batch k's k_setup zeroes the set
// of batch k + 1, last used by batch k - 2, whose raster its setup stream has waited for -- no memset
// node between two batches).
// Only the append positions and the overflow flags live here; statistics go to per-block slots.
// C_BUSY: entries of the busy-tile list (k_setup / k_ghost).  The host reads the first C_NCOUNTERS
// words of a set.  k_raster's work tickets live in N_WORKQ queues, one 128-B line each from C_WORK
// (one queue per XCD-sized group of workgroups: a same-address returning atomic serialises).
constexpr int C_OVERFLOW = 0, C_SPILL = 1, C_FRAG = 2, C_SLIVER = 3, C_BUSY = 4, C_NCOUNTERS = 5;
constexpr int N_WORKQ = 8, WORKQ_STRIDE = 32, C_WORK = 32;
constexpr int CSET = C_WORK + N_WORKQ * WORKQ_STRIDE;   // words per counter set (N_CSETS sets)
constexpr int N_CSETS = 3;
constexpr uint32_t OV_SPILL = 1u, OV_FRAG = 2u;

// Timing-experiment switches (frame flags bits 8+; results are WRONG with any of them set): they
// let bench --debug-flags attribute kernel time to phases.  Never set by the product path.
constexpr uint32_t DBG_SKIP_GHOST = 1u << 8, DBG_SKIP_SHADE = 1u << 9, DBG_CLEAR_ONLY = 1u << 10,
                   DBG_SKIP_BIN = 1u << 11, DBG_SKIP_CLEAR = 1u << 12,
                   DBG_TWICE = 1u << 13, DBG_SKIP_PAIRS = 1u << 14, DBG_SKIP_TILE_STORES = 1u << 15;
constexpr uint32_t DBG_MASK = 0xffu << 8;   // dropped from the caller's flags outside the experiments build
// The DBG_* checks are compiled only into the experiments build (-DSHS_TIMING_EXPERIMENTS): the
// product kernels carry none of their code (DBG_TWICE alone inlined the whole raster tile twice).
#ifdef SHS_TIMING_EXPERIMENTS
constexpr bool DBG_BUILD = true;
#else
constexpr bool DBG_BUILD = false;
#endif
#define SHS_DBG(fp, bit) (::shs_dev::DBG_BUILD && ((fp).flags & (bit)))
// Raster inner loop (frame flags bit 16, set by the context from SHS_OPT_RASTER_LOOP): per-pixel
// candidate loop instead of (candidate, pixel) pair tasks.  Results are identical either way.
constexpr uint32_t RF_PER_PIXEL = 1u << 16;
// Binned frames without per-triangle records in HBM (frame flags bit 17; SHS_LEGACY_NORECS=1, a
// measured alternative, off by default): k_setup writes only the bin box and a draw|flags word of each
// triangle (12 B instead of the 184-B TriRec + ShadeRec), and k_raster recomputes a staged candidate's
// record -- and a winner's shading varyings -- from the resident mesh with the identical arithmetic (a
// quad of lanes per candidate, as k_setup).  Unbounded slivers (TRI_UNBOUNDED) still store their
// record for k_ghost.
constexpr uint32_t RF_NO_RECS = 1u << 17;
// Varyings shared by the batch's frames (frame flags bit 18, set by the host): every frame's draws have
// frame 0's meshes, Phong / Blinn-Phong shading and model matrices (a static scene seen from a batch of
// camera poses), so each triangle's ShadeRec -- world positions and normals of its corners, which
// depend on the model matrix alone -- is the same in every frame.  Frame 0's k_setup blocks store it
// once, the other frames' skip the normals and the varyings, and every frame's winners read frame 0's
// copy (frame_view).  The draw uniforms a winner shades with come from its TriRec's per-frame draw.
constexpr uint32_t RF_SHARED_VARY = 1u << 18;
// Scan-mode batches without ghost waves (frame flags bit 19, set by the host): a setup wave that finds
// unbounded slivers among its own triangles enumerates their tile-clamp pixels itself, from the
// records it keeps in LDS, instead of ghost blocks recomputing every triangle's record.
constexpr uint32_t RF_GHOST_INLINE = 1u << 19;
// Bin-mode batches whose bin tiles' raster rows run on one XCD (frame flags bit 20, set by the host):
// a bin tile's first appender lists its four raster rows as one 4-aligned group of the busy list
// (BUSY_SKIP pads the rows below the screen), and k_raster deals busy items so that the four rows of a
// group land on the same ticket queue -- the same XCD, whose L2 then serves the group's bin list, boxes
// and records to the three rows after the first.
constexpr uint32_t RF_XCD_ROWS = 1u << 20;
constexpr uint32_t BUSY_SKIP = 0xffffffffu;   // a padding entry of the busy list: no tile

// Uniforms of up to KARG_DRAWS draws travel in the kernel arguments (no per-frame copy);
// larger scenes read the device draw table.
constexpr int KARG_DRAWS = 6;

// A pixel the reference's tile clamp makes an unbounded sliver visit outside its bbox and whose
// barycentrics pass (rare): resolved by k_raster like any other candidate.
struct alignas(16) GhostFrag {
    uint32_t xy;     // x | y << 16
    float z;
    uint32_t id;     // submission index
    float v, w;      // barycentrics for shading (u = (1 - v) - w)
    uint32_t frame;  // frame of the batch
    uint32_t pad[2];
};

struct FrameParams {
    int32_t W, H;
    int32_t rtw, rth;                // reference tile-job size (80x80)
    int32_t rank, count;             // shard ownership of 32x32 bin tiles (tile % count == rank)
    int32_t tiles_x, tiles_y;        // bin tiles (raster tiles across == tiles_x)
    int32_t rtiles_y;                // raster tile rows
    int32_t rt_x, rt_y;              // reference tiles across / down
    int32_t n_tris, n_draws;
    uint32_t clear_rgba;
    uint32_t flags;
    uint32_t bin_cap;                // per-bin-tile capacity
    uint32_t spill_cap;
    uint32_t frag_cap;               // ghost fragment capacity
    uint32_t ghost_slices;           // ghost waves per GHOST_GROUP triangles (k_setup)
    uint32_t parity;                 // counter set used by this batch
    uint32_t zero_set;               // counter set k_setup zeroes (the next batch's)
    uint32_t scan_mode;              // 1: no bins, busy raster tiles scan all bin boxes (small scenes)
    uint32_t ghost_list;             // 1: k_setup lists the unbounded slivers, k_ghost enumerates them
                                     // (binned scenes); 0: k_setup's ghost waves (scan-mode scenes)
    int32_t setup_blocks, ghost_blocks, clear_blocks;   // k_setup block roles, in this order (no
                                                        // clear blocks: k_raster clears)
    int32_t n_owned_rt;              // raster tiles of the owned bin tiles (4 per bin tile), per frame
    int32_t setup_grid;              // k_setup grid (k_raster's timeline slots follow)
    // Frame batches: n_frames frames of this size, each with its own n_draws draws (draw table entry
    // f * n_draws + i) and its own framebuffers / workspace (FrameBuffers strides below).  k_setup runs
    // frame_blocks (= setup_blocks + ghost_blocks) blocks per frame; k_raster's persistent grid walks
    // the n_frames * n_owned_rt raster tiles of the whole batch.
    int32_t n_frames;
    int32_t frame_blocks;
    uint32_t epoch;                  // busy[] value that means "busy in this launch" (never 0)
};

// Device buffers.  "per frame" buffers hold n_frames consecutive copies (frame_view() offsets them);
// the others are shared by the batch.
struct FrameBuffers {
    const DrawGPU *draws;            // device draw table (n_frames * n_draws > KARG_DRAWS)
    const int32_t *bdraw;            // per setup block: the frame-local draw of its first triangle when
                                     // every frame has the same draw layout (device table only), or null
    TriHot *recs;                    // per frame: n_tris
    float4 *rext;                    // per frame: n_tris float bboxes (fminx, fmaxx, fminy, fmaxy), ghosts only
    ShadeRec *shade;                 // per frame: n_tris
    uint32_t *tile_count;            // per frame: n_bin_tiles counts (zeroed before each launch)
    uint32_t *bins;                  // per frame: n_bin_tiles * bin_cap
    uint2 *spill;                    // (f * n_bin_tiles + bin tile, tri) pairs beyond bin_cap
    GhostFrag *frags;                // tile-clamp pixels of unbounded slivers that pass (frag_cap)
    uint32_t *slivers;               // n_frames * n_tris: unbounded slivers, f * n_tris + tri (ghost_list)
    uint2 *boxes;                    // per frame: n_tris packed bin boxes (gbx, gby); empty for culled
    int32_t *tdraw;                  // per frame: n_tris, the triangle's draw in the frame's slice (RF_NO_RECS)
    uint32_t *counters;              // 2 * CSET
    uint32_t *busy;                  // per frame, per raster tile: == fp.epoch when the tile has
                                     // candidates / fragments in this launch (no reset needed)
    uint32_t *busy_list;             // C_BUSY entries f * n_raster_tiles + raster tile, each busy tile of
                                     // the batch once (capacity n_frames * n_raster_tiles)
    uint4 *blk_stat;                 // per setup block: (set up, ghost, unbounded, bin entries)
    uint2 *rstat;                    // per raster block: (covered pixels, fullest bin seen)
    uint64_t *timeline;              // optional: TL_STRIDE slots per workgroup, k_setup then k_raster:
                                     // start, end, then phase marks of thread 0 (first busy tile)
    uint8_t *color;                  // per frame: W*H*4, canvas rows
    float *depth;                    // per frame: W*H, screen rows
    float4 *prequant;                // per frame: W*H (optional)
    uint32_t *present;               // per frame: W*H RGBA8 SDL staging, rows top-down (optional,
                                     // SHS_FRAME_PRESENT: Canvas::copy_to_SDLSurface's layout)
    uint32_t *ov_host;               // the slot's overflow word in mapped host memory: set to 1 with
                                     // every overflow bit (read by the host before superseding)
};

// A capacity overflow: the counter-set bit (finish_frame / check_pass read it) and the mapped host
// word the host reads when the batch is superseded (a system-scope vector store, rare).
__device__ __forceinline__ void raise_overflow(uint32_t *word, uint32_t bit, uint32_t *ov_host) {
    atomicOr(word, bit);
    if (ov_host) __hip_atomic_store(ov_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The buffers of frame f of the batch (shared buffers unchanged).
__device__ __forceinline__ FrameBuffers frame_view(const FrameParams &fp, const FrameBuffers &fb, int f) {
    FrameBuffers v = fb;
    const size_t nt = (size_t)fp.n_tris, n_bt = (size_t)fp.tiles_x * fp.tiles_y;
    const size_t npx = (size_t)fp.W * fp.H, n_rt = (size_t)fp.tiles_x * fp.rtiles_y;
    v.recs += f * nt;
    v.rext += f * nt;
    if (!(fp.flags & RF_SHARED_VARY)) v.shade += f * nt;
    v.boxes += f * nt;
    if (v.tdraw) v.tdraw += f * nt;
    v.tile_count += f * n_bt;
    v.bins += f * n_bt * fp.bin_cap;
    v.busy += f * n_rt;
    v.color += f * npx * 4;
    v.depth += f * npx;
    if (v.prequant) v.prequant += f * npx;
    if (v.present) v.present += f * npx;
    return v;
}

constexpr int TL_STRIDE = 12;

struct KArgDraws {
    DrawGPU d[KARG_DRAWS];
};

// ---- GLM scalar semantics (glm/detail/func_common.inl) -------------------------------------
__device__ __forceinline__ float g_min(float x, float y) { return (y < x) ? y : x; }
__device__ __forceinline__ float g_max(float x, float y) { return (x < y) ? y : x; }
__device__ __forceinline__ float g_clamp01(float x) { return g_min(g_max(x, 0.0f), 1.0f); }

struct f3 { float x, y, z; };
__device__ __forceinline__ float dot3(f3 a, f3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
__device__ __forceinline__ f3 sc3(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 add3(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 normalize3(f3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return sc3(v, inv); }

// glm mat4*vec4 with w = 1: (m0*x + m1*y) + (m2*z + m3*1)
__device__ __forceinline__ void m4p(const float *m, float x, float y, float z, float &ox, float &oy, float &oz, float &ow) {
    ox = (m[0] * x + m[4] * y) + (m[8] * z + m[12] * 1.0f);
    oy = (m[1] * x + m[5] * y) + (m[9] * z + m[13] * 1.0f);
    oz = (m[2] * x + m[6] * y) + (m[10] * z + m[14] * 1.0f);
    ow = (m[3] * x + m[7] * y) + (m[11] * z + m[15] * 1.0f);
}
// glm mat3*vec3: left to right
__device__ __forceinline__ f3 m3v(const float *m, f3 v) {
    return {m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z, m[2] * v.x + m[5] * v.y + m[8] * v.z};
}

// Canvas::barycentric_coordinate body after the per-triangle part (shs_renderer.hpp:809-820) and
// draw_triangle_tile's inside test (blinn_phong_shading.cpp:226: u < 0 || v < 0 || w < 0 rejects);
// the |denom| < 1e-5 early-out is per triangle and culled in k_setup.  Returns true when the pixel
// passes, with (u, v, w) rounded exactly as the reference.
//
// Exact early-out: v = nv / denom is certainly negative (so the pixel is rejected) when nv and
// denom have opposite signs and |nv| > |denom| * 2^-100 -- the quotient is then a nonzero negative
// float (no underflow to -0, which would pass).  NaN or infinite numerators/denominators never take
// the early-out (every comparison with NaN is false; |denom| = inf makes the threshold inf).  The
// two divides, the costliest part, then run only for pixels inside or at the edge of the triangle.
__device__ __forceinline__ bool bary_pass(const TriRec &r, float Px, float Py, float &u, float &v, float &w) {
    const float vpx = Px - r.ax, vpy = Py - r.ay;
    const float t0 = vpx * r.v0x, t1 = vpy * r.v0y;
    const float d20 = t0 + t1;
    const float t2 = vpx * r.v1x, t3 = vpy * r.v1y;
    const float d21 = t2 + t3;
    const float nv = r.d11 * d20 - r.d01 * d21;
    const float nw = r.d00 * d21 - r.d01 * d20;
    const float thr = fabsf(r.denom) * 0x1p-100f;   // exact: |denom| >= 1e-5 keeps it normal
    const bool dneg = r.denom < 0.0f;
    if (((nv < 0.0f) != dneg && fabsf(nv) > thr) || ((nw < 0.0f) != dneg && fabsf(nw) > thr)) return false;
    v = nv / r.denom;
    w = nw / r.denom;
    u = (1.0f - v) - w;
    return !(u < 0 || v < 0 || w < 0);
}

}  // namespace shs_dev
