/*
 * shs_gpu.h -- C ABI of libshs_gpu.so, the MI355X (gfx950) replacement for the shs_renderer
 * triangle scan-conversion hot path.
 *
 * The reference has no C ABI/FFI; it has three C++ seams, and every entry point
 * below names the seam it replaces.  Paths are relative to /root/reference/cpp-folders/src/.
 *
 *   Seam 1 (legacy draw-call seam): RendererSystem::process(dt) -> draw_triangle_tile(Canvas&,
 *     ZBuffer&, verts, norms, std::function VS, std::function FS, tile_min, tile_max)
 *     hello-3d-primitives/hello_pipeline_blinn_phong_shading.cpp:189-313 (and the Phong :204,
 *     Gouraud :186-236, Flat :194-247 copies).  Replaced by shs_render_legacy(): the std::function
 *     shaders become the shading-model enum + POD uniform block of shs_legacy_draw, the per-tile job
 *     loop becomes one enqueue on the context's HIP stream.
 *   Seam 2 (library rasterize_mesh) and Seam 3 (the PassShadowMap / PassPBRForward IRenderPass
 *     bodies, Forward+ light culling): the "Library path" section below.
 *
 * Conventions: every function returns int status (0 = SHS_OK), never throws; a
 * context is used by one host thread at a time; host buffers are caller-owned and use the exact
 * reference layouts (RGBA8 canvas rows bottom-up, f32 depth in screen rows for the legacy path);
 * matrices are column-major float[16] exactly as glm::mat4 stores them.  No torch types cross.
 */
#ifndef SHS_GPU_H
#define SHS_GPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHS_OK 0
#define SHS_ERR_INVALID (-1)     /* bad argument (null pointer, bad size, unknown id)      */
#define SHS_ERR_HIP (-2)         /* HIP runtime error (message via shs_last_error)         */
#define SHS_ERR_NO_DEVICE (-3)   /* no gfx950 device / device index out of range           */
#define SHS_ERR_OVERFLOW (-4)    /* internal bin capacity exceeded; frame re-issued        */

/* Shading models of the legacy pipelines (the FS/VS pairs each hello_pipeline_* demo binds). */
#define SHS_SHADING_FLAT 0         /* hello_pipeline_flat_shading.cpp:46-98         */
#define SHS_SHADING_GOURAUD 1      /* hello_pipeline_gouraud_shading.cpp:46-89       */
#define SHS_SHADING_PHONG 2        /* hello_pipeline_phong_shading.cpp:47-108        */
#define SHS_SHADING_BLINN_PHONG 3  /* hello_pipeline_blinn_phong_shading.cpp:48-97   */

typedef struct shs_ctx shs_ctx;

/* One legacy draw = one object of the scene loop (blinn_phong_shading.cpp:272-305): the
 * reference's `Uniforms` POD (:36-42) plus the mesh handle and shading model.
 *   model      : Uniforms::model; for SHS_SHADING_FLAT this is Uniforms::mv (flat_shading.cpp:35)
 *   light_dir  : Uniforms::light_dir (world); for SHS_SHADING_FLAT: Uniforms::light_dir_view      */
typedef struct shs_legacy_draw {
    int32_t mesh_id;
    int32_t shading;
    float mvp[16];
    float model[16];
    float light_dir[3];
    float camera_pos[3];
    uint8_t color[4];
} shs_legacy_draw;

/* Per-frame description.  ref_tile_w/h are the reference's tile-job size (TILE_SIZE_X/Y = 80,
 * blinn_phong_shading.cpp:29-30): the legacy raster clamps each triangle's bounding box to the
 * tile that runs it, and the GPU path reproduces that visited-pixel set exactly.
 * shard_rank/shard_count select the GPU tiles (shs_gpu_tile_size() px square, row-major) this
 * device owns (tile % count == rank);
 * (0,1) renders the whole frame. */
typedef struct shs_frame_desc {
    int32_t width, height;
    int32_t ref_tile_w, ref_tile_h;
    int32_t shard_rank, shard_count;
    uint32_t flags;               /* SHS_FRAME_* */
    uint8_t clear_color[4];       /* Canvas::fill_pixel colour, {0,0,0,255} in every demo      */
} shs_frame_desc;

#define SHS_FRAME_PREQUANT 1u     /* also keep the shader's pre-truncation floats (tests)     */
#define SHS_FRAME_PRESENT 2u      /* also write the SDL present staging (shs_resolve_present)  */

typedef struct shs_raster_stats {
    uint64_t tri_input;           /* triangles submitted (rasterizer.hpp:208 tri_input)        */
    uint64_t tri_setup;           /* triangles surviving setup culls (area<=0, |denom|<1e-5)   */
    uint64_t tri_ghost;           /* slivers whose tile-clamp pixels near the bbox are tested   */
    uint64_t bin_entries;         /* (tile, triangle) pairs binned                              */
    uint64_t covered_pixels;      /* final pixels with depth != clear (shaded Mpix/s numerator) */
    uint64_t tri_ghost_unbounded; /* ... with no error bound: every visited pixel tested        */
    uint64_t spilled;             /* bin entries beyond the per-tile capacity                    */
    uint64_t max_tile_bin;        /* fullest 32x32 tile's triangle count                         */
    uint64_t ghost_fragments;     /* passing tile-clamp pixels of unbounded slivers outside bbox */
} shs_raster_stats;

/* ---- context ---------------------------------------------------------------------------- */
int shs_create(int device, shs_ctx **out);
int shs_destroy(shs_ctx *ctx);
const char *shs_last_error(shs_ctx *ctx);
/* Run on a caller-provided hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL
 * restores the context's own stream. */
int shs_set_stream(shs_ctx *ctx, void *hip_stream);
void *shs_get_stream(shs_ctx *ctx);
int shs_synchronize(shs_ctx *ctx);

/* ---- geometry (replaces the ModelGeometry vectors the tile jobs read,
 *      shs_renderer.hpp:1296-1298; uploaded once, device resident) ------------------------ */
int shs_mesh_upload_soup(shs_ctx *ctx, const float *positions, const float *normals, int32_t n_tris,
                         int32_t *mesh_id);
int shs_mesh_release(shs_ctx *ctx, int32_t mesh_id);
/* A handle in dst to src's uploaded mesh (legacy soup or library MeshData), on the same device, without
 * a copy: frames in flight on several contexts read one device copy of each mesh.  The buffers stay
 * src's: src must not release the mesh, nor be destroyed, while dst may still read it; releasing the
 * shared handle in dst (or destroying dst) frees nothing. */
int shs_mesh_share(shs_ctx *dst, shs_ctx *src, int32_t src_mesh_id, int32_t *mesh_id);

/* ---- the hot path (Seam 1) --------------------------------------------------------------- */
/* Clears the frame (Canvas::fill_pixel + ZBuffer::clear) and rasterises all draws in order,
 * asynchronously on the context stream.  Results stay in device memory until shs_resolve. */
int shs_render_legacy(shs_ctx *ctx, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws);

/* Superseding: a render call while the previous batch is still in flight does not wait for it, but
 * it reads that batch's capacity-overflow word first (final once the batch's setup is, copied to
 * pinned memory beside its raster); an overflowed batch is finished -- re-issued with grown
 * capacities -- before the new one is enqueued, so work queued behind a batch on the stream never
 * sees an incomplete frame. */
/* A batch of n_frames frames (1 <= n_frames <= SHS_MAX_BATCH_FRAMES) of one frame description, e.g.
 * the next n_frames camera poses of a render-ahead host or the views of a multi-view capture: frame f
 * draws draws[f * n_draws .. f * n_draws + n_draws - 1], in that order, and every frame must submit
 * the same number of triangles.  Each frame has its own device framebuffers (frame f's colour at
 * byte f*W*H*4 of the colour plane shs_device_framebuffers returns, its depth at float f*W*H); the
 * frames are independent -- each equals the frame shs_render_legacy renders from its draws.  One
 * k_setup + one k_raster launch cover the whole batch.  shs_render_legacy(ctx, frame, draws, n) is
 * shs_render_legacy_batch(ctx, frame, draws, n, 1).  Statistics (shs_get_stats) are batch totals. */
#define SHS_MAX_BATCH_FRAMES 1024
int shs_render_legacy_batch(shs_ctx *ctx, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws,
                            int32_t n_frames);

/* Copy the frame into caller-owned host buffers (blocking).  color: W*H*4 bytes, canvas rows
 * (Canvas::buffer() layout); depth: W*H floats, screen rows (ZBuffer::buffer() as the legacy
 * pipelines index it).  Either pointer may be NULL.  shs_resolve = frame 0 of the last batch. */
int shs_resolve(shs_ctx *ctx, uint8_t *color, float *depth);
int shs_resolve_frame(shs_ctx *ctx, int32_t frame_index, uint8_t *color, float *depth);
/* Present staging (SHS_FRAME_PRESENT), written by the same launch as the canvas: the RGBA32 surface
 * Canvas::copy_to_SDLSurface fills (shs_renderer.hpp:833-848) -- surface row h-1-y holds canvas row
 * y, SDL_MapRGBA into create_sdl_surface's little-endian RGBA32 masks (:850-856) is the Color bytes.
 * shs_resolve_present copies it into a caller surface (pixels + pitch in bytes >= W*4), replacing
 * the per-pixel copy loop; shs_present_device returns the device pointer (W*H words, rows top-down).
 * shs_present_device and shs_device_framebuffers first finish the batch (wait for it; a capacity
 * overflow re-issues it), so the pointer holds the final frame.  The pointer aliases the context's
 * buffers: it is valid until the next shs_render_legacy* call on this context (which rewrites them,
 * and reallocates them when the frame or batch grows); call again per batch. */
int shs_resolve_present(shs_ctx *ctx, int32_t frame_index, uint8_t *pixels, int32_t pitch);
int shs_present_device(shs_ctx *ctx, int32_t frame_index, void **present_dev);
/* Pre-truncation shader floats, W*H*4 (canvas rows), only when SHS_FRAME_PREQUANT was set:
 * shs_resolve_prequant_frame for frame frame_index of the batch, shs_resolve_prequant for frame 0. */
int shs_resolve_prequant(shs_ctx *ctx, float *prequant);
int shs_resolve_prequant_frame(shs_ctx *ctx, int32_t frame_index, float *prequant);
/* Device pointers of the current batch's colour / depth planes (zero-copy hand-off to torch / RCCL);
 * finished and valid as for shs_present_device. */
int shs_device_framebuffers(shs_ctx *ctx, void **color_dev, void **depth_dev);
int shs_get_stats(shs_ctx *ctx, shs_raster_stats *stats);

/* Per-kernel device timing of the last frame, recorded with HIP events on the context stream
 * (k_setup, k_ghost, unused, k_raster) in milliseconds.  Enabled by shs_enable_timing(ctx, 1). */
int shs_enable_timing(shs_ctx *ctx, int enable);
int shs_last_kernel_ms(shs_ctx *ctx, float *ms4);
/* Sums of the same four kernel durations over every frame enqueued since shs_timing_reset
 * (events recorded on the context stream around each kernel, harvested lazily). */
int shs_timing_reset(shs_ctx *ctx);
int shs_timing_read(shs_ctx *ctx, double *sum_ms4, int64_t *n_frames);

/* ---- host helpers: GLM restatements the reference host code computes with glm -----------
 * (Camera3D::update shs_renderer.hpp:1224-1236; MonkeyObject::get_world_matrix
 *  blinn_phong_shading.cpp:122-128).  The drop-in host keeps its own glm code; these exist so
 *  non-C++ callers (tests, bench) can build identical uniforms. */
int shs_camera3d(const float position[3], float horizontal_angle, float vertical_angle, float fov_deg,
                 float z_near, float z_far, float view16[16], float proj16[16]);
int shs_model_trs(const float position[3], float rotation_deg_y, const float scale[3], float out16[16]);
int shs_mat4_mul(const float a16[16], const float b16[16], float out16[16]);
int shs_mat4_inverse(const float m16[16], float out16[16]);

/* Debug / test hook: copy the last frame's per-triangle raster records (64 B each, layout
 * shs_dev::TriHot in csrc/shs_device.hpp: the pixel-independent barycentric terms, screen z, a
 * draw | flags << 29 word and the packed bin box) into caller memory; returns the count via n_out.
 * Records of culled triangles are not written by the legacy setup (stale entries). */
int shs_debug_records(shs_ctx *ctx, void *out, int64_t capacity, int64_t *n_out);

/* Tuning knobs.  SHS_OPT_BIN_CAPACITY: initial per-tile bin capacity (entries past it spill to a
 * global list and stay exact; the context grows the capacity to the fullest tile it observes). */
#define SHS_OPT_BIN_CAPACITY 1
/* SHS_OPT_RASTER_MODE: 0 auto (small scenes scan every triangle's bin box per tile, large scenes
 * build per-tile bins), 1 force scan, 2 force bins.  Results are identical in every mode. */
#define SHS_OPT_RASTER_MODE 2
/* SHS_OPT_TIMELINE: 1 = record every workgroup's start / end time (s_memrealtime, 100 MHz) of the
 * frames that follow (profiling aid; read with shs_debug_timeline / shs_lib_debug_timeline), 2 = the
 * same, with the library's shadow-pass raster recorded instead of the camera pass's, 0 = off. */
#define SHS_OPT_TIMELINE 3
/* SHS_OPT_RASTER_LOOP: 1 = (candidate, pixel) pair tasks dealt over the waves (default), 0 = each
 * thread loops over the tile's candidates for its own pixel.  Results are identical in both. */
#define SHS_OPT_RASTER_LOOP 4
/* SHS_OPT_SPILL_CAPACITY / SHS_OPT_FRAG_CAPACITY (tests): reallocate the legacy workspaces' global
 * bin-spill list / ghost-fragment list to `value` entries.  A batch that needs more raises its
 * overflow flag and is re-issued with grown lists when it is finished (synchronise, resolve, present,
 * superseded); results are identical. */
#define SHS_OPT_SPILL_CAPACITY 5
#define SHS_OPT_FRAG_CAPACITY 6
/* SHS_OPT_LIB_PART: library camera passes split a busy 32x8 raster tile whose candidate list holds more
 * than `value` entries into ceil(n / value) parts (at most 16) rendered by several workgroups at once,
 * part j over list positions [j n / k, (j + 1) n / k) of the whole tile; the parts merge their keys
 * with 64-bit atomicMin and the last one writes the winners (results identical).  -1: 512 for
 * tile-sharded passes, off otherwise; 0 (default): off (measured slower). */
#define SHS_OPT_LIB_PART 7
/* SHS_OPT_SHARD_CULL: 1 = each setup workgroup of a tile-sharded camera pass first keeps the triangles
 * of its inputs that can reach the rank's tiles (positions only) and sets up only those; 0 (default) =
 * every rank sets up every triangle, dropping the ones off its tiles after the transform.  Results
 * identical. */
#define SHS_OPT_SHARD_CULL 8
/* SHS_OPT_SHARD_LAYOUT: which 32x32 bin tiles a tile-sharded library frame's rank owns.
 * SHS_SHARD_INTERLEAVED (default): tile % count == rank.  SHS_SHARD_REGIONS: one rectangle per rank,
 * from a recursive bisection of the bin grid at equal predicted cost, predicted from the context's
 * previous camera pass (the bin-tile bounds of its 256-triangle setup blocks; the first pass, or one
 * after a resize, splits by pixels).  Every rank derives the same rectangles from the same frames, with
 * no exchange; a rank then skips whole setup blocks whose bounds miss its rectangle.  Applies to
 * shs_light_cull, shs_render_pbr_forward, shs_tonemap and shs_tiles_* of sharded library frames (the
 * legacy path stays interleaved).  Images identical; a region-sharded pass's statistics count only the
 * setup blocks that reach the rank. */
#define SHS_OPT_SHARD_LAYOUT 9
#define SHS_SHARD_INTERLEAVED 0
#define SHS_SHARD_REGIONS 1
/* SHS_OPT_SHARD_ROOT_SHARE: rank 0's share of a region layout's predicted cost, in permille of the other
 * ranks' (default 1000).  Rank 0 also unpacks every peer's tiles of the gathered frame; a smaller share
 * leaves it room for that.  Every rank must use the same value. */
#define SHS_OPT_SHARD_ROOT_SHARE 10
/* SHS_OPT_SHADOW_FOOTPRINT: 1 = shs_render_shadow_map records the pass (light camera computed and
 * returned as before) and the next shs_render_pbr_forward enqueues it over only the 32x32 shadow-map
 * tiles that pass's pixels can read: for each draw with `shadow`, the light-space bounds of (its world
 * box) ∩ (the camera frustum slice of the pixels the rank shades -- its region, or the whole frame),
 * widened by the PCF reach (shadow_sample.hpp:65-104) -- so a region-sharded rank renders only its own
 * shadow footprint and no shadow map crosses between ranks.  Texels outside are not written that pass;
 * the frame's images are identical.  A later camera pass that samples the same map (another view or
 * region) and reads beyond the rendered tiles enqueues the shadow pass again over the union first;
 * releasing a caster mesh of a footprint-restricted map renders the map whole first.
 * shs_resolve_shadow_map of a recorded pass renders it whole.
 * 0 (default): every shadow pass renders the whole map when it is called. */
#define SHS_OPT_SHADOW_FOOTPRINT 11
/* SHS_OPT_LEGACY_PIPELINE: 1 = multi-draw scan-mode legacy batches (shs_render_legacy_batch with more
 * than 6 draws in all, scenes up to 4096 triangles) are pipelined: batch k's raster runs in the same
 * launch as batch k + 1's setup, or at the next call that needs the frames (shs_synchronize, every
 * resolve / present / tiles call, a non-pipelined render, shs_set_stream).  The frames are identical;
 * what changes is that a batch's frames are final only after such a call -- work the caller queues on
 * the context stream right after shs_render_legacy_batch does not see them.  0 (default): off. */
#define SHS_OPT_LEGACY_PIPELINE 12
int shs_set_option(shs_ctx *ctx, int option, int64_t value);
/* The regions of the last region-sharded camera pass: rects[4 r .. 4 r + 3] = (bx0, by0, bx1, by1) of
 * rank r, bin tiles, inclusive (bx1 < bx0: rank r owns nothing). */
int shs_get_shard_regions(shs_ctx *ctx, int32_t shard_count, int32_t *rects);
/* Host-only (no device): the region balance itself, for tests -- blocks[4 i .. 4 i + 3] = k_lib_setup's
 * per-block record (bx0 | bx1 << 16, by0 | by1 << 16, triangles, 1 bounded / 2 estimate / 0 none). */
int shs_shard_balance_rects(const uint32_t *blocks, int32_t n_blocks, int32_t width, int32_t height, int32_t shard_count,
                            int32_t root_permille, int32_t *rects);

/* Debug / profiling hook: the last frame's workgroup timeline.  out[0..7] = {k_setup grid, k_raster
 * grid, setup blocks, ghost blocks, clear blocks, stride S, 0, 0} (k_setup's block roles in that
 * order), then S slots per k_setup workgroup followed by S per k_raster workgroup: start, end, and
 * phase marks of the workgroup's thread 0 (0 where a phase did not run). */
int shs_debug_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out);
/* Debug / profiling hook: the last camera pass's (SHS_OPT_TIMELINE 2: shadow pass's) k_lib_raster workgroup timeline,
 * 16 uint64 per workgroup: start, end, summed ticks of gather / stage + pairs / resolve + shade over
 * its busy tiles, clear ticks, busy tiles, cleared tiles, staging passes, pairs, candidates, longest
 * busy tile, and (deep camera raster) the staging passes' selection + record + span ticks and segment
 * ticks, all busy tiles' ticks, the last busy tile's end (s_memrealtime, 100 MHz).  out = NULL: *n_out = the count only. */
int shs_lib_debug_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out);
/* The same for the last camera pass's k_lib_setup: 6 uint64 per workgroup -- start, after its
 * triangles, after the deferred marks, end, large primitives, deferred union width x height. */
int shs_lib_debug_setup_timeline(shs_ctx *ctx, uint64_t *out, int64_t capacity, int64_t *n_out);

/* Library/ABI version for integration checks; edge of the square GPU screen tile (shard unit). */
int shs_abi_version(void);
int shs_gpu_tile_size(void);

/* =========================================================================================
 * Library path -- Seam 2 (rasterize_mesh, shs-renderer-lib/include/shs/sw_render/rasterizer.hpp
 * :181-442) and Seam 3 (PassShadowMap, passes/pass_shadow_map.hpp:44-206; PassPBRForward,
 * passes/pass_pbr_forward.hpp:49-214).  The std::function ShaderProgram becomes a program enum
 * + the POD uniform block below.  Paths relative to shs-renderer-lib/include/shs/.
 * ========================================================================================= */
#define SHS_PROGRAM_PBR_MR 0        /* make_pbr_mr_program          shader/builtin_shaders.hpp:154-214 */
#define SHS_PROGRAM_BLINN_PHONG 1   /* make_blinn_phong_program     :105-152                         */
#define SHS_PROGRAM_DEBUG_ALBEDO 2  /* make_debug_view_shader_program(DebugViewMode) :221-245        */
#define SHS_PROGRAM_DEBUG_NORMAL 3
#define SHS_PROGRAM_DEBUG_DEPTH 4

#define SHS_CULL_NONE 0             /* RasterizerCullMode (rasterizer.hpp:26-31) */
#define SHS_CULL_BACK 1
#define SHS_CULL_FRONT 2

/* MeshData (resources/mesh.hpp:23-43): n_verts vec3 positions; normals / uvs may be shorter than
 * positions (missing entries read as (0,1,0) / (0,0), rasterizer.hpp:196-202) or NULL; indices NULL
 * = non-indexed soup (3 consecutive positions per triangle).  Device resident from here on, a mesh of
 * more than 256 triangles stored in the spatial (Morton) order of its triangles' centroids; the
 * submission order -- z ties, clipped fans, draws without a depth target -- stays the MeshData order. */
int shs_mesh_upload(shs_ctx *ctx, const float *positions, int32_t n_verts, const float *normals, int32_t n_normals,
                    const float *uvs, int32_t n_uvs, const uint32_t *indices, int64_t n_indices, int32_t *mesh_id);

/* Texture2DData (resources/texture.hpp:23-49): w * h Color texels (RGBA8, texel (x, y) at byte
 * 4 * (y * w + x)), device resident from here on.  *tex_id is >= 1 (the TextureAssetHandle convention,
 * resource_registry.hpp:62-66: 0 = no texture).  The PBR and Blinn-Phong programs sample it at the
 * perspective-correct UV0 varying with sample_texture2d_bilinear_repeat_linear (shader/
 * builtin_shaders.hpp:25-55; the sRGB decode uses the host's std::pow values).  A texture that fails
 * Texture2DData::valid() is not uploaded: the caller passes 0, as the sampler then returns vec3(1). */
int shs_texture_upload(shs_ctx *ctx, const uint8_t *rgba, int32_t w, int32_t h, int32_t *tex_id);
int shs_texture_release(shs_ctx *ctx, int32_t tex_id);

/* One rasterize_mesh call as PassPBRForward issues it per RenderItem: the ShaderUniforms fields the
 * builtin programs read (shader/types.hpp:87-116) and RasterizerConfig's cull mode / front face.
 * shadow != 0: u.shadow_map = the context's shadow map (last shs_render_shadow_map). */
typedef struct shs_lib_draw {
    int32_t mesh_id;
    int32_t program;              /* SHS_PROGRAM_* */
    int32_t cull_mode;            /* SHS_CULL_* */
    int32_t front_face_ccw;
    float model[16], viewproj[16], prev_model[16], prev_viewproj[16];
    float light_dir_ws[3], light_color[3], light_intensity, camera_pos[3];
    float base_color[3], metallic, roughness, ao;
    int32_t shadow;
    float light_viewproj[16];
    float shadow_bias_const, shadow_bias_slope;
    int32_t shadow_pcf_radius;
    float shadow_pcf_step, shadow_strength;
    int32_t enable_motion_vectors;
    int32_t base_color_tex;       /* u.base_color_tex: a shs_texture_upload id, 0 = none (sample = vec3(1)) */
} shs_lib_draw;

#define SHS_LIB_DEPTH_MOTION 1u   /* RasterizerTarget::depth_motion present: z test, depth + motion */
#define SHS_LIB_BG_GRADIENT 2u    /* PassPBRForward's no-sky background gradient, else clear_hdr     */

/* The pass's render targets: RT_ColorHDR (W*H RGBA32F, rows y-up) and RT_ColorDepthMotion (depth
 * cleared to 1 with zn / zf for the linear depth, motion cleared to 0).  shard_rank / shard_count as
 * in shs_frame_desc (32x32 tiles, tile % count == rank). */
typedef struct shs_lib_frame {
    int32_t width, height;
    int32_t shard_rank, shard_count;
    uint32_t flags;               /* SHS_LIB_* */
    float zn, zf;
    float clear_hdr[4];
} shs_lib_frame;

typedef struct shs_lib_stats {
    uint64_t tri_input;           /* RasterizerStats (rasterizer.hpp:48-53) */
    uint64_t tri_after_clip;
    uint64_t tri_raster;
    uint64_t covered_pixels;      /* pixels whose depth != clear (shaded Mpix/s numerator) */
    uint64_t max_tile_bin;
    uint64_t spilled;
    uint64_t clipped_extra;       /* fan triangles beyond the first of clipped input triangles */
} shs_lib_stats;
/* A tile-sharded pass (shard_count > 1) skips the clipping of triangles whose fans cannot reach its
 * tiles: its tri_after_clip / tri_raster / clipped_extra leave those out. */

/* PassPBRForward::execute: clear (gradient / clear_hdr, depth 1, motion 0) and one rasterize_mesh per
 * draw, in order, asynchronously on the context stream. */
int shs_render_pbr_forward(shs_ctx *ctx, const shs_lib_frame *frame, const shs_lib_draw *draws, int32_t n_draws);
/* Copy the pass's targets into caller-owned buffers: hdr W*H*4 floats, depth W*H, motion W*H*2
 * (row y = bottom-up, exactly PixelBuffer2D::at(x, y)); any pointer may be NULL. */
int shs_resolve_lib(shs_ctx *ctx, float *hdr, float *depth, float *motion);
int shs_get_lib_stats(shs_ctx *ctx, shs_lib_stats *stats);
/* Device pointers of the pass's targets; the pass chain is finished first (a capacity overflow
 * re-issues it), valid until the next shs_render_pbr_forward on this context. */
int shs_lib_device_targets(shs_ctx *ctx, void **hdr_dev, void **depth_dev, void **motion_dev);
/* Kernel durations of the library passes enqueued since shs_lib_timing_reset while
 * shs_enable_timing(ctx, 1) is on (HIP events on the context stream): sum_ms4 = {shadow k_lib_setup,
 * shadow k_lib_raster, camera k_lib_setup, camera k_lib_raster}; n_passes2 = {shadow, camera} passes. */
int shs_lib_timing_reset(shs_ctx *ctx);
int shs_lib_timing_read(shs_ctx *ctx, double sum_ms4[4], int64_t n_passes2[2]);

/* A shadow caster (RenderItem with casts_shadow): mesh + model matrix. */
typedef struct shs_shadow_caster {
    int32_t mesh_id;
    float model[16];
} shs_shadow_caster;

/* PassShadowMap::execute into the context's RT_ShadowDepth (w*h f32, cleared to 1): scene AABB of the
 * casters' mesh bounds, build_dir_light_camera_aabb(sun_dir, aabb, 10, w) (camera/light_camera.hpp
 * :33-98), then the depth pass.  light_viewproj_out (optional) receives ctx.shadow.light_viewproj. */
int shs_render_shadow_map(shs_ctx *ctx, int32_t w, int32_t h, const float sun_dir[3], const shs_shadow_caster *casters,
                          int32_t n_casters, float light_viewproj_out[16]);
int shs_resolve_shadow_map(shs_ctx *ctx, float *depth);
/* The bin tiles (32x32 texels, inclusive) the last enqueued shadow pass rendered: the whole map, or
 * under SHS_OPT_SHADOW_FOOTPRINT the camera pass's footprint (rect[2] < rect[0]: none, or still recorded). */
int shs_get_shadow_region(shs_ctx *ctx, int32_t rect[4]);
/* Host-only (no device): the footprint itself, for tests -- the texels (inclusive; texel_rect[2] <
 * texel_rect[0]: none) of an sm_w x sm_h map, through light_viewproj, that a PCF of `reach` texels reads
 * from points of the world box [world_min, world_max] whose camera_viewproj projection falls on the pixel
 * rectangle px_rect = {x0, y0, x1, y1} (inclusive, rows y up) of a width x height frame. */
int shs_shadow_footprint(const float light_viewproj[16], int32_t sm_w, int32_t sm_h, const float camera_viewproj[16],
                         int32_t width, int32_t height, const int32_t px_rect[4], const float world_min[3],
                         const float world_max[3], int32_t reach, int32_t texel_rect[4]);
/* Host-only, for tests: the same footprint per row of row_h texels (row r: texel rows r * row_h ..
 * r * row_h + row_h - 1, r < n_rows) -- the texel columns [x0[r], x1[r]] (x1[r] < x0[r]: none) read there,
 * from the convex hull of the footprint polytope's light-space image (round 6: a footprint shadow pass
 * renders only these 32-texel rows' spans of its rectangle). */
int shs_shadow_footprint_rows(const float light_viewproj[16], int32_t sm_w, int32_t sm_h, const float camera_viewproj[16],
                              int32_t width, int32_t height, const int32_t px_rect[4], const float world_min[3],
                              const float world_max[3], int32_t reach, int32_t row_h, int32_t n_rows, int32_t *x0,
                              int32_t *x1);

/* ---- Forward+ light-list binning ---------------------------------------
 * CullingLightGPU (lighting/light_types.hpp:141-166), the std430 record the reference uploads for
 * its GPU light culling; 160 B. */
typedef struct shs_culling_light {
    float position_range[4];      /* xyz position, w range                                       */
    float color_intensity[4];
    float direction_spot[4];
    float axis_spot_outer[4];
    float up_shape_x[4];
    float shape_attenuation[4];   /* x shape, y attenuation power, z bias, w cutoff              */
    uint32_t type_shape_flags[4]; /* x LightType, y culling shape, z flags, w attenuation model   */
    float cull_sphere[4];
    float cull_aabb_min[4];
    float cull_aabb_max[4];
} shs_culling_light;

#define SHS_LIGHT_CULL_NONE 0         /* culling_mode of fp_stress_light_cull.comp             */
#define SHS_LIGHT_CULL_TILED 1
#define SHS_LIGHT_CULL_TILED_DEPTH 2  /* tiles + per-tile depth range (fp_stress_depth_reduce) */
#define SHS_LIGHT_CULL_CLUSTERED 3

/* The CameraUBO fields the culling reads.  depth_linear: the depth range of mode 2 is reduced from
 * the context's library depth buffer (linear view depth, rasterizer.hpp:354-357); 0 = perspective
 * LH_NO depth as the Vulkan depth_reduce shader assumes.  shard_rank / shard_count: only the lists of
 * owned 32x32 tiles are built (others get count 0). */
typedef struct shs_light_cull_desc {
    int32_t width, height;
    uint32_t tile_size, max_per_tile, mode, z_slices;
    float view[16], proj[16];
    float zn, zf;
    int32_t depth_linear;
    int32_t shard_rank, shard_count;
} shs_light_cull_desc;

/* Upload the frame's local light set (replaces the LightBuffer SSBO). */
int shs_lights_upload(shs_ctx *ctx, const shs_culling_light *lights, int32_t n_lights);
/* fp_stress_light_cull.comp (+ fp_stress_depth_reduce.comp for mode 2, over the last library depth)
 * into device tile lists: counts[n_lists], indices[n_lists * max_per_tile], ascending light index.
 * Draws with SHS_PROGRAM_FORWARD_PLUS read these lists. */
int shs_light_cull(shs_ctx *ctx, const shs_light_cull_desc *desc);
/* counts: n_lists; indices: n_lists * max_per_tile (entries past the count are undefined); ranges:
 * tiles * 2 floats (mode 2).  Any pointer may be NULL. */
int shs_resolve_light_lists(shs_ctx *ctx, uint32_t *counts, uint32_t *indices, float *ranges);
#define SHS_PROGRAM_FORWARD_PLUS 5  /* per-pixel point lights from the tile lists (light_runtime.hpp:321-333) */

/* ---- the software library's CPU light binning -----------------------------
 * build_light_bin_culling (shs-renderer-lib/include/shs/lighting/light_culling_runtime.hpp:266-371):
 * cull_lights_tiled / cull_lights_tiled_view_depth_range / cull_lights_clustered
 * (lighting/jolt_light_culling.hpp:135-412) -- per bin, the cell of make_screen_tile_cell (:95-133)
 * against every camera-frustum-visible light with classify_vs_cell (geometry/jolt_culling.hpp:129-257).
 * The lights are the SceneShapes' world AABBs (min xyz, max xyz; SceneShape::world_aabb()): the
 * binning reads only those and the bounding sphere Jolt derives from them.  Lists hold local light
 * indices in ascending order: counts[bin] = every match, indices[bin * max_per_bin + k] the first
 * max_per_bin (use max_per_bin = n_lights for the reference's unbounded vectors).  Bins are tile-row-
 * major (top-origin tile rows), clusters slice-major; bins_xyz = (bins_x, bins_y, bins_z), all 0 for
 * SHS_LIGHT_CULL_NONE or no lights.  Synchronous: host arrays in, host arrays out. */
typedef struct shs_light_bin_desc {
    int32_t width, height;
    uint32_t tile_size;           /* LightBinCullingConfig::tile_size (16)                        */
    uint32_t mode;                /* SHS_LIGHT_CULL_NONE / _TILED / _TILED_DEPTH / _CLUSTERED       */
    uint32_t z_slices;            /* cluster_depth_slices (16)                                    */
    uint32_t max_per_bin;
    float view_proj[16];
    float z_near, z_far;          /* LightBinCullingConfig::z_near / z_far                         */
    const float *tile_min_view_depth;   /* mode 2: tiles_x * tiles_y linear view depths each, or NULL */
    const float *tile_max_view_depth;
    int32_t n_depth_tiles;
} shs_light_bin_desc;
int shs_light_bin_culling(shs_ctx *ctx, const shs_light_bin_desc *desc, const float *light_aabbs, int32_t n_lights,
                          uint32_t bins_xyz[3], uint32_t *counts, uint32_t *indices);

/* ---- multi-GPU tile shards -------------------------------------------------------
 * A frame rendered with shard_rank / shard_count holds only its own 32x32 tiles (tile % count ==
 * rank, or its region: SHS_OPT_SHARD_LAYOUT).  shs_tiles_pack writes them into a caller-owned DEVICE buffer (e.g. a torch tensor on the
 * context's device) -- one 32x32-padded block per owned tile, planes colour / depth / motion --
 * for an RCCL gather; rank 0 calls shs_tiles_unpack once per peer to compose the full frame.  Both
 * are enqueued on the context stream (see shs_set_stream). */
#define SHS_TARGET_LEGACY 0   /* shs_render_legacy frame: RGBA8 canvas rows + f32 depth  */
#define SHS_TARGET_LIB 1      /* library frame: RGBA32F HDR (+ depth + motion)           */
#define SHS_TARGET_PRESENT 2  /* legacy SDL staging (SHS_FRAME_PRESENT): RGBA8, 4 B/px    */
#define SHS_TARGET_LIB_PRESENT 3 /* tonemap present staging (SHS_TONEMAP_PRESENT): RGBA8  */
int shs_tiles_packed_words(shs_ctx *ctx, int target, int32_t shard_count, int64_t *words_per_rank);   /* the largest rank's */
/* The packed size of one rank's tiles (regions differ in size). */
int shs_tiles_rank_words(shs_ctx *ctx, int target, int32_t shard_rank, int32_t shard_count, int64_t *words);
/* shs_tiles_pack first makes the frame final: it waits for the frame's setup (not its raster) and,
 * if a capacity overflowed, re-issues it; the pack is then enqueued on the context stream behind it,
 * so the packed tiles are final without a host wait for the render. */
int shs_tiles_pack(shs_ctx *ctx, int target, int32_t shard_rank, int32_t shard_count, void *dst_dev);
int shs_tiles_unpack(shs_ctx *ctx, int target, int32_t shard_rank, int32_t shard_count, const void *src_dev);
/* shs_tiles_unpack of several ranks' packed buffers in one launch (rank 0's side of the gather):
 * src_dev[r] = rank r's packed buffer, or NULL to skip rank r (rank 0 itself, empty ranks). */
int shs_tiles_unpack_ranks(shs_ctx *ctx, int target, int32_t count, const void *const *src_dev);

/* Host GLM restatements for non-C++ callers (camera/convention.hpp; pass_pbr_forward.hpp:136-141). */
int shs_look_at_lh(const float eye[3], const float center[3], const float up[3], float out16[16]);
int shs_perspective_lh_no(float fovy_radians, float aspect, float zn, float zf, float out16[16]);
int shs_model_euler(const float pos[3], const float rot_euler[3], const float scl[3], float out16[16]);
int shs_dir_light_camera_aabb(const float sun_dir[3], const float aabb_min[3], const float aabb_max[3], float extra_margin,
                              uint32_t resolution, float view16[16], float proj16[16], float viewproj16[16]);

/* ---- after the path: PassTonemap + present staging ------------------------
 * PassTonemap::execute (shs-renderer-lib/include/shs/passes/pass_tonemap.hpp:36-83) over the last
 * camera pass's HDR target, and the SDL texture staging of upload_ldr_to_rgba8
 * (exp-plumbing/hello_pass_basics.cpp:102-119), in one launch on the context stream.  The bytes are
 * the reference's: the host derives, with its own std::pow / std::lround, the 255 thresholds in
 * x = c / (1 + c) where the byte changes, and the kernel counts thresholds. */
#define SHS_TONEMAP_LDR 1u      /* RT_ColorLDR: W*H RGBA8, rows y up, alpha 255 */
#define SHS_TONEMAP_PRESENT 2u  /* RGBA8 staging for SDL_UpdateTexture: rows top-down, alpha 255 */
typedef struct shs_tonemap_desc {
    float exposure;             /* FrameParams::pass.tonemap.exposure (clamped to >= 0.0001 as the pass does) */
    float gamma;                /* ...gamma (clamped to >= 0.001) */
    uint32_t flags;             /* SHS_TONEMAP_* targets to write (at least one) */
} shs_tonemap_desc;
int shs_tonemap(shs_ctx *ctx, const shs_tonemap_desc *desc);
/* Fused PassTonemap: with desc non-NULL, every later shs_render_pbr_forward also writes desc's
 * targets from its shading kernel (one launch, no HDR re-read; the bytes are shs_tonemap's), and the
 * frame counts as tonemapped (shs_resolve_ldr, shs_motion_blur, SHS_TARGET_LIB_PRESENT tiles) without
 * a shs_tonemap call.  NULL turns it off.  The reference runs PassTonemap as a separate pass
 * (pass_tonemap.hpp:36-83); this only fuses it into the producer. */
int shs_lib_fuse_tonemap(shs_ctx *ctx, const shs_tonemap_desc *desc);
/* Copy the tonemapped targets into caller-owned W*H*4-byte buffers (either may be NULL). */
int shs_resolve_ldr(shs_ctx *ctx, uint8_t *ldr, uint8_t *present);
/* Device pointers of the tonemap targets (the pass chain finished first, as shs_lib_device_targets). */
int shs_ldr_device_targets(shs_ctx *ctx, void **ldr_dev, void **present_dev);
/* PassMotionBlur::execute (shs-renderer-lib/include/shs/passes/pass_motion_blur.hpp:38-170) on the
 * last tonemap's RT_ColorLDR (SHS_TONEMAP_LDR) with the camera pass's depth / motion planes
 * (SHS_LIB_DEPTH_MOTION), into a separate RT_ColorLDR (+ its present staging with
 * SHS_MOTION_BLUR_PRESENT).  Fields are FrameParams::pass.motion_blur (frame/frame_params.hpp:49-57)
 * and FrameParams::dt; enable = 0 copies the input, as the pass does. */
#define SHS_MOTION_BLUR_PRESENT 1u
typedef struct shs_motion_blur_desc {
    int32_t enable;
    int32_t samples;            /* default 10, clamped to [4, 32] */
    float strength;             /* 1 */
    float max_velocity_px;      /* 20 */
    float min_velocity_px;      /* 0.25 */
    float depth_reject;         /* 0.08 */
    float dt;                   /* FrameParams::dt, seconds */
    uint32_t flags;             /* SHS_MOTION_BLUR_* */
} shs_motion_blur_desc;
int shs_motion_blur(shs_ctx *ctx, const shs_motion_blur_desc *desc);
/* Copy the blurred RT_ColorLDR (rows y up) and / or its present staging (rows top-down). */
int shs_resolve_motion_blur(shs_ctx *ctx, uint8_t *ldr, uint8_t *present);
/* ---- software occlusion pass ------------------------------------------------
 * culling_sw::run_software_occlusion_pass (shs-renderer-lib/include/shs/geometry/culling_software.hpp
 * :229-331) as scene_culling.hpp:187-219 drives it: the frustum-visible objects in view-depth order
 * (view z of the world AABB centre), each tested against the occlusion depth with its screen rect
 * (project_aabb_to_screen_rect + is_rect_occluded) and, when visible, depth-rasterized into it
 * (rasterize_mesh_depth_transformed).  Synchronous: the visible list feeds the host's draw list. */
typedef struct shs_occluder {
    int32_t mesh_id;            /* indexed shs_mesh_upload mesh (DebugMesh vertices + indices) */
    float model[16];            /* the instance transform (column-major) */
    float aabb_min[3], aabb_max[3];   /* world AABB (SceneElement::geometry.world_aabb()) */
} shs_occluder;
typedef struct shs_occlusion_desc {
    int32_t width, height;      /* occlusion buffer (OCC_W x OCC_H) */
    float view[16], view_proj[16];
    float depth_epsilon;        /* 1e-4 in the reference */
    int32_t enable;             /* 0: every frustum-visible object is visible */
} shs_occlusion_desc;
/* occluded[n_objects] (1 = occluded; 0 for objects not frustum-visible), visible[] in visit order
 * (capacity n_frustum_visible), *n_visible, depth W*H (y * W + x, may be NULL). */
int shs_occlusion_pass(shs_ctx *ctx, const shs_occlusion_desc *desc, const shs_occluder *objects, int32_t n_objects,
                       const uint32_t *frustum_visible, int32_t n_frustum_visible, uint8_t *occluded,
                       uint32_t *visible, int32_t *n_visible, float *depth);

/* ---- debug_draw colour + depth raster ----------------------------------------
 * shs::debug_draw (shs-renderer-lib/include/shs/sw_render/debug_draw.hpp): draw_filled_triangle
 * (:60-109) and draw_mesh_blinn_phong_transformed (:147-203), the lit-surface draw of the culling
 * demos (hello_occlusion_culling_sw.cpp:387-407, hello_culling_sw.cpp:315).  rgba is the RT_ColorLDR
 * (W*H Color, y * W + x, the rows as the canvas holds them) and depth the std::span<float> depth
 * buffer (y * W + x); both are read and written in place, exactly as a sequential draw of the list in
 * submission order leaves them.  Synchronous. */
typedef struct shs_debug_draw_desc {
    int32_t width, height;      /* canvas_w, canvas_h (== rt.w, rt.h) */
    float view_proj[16];        /* vp (column-major) */
    float camera_pos[3];
    float light_dir_ws[3];
} shs_debug_draw_desc;
typedef struct shs_debug_mesh {
    int32_t mesh_id;            /* indexed shs_mesh_upload mesh (DebugMesh vertices + indices) */
    float model[16];            /* column-major */
    float base_color[3];
} shs_debug_mesh;
/* The meshes in order, each draw_mesh_blinn_phong_transformed.  tri_lit (may be NULL): 4 floats per
 * triangle in submission order -- lit.rgb before the byte conversion (0 when the triangle is culled
 * before shading) and 1.0 when the triangle passes draw_filled_triangle's area test (0.0 otherwise). */
int shs_debug_draw_meshes(shs_ctx *ctx, const shs_debug_draw_desc *desc, const shs_debug_mesh *meshes,
                          int32_t n_meshes, uint8_t *rgba, float *depth, float *tri_lit);
typedef struct shs_debug_triangle {
    float p0[2], p1[2], p2[2];  /* screen points (pixels) */
    float z[3];                 /* depths z0, z1, z2 */
    uint8_t rgba[4];            /* Color */
} shs_debug_triangle;
/* draw_filled_triangle for each triangle in order. */
int shs_debug_fill_triangles(shs_ctx *ctx, int32_t width, int32_t height, const shs_debug_triangle *tris,
                             int32_t n_tris, uint8_t *rgba, float *depth);

/* ---- Canvas-API multi-pass extras --------------------------------------------
 * hello-render-target/ demos, paths relative to cpp-folders/src/hello-render-target/.  Colour buffers are
 * shs::Canvas pixels (W*H Color), depth the ZBuffer (view z, FLT_MAX = empty) and velocity the
 * Buffer<glm::vec2>, all indexed y * W + x as the passes index raw().  Host buffers: synchronous;
 * flags SHS_CANVAS_DEVICE: device buffers, enqueued on the context stream (shs_set_stream): the
 * caller orders that stream against whatever produces the inputs and consumes the outputs -- run
 * the context on the producer's stream (as the Python host does with torch's current stream) or
 * make the streams wait on events. */
#define SHS_CANVAS_DEVICE 1u
#define SHS_CANVAS_MAX_AUTOFOCUS_RADIUS 32
typedef struct shs_canvas_motion_blur_desc {
    int32_t width, height;
    float curr_view[16], curr_proj[16], prev_view[16], prev_proj[16];   /* column-major */
    int32_t samples;            /* MB_SAMPLES (12) */
    float strength;             /* MB_STRENGTH (0.85) */
    float w_obj, w_cam;         /* MB_W_OBJ (1), MB_W_CAM (0.35) */
    int32_t soft_knee;          /* MB_SOFT_KNEE (1) */
    float knee_px;              /* MB_KNEE_PIXELS (18) */
    float max_px;               /* MB_MAX_PIXELS (22) */
} shs_canvas_motion_blur_desc;
/* combined_motion_blur_pass (hello_pbr.cpp:1128-1252): src, depth, velocity -> dst. */
int shs_canvas_motion_blur(shs_ctx *ctx, const shs_canvas_motion_blur_desc *desc, const uint8_t *src, const float *depth,
                           const float *velocity, uint8_t *dst, uint32_t flags);
/* gaussian_blur_pass (hello_depth_of_field.cpp:175-251): one 5-tap axis, src -> dst. */
int shs_canvas_gaussian_blur(shs_ctx *ctx, int32_t width, int32_t height, const uint8_t *src, uint8_t *dst,
                             int32_t horizontal, uint32_t flags);
typedef struct shs_canvas_dof_desc {
    int32_t width, height;
    int32_t blur_iterations;    /* BLUR_ITERATIONS (3) */
    int32_t autofocus_radius;   /* AUTOFOCUS_RADIUS (6), at most SHS_CANVAS_MAX_AUTOFOCUS_RADIUS */
    int32_t focus_x, focus_y;   /* the autofocus centre (CANVAS_WIDTH / 2, CANVAS_HEIGHT / 2) */
    float range;                /* dof_range (24) */
    float max_blur;             /* dof_maxblur (0.6) */
} shs_canvas_dof_desc;
/* The depth-of-field step of hello_depth_of_field.cpp:786-812: color (ping.color) is the sharp frame
 * in and the composite out; blur_out (may be NULL) receives the final blur (pong.color); focus_depth
 * (may be NULL, host) the autofocus depth. */
int shs_canvas_dof(shs_ctx *ctx, const shs_canvas_dof_desc *desc, uint8_t *color, const float *depth, uint8_t *blur_out,
                   float *focus_depth, uint32_t flags);

/* ---- multi-GPU from one host process (SURVEY.md 5 "Distributed communication backend", 8e) ---------
 * The reference host is one C++ process driving one render loop (hello_pipeline_blinn_phong_shading.cpp
 * :369-455; PluggablePipeline::execute, pipeline/pluggable_pipeline.hpp:980).  A group is n contexts
 * in this process, context r on devices[r] (a device may repeat), each rendering the 32x32 tiles with
 * tile % n == r of every frame.  Per-rank work (uploads, passes) runs on one host worker thread per
 * rank, so the enqueue cost does not serialise over the GPUs.  shs_group_gather composes a frame on
 * rank 0's context: every rank packs its tiles on its own stream, copies them to rank 0's device
 * (hipMemcpyPeerAsync: xGMI between MI355X peers) and rank 0 unpacks them -- all stream-ordered, no
 * host wait, receive buffers double-buffered so the next frame's render overlaps this one's transfer.
 * Rank 0's context then resolves the full frame with the single-context calls (shs_resolve_lib,
 * shs_resolve_ldr, shs_resolve, shs_resolve_present).  Geometry, textures and lights are uploaded to
 * every rank (the ids agree across ranks when every rank uploads the same sequence). */
typedef struct shs_group shs_group;
int shs_group_create(const int32_t *devices, int32_t n, shs_group **out);
int shs_group_destroy(shs_group *g);
const char *shs_group_last_error(shs_group *g);
int shs_group_size(shs_group *g);
/* The rank's context (for the single-context calls; do not destroy it). */
int shs_group_context(shs_group *g, int32_t rank, shs_ctx **ctx);
/* Replicated uploads: the same call on every rank; *id is the (common) id. */
int shs_group_mesh_upload(shs_group *g, const float *positions, int32_t n_verts, const float *normals, int32_t n_normals,
                          const float *uvs, int32_t n_uvs, const uint32_t *indices, int64_t n_indices, int32_t *mesh_id);
int shs_group_mesh_upload_soup(shs_group *g, const float *positions, const float *normals, int32_t n_tris, int32_t *mesh_id);
int shs_group_texture_upload(shs_group *g, const uint8_t *rgba, int32_t w, int32_t h, int32_t *tex_id);
int shs_group_lights_upload(shs_group *g, const shs_culling_light *lights, int32_t n_lights);
/* shs_set_option on every rank's context (e.g. SHS_OPT_SHARD_LAYOUT). */
int shs_group_set_option(shs_group *g, int option, int64_t value);
int shs_group_lib_fuse_tonemap(shs_group *g, const shs_tonemap_desc *desc);
/* Sharded passes: rank r runs the call with shard_rank = r, shard_count = n (the frame's own shard
 * fields are ignored).  The shadow map is rendered whole on every rank (every rank's PCF reads all of it). */
int shs_group_light_cull(shs_group *g, const shs_light_cull_desc *desc);
int shs_group_render_shadow_map(shs_group *g, int32_t w, int32_t h, const float sun_dir[3], const shs_shadow_caster *casters,
                                int32_t n_casters, float light_viewproj_out[16]);
int shs_group_render_pbr_forward(shs_group *g, const shs_lib_frame *frame, const shs_lib_draw *draws, int32_t n_draws);
int shs_group_render_legacy(shs_group *g, const shs_frame_desc *frame, const shs_legacy_draw *draws, int32_t n_draws);
/* Compose the last frame's target (SHS_TARGET_*) on rank 0's context, asynchronously. */
int shs_group_gather(shs_group *g, int target);
int shs_group_synchronize(shs_group *g);

/* Host-only (no device): the byte thresholds for gamma (thr[0] = 0; +inf where a byte is never
 * reached).  Exposed for the parity tests. */
int shs_tonemap_thresholds(float gamma, float thr[256]);

#ifdef __cplusplus
}
#endif
#endif
