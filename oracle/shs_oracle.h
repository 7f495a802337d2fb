/*
 * shs_oracle.h -- CPU restatement of the shs_renderer legacy triangle scan-conversion path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / CPU baseline.  The product path
 * (libshs_gpu.so) never links, loads or calls it.
 *
 * PARITY UNPINNED: the reference (sharavsambuu/leisure-software-renderer) ships no golden vectors
 * or known-answer tests for this path and cannot be compiled here
 * (glm, SDL2, assimp absent), so this restatement is pinned only by its own analytic known-answer
 * tests (tests/test_oracle.py).  GLM operation order (mat*vec, dot, normalize, inverse, pow) is
 * restated from GLM's published headers (vcpkg classic mode, unversioned) -- see DESIGN.md.
 *
 * Layout conventions follow the reference exactly:
 *   color  : RGBA8, W*H*4 bytes, CANVAS rows (y up: row = H-1-y_screen) -- Canvas::draw_pixel_screen_space
 *            (cpp-folders/src/hello-shs-renderer/shs_renderer.hpp:792-796)
 *   depth  : float, W*H, SCREEN rows (y down) -- ZBuffer::test_and_set_depth(px, py)
 *            (hello_pipeline_blinn_phong_shading.cpp:231; shs_renderer.hpp:660-670)
 *   matrices: column-major float[16] exactly like glm::mat4 (m[col*4+row]).
 */
#ifndef SHS_ORACLE_H
#define SHS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ora_shading {
    ORA_FLAT = 0,        /* hello_pipeline_flat_shading.cpp:46-98        */
    ORA_GOURAUD = 1,     /* hello_pipeline_gouraud_shading.cpp:46-89      */
    ORA_PHONG = 2,       /* hello_pipeline_phong_shading.cpp:47-108       */
    ORA_BLINN_PHONG = 3  /* hello_pipeline_blinn_phong_shading.cpp:48-97  */
};

typedef struct ora_draw {
    int32_t shading;           /* enum ora_shading */
    int32_t n_tris;
    const float *positions;    /* 9*n_tris floats: triangle soup (ModelGeometry::triangles) */
    const float *normals;      /* 9*n_tris floats (ModelGeometry::normals)                  */
    float mvp[16];             /* Uniforms::mvp   = proj*view*model                         */
    float model[16];           /* Uniforms::model (Flat: Uniforms::mv)                      */
    float light_dir[3];        /* Uniforms::light_dir (Flat: light_dir_view)                */
    float camera_pos[3];       /* Uniforms::camera_pos                                      */
    uint8_t color[4];          /* Uniforms::color                                           */
} ora_draw;

/* RendererSystem::process + draw_triangle_tile (hello_pipeline_*_shading.cpp), one job per
 * tile_w x tile_h tile on n_threads workers.  prequant (optional, W*H*4 floats, canvas rows)
 * receives the fragment shader's value just before the (uint8_t) truncation of the final
 * fragment of every pixel (r,g,b, and 1.0 in .w for written pixels, 0 otherwise).
 * Returns 0 on success. */
int ora_render_legacy(int W, int H, int tile_w, int tile_h, int n_threads,
                      const ora_draw *draws, int n_draws,
                      uint8_t *color_out, float *depth_out, float *prequant_out);

/* Per-triangle raster setup exactly as draw_triangle_tile computes it (VS + clip_to_screen);
 * out: 9 floats per triangle (sx,sy,sz per corner), used by tests to build edge cases. */
int ora_screen_coords(int W, int H, const ora_draw *d, float *out9);

/* Canvas::barycentric_coordinate (shs_renderer.hpp:802-821) for a single point. */
void ora_barycentric(const float *tri6, float px, float py, float *out3);

/* GLM restatements used to build uniforms in tests (glm/gtc/matrix_transform.inl). */
void ora_mat4_inverse(const float *m, float *out);
void ora_mat4_mul(const float *a, const float *b, float *out);

/* 64-bit FNV-1a (demo_forward_classic_renderpath.cpp:1102-1116 pattern). */
uint64_t ora_fnv1a64(const void *data, uint64_t nbytes);

/* ===== Library path (shs_oracle_lib.c): shs-renderer-lib/include/shs/ ======================== */

enum ora_program {                 /* the ShaderProgram the pass binds (pass_pbr_forward.hpp:100-108) */
    ORA_PROGRAM_PBR_MR = 0,        /* make_pbr_mr_program       shader/builtin_shaders.hpp:154-214 */
    ORA_PROGRAM_BLINN_PHONG = 1,   /* make_blinn_phong_program  :105-152                          */
    ORA_PROGRAM_DEBUG_ALBEDO = 2,  /* make_debug_view_shader_program(Albedo|Normal|Depth) :221-245 */
    ORA_PROGRAM_DEBUG_NORMAL = 3,
    ORA_PROGRAM_DEBUG_DEPTH = 4,
    ORA_PROGRAM_FORWARD_PLUS = 5   /* per-pixel point lights from the tile lists (shs_oracle_light.c) */
};

/* CullingLightGPU (include/shs/lighting/light_types.hpp:141-166), 160 B */
typedef struct ora_culling_light {
    float position_range[4], color_intensity[4], direction_spot[4], axis_spot_outer[4], up_shape_x[4];
    float shape_attenuation[4];
    uint32_t type_shape_flags[4];
    float cull_sphere[4], cull_aabb_min[4], cull_aabb_max[4];
} ora_culling_light;

/* The CameraUBO fields fp_stress_light_cull.comp / fp_stress_depth_reduce.comp read. */
typedef struct ora_light_cull_desc {
    int32_t width, height;
    uint32_t tile_size, max_per_tile, mode, z_slices;   /* mode: 0 none, 1 tiled, 2 tiled depth range, 3 clustered */
    float view[16], proj[16];
    float zn, zf;
    int32_t depth_linear;                               /* depth input holds linear view depth (library RT) */
} ora_light_cull_desc;
enum ora_cull { ORA_CULL_NONE = 0, ORA_CULL_BACK = 1, ORA_CULL_FRONT = 2 };  /* RasterizerCullMode */

/* MeshData (resources/mesh.hpp:23-43): vec3 positions / normals, vec2 uvs, u32 indices (NULL:
 * non-indexed soup, 3 consecutive positions per triangle).  Normals / uvs may be shorter than
 * positions: missing entries read as (0,1,0) / (0,0) (rasterizer.hpp:196-202). */
typedef struct ora_mesh {
    const float *positions;
    const float *normals;
    const float *uvs;
    int32_t n_verts, n_normals, n_uvs;
    const uint32_t *indices;
    int64_t n_indices;
} ora_mesh;

/* One rasterize_mesh call: mesh + the ShaderUniforms fields the builtin programs read
 * (shader/types.hpp:87-116) + RasterizerConfig's cull mode / front face (rasterizer.hpp:33-40). */
typedef struct ora_lib_draw {
    ora_mesh mesh;
    int32_t program, cull_mode, front_face_ccw, shadow;  /* shadow: u.shadow_map != nullptr */
    float model[16], viewproj[16], prev_model[16], prev_viewproj[16];
    float light_dir_ws[3], light_color[3], light_intensity, camera_pos[3];
    float base_color[3], metallic, roughness, ao;
    float light_viewproj[16];
    float shadow_bias_const, shadow_bias_slope;
    int32_t shadow_pcf_radius;
    float shadow_pcf_step, shadow_strength;
    int32_t enable_motion_vectors;
    /* u.base_color_tex (shader/types.hpp:105): Texture2DData texels (Color RGBA8, y * w + x), NULL = none */
    const uint8_t *base_color_tex;
    int32_t tex_w, tex_h;
} ora_lib_draw;

/* RasterizerTarget: hdr (RT_ColorHDR, W*H*4 floats, rows y-up) and optionally depth_motion
 * (RT_ColorDepthMotion depth W*H + motion W*H*2; NULL depth = no depth test).  The shadow map the
 * programs sample (RT_ShadowDepth, shadow_w*shadow_h).  bg_gradient: PassPBRForward's no-sky
 * background (pass_pbr_forward.hpp:71-84), else clear_hdr. */
typedef struct ora_lib_target {
    int32_t W, H;
    float zn, zf;
    int32_t bg_gradient;
    float clear_hdr[4];
    float *hdr, *depth, *motion;
    const float *shadow;
    int32_t shadow_w, shadow_h;
    /* ORA_PROGRAM_FORWARD_PLUS: the light set and the lists of ora_light_cull with this desc */
    const ora_culling_light *lights;
    int32_t n_lights;
    const uint32_t *tile_counts, *tile_indices;
    const ora_light_cull_desc *cull;
} ora_lib_target;

typedef struct ora_shadow_caster {   /* RenderItem with casts_shadow (scene/scene_types.hpp:78-87) */
    ora_mesh mesh;
    float model[16];
} ora_shadow_caster;

/* rasterize_mesh (sw_render/rasterizer.hpp:181-442); stats3 += {tri_input, tri_after_clip, tri_raster} */
void ora_rasterize_mesh(const ora_lib_target *t, const ora_lib_draw *d, uint64_t *stats3);
/* PassPBRForward::execute (passes/pass_pbr_forward.hpp:49-214): clears + one rasterize_mesh per draw */
int ora_pbr_forward(const ora_lib_target *t, const ora_lib_draw *draws, int n_draws, uint64_t *stats3);
/* sample_texture2d_bilinear_repeat_linear (builtin_shaders.hpp:33-55) over rgba (w x h Color texels) */
void ora_sample_texture(const uint8_t *rgba, int32_t w, int32_t h, float u, float v, float out3[3]);
/* Threads for rasterize_mesh's row-parallel split of big bboxes (rasterizer.hpp:424-436; default 1). */
void ora_set_lib_threads(int n);
/* PassShadowMap::execute (passes/pass_shadow_map.hpp:44-206) into sm[SW*SH]; returns the light viewproj */
int ora_shadow_map(int SW, int SH, const float *sun_dir3, const ora_shadow_caster *casters, int n_casters, float *sm,
                   float *light_viewproj_out);
/* build_dir_light_camera_aabb (camera/light_camera.hpp:33-98) */
void ora_dir_light_camera_aabb(const float *sun_dir3, const float *mn3, const float *mx3, float extra_margin,
                               uint32_t res, float *view, float *proj, float *viewproj);
void ora_look_at_lh(const float *eye3, const float *center3, const float *up3, float *out16);

/* Light lists (shs_oracle_light.c).  ora_light_project: per light {cx, cy, radius_px, view_depth,
 * cull radius, 0, 0, valid} (project_light_screen, tile independent).  ora_depth_reduce: per tile
 * (min, max) linear view depth of depth[W*H] (rows y-up), (0,0) when empty.  ora_light_cull: counts
 * per list and max_per_tile indices per list (ranges2 used by mode 2). */
void ora_light_project(const ora_light_cull_desc *d, const ora_culling_light *lights, int n, float *out8);
void ora_depth_reduce(const ora_light_cull_desc *d, const float *depth, float *ranges2);
void ora_light_cull(const ora_light_cull_desc *d, const ora_culling_light *lights, int n, const float *ranges2,
                    uint32_t *counts, uint32_t *indices);
void ora_point_light_accumulate(const ora_culling_light *L, const float *world, const float *N, const float *V,
                                const float *base, float *lit);
float ora_mat4_determinant(const float *m);

/* PassTonemap (passes/pass_tonemap.hpp:36-83) + upload_ldr_to_rgba8 (exp-plumbing/hello_pass_basics.cpp:102-119):
 * hdr W*H*4 floats (rows y up) -> ldr (rows y up) and / or present (rows top-down), W*H*4 bytes. */
uint8_t ora_tonemap_channel(float s, float exposure, float inv_gamma);
void ora_tonemap(const float *hdr, int W, int H, float exposure, float gamma, uint8_t *ldr, uint8_t *present);
/* PassMotionBlur (passes/pass_motion_blur.hpp:38-170): src / dst W*H*4 bytes, depth W*H, motion W*H*2
 * (all rows y up). */
void ora_motion_blur(const uint8_t *src, const float *depth, const float *motion, int W, int H, int enable,
                     int samples, float strength, float max_velocity_px, float min_velocity_px, float depth_reject,
                     float dt, uint8_t *dst);

/* culling_sw::run_software_occlusion_pass (geometry/culling_software.hpp:229-331) as scene_culling.hpp
 * :187-219 drives it.  One object: an indexed DebugMesh (positions xyz, indices) + model + world AABB.
 * Writes occluded[n_objects] (0 for objects not frustum-visible), visible_out (sorted visit order),
 * depth W*H (rows as the reference indexes them: y * W + x); returns the visible count. */
typedef struct ora_occ_object {
    const float *pos;
    int32_t n_verts;
    const uint32_t *idx;
    int32_t n_idx;
    float model[16];
    float aabb_min[3], aabb_max[3];
} ora_occ_object;
int ora_occlusion_pass(const ora_occ_object *objs, int n_objects, const uint32_t *frustum_visible, int n_fv, int enable,
                       float *depth, int W, int H, const float *view16, const float *vp16, float eps,
                       uint8_t *occluded, uint32_t *visible_out);

#ifdef __cplusplus
}
#endif

/* shs_oracle_camera.c: Camera3D::update / glm::perspectiveLH / glm::lookAtLH / the monkey model
 * matrix and the legacy MVP, restated independently of the product's host helpers. */
void ora_camera3d(const float pos[3], float horizontal_angle, float vertical_angle, float fov, float zn, float zf,
                  float view16[16], float proj16[16]);
void ora_model_trs(const float pos[3], float rot_deg_y, const float scl[3], float out16[16]);
void ora_perspective_lh_no(float fovy, float aspect, float zn, float zf, float out16[16]);
void ora_legacy_mvp(const float view16[16], const float proj16[16], const float model16[16], int flat, float mvp16[16],
                    float mv16[16]);

/* shs_oracle_lightbin.c: build_light_bin_culling (light_culling_runtime.hpp:266-371) over lights given as
 * world AABBs (min xyz, max xyz per light: SceneShape::world_aabb()).  Lists: counts[bin] (all matches)
 * and indices[bin * max_per_bin + k] (the first max_per_bin, ascending); bins tile-row-major, clusters
 * slice-major; bins_xyz = (bins_x, bins_y, bins_z), all 0 for mode None / no lights. */
typedef struct ora_light_bin_desc {
    int32_t width, height;
    uint32_t tile_size, mode, z_slices, max_per_bin;
    float view_proj[16];
    float z_near, z_far;
    const float *tile_min_view_depth, *tile_max_view_depth;   /* mode 2, tiles_x * tiles_y each */
    int32_t n_depth_tiles;
} ora_light_bin_desc;
int ora_light_bin_culling(const ora_light_bin_desc *d, const float *aabbs, int n_lights, uint32_t *bins_xyz,
                          uint32_t *counts, uint32_t *indices);

/* shs_oracle_debugdraw.c: debug_draw::draw_filled_triangle (sw_render/debug_draw.hpp:60-109) and
 * draw_mesh_blinn_phong_transformed (:147-203).  rgba W*H*4 and depth W*H (y * W + x) in place;
 * tri_lit (may be NULL) 4 floats per triangle: lit rgb before the byte conversion (0 when culled
 * before shading), 1.0 when the triangle reaches the pixel loop.  Returns the triangle count. */
void ora_draw_filled_triangle(uint8_t *rgba, float *depth, int W, int H, const float *p0, float z0, const float *p1,
                              float z1, const float *p2, float z2, const uint8_t *c);
typedef struct ora_dd_mesh {
    const float *pos;
    int32_t n_verts;
    const uint32_t *idx;
    int32_t n_idx;
    float model[16];
    float base[3];
} ora_dd_mesh;
int ora_debug_draw_meshes(const ora_dd_mesh *meshes, int n_meshes, int W, int H, const float *vp, const float *cam,
                          const float *light_dir, uint8_t *rgba, float *depth, float *tri_lit);

/* shs_oracle_canvas_post.c: the Canvas-API multi-pass extras (hello-render-target/hello_pbr.cpp:1051-1252,
 * hello_depth_of_field.cpp:175-343, 786-812).  Colours 4 bytes per pixel, buffers y * W + x. */
void ora_canvas_motion_blur(const uint8_t *src, const float *depth, const float *vel, uint8_t *dst, int W, int H,
                            const float *curr_view, const float *curr_proj, const float *prev_view,
                            const float *prev_proj, int samples, float strength, float w_obj, float w_cam,
                            int soft_knee, float knee, float max_px);
void ora_canvas_gaussian(const uint8_t *src, uint8_t *dst, int W, int H, int horizontal);
float ora_canvas_autofocus(const float *depth, int W, int H, int cx, int cy, int radius);
float ora_canvas_dof(uint8_t *color, const float *depth, uint8_t *blur_out, int W, int H, int iterations, int radius,
                     int cx, int cy, float range, float max_blur);

#endif
