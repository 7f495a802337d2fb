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

#ifdef __cplusplus
}
#endif
#endif
