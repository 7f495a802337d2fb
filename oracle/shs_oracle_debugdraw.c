/* shs_oracle_debugdraw.c -- TEST INFRASTRUCTURE ONLY (the checker of SURVEY.md 8f row 2's debug_draw
 * raster; never linked into the product).  A sequential CPU restatement of shs::debug_draw
 * (shs-renderer-lib/include/shs/sw_render/debug_draw.hpp, paths relative to
 * /root/reference/cpp-folders/src/):
 *   edge_fn (:35-37), project_world_to_screen (:40-58), draw_filled_triangle (:60-109),
 *   draw_mesh_blinn_phong_transformed (:147-203).
 * GLM op order as elsewhere in the oracle: mat4 * vec4 = (m0 x + m1 y) + (m2 z + m3 w), dot =
 * (x x + y y) + z z, normalize v * (1 / sqrt(dot)), cross (x.y y.z - y.y x.z, ...); glm::clamp =
 * min(max(x, lo), hi) with glm's (a < b) selections; std::pow(float, float) = powf. */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "shs_oracle.h"

static void dd_m4v(const float *m, float x, float y, float z, float w, float *o) {
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w);
}

static float dd_edge(const float *a, const float *b, const float *p) {
    return (p[0] - a[0]) * (b[1] - a[1]) - (p[1] - a[1]) * (b[0] - a[0]);
}

static int dd_project(const float *w, const float *vp, int W, int H, float *xy, float *z) {
    float c[4];
    dd_m4v(vp, w[0], w[1], w[2], 1.0f, c);
    if (c[3] <= 0.001f) return 0;
    const float n[3] = {c[0] / c[3], c[1] / c[3], c[2] / c[3]};
    if (n[2] < -1.0f || n[2] > 1.0f) return 0;
    xy[0] = (n[0] + 1.0f) * 0.5f * (float)W;
    xy[1] = (n[1] + 1.0f) * 0.5f * (float)H;
    *z = n[2] * 0.5f + 0.5f;
    return 1;
}

static float dd_min(float a, float b) { return (b < a) ? b : a; }
static float dd_max(float a, float b) { return (a < b) ? b : a; }
static float dd_dot(const float *a, const float *b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static void dd_normalize(float *v) {
    const float s = 1.0f / sqrtf(dd_dot(v, v));
    v[0] *= s; v[1] *= s; v[2] *= s;
}
static uint8_t dd_u8(float v) {   /* static_cast<uint8_t>(std::clamp(v * 255, 0, 255)) */
    const float s = v * 255.0f;
    const float c = (s < 0.0f) ? 0.0f : ((255.0f < s) ? 255.0f : s);
    return (uint8_t)c;
}

void ora_draw_filled_triangle(uint8_t *rgba, float *depth, int W, int H, const float *p0, float z0, const float *p1,
                              float z1, const float *p2, float z2, const uint8_t *c) {
    const float area = dd_edge(p0, p1, p2);
    if (fabsf(area) <= 1e-6f) return;
    const float min_xf = dd_min(p0[0], dd_min(p1[0], p2[0])), min_yf = dd_min(p0[1], dd_min(p1[1], p2[1]));
    const float max_xf = dd_max(p0[0], dd_max(p1[0], p2[0])), max_yf = dd_max(p0[1], dd_max(p1[1], p2[1]));
    int min_x = (int)floorf(min_xf), min_y = (int)floorf(min_yf);
    int max_x = (int)ceilf(max_xf), max_y = (int)ceilf(max_yf);
    if (min_x < 0) min_x = 0;
    if (min_y < 0) min_y = 0;
    if (max_x > W - 1) max_x = W - 1;
    if (max_y > H - 1) max_y = H - 1;
    if (min_x > max_x || min_y > max_y) return;
    const int ccw = area > 0.0f;
    for (int y = min_y; y <= max_y; ++y)
        for (int x = min_x; x <= max_x; ++x) {
            const float p[2] = {(float)x + 0.5f, (float)y + 0.5f};
            const float w0 = dd_edge(p1, p2, p), w1 = dd_edge(p2, p0, p), w2 = dd_edge(p0, p1, p);
            const int inside = ccw ? (w0 >= 0.0f && w1 >= 0.0f && w2 >= 0.0f) : (w0 <= 0.0f && w1 <= 0.0f && w2 <= 0.0f);
            if (!inside) continue;
            const float iw0 = w0 / area, iw1 = w1 / area, iw2 = w2 / area;
            const float d = iw0 * z0 + iw1 * z1 + iw2 * z2;
            if (d < 0.0f || d > 1.0f) continue;
            const size_t di = (size_t)y * (size_t)W + (size_t)x;
            if (d < depth[di]) {
                depth[di] = d;
                memcpy(rgba + 4 * di, c, 4);
            }
        }
}

int ora_debug_draw_meshes(const ora_dd_mesh *meshes, int n_meshes, int W, int H, const float *vp, const float *cam,
                          const float *light_dir, uint8_t *rgba, float *depth, float *tri_lit) {
    float L[3] = {-light_dir[0], -light_dir[1], -light_dir[2]};
    dd_normalize(L);
    int g = 0;
    for (int m = 0; m < n_meshes; ++m) {
        const ora_dd_mesh *o = &meshes[m];
        for (int i = 0; i + 2 < o->n_idx; i += 3, ++g) {
            float *lit_out = tri_lit ? tri_lit + 4 * (size_t)g : NULL;
            if (lit_out) lit_out[0] = lit_out[1] = lit_out[2] = lit_out[3] = 0.0f;
            float p[3][3], s[3][2], z[3] = {1.0f, 1.0f, 1.0f};
            int ok = 1;
            for (int k = 0; k < 3; ++k) {
                const uint32_t id = o->idx[i + k];
                if (id >= (uint32_t)o->n_verts) { ok = 0; break; }   /* the reference indexes out of range (UB) */
                const float *lp = o->pos + 3 * (size_t)id;
                float c[4];
                dd_m4v(o->model, lp[0], lp[1], lp[2], 1.0f, c);
                p[k][0] = c[0]; p[k][1] = c[1]; p[k][2] = c[2];
            }
            if (!ok) continue;
            for (int k = 0; k < 3 && ok; ++k) ok = dd_project(p[k], vp, W, H, s[k], &z[k]);
            if (!ok) continue;
            const float a[3] = {p[2][0] - p[0][0], p[2][1] - p[0][1], p[2][2] - p[0][2]};
            const float b[3] = {p[1][0] - p[0][0], p[1][1] - p[0][1], p[1][2] - p[0][2]};
            float n[3] = {a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]};
            if (dd_dot(n, n) <= 1e-10f) continue;
            dd_normalize(n);
            const float third = 1.0f / 3.0f;
            float V[3], Hh[3];
            for (int k = 0; k < 3; ++k) {
                const float centroid = ((p[0][k] + p[1][k]) + p[2][k]) * third;
                V[k] = cam[k] - centroid;
            }
            dd_normalize(V);
            for (int k = 0; k < 3; ++k) Hh[k] = L[k] + V[k];
            dd_normalize(Hh);
            const float ndotl = dd_max(0.0f, dd_dot(n, L));
            const float ndoth = dd_max(0.0f, dd_dot(n, Hh));
            const float diffuse = 0.72f * ndotl;
            const float specular = (ndotl > 0.0f) ? (0.35f * powf(ndoth, 32.0f)) : 0.0f;
            float lit[3];
            uint8_t col[4];
            for (int k = 0; k < 3; ++k) {
                const float v = o->base[k] * (0.18f + diffuse) + specular;
                const float mx = (v < 0.0f) ? 0.0f : v;        /* glm::max(x, 0) */
                lit[k] = (1.0f < mx) ? 1.0f : mx;              /* glm::min(., 1) */
                col[k] = dd_u8(lit[k]);
            }
            col[3] = 255;
            if (lit_out) {
                lit_out[0] = lit[0]; lit_out[1] = lit[1]; lit_out[2] = lit[2];
                const float area = dd_edge(s[0], s[1], s[2]);
                lit_out[3] = fabsf(area) <= 1e-6f ? 0.0f : 1.0f;
            }
            ora_draw_filled_triangle(rgba, depth, W, H, s[0], z[0], s[1], z[1], s[2], z[2], col);
        }
    }
    return g;
}
