/*
 * shs_oracle.c -- CPU restatement (oracle) of the shs_renderer legacy scan-conversion path.
 *
 * TEST INFRASTRUCTURE ONLY (see shs_oracle.h).  PARITY UNPINNED (no reference golden vectors).
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off, no -ffast-math), output in oracle/_build/.
 *
 * Every function cites the reference line it restates.  Paths are relative to
 * /root/reference/cpp-folders/src/.
 */
#include "shs_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

/* ---- GLM scalar semantics (glm/detail/func_common.inl) --------------------------------- */
static inline float g_min(float x, float y) { return (y < x) ? y : x; }   /* glm::min */
static inline float g_max(float x, float y) { return (x < y) ? y : x; }   /* glm::max */
static inline float g_clamp(float x, float lo, float hi) { return g_min(g_max(x, lo), hi); }

/* glm::dot: tmp = a*b; (tmp.x + tmp.y) + tmp.z  (func_geometric.inl compute_dot) */
static inline float dot3(v3 a, v3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
static inline float dot2(v2 a, v2 b) { float x = a.x * b.x, y = a.y * b.y; return x + y; }
static inline v3 v3s(v3 a, float s) { v3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static inline v3 v3add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static inline v3 v3sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static inline v3 v3mul(v3 a, v3 b) { v3 r = {a.x * b.x, a.y * b.y, a.z * b.z}; return r; }
/* glm::normalize: v * inversesqrt(dot(v,v)), inversesqrt(x) = 1/sqrt(x) */
static inline v3 normalize3(v3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return v3s(v, inv); }

/* glm mat4 * vec4: (m0*v.x + m1*v.y) + (m2*v.z + m3*v.w)  (type_mat4x4.inl operator*) */
static inline v4 m4v4(const float *m, v4 v) {
    v4 r;
    r.x = (m[0] * v.x + m[4] * v.y) + (m[8] * v.z + m[12] * v.w);
    r.y = (m[1] * v.x + m[5] * v.y) + (m[9] * v.z + m[13] * v.w);
    r.z = (m[2] * v.x + m[6] * v.y) + (m[10] * v.z + m[14] * v.w);
    r.w = (m[3] * v.x + m[7] * v.y) + (m[11] * v.z + m[15] * v.w);
    return r;
}
/* glm mat3 * vec3: m[0][r]*x + m[1][r]*y + m[2][r]*z  (type_mat3x3.inl); m3 is column-major [9] */
static inline v3 m3v3(const float *m, v3 v) {
    v3 r;
    r.x = m[0] * v.x + m[3] * v.y + m[6] * v.z;
    r.y = m[1] * v.x + m[4] * v.y + m[7] * v.z;
    r.z = m[2] * v.x + m[5] * v.y + m[8] * v.z;
    return r;
}

/* glm::inverse for mat4 (detail/func_matrix.inl compute_inverse<4,4>) */
void ora_mat4_inverse(const float *mm, float *out) {
#define M(c, r) mm[(c) * 4 + (r)]
    float c00 = M(2,2) * M(3,3) - M(3,2) * M(2,3);
    float c02 = M(1,2) * M(3,3) - M(3,2) * M(1,3);
    float c03 = M(1,2) * M(2,3) - M(2,2) * M(1,3);
    float c04 = M(2,1) * M(3,3) - M(3,1) * M(2,3);
    float c06 = M(1,1) * M(3,3) - M(3,1) * M(1,3);
    float c07 = M(1,1) * M(2,3) - M(2,1) * M(1,3);
    float c08 = M(2,1) * M(3,2) - M(3,1) * M(2,2);
    float c10 = M(1,1) * M(3,2) - M(3,1) * M(1,2);
    float c11 = M(1,1) * M(2,2) - M(2,1) * M(1,2);
    float c12 = M(2,0) * M(3,3) - M(3,0) * M(2,3);
    float c14 = M(1,0) * M(3,3) - M(3,0) * M(1,3);
    float c15 = M(1,0) * M(2,3) - M(2,0) * M(1,3);
    float c16 = M(2,0) * M(3,2) - M(3,0) * M(2,2);
    float c18 = M(1,0) * M(3,2) - M(3,0) * M(1,2);
    float c19 = M(1,0) * M(2,2) - M(2,0) * M(1,2);
    float c20 = M(2,0) * M(3,1) - M(3,0) * M(2,1);
    float c22 = M(1,0) * M(3,1) - M(3,0) * M(1,1);
    float c23 = M(1,0) * M(2,1) - M(2,0) * M(1,1);
    float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    float vv0[4] = {M(1,0), M(0,0), M(0,0), M(0,0)};
    float vv1[4] = {M(1,1), M(0,1), M(0,1), M(0,1)};
    float vv2[4] = {M(1,2), M(0,2), M(0,2), M(0,2)};
    float vv3[4] = {M(1,3), M(0,3), M(0,3), M(0,3)};
    float inv[4][4];
    const float sa[4] = {+1.f, -1.f, +1.f, -1.f}, sb[4] = {-1.f, +1.f, -1.f, +1.f};
    for (int i = 0; i < 4; ++i) {
        float i0 = (vv1[i] * f0[i] - vv2[i] * f1[i]) + vv3[i] * f2[i];
        float i1 = (vv0[i] * f0[i] - vv2[i] * f3[i]) + vv3[i] * f4[i];
        float i2 = (vv0[i] * f1[i] - vv1[i] * f3[i]) + vv3[i] * f5[i];
        float i3 = (vv0[i] * f2[i] - vv1[i] * f4[i]) + vv2[i] * f5[i];
        inv[0][i] = i0 * sa[i];
        inv[1][i] = i1 * sb[i];
        inv[2][i] = i2 * sa[i];
        inv[3][i] = i3 * sb[i];
    }
    float d0 = M(0,0) * inv[0][0], d1 = M(0,1) * inv[1][0], d2 = M(0,2) * inv[2][0], d3 = M(0,3) * inv[3][0];
    float det = (d0 + d1) + (d2 + d3);
    float one_over = 1.0f / det;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = inv[c][r] * one_over;
#undef M
}

/* glm mat4 * mat4: Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3] */
void ora_mat4_mul(const float *a, const float *b, float *out) {
    float t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) + a[2 * 4 + r] * b[c * 4 + 2]) +
                           a[3 * 4 + r] * b[c * 4 + 3];
    memcpy(out, t, sizeof t);
}

uint64_t ora_fnv1a64(const void *data, uint64_t n) {
    const uint8_t *p = (const uint8_t *)data;
    uint64_t h = 1469598103934665603ULL;
    for (uint64_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

/* ---- shs_renderer primitives -------------------------------------------------------------- */

/* Canvas::clip_to_screen (shs_renderer.hpp:823-831) */
static inline v3 clip_to_screen(v4 c, int W, int H) {
    v3 ndc = {c.x / c.w, c.y / c.w, c.z / c.w};
    v3 s;
    s.x = (ndc.x + 1.0f) * 0.5f * (float)(W - 1);
    s.y = (1.0f - ndc.y) * 0.5f * (float)(H - 1);
    s.z = ndc.z;
    return s;
}

/* Canvas::barycentric_coordinate (shs_renderer.hpp:802-821).  Note the float-vs-double compare. */
static inline v3 barycentric(v2 P, v2 A, v2 B, v2 C) {
    v2 v0 = {B.x - A.x, B.y - A.y};
    v2 v1 = {C.x - A.x, C.y - A.y};
    v2 vp = {P.x - A.x, P.y - A.y};
    float d00 = dot2(v0, v0), d01 = dot2(v0, v1), d11 = dot2(v1, v1);
    float d20 = dot2(vp, v0), d21 = dot2(vp, v1);
    float denom = d00 * d11 - d01 * d01;
    if ((double)fabsf(denom) < 1e-5) { v3 r = {-1.f, -1.f, -1.f}; return r; }
    float v = (d11 * d20 - d01 * d21) / denom;
    float w = (d00 * d21 - d01 * d20) / denom;
    float u = 1.0f - v - w;
    v3 r = {u, v, w};
    return r;
}

void ora_barycentric(const float *t, float px, float py, float *o) {
    v2 P = {px, py}, A = {t[0], t[1]}, B = {t[2], t[3]}, C = {t[4], t[5]};
    v3 r = barycentric(P, A, B, C);
    o[0] = r.x; o[1] = r.y; o[2] = r.z;
}

typedef struct {
    v4 position;
    v3 normal;
    v3 world_pos;   /* Gouraud smuggles its colour through world_pos (gouraud_shading.cpp:71) */
} varyings;

/* normal matrix mat3(transpose(inverse(model))) -- recomputed per vertex exactly as the
 * reference shaders do (blinn_phong_shading.cpp:54) */
static inline void normal_matrix(const float *model, float *n3) {
    float inv[16];
    ora_mat4_inverse(model, inv);
    /* mat3(transpose(inv))[c][r] = inv[r][c] */
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) n3[c * 3 + r] = inv[r * 4 + c];
}

static inline v3 pos_of(const float *p) { v3 r = {p[0], p[1], p[2]}; return r; }

/* Vertex shaders ---------------------------------------------------------------------------- */
static varyings vertex_shader(const ora_draw *d, v3 p, v3 n) {
    varyings o;
    v4 p4 = {p.x, p.y, p.z, 1.0f};
    o.position = m4v4(d->mvp, p4);
    if (d->shading == ORA_FLAT) {
        /* flat_shading.cpp:46-61: normal = mat3(mv) * n (no normalize) */
        float m3[9];
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) m3[c * 3 + r] = d->model[c * 4 + r];
        o.normal = m3v3(m3, n);
        o.world_pos.x = o.world_pos.y = o.world_pos.z = 0.0f;
        return o;
    }
    v4 w4 = m4v4(d->model, p4);
    v3 world = {w4.x, w4.y, w4.z};
    float n3[9];
    normal_matrix(d->model, n3);
    v3 nrm = normalize3(m3v3(n3, n));
    if (d->shading == ORA_GOURAUD) {
        /* gouraud_shading.cpp:46-77: Blinn-Phong lighting per vertex, shininess 32 */
        v3 neg = {-d->light_dir[0], -d->light_dir[1], -d->light_dir[2]};
        v3 lightDir = normalize3(neg);
        v3 cam = {d->camera_pos[0], d->camera_pos[1], d->camera_pos[2]};
        v3 viewDir = normalize3(v3sub(cam, world));
        float ambient = 0.15f * 1.0f;
        float diff = g_max(dot3(nrm, lightDir), 0.0f);
        v3 halfway = normalize3(v3add(lightDir, viewDir));
        float spec = powf(g_max(dot3(nrm, halfway), 0.0f), 32.0f);
        float specular = (0.5f * spec) * 1.0f;
        v3 ocol = {(float)d->color[0] / 255.0f, (float)d->color[1] / 255.0f, (float)d->color[2] / 255.0f};
        float s = (ambient + diff * 1.0f) + specular;
        v3 fc = {s * ocol.x, s * ocol.y, s * ocol.z};
        fc.x = g_clamp(fc.x, 0.0f, 1.0f); fc.y = g_clamp(fc.y, 0.0f, 1.0f); fc.z = g_clamp(fc.z, 0.0f, 1.0f);
        o.world_pos = fc;
        o.normal = nrm;
        return o;
    }
    o.world_pos = world;
    o.normal = nrm;
    return o;
}

/* Fragment shaders: return pre-truncation floats (r,g,b) and the uint8 colour --------------- */
static inline uint8_t trunc_u8(float x) { return (uint8_t)x; }

static void fragment_shader(const ora_draw *d, v3 in_normal, v3 in_world, float *pre, uint8_t *rgba) {
    if (d->shading == ORA_FLAT) {
        /* flat_shading.cpp:69-98 */
        v3 n = normalize3(in_normal);
        v3 ld = {d->light_dir[0], d->light_dir[1], d->light_dir[2]};
        v3 l = normalize3(ld);
        float diffuse = g_max(dot3(n, l), 0.0f);
        float intensity = 0.2f + diffuse;
        if (intensity > 1.0f) intensity = 1.0f;
        pre[0] = (float)d->color[0] * intensity;
        pre[1] = (float)d->color[1] * intensity;
        pre[2] = (float)d->color[2] * intensity;
    } else if (d->shading == ORA_GOURAUD) {
        /* gouraud_shading.cpp:80-89 */
        pre[0] = in_world.x * 255.0f;
        pre[1] = in_world.y * 255.0f;
        pre[2] = in_world.z * 255.0f;
    } else {
        v3 norm = normalize3(in_normal);
        v3 neg = {-d->light_dir[0], -d->light_dir[1], -d->light_dir[2]};
        v3 lightDir = normalize3(neg);
        v3 cam = {d->camera_pos[0], d->camera_pos[1], d->camera_pos[2]};
        v3 viewDir = normalize3(v3sub(cam, in_world));
        float ambient = 0.15f * 1.0f;
        float diff = g_max(dot3(norm, lightDir), 0.0f);
        float specular;
        if (d->shading == ORA_PHONG) {
            /* phong_shading.cpp:70-108: reflect(-L, N) = I - N*dot(N,I)*2; pow(float,int)
             * resolves to std::pow(double,double) (int shininess), narrowed to float */
            v3 I = {-lightDir.x, -lightDir.y, -lightDir.z};
            float dn = dot3(norm, I);
            v3 t = v3s(v3s(norm, dn), 2.0f);
            v3 reflectDir = v3sub(I, t);
            float spec = (float)pow((double)g_max(dot3(viewDir, reflectDir), 0.0f), 32.0);
            specular = (0.8f * spec) * 1.0f;
        } else {
            /* blinn_phong_shading.cpp:63-97: powf(max(N.H,0), 64) */
            v3 halfway = normalize3(v3add(lightDir, viewDir));
            float spec = powf(g_max(dot3(norm, halfway), 0.0f), 64.0f);
            specular = (0.5f * spec) * 1.0f;
        }
        v3 ocol = {(float)d->color[0] / 255.0f, (float)d->color[1] / 255.0f, (float)d->color[2] / 255.0f};
        float s = (ambient + diff * 1.0f) + specular;
        v3 res = {s * ocol.x, s * ocol.y, s * ocol.z};
        res.x = g_clamp(res.x, 0.0f, 1.0f); res.y = g_clamp(res.y, 0.0f, 1.0f); res.z = g_clamp(res.z, 0.0f, 1.0f);
        pre[0] = res.x * 255.0f;
        pre[1] = res.y * 255.0f;
        pre[2] = res.z * 255.0f;
    }
    rgba[0] = trunc_u8(pre[0]);
    rgba[1] = trunc_u8(pre[1]);
    rgba[2] = trunc_u8(pre[2]);
    rgba[3] = 255;
}

typedef struct {
    int W, H;
    uint8_t *color;
    float *depth;
    float *pre;
} target;

/* draw_triangle_tile (hello_pipeline_blinn_phong_shading.cpp:189-242; identical body in the
 * Phong :204, Gouraud :186-236 and Flat :194-247 pipelines; the interpolated varying differs) */
static void draw_triangle_tile(target *t, const ora_draw *d, const float *pos9, const float *nrm9,
                               int tminx, int tminy, int tmaxx, int tmaxy) {
    varyings vout[3];
    v3 sc[3];
    for (int i = 0; i < 3; ++i) {
        vout[i] = vertex_shader(d, pos_of(pos9 + 3 * i), pos_of(nrm9 + 3 * i));
        sc[i] = clip_to_screen(vout[i].position, t->W, t->H);
    }
    v2 bmin = {(float)tmaxx, (float)tmaxy};
    v2 bmax = {(float)tminx, (float)tminy};
    v2 v2d[3] = {{sc[0].x, sc[0].y}, {sc[1].x, sc[1].y}, {sc[2].x, sc[2].y}};
    for (int i = 0; i < 3; ++i) {
        bmin.x = g_max((float)tminx, g_min(bmin.x, v2d[i].x));
        bmin.y = g_max((float)tminy, g_min(bmin.y, v2d[i].y));
        bmax.x = g_min((float)tmaxx, g_max(bmax.x, v2d[i].x));
        bmax.y = g_min((float)tmaxy, g_max(bmax.y, v2d[i].y));
    }
    if (bmin.x > bmax.x || bmin.y > bmax.y) return;
    float area = (v2d[1].x - v2d[0].x) * (v2d[2].y - v2d[0].y) - (v2d[1].y - v2d[0].y) * (v2d[2].x - v2d[0].x);
    if (area <= 0) return;

    for (int px = (int)bmin.x; px <= (int)bmax.x; px++) {
        for (int py = (int)bmin.y; py <= (int)bmax.y; py++) {
            v2 P = {(float)px + 0.5f, (float)py + 0.5f};
            v3 bc = barycentric(P, v2d[0], v2d[1], v2d[2]);
            if (bc.x < 0 || bc.y < 0 || bc.z < 0) continue;
            float z = bc.x * sc[0].z + bc.y * sc[1].z + bc.z * sc[2].z;
            /* ZBuffer::test_and_set_depth (shs_renderer.hpp:660-670), screen-row indexing */
            if (px < 0 || px >= t->W || py < 0 || py >= t->H) continue;
            float *dz = &t->depth[(size_t)py * t->W + px];
            if (!(z < *dz)) continue;
            *dz = z;
            v3 in_n = {0, 0, 0}, in_w = {0, 0, 0};
            if (d->shading == ORA_GOURAUD) {
                in_w = v3add(v3add(v3s(vout[0].world_pos, bc.x), v3s(vout[1].world_pos, bc.y)), v3s(vout[2].world_pos, bc.z));
            } else {
                in_n = normalize3(v3add(v3add(v3s(vout[0].normal, bc.x), v3s(vout[1].normal, bc.y)), v3s(vout[2].normal, bc.z)));
                if (d->shading != ORA_FLAT)
                    in_w = v3add(v3add(v3s(vout[0].world_pos, bc.x), v3s(vout[1].world_pos, bc.y)), v3s(vout[2].world_pos, bc.z));
            }
            float pre[3];
            uint8_t rgba[4];
            fragment_shader(d, in_n, in_w, pre, rgba);
            /* Canvas::draw_pixel_screen_space (shs_renderer.hpp:792-796) */
            int yc = (t->H - 1) - py;
            if (yc < 0 || yc >= t->H) continue;
            size_t o = (size_t)yc * t->W + px;
            memcpy(&t->color[o * 4], rgba, 4);
            if (t->pre) { t->pre[o * 4 + 0] = pre[0]; t->pre[o * 4 + 1] = pre[1]; t->pre[o * 4 + 2] = pre[2]; t->pre[o * 4 + 3] = 1.0f; }
        }
    }
}

typedef struct {
    target *t;
    const ora_draw *draws;
    int n_draws, tile_w, tile_h, cols, rows;
    atomic_int next;
} job_ctx;

/* One tile job (hello_pipeline_blinn_phong_shading.cpp:266-308): objects outer, triangles inner */
static void run_tile(job_ctx *c, int tile) {
    int tx = tile % c->cols, ty = tile / c->cols;
    int tminx = tx * c->tile_w, tminy = ty * c->tile_h;
    int tmaxx = ((tx + 1) * c->tile_w < c->t->W ? (tx + 1) * c->tile_w : c->t->W) - 1;
    int tmaxy = ((ty + 1) * c->tile_h < c->t->H ? (ty + 1) * c->tile_h : c->t->H) - 1;
    for (int di = 0; di < c->n_draws; ++di) {
        const ora_draw *d = &c->draws[di];
        for (int i = 0; i < d->n_tris; ++i)
            draw_triangle_tile(c->t, d, d->positions + 9 * (size_t)i, d->normals + 9 * (size_t)i, tminx, tminy, tmaxx, tmaxy);
    }
}

static void *worker(void *arg) {
    job_ctx *c = (job_ctx *)arg;
    int n = c->cols * c->rows;
    for (;;) {
        int t = atomic_fetch_add(&c->next, 1);
        if (t >= n) break;
        run_tile(c, t);
    }
    return NULL;
}

/* The tile-job executor: worker threads created once and reused across frames, as the reference's
   ThreadedPriorityJobSystem (hello-shs-renderer/shs_renderer.hpp:1534-1564) keeps its workers for the
   whole run.  A frame publishes its job context, wakes the workers, and waits until each has drained the
   shared tile counter -- the reference's WaitGroup (:1597-1630); the submitting thread runs no tile,
   as the reference's render loop only waits.  (Until round 4 the threads were created and joined every
   frame, which at 256 threads cost more than the frame.) */
typedef struct {
    pthread_t th[256];
    int n;
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    unsigned gen;
    int busy, quit;
    job_ctx *job;
} tile_pool;
static tile_pool g_pool = {.mu = PTHREAD_MUTEX_INITIALIZER, .go = PTHREAD_COND_INITIALIZER, .done = PTHREAD_COND_INITIALIZER};
static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;

static void *pool_worker(void *arg) {
    unsigned seen = (unsigned)(uintptr_t)arg;   /* the generation at creation: later frames wake it */
    pthread_mutex_lock(&g_pool.mu);
    for (;;) {
        while (!g_pool.quit && g_pool.gen == seen) pthread_cond_wait(&g_pool.go, &g_pool.mu);
        if (g_pool.quit) break;
        seen = g_pool.gen;
        job_ctx *c = g_pool.job;
        pthread_mutex_unlock(&g_pool.mu);
        worker(c);
        pthread_mutex_lock(&g_pool.mu);
        if (--g_pool.busy == 0) pthread_cond_signal(&g_pool.done);
    }
    pthread_mutex_unlock(&g_pool.mu);
    return NULL;
}

/* (caller holds g_pool_lock) the pool with n workers; returns the workers running.  The request is
 * remembered apart from the count started: when pthread_create falls short (thread limits), later
 * frames with the same request keep the smaller pool instead of re-creating it every frame. */
static int g_pool_req = 0;
static int pool_resize(int n) {
    if (g_pool.n == n || (g_pool_req == n && g_pool.n > 0)) return g_pool.n;
    g_pool_req = n;
    pthread_mutex_lock(&g_pool.mu);
    g_pool.quit = 1;
    pthread_cond_broadcast(&g_pool.go);
    pthread_mutex_unlock(&g_pool.mu);
    for (int i = 0; i < g_pool.n; ++i) pthread_join(g_pool.th[i], NULL);
    g_pool.n = 0;
    g_pool.quit = 0;
    for (int i = 0; i < n; ++i) {
        if (pthread_create(&g_pool.th[i], NULL, pool_worker, (void *)(uintptr_t)g_pool.gen) != 0) break;
        g_pool.n++;
    }
    return g_pool.n;
}

/* (caller holds g_pool_lock) one frame's tiles over the pool */
static void pool_run(job_ctx *c) {
    pthread_mutex_lock(&g_pool.mu);
    g_pool.job = c;
    g_pool.busy = g_pool.n;
    g_pool.gen++;
    pthread_cond_broadcast(&g_pool.go);
    while (g_pool.busy > 0) pthread_cond_wait(&g_pool.done, &g_pool.mu);
    pthread_mutex_unlock(&g_pool.mu);
}

int ora_render_legacy(int W, int H, int tile_w, int tile_h, int n_threads, const ora_draw *draws, int n_draws,
                      uint8_t *color_out, float *depth_out, float *prequant_out) {
    if (W <= 0 || H <= 0 || tile_w <= 0 || tile_h <= 0 || !color_out || !depth_out) return -1;
    target t = {W, H, color_out, depth_out, prequant_out};
    /* Canvas::fill_pixel(black) (shs_renderer.hpp:859-866) + ZBuffer::clear (FLT_MAX, :677-680) */
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        color_out[i * 4 + 0] = 0; color_out[i * 4 + 1] = 0; color_out[i * 4 + 2] = 0; color_out[i * 4 + 3] = 255;
        depth_out[i] = FLT_MAX;
    }
    if (prequant_out) memset(prequant_out, 0, sizeof(float) * 4 * (size_t)W * H);
    job_ctx c;
    c.t = &t; c.draws = draws; c.n_draws = n_draws; c.tile_w = tile_w; c.tile_h = tile_h;
    c.cols = (W + tile_w - 1) / tile_w; c.rows = (H + tile_h - 1) / tile_h;
    atomic_init(&c.next, 0);
    if (n_threads <= 1) { worker(&c); return 0; }
    if (n_threads > 256) n_threads = 256;
    pthread_mutex_lock(&g_pool_lock);   /* one frame at a time on the pool */
    if (pool_resize(n_threads) == 0) worker(&c);   /* no thread could be started */
    else pool_run(&c);
    pthread_mutex_unlock(&g_pool_lock);
    return 0;
}

int ora_screen_coords(int W, int H, const ora_draw *d, float *out) {
    for (int i = 0; i < d->n_tris; ++i)
        for (int k = 0; k < 3; ++k) {
            const float *p = d->positions + 9 * (size_t)i + 3 * k, *n = d->normals + 9 * (size_t)i + 3 * k;
            varyings v = vertex_shader(d, pos_of(p), pos_of(n));
            v3 s = clip_to_screen(v.position, W, H);
            out[9 * (size_t)i + 3 * k + 0] = s.x; out[9 * (size_t)i + 3 * k + 1] = s.y; out[9 * (size_t)i + 3 * k + 2] = s.z;
        }
    return 0;
}
