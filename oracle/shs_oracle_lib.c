/*
 * shs_oracle_lib.c -- CPU restatement (oracle) of the shs-renderer-lib software raster path:
 * rasterize_mesh, the builtin PBR / Blinn-Phong / debug programs, the shadow-map pass and the
 * directional shadow sampling.
 *
 * TEST INFRASTRUCTURE ONLY (see shs_oracle.h).  PARITY UNPINNED (no reference golden vectors; glm
 * operation order restated from GLM's published headers, unversioned in the reference build).
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off, no -ffast-math).
 *
 * Paths below are relative to /root/reference/cpp-folders/src/shs-renderer-lib/include/shs/.
 */
#include "shs_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

#define PI_F 3.14159265358979323846264338327950288f   /* glm::pi<float>() */

/* ---- GLM / std scalar semantics -------------------------------------------------------------- */
static inline float g_min(float x, float y) { return (y < x) ? y : x; }        /* glm::min   */
static inline float g_max(float x, float y) { return (x < y) ? y : x; }        /* glm::max   */
static inline float g_clamp(float x, float lo, float hi) { return g_min(g_max(x, lo), hi); }  /* glm::clamp */
static inline float s_max(float a, float b) { return (a < b) ? b : a; }        /* std::max(a, b) */
static inline float s_min(float a, float b) { return (b < a) ? b : a; }        /* std::min(a, b) */
static inline float s_clamp(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }  /* std::clamp */
static inline int s_clampi(int v, int lo, int hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }
/* glm::mix(x, y, a) = x * (1 - a) + y * a (func_common.inl compute_mix) */
static inline float g_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline float dot3(v3 a, v3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
static inline v3 v3s(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 v3add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v3sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v3mul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 v3neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline v3 normalize3(v3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return v3s(v, inv); }
static inline v3 v3mix(v3 a, v3 b, float t) { return V3(g_mix(a.x, b.x, t), g_mix(a.y, b.y, t), g_mix(a.z, b.z, t)); }
static inline v3 v3gmax(v3 a, v3 b) { return V3(g_max(a.x, b.x), g_max(a.y, b.y), g_max(a.z, b.z)); }
/* glm::reflect(I, N) = I - N * dot(N, I) * 2 */
static inline v3 reflect3(v3 I, v3 N) { return v3sub(I, v3s(v3s(N, dot3(N, I)), 2.0f)); }

/* glm mat4 * vec4 (type_mat4x4.inl): (m0*x + m1*y) + (m2*z + m3*w) */
static inline v4 m4v4(const float *m, v4 v) {
    v4 r;
    r.x = (m[0] * v.x + m[4] * v.y) + (m[8] * v.z + m[12] * v.w);
    r.y = (m[1] * v.x + m[5] * v.y) + (m[9] * v.z + m[13] * v.w);
    r.z = (m[2] * v.x + m[6] * v.y) + (m[10] * v.z + m[14] * v.w);
    r.w = (m[3] * v.x + m[7] * v.y) + (m[11] * v.z + m[15] * v.w);
    return r;
}
/* glm mat3 * vec3 (type_mat3x3.inl), m column-major [9] */
static inline v3 m3v3(const float *m, v3 v) {
    return V3(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z, m[2] * v.x + m[5] * v.y + m[8] * v.z);
}

/* glm::determinant(mat3) (func_matrix.inl compute_determinant<3,3>) */
static float det3(const float *m) {
#define M3(c, r) m[(c) * 3 + (r)]
    return (M3(0,0) * (M3(1,1) * M3(2,2) - M3(2,1) * M3(1,2))
          - M3(1,0) * (M3(0,1) * M3(2,2) - M3(2,1) * M3(0,2)))
          + M3(2,0) * (M3(0,1) * M3(1,2) - M3(1,1) * M3(0,2));
}
/* glm::inverse(mat3) (func_matrix.inl compute_inverse<3,3>) */
static void inverse3(const float *m, float *o) {
    const float one_over = 1.0f / det3(m);
    o[0 * 3 + 0] = +(M3(1,1) * M3(2,2) - M3(2,1) * M3(1,2)) * one_over;
    o[1 * 3 + 0] = -(M3(1,0) * M3(2,2) - M3(2,0) * M3(1,2)) * one_over;
    o[2 * 3 + 0] = +(M3(1,0) * M3(2,1) - M3(2,0) * M3(1,1)) * one_over;
    o[0 * 3 + 1] = -(M3(0,1) * M3(2,2) - M3(2,1) * M3(0,2)) * one_over;
    o[1 * 3 + 1] = +(M3(0,0) * M3(2,2) - M3(2,0) * M3(0,2)) * one_over;
    o[2 * 3 + 1] = -(M3(0,0) * M3(2,1) - M3(2,0) * M3(0,1)) * one_over;
    o[0 * 3 + 2] = +(M3(0,1) * M3(1,2) - M3(1,1) * M3(0,2)) * one_over;
    o[1 * 3 + 2] = -(M3(0,0) * M3(1,2) - M3(1,0) * M3(0,2)) * one_over;
    o[2 * 3 + 2] = +(M3(0,0) * M3(1,1) - M3(1,0) * M3(0,1)) * one_over;
#undef M3
}
/* glm::determinant(mat4) (func_matrix.inl compute_determinant<4,4>) */
float ora_mat4_determinant(const float *mm) {
#define M(c, r) mm[(c) * 4 + (r)]
    const float s00 = M(2,2) * M(3,3) - M(3,2) * M(2,3);
    const float s01 = M(2,1) * M(3,3) - M(3,1) * M(2,3);
    const float s02 = M(2,1) * M(3,2) - M(3,1) * M(2,2);
    const float s03 = M(2,0) * M(3,3) - M(3,0) * M(2,3);
    const float s04 = M(2,0) * M(3,2) - M(3,0) * M(2,2);
    const float s05 = M(2,0) * M(3,1) - M(3,0) * M(2,1);
    const float c0 = +((M(1,1) * s00 - M(1,2) * s01) + M(1,3) * s02);
    const float c1 = -((M(1,0) * s00 - M(1,2) * s03) + M(1,3) * s04);
    const float c2 = +((M(1,0) * s01 - M(1,1) * s03) + M(1,3) * s05);
    const float c3 = -((M(1,0) * s02 - M(1,1) * s04) + M(1,2) * s05);
    return ((M(0,0) * c0 + M(0,1) * c1) + M(0,2) * c2) + M(0,3) * c3;
#undef M
}

/* ---- rasterizer.hpp ------------------------------------------------------------------------- */
/* detail::RasterVertex (:57-67) with the VertexOut varyings the builtin VS sets (builtin_shaders.hpp
 * :98-101): WorldPos = (world, 1), NormalWS = (n, 0), UV0 = (uv, 0, 0), Color0 = vin.color = (1,1,1,1). */
typedef struct {
    v4 clip;
    v4 var[4];          /* WorldPos, NormalWS, UV0, Color0 */
    v3 world_pos;
    v3 normal_ws;
    v2 uv;
} rvert;

/* detail::lerp_rv (:69-79) */
static rvert lerp_rv(const rvert *a, const rvert *b, float t) {
    rvert o;
    o.clip.x = g_mix(a->clip.x, b->clip.x, t); o.clip.y = g_mix(a->clip.y, b->clip.y, t);
    o.clip.z = g_mix(a->clip.z, b->clip.z, t); o.clip.w = g_mix(a->clip.w, b->clip.w, t);
    for (int i = 0; i < 4; ++i) {
        o.var[i].x = g_mix(a->var[i].x, b->var[i].x, t); o.var[i].y = g_mix(a->var[i].y, b->var[i].y, t);
        o.var[i].z = g_mix(a->var[i].z, b->var[i].z, t); o.var[i].w = g_mix(a->var[i].w, b->var[i].w, t);
    }
    o.world_pos = v3mix(a->world_pos, b->world_pos, t);
    o.normal_ws = normalize3(v3mix(a->normal_ws, b->normal_ws, t));
    o.uv.x = g_mix(a->uv.x, b->uv.x, t); o.uv.y = g_mix(a->uv.y, b->uv.y, t);
    return o;
}

static float plane_dist(const rvert *v, int p) {   /* plane_dist_left .. far (:81-109) */
    switch (p) {
        case 0: return v->clip.x + v->clip.w;
        case 1: return v->clip.w - v->clip.x;
        case 2: return v->clip.y + v->clip.w;
        case 3: return v->clip.w - v->clip.y;
        case 4: return v->clip.z + v->clip.w;
        default: return v->clip.w - v->clip.z;
    }
}

/* detail::clip_polygon_plane (:111-152).  A convex polygon gains at most one vertex per plane
 * (3 + 6); MAX_POLY bounds the arrays for a rounding-induced non-convex one (never reached in the
 * test scenes; the GPU path applies the identical cap). */
#define MAX_POLY 16
static int clip_polygon_plane(const rvert *in, int n, rvert *out, int p) {
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const rvert *cur = &in[i], *nxt = &in[(i + 1) % n];
        const float da = plane_dist(cur, p), db = plane_dist(nxt, p);
        const int cur_in = da >= 0.0f, nxt_in = db >= 0.0f;
        if (m > MAX_POLY - 2) break;
        if (cur_in && nxt_in) {
            out[m++] = *nxt;
        } else if (cur_in && !nxt_in) {
            const float denom = da - db;
            if (fabsf(denom) > 1e-8f) out[m++] = lerp_rv(cur, nxt, da / denom);
        } else if (!cur_in && nxt_in) {
            const float denom = da - db;
            if (fabsf(denom) > 1e-8f) out[m++] = lerp_rv(cur, nxt, da / denom);
            out[m++] = *nxt;
        }
    }
    return m;
}

static int fully_inside_clip(const rvert *v) {   /* :232-240 */
    const v4 c = v->clip;
    if (!(c.w > 0.0f)) return 0;
    return (c.x >= -c.w && c.x <= c.w) && (c.y >= -c.w && c.y <= c.w) && (c.z >= -c.w && c.z <= c.w);
}

/* barycentric_2d (:167-179) */
static inline v3 barycentric_2d(v2 p, v2 a, v2 b, v2 c) {
    const v2 v0 = {b.x - a.x, b.y - a.y}, v1 = {c.x - a.x, c.y - a.y}, vp = {p.x - a.x, p.y - a.y};
    const float den = v0.x * v1.y - v1.x * v0.y;
    if (fabsf(den) < 1e-8f) return V3(-1.0f, -1.0f, -1.0f);
    const float inv_den = 1.0f / den;
    const float v = (vp.x * v1.y - v1.x * vp.y) * inv_den;
    const float w = (v0.x * vp.y - vp.x * v0.y) * inv_den;
    const float u = 1.0f - v - w;
    return V3(u, v, w);
}

/* ---- builtin_shaders.hpp / shadow_sample.hpp ---------------------------------------------------- */
/* shadow_visibility_dir (shadow_sample.hpp:65-104) with ShadowParams built as the builtin FS does */
static float shadow_visibility_dir(const ora_lib_target *t, const ora_lib_draw *u, v3 pos, float ndotl) {
    const v4 p = m4v4(u->light_viewproj, (v4){pos.x, pos.y, pos.z, 1.0f});
    if (fabsf(p.w) < 1e-8f) return 1.0f;
    const float nx = p.x / p.w, ny = p.y / p.w, nz = p.z / p.w;
    const float su = nx * 0.5f + 0.5f, sv = ny * 0.5f + 0.5f, sz = nz * 0.5f + 0.5f;
    if (su < 0.0f || su > 1.0f || sv < 0.0f || sv > 1.0f) return 1.0f;
    const float slope = 1.0f - s_clamp(ndotl, 0.0f, 1.0f);
    const float bias = u->shadow_bias_const + u->shadow_bias_slope * slope;
    const float z_test = sz - bias;
    const float fx = su * (float)(t->shadow_w - 1), fy = sv * (float)(t->shadow_h - 1);
    const int cx = (int)roundf(fx), cy = (int)roundf(fy);
    const int r = u->shadow_pcf_radius > 0 ? u->shadow_pcf_radius : 0;   /* std::max(0, ...) twice */
    if (r == 0) {
        const float z_ref = t->shadow[(size_t)s_clampi(cy, 0, t->shadow_h - 1) * t->shadow_w + s_clampi(cx, 0, t->shadow_w - 1)];
        return (z_test <= z_ref) ? 1.0f : 0.0f;
    }
    const float pcf_step = s_max(1.0f, u->shadow_pcf_step);
    const int rs = (int)roundf(pcf_step);
    const int step = rs > 1 ? rs : 1;
    int count = 0, lit = 0;
    for (int oy = -r; oy <= r; oy++)
        for (int ox = -r; ox <= r; ox++) {
            const int x = s_clampi(cx + ox * step, 0, t->shadow_w - 1), y = s_clampi(cy + oy * step, 0, t->shadow_h - 1);
            lit += (z_test <= t->shadow[(size_t)y * t->shadow_w + x]) ? 1 : 0;
            count++;
        }
    return (count > 0) ? (float)lit / (float)count : 1.0f;
}

/* eval_fake_ibl (builtin_shaders.hpp:57-85) */
static v3 eval_fake_ibl(v3 N, v3 V, v3 base, float metallic, float roughness, float ao) {
    const v3 n = normalize3(N), v = normalize3(V);
    const v3 r = reflect3(v3neg(v), n);
    const v3 zen = V3(0.32f, 0.46f, 0.72f), hor = V3(0.62f, 0.66f, 0.72f), gnd = V3(0.16f, 0.15f, 0.14f);
    const float up_n = s_clamp(n.y * 0.5f + 0.5f, 0.0f, 1.0f);
    const float up_r = s_clamp(r.y * 0.5f + 0.5f, 0.0f, 1.0f);
    const v3 env_n = v3mix(gnd, v3mix(hor, zen, up_n), up_n);
    const v3 env_r = v3mix(gnd, v3mix(hor, zen, up_r), up_r);
    const float m = s_clamp(metallic, 0.0f, 1.0f), rgh = s_clamp(roughness, 0.0f, 1.0f);
    const v3 F0 = v3mix(V3(0.04f, 0.04f, 0.04f), v3gmax(base, V3(0.0f, 0.0f, 0.0f)), m);
    const float fres = powf(1.0f - s_max(0.0f, dot3(n, v)), 5.0f);
    const v3 F = v3add(F0, v3s(v3sub(V3(1.0f, 1.0f, 1.0f), F0), fres));
    const v3 kd = v3s(v3sub(V3(1.0f, 1.0f, 1.0f), F), 1.0f - m);
    const v3 diffuse_ibl = v3s(v3mul(v3mul(kd, base), env_n), 0.12f);
    const float spec_strength = 0.02f + (1.0f - rgh) * 0.18f;
    const v3 spec_ibl = v3s(v3mul(env_r, F), spec_strength);
    return v3s(v3add(diffuse_ibl, spec_ibl), s_clamp(ao, 0.0f, 1.0f));
}

typedef struct {
    v3 world_pos, normal_ws;
    v2 uv;
    float depth01;
    int px, py;
} frag_in;

/* Forward+ per-pixel lighting (shs_oracle_light.c): the tile list of the pixel as fp_stress_scene.frag
 * :644-685 selects it (saturated list -> every light), each light through PointLightModel::sample,
 * combined like hello_light_types_culling_sw.cpp:404-416 (ambient hemisphere + sum, clamped). */
static v3 forward_plus(const ora_lib_target *t, const ora_lib_draw *u, const frag_in *fin) {
    const ora_light_cull_desc *d = t->cull;
    const v3 N = normalize3(fin->normal_ws);
    const v3 cam = V3(u->camera_pos[0], u->camera_pos[1], u->camera_pos[2]);
    v3 V = v3sub(cam, fin->world_pos);
    const float len2 = dot3(V, V);
    V = len2 <= 1e-10f ? V3(0.0f, 0.0f, 1.0f) : v3s(V, 1.0f / sqrtf(len2));        /* normalize_or */
    const float hemi = 0.5f + 0.5f * s_clamp(N.y, -1.0f, 1.0f);
    const float amb = 0.22f + 0.12f * hemi;                                         /* kAmbientBase / Hemi */
    float lit[3] = {u->base_color[0] * amb, u->base_color[1] * amb, u->base_color[2] * amb};
    const float w[3] = {fin->world_pos.x, fin->world_pos.y, fin->world_pos.z}, n[3] = {N.x, N.y, N.z}, vv[3] = {V.x, V.y, V.z};
    const uint32_t ts = d->tile_size > 0 ? d->tile_size : 1u, maxp = d->max_per_tile > 0 ? d->max_per_tile : 1u;
    const uint32_t tx_n = ((uint32_t)t->W + ts - 1) / ts, ty_n = ((uint32_t)t->H + ts - 1) / ts;
    uint32_t tx = (uint32_t)fin->px / ts, ty = (uint32_t)(t->H - 1 - fin->py) / ts;   /* gl_FragCoord rows y-down */
    if (tx > tx_n - 1) tx = tx_n - 1;
    if (ty > ty_n - 1) ty = ty_n - 1;
    uint32_t list = ty * tx_n + tx;
    if (d->mode == 3u) {
        const uint32_t zs = d->z_slices > 0 ? d->z_slices : 1u;
        const v4 vw = m4v4(d->view, (v4){w[0], w[1], w[2], 1.0f});
        const float view_depth = s_max(0.001f, vw.z);
        const float near_z = s_max(d->zn, 0.001f), far_z = s_max(d->zf, near_z + 0.01f);
        const float dd = g_clamp(view_depth, near_z, far_z);
        const float tt = logf(dd / near_z) / s_max(logf(far_z / near_z), 1e-6f);
        const float zi = g_clamp(floorf(tt * (float)zs), 0.0f, (float)(zs - 1u));
        list = ((uint32_t)zi * ty_n + ty) * tx_n + tx;
    }
    const uint32_t count = d->mode == 0u ? maxp : (t->tile_counts[list] < maxp ? t->tile_counts[list] : maxp);
    const float base[3] = {u->base_color[0], u->base_color[1], u->base_color[2]};
    if (count >= maxp) {
        for (int i = 0; i < t->n_lights; ++i) ora_point_light_accumulate(&t->lights[i], w, n, vv, base, lit);
    } else {
        for (uint32_t i = 0; i < count; ++i) {
            const uint32_t idx = t->tile_indices[(size_t)list * maxp + i];
            if ((int)idx < t->n_lights) ora_point_light_accumulate(&t->lights[idx], w, n, vv, base, lit);
        }
    }
    return V3(g_clamp(lit[0], 0.0f, 1.0f), g_clamp(lit[1], 0.0f, 1.0f), g_clamp(lit[2], 0.0f, 1.0f));
}

/* srgb_to_linear_rgb (builtin_shaders.hpp:25-31): std::pow((float)c / 255.0f, 2.2f) per channel */
static v3 srgb_to_linear_rgb(const uint8_t *c) {
    return V3(powf((float)c[0] / 255.0f, 2.2f), powf((float)c[1] / 255.0f, 2.2f), powf((float)c[2] / 255.0f, 2.2f));
}

/* sample_texture2d_bilinear_repeat_linear (builtin_shaders.hpp:33-55): no texture -> vec3(1); repeat
 * wrap u - floor(u); bilinear between the four srgb_to_linear_rgb texels with glm::mix. */
static v3 sample_texture2d_bilinear_repeat_linear(const ora_lib_draw *u, v2 uv) {
    if (!u->base_color_tex || u->tex_w <= 0 || u->tex_h <= 0) return V3(1.0f, 1.0f, 1.0f);
    const int w = u->tex_w, h = u->tex_h;
    const float uu = uv.x - floorf(uv.x);
    const float vv = uv.y - floorf(uv.y);
    const float fx = uu * (float)(w - 1);
    const float fy = vv * (float)(h - 1);
    const int x0 = (int)floorf(fx);
    const int y0 = (int)floorf(fy);
    const int x1 = x0 + 1 < w - 1 ? x0 + 1 : w - 1;   /* std::min(x0 + 1, tex->w - 1) */
    const int y1 = y0 + 1 < h - 1 ? y0 + 1 : h - 1;
    const float tx = fx - (float)x0;
    const float ty = fy - (float)y0;
    const uint8_t *T = u->base_color_tex;
    const v3 c00 = srgb_to_linear_rgb(T + 4 * ((size_t)y0 * w + x0));
    const v3 c10 = srgb_to_linear_rgb(T + 4 * ((size_t)y0 * w + x1));
    const v3 c01 = srgb_to_linear_rgb(T + 4 * ((size_t)y1 * w + x0));
    const v3 c11 = srgb_to_linear_rgb(T + 4 * ((size_t)y1 * w + x1));
    const v3 cx0 = v3mix(c00, c10, tx);
    const v3 cx1 = v3mix(c01, c11, tx);
    return v3mix(cx0, cx1, ty);
}

/* The sampler alone (known-answer tests). */
void ora_sample_texture(const uint8_t *rgba, int32_t w, int32_t h, float u, float v, float out3[3]) {
    ora_lib_draw d;
    memset(&d, 0, sizeof d);
    d.base_color_tex = rgba;
    d.tex_w = w;
    d.tex_h = h;
    const v3 c = sample_texture2d_bilinear_repeat_linear(&d, (v2){u, v});
    out3[0] = c.x; out3[1] = c.y; out3[2] = c.z;
}

/* The builtin fragment programs (builtin_shaders.hpp:105-245); albedo_tex = the base_color_tex sample
 * at fin.uv (:113, :162). */
static v4 fragment(const ora_lib_target *t, const ora_lib_draw *u, const frag_in *fin) {
    v4 o = {0.0f, 0.0f, 0.0f, 1.0f};
    const v3 albedo_tex = sample_texture2d_bilinear_repeat_linear(u, fin->uv);
    const v3 bc = V3(u->base_color[0], u->base_color[1], u->base_color[2]);
    const v3 cam = V3(u->camera_pos[0], u->camera_pos[1], u->camera_pos[2]);
    const v3 ldir = V3(u->light_dir_ws[0], u->light_dir_ws[1], u->light_dir_ws[2]);
    const v3 lcol = V3(u->light_color[0], u->light_color[1], u->light_color[2]);
    const int use_shadow = u->shadow && t->shadow != NULL;
    if (u->program == ORA_PROGRAM_DEBUG_ALBEDO) {          /* :227-231 */
        o.x = bc.x; o.y = bc.y; o.z = bc.z;
        return o;
    }
    if (u->program == ORA_PROGRAM_DEBUG_NORMAL) {          /* :232-237 */
        const v3 n = v3add(v3s(normalize3(fin->normal_ws), 0.5f), V3(0.5f, 0.5f, 0.5f));
        o.x = n.x; o.y = n.y; o.z = n.z;
        return o;
    }
    if (u->program == ORA_PROGRAM_FORWARD_PLUS) {
        const v3 c = forward_plus(t, u, fin);
        o.x = c.x; o.y = c.y; o.z = c.z;
        return o;
    }
    if (u->program == ORA_PROGRAM_DEBUG_DEPTH) {           /* :238-241 */
        const float d = s_clamp(fin->depth01, 0.0f, 1.0f);
        o.x = d; o.y = d; o.z = d;
        return o;
    }
    if (u->program == ORA_PROGRAM_BLINN_PHONG) {           /* make_blinn_phong_program :111-150 */
        const v3 albedo = v3gmax(v3mul(bc, albedo_tex), V3(0.0f, 0.0f, 0.0f));
        const v3 N = normalize3(fin->normal_ws);
        const v3 L = normalize3(v3neg(ldir));
        const v3 V = normalize3(v3sub(cam, fin->world_pos));
        const v3 H = normalize3(v3add(L, V));
        const float NdotL = s_max(0.0f, dot3(N, L));
        const float NdotH = s_max(0.0f, dot3(N, H));
        const float rough = s_clamp(u->roughness, 0.0f, 1.0f);
        const float metal = s_clamp(u->metallic, 0.0f, 1.0f);
        const float spec_pow = s_max(4.0f, 8.0f + (1.0f - rough) * 120.0f);
        const float spec_norm = (spec_pow + 2.0f) / (2.0f * PI_F);
        const float spec_f0 = 0.04f + 0.96f * metal;
        const float spec = ((powf(NdotH, spec_pow) * spec_norm) * spec_f0) * NdotL;
        const v3 kd = V3(1.0f - metal, 1.0f - metal, 1.0f - metal);
        const v3 diffuse = v3s(v3mul(kd, albedo), NdotL / PI_F);
        float vis = 1.0f;
        if (use_shadow && NdotL > 0.0f) {
            vis = shadow_visibility_dir(t, u, fin->world_pos, NdotL);
            vis = g_mix(1.0f, vis, s_clamp(u->shadow_strength, 0.0f, 1.0f));
        }
        const v3 direct = v3s(v3s(v3mul(v3add(diffuse, V3(spec, spec, spec)), lcol), u->light_intensity), vis);
        const v3 ibl = eval_fake_ibl(N, V, albedo, u->metallic, u->roughness, u->ao);
        const v3 c = v3add(direct, ibl);
        o.x = c.x; o.y = c.y; o.z = c.z;
        return o;
    }
    /* make_pbr_mr_program :160-212 */
    const v3 N = normalize3(fin->normal_ws);
    const v3 V = normalize3(v3sub(cam, fin->world_pos));
    const v3 L = normalize3(v3neg(ldir));
    const v3 H = normalize3(v3add(V, L));
    const float NdotL = s_max(0.0f, dot3(N, L));
    const float NdotV = s_max(0.0f, dot3(N, V));
    const float NdotH = s_max(0.0f, dot3(N, H));
    const float VdotH = s_max(0.0f, dot3(V, H));
    const float rough = s_clamp(u->roughness, 0.04f, 1.0f);
    const float metal = s_clamp(u->metallic, 0.0f, 1.0f);
    const v3 albedo = v3gmax(v3mul(bc, albedo_tex), V3(0.0f, 0.0f, 0.0f));
    const v3 F0 = v3mix(V3(0.04f, 0.04f, 0.04f), albedo, metal);
    const float a = rough * rough;
    const float a2 = a * a;
    const float denomD = (NdotH * NdotH) * (a2 - 1.0f) + 1.0f;
    const float D = a2 / ((PI_F * denomD) * denomD + 1e-7f);
    const float k = ((a + 1.0f) * (a + 1.0f)) * 0.125f;
    const float g1v = NdotV / ((NdotV * (1.0f - k) + k) + 1e-7f);
    const float g1l = NdotL / ((NdotL * (1.0f - k) + k) + 1e-7f);
    const float G = g1v * g1l;
    const v3 F = v3add(F0, v3s(v3sub(V3(1.0f, 1.0f, 1.0f), F0), powf(1.0f - VdotH, 5.0f)));
    const float sden = s_max((4.0f * NdotL) * NdotV, 1e-6f);
    const v3 DGF = v3s(F, D * G);
    const v3 spec = V3(DGF.x / sden, DGF.y / sden, DGF.z / sden);
    const v3 kd = v3s(v3sub(V3(1.0f, 1.0f, 1.0f), F), 1.0f - metal);
    const v3 diff = v3s(v3mul(kd, albedo), 1.0f / PI_F);
    const v3 radiance = v3s(lcol, u->light_intensity);
    float vis = 1.0f;
    if (use_shadow && NdotL > 0.0f) {
        vis = shadow_visibility_dir(t, u, fin->world_pos, NdotL);
        vis = g_mix(1.0f, vis, s_clamp(u->shadow_strength, 0.0f, 1.0f));
    }
    const v3 direct = (NdotL > 0.0f && NdotV > 0.0f) ? v3s(v3s(v3mul(v3add(diff, spec), radiance), NdotL), vis)
                                                     : V3(0.0f, 0.0f, 0.0f);
    const v3 ibl = eval_fake_ibl(N, V, albedo, metal, rough, u->ao);
    const v3 c = v3add(direct, ibl);
    o.x = c.x; o.y = c.y; o.z = c.z;
    return o;
}

/* make_default_vertex_out (builtin_shaders.hpp:87-103) */
static rvert vertex_out(const ora_lib_draw *u, v3 p, v3 n, v2 uv) {
    rvert o;
    const v4 wp4 = m4v4(u->model, (v4){p.x, p.y, p.z, 1.0f});
    o.world_pos = V3(wp4.x, wp4.y, wp4.z);
    o.clip = m4v4(u->viewproj, wp4);
    float nm[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) nm[c * 3 + r] = u->model[c * 4 + r];   /* glm::mat3(model) */
    if (fabsf(det3(nm)) > 1e-8f) {
        float inv[9], tr[9];
        inverse3(nm, inv);
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) tr[c * 3 + r] = inv[r * 3 + c];     /* glm::transpose */
        memcpy(nm, tr, sizeof nm);
    }
    o.normal_ws = normalize3(m3v3(nm, n));
    o.uv = uv;
    o.var[0] = (v4){o.world_pos.x, o.world_pos.y, o.world_pos.z, 1.0f};
    o.var[1] = (v4){o.normal_ws.x, o.normal_ws.y, o.normal_ws.z, 0.0f};
    o.var[2] = (v4){uv.x, uv.y, 0.0f, 0.0f};
    o.var[3] = (v4){1.0f, 1.0f, 1.0f, 1.0f};
    return o;
}

/* ShaderVertex read_v (rasterizer.hpp:196-202): normal (0,1,0) and uv (0,0) when absent */
static void read_vertex(const ora_mesh *m, uint32_t idx, v3 *p, v3 *n, v2 *uv) {
    *p = V3(m->positions[3 * (size_t)idx], m->positions[3 * (size_t)idx + 1], m->positions[3 * (size_t)idx + 2]);
    *n = (int64_t)idx < m->n_normals ? V3(m->normals[3 * (size_t)idx], m->normals[3 * (size_t)idx + 1], m->normals[3 * (size_t)idx + 2])
                                     : V3(0.0f, 1.0f, 0.0f);
    uv->x = (int64_t)idx < m->n_uvs ? m->uvs[2 * (size_t)idx] : 0.0f;
    uv->y = (int64_t)idx < m->n_uvs ? m->uvs[2 * (size_t)idx + 1] : 0.0f;
}

static int64_t mesh_tris(const ora_mesh *m) { return m->indices ? m->n_indices / 3 : m->n_verts / 3; }

/* One triangle's pixel loop (rasterizer.hpp:336-420) over rows [y0, y1): the unit the reference's
 * row-parallel split (parallel_for_1d over bbox rows, :424-436) hands to its job system. */
typedef struct row_job {
    const ora_lib_target *t;
    const ora_lib_draw *u;
    v2 s[3];
    float iw[3], zw[3];
    v4 varw[3][3];
    float c2p[16];
    int minx, maxx, miny, maxy, W, H, depth_motion, write_motion;
    int next_chunk, n_chunks, grain;
    pthread_mutex_t lock;
} row_job;

static void raster_rows(row_job *j, int y0, int y1) {
    for (int y = y0; y < y1; ++y)
        for (int x = j->minx; x <= j->maxx; ++x) {
            const v2 p = {(float)x + 0.5f, (float)y + 0.5f};
            const v3 bc = barycentric_2d(p, j->s[0], j->s[1], j->s[2]);
            if (bc.x < 0.0f || bc.y < 0.0f || bc.z < 0.0f) continue;
            const float denom = (bc.x * j->iw[0] + bc.y * j->iw[1]) + bc.z * j->iw[2];
            if (denom <= 1e-10f) continue;
            const float inv_denom = 1.0f / denom;
            const float z_clip = (bc.x * j->zw[0] + bc.y * j->zw[1]) + bc.z * j->zw[2];
            const float z_ndc = z_clip * inv_denom;
            float z01 = g_clamp(z_ndc * 0.5f + 0.5f, 0.0f, 1.0f);
            const size_t o = (size_t)y * j->W + x;
            if (j->depth_motion) {
                const float view_z = 1.0f / denom;
                if (j->t->zf > j->t->zn + 1e-6f) z01 = g_clamp((view_z - j->t->zn) / (j->t->zf - j->t->zn), 0.0f, 1.0f);
                if (z01 >= j->t->depth[o]) continue;
                j->t->depth[o] = z01;
            }
            float fv[3][4];
            for (int q = 0; q < 3; ++q) {
                fv[q][0] = ((bc.x * j->varw[0][q].x + bc.y * j->varw[1][q].x) + bc.z * j->varw[2][q].x) * inv_denom;
                fv[q][1] = ((bc.x * j->varw[0][q].y + bc.y * j->varw[1][q].y) + bc.z * j->varw[2][q].y) * inv_denom;
                fv[q][2] = ((bc.x * j->varw[0][q].z + bc.y * j->varw[1][q].z) + bc.z * j->varw[2][q].z) * inv_denom;
            }
            frag_in fin;
            fin.world_pos = V3(fv[0][0], fv[0][1], fv[0][2]);           /* the WorldPos varying wins (:375-378) */
            fin.normal_ws = normalize3(V3(fv[1][0], fv[1][1], fv[1][2])); /* NormalWS (:379-382) */
            fin.uv.x = fv[2][0]; fin.uv.y = fv[2][1];                    /* UV0 (:383-387) */
            if (j->write_motion) {                                          /* :388-411 */
                const v4 cw = {fin.world_pos.x, fin.world_pos.y, fin.world_pos.z, 1.0f};
                const v4 pw = m4v4(j->c2p, cw);
                const v4 cc = m4v4(j->u->viewproj, cw);
                const v4 pc = m4v4(j->u->prev_viewproj, pw);
                float mx = 0.0f, my = 0.0f;
                if (fabsf(cc.w) > 1e-8f && fabsf(pc.w) > 1e-8f) {
                    const float cnx = cc.x / cc.w, cny = cc.y / cc.w, pnx = pc.x / pc.w, pny = pc.y / pc.w;
                    float vx = ((cnx - pnx) * 0.5f) * (float)j->W, vy = ((cny - pny) * 0.5f) * (float)j->H;
                    const float len = sqrtf(vx * vx + vy * vy);
                    if (len > 96.0f && len > 1e-6f) {
                        const float sc = 96.0f / len;
                        vx *= sc; vy *= sc;
                    }
                    mx = vx; my = vy;
                }
                j->t->motion[2 * o] = mx; j->t->motion[2 * o + 1] = my;
            }
            fin.depth01 = z01;
            fin.px = x;
            fin.py = y;
            const v4 c = fragment(j->t, j->u, &fin);
            j->t->hdr[4 * o] = c.x; j->t->hdr[4 * o + 1] = c.y; j->t->hdr[4 * o + 2] = c.z; j->t->hdr[4 * o + 3] = c.w;
        }
}

static int g_lib_threads = 1;   /* 1: sequential (the reference without a job system) */

void ora_set_lib_threads(int n) { g_lib_threads = n < 1 ? 1 : n; }

static void *row_worker(void *arg) {
    row_job *j = (row_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->lock);
        const int c = j->next_chunk++;
        pthread_mutex_unlock(&j->lock);
        if (c >= j->n_chunks) return NULL;
        const int y0 = j->miny + c * j->grain;
        const int y1 = y0 + j->grain < j->maxy + 1 ? y0 + j->grain : j->maxy + 1;
        raster_rows(j, y0, y1);
    }
}

/* RasterizerConfig defaults (rasterizer.hpp:37-39): parallel_min_rows 8, parallel_min_pixels 128*128.
 * Rows are disjoint, so the result equals the sequential loop's. */
static void raster_triangle(row_job *j) {
    const int rows = j->maxy - j->miny + 1, pixels = (j->maxx - j->minx + 1) * rows;
    if (g_lib_threads <= 1 || rows < 8 || pixels < 128 * 128) {
        raster_rows(j, j->miny, j->maxy + 1);
        return;
    }
    j->grain = 8;
    j->n_chunks = (rows + j->grain - 1) / j->grain;
    j->next_chunk = 0;
    pthread_mutex_init(&j->lock, NULL);
    pthread_t th[64];
    const int n = g_lib_threads < 64 ? g_lib_threads : 64;
    for (int i = 1; i < n; ++i) pthread_create(&th[i], NULL, row_worker, j);
    row_worker(j);
    for (int i = 1; i < n; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j->lock);
}

/* rasterize_mesh (rasterizer.hpp:181-442); big bboxes row-parallel on g_lib_threads threads as the
 * reference's job system splits them (disjoint rows: the result equals the sequential order). */
void ora_rasterize_mesh(const ora_lib_target *t, const ora_lib_draw *u, uint64_t *stats3) {
    const int W = t->W, H = t->H;
    const ora_mesh *m = &u->mesh;
    if (!t->hdr || m->n_verts <= 0 || W <= 0 || H <= 0) return;
    const int64_t tri_count = mesh_tris(m);
    const int depth_motion = t->depth != NULL;
    const int write_motion = depth_motion && t->motion != NULL && u->enable_motion_vectors;
    float c2p[16];   /* curr_to_prev_model (:296-308) */
    if (write_motion) {
        if (fabsf(ora_mat4_determinant(u->model)) > 1e-10f) {
            float inv[16];
            ora_mat4_inverse(u->model, inv);
            ora_mat4_mul(u->prev_model, inv, c2p);
        } else {
            memset(c2p, 0, sizeof c2p);
            c2p[0] = c2p[5] = c2p[10] = c2p[15] = 1.0f;
        }
    }
    for (int64_t ti = 0; ti < tri_count; ++ti) {
        stats3[0]++;
        uint32_t id[3];
        for (int k = 0; k < 3; ++k) id[k] = m->indices ? m->indices[ti * 3 + k] : (uint32_t)(ti * 3 + k);
        if ((int64_t)id[0] >= m->n_verts || (int64_t)id[1] >= m->n_verts || (int64_t)id[2] >= m->n_verts) continue;
        rvert poly[2][MAX_POLY];
        for (int k = 0; k < 3; ++k) {
            v3 p, n; v2 uv;
            read_vertex(m, id[k], &p, &n, &uv);
            poly[0][k] = vertex_out(u, p, n, uv);
        }
        int n = 3, cur = 0;
        if (!(fully_inside_clip(&poly[0][0]) && fully_inside_clip(&poly[0][1]) && fully_inside_clip(&poly[0][2]))) {
            for (int p = 0; p < 6 && n > 0; ++p) {
                n = clip_polygon_plane(poly[cur], n, poly[cur ^ 1], p);
                cur ^= 1;
            }
        }
        if (n < 3) continue;
        const rvert *P = poly[cur];
        for (int k = 1; k + 1 < n; ++k) {
            stats3[1]++;
            const rvert *r[3] = {&P[0], &P[k], &P[k + 1]};
            v3 nd[3];
            int finite = 1;
            for (int j = 0; j < 3; ++j) {
                nd[j] = V3(r[j]->clip.x / r[j]->clip.w, r[j]->clip.y / r[j]->clip.w, r[j]->clip.z / r[j]->clip.w);
                finite = finite && isfinite(nd[j].x) && isfinite(nd[j].y) && isfinite(nd[j].z);
            }
            if (!finite) continue;
            v2 s[3];
            for (int j = 0; j < 3; ++j) {
                s[j].x = (nd[j].x * 0.5f + 0.5f) * (float)(W - 1);
                s[j].y = (nd[j].y * 0.5f + 0.5f) * (float)(H - 1);
            }
            const v2 e0 = {s[1].x - s[0].x, s[1].y - s[0].y}, e1 = {s[2].x - s[0].x, s[2].y - s[0].y};
            const float area2 = e0.x * e1.y - e0.y * e1.x;
            if (fabsf(area2) < 1e-10f) continue;
            const int tri_ccw = area2 > 0.0f;
            const int is_front = (tri_ccw == (u->front_face_ccw != 0));
            if (u->cull_mode == ORA_CULL_BACK && !is_front) continue;
            if (u->cull_mode == ORA_CULL_FRONT && is_front) continue;
            const float minx_f = s_min(s_min(s[0].x, s[1].x), s[2].x), maxx_f = s_max(s_max(s[0].x, s[1].x), s[2].x);
            const float miny_f = s_min(s_min(s[0].y, s[1].y), s[2].y), maxy_f = s_max(s_max(s[0].y, s[1].y), s[2].y);
            int minx = (int)floorf(minx_f); if (minx < 0) minx = 0;
            int maxx = (int)ceilf(maxx_f); if (maxx > W - 1) maxx = W - 1;
            int miny = (int)floorf(miny_f); if (miny < 0) miny = 0;
            int maxy = (int)ceilf(maxy_f); if (maxy > H - 1) maxy = H - 1;
            if (minx > maxx || miny > maxy) continue;
            stats3[2]++;
            float iw[3], zw[3];
            v4 varw[3][3];
            for (int j = 0; j < 3; ++j) {
                iw[j] = 1.0f / r[j]->clip.w;
                zw[j] = r[j]->clip.z * iw[j];
                for (int q = 0; q < 3; ++q) {   /* WorldPos, NormalWS, UV0 (Color0 is never read) */
                    varw[j][q].x = r[j]->var[q].x * iw[j]; varw[j][q].y = r[j]->var[q].y * iw[j];
                    varw[j][q].z = r[j]->var[q].z * iw[j]; varw[j][q].w = r[j]->var[q].w * iw[j];
                }
            }
            row_job job;
            job.t = t; job.u = u; job.W = W; job.H = H;
            job.depth_motion = depth_motion; job.write_motion = write_motion;
            memcpy(job.s, s, sizeof job.s);
            memcpy(job.iw, iw, sizeof job.iw);
            memcpy(job.zw, zw, sizeof job.zw);
            memcpy(job.varw, varw, sizeof job.varw);
            if (write_motion) memcpy(job.c2p, c2p, sizeof job.c2p);
            job.minx = minx; job.maxx = maxx; job.miny = miny; job.maxy = maxy;
            raster_triangle(&job);
        }
    }
}

/* PassPBRForward::execute (passes/pass_pbr_forward.hpp:49-214) without a sky: background gradient
 * (:71-84), motion->clear_all() (depth 1, motion 0; :87-98), then rasterize_mesh per item. */
int ora_pbr_forward(const ora_lib_target *t, const ora_lib_draw *draws, int n_draws, uint64_t *stats3) {
    if (!t || !t->hdr || t->W <= 0 || t->H <= 0 || (n_draws > 0 && !draws)) return -1;
    const int W = t->W, H = t->H;
    for (int y = 0; y < H; ++y) {
        float c[4];
        if (t->bg_gradient) {
            const float tt = (float)y / (float)(H - 1 > 1 ? H - 1 : 1);
            c[0] = 0.06f + 0.08f * tt; c[1] = 0.08f + 0.10f * tt; c[2] = 0.12f + 0.12f * tt; c[3] = 1.0f;
        } else {
            memcpy(c, t->clear_hdr, sizeof c);
        }
        for (int x = 0; x < W; ++x) memcpy(&t->hdr[4 * ((size_t)y * W + x)], c, sizeof c);
    }
    if (t->depth)
        for (size_t i = 0; i < (size_t)W * H; ++i) t->depth[i] = 1.0f;
    if (t->motion) memset(t->motion, 0, sizeof(float) * 2 * (size_t)W * H);
    stats3[0] = stats3[1] = stats3[2] = 0;
    for (int i = 0; i < n_draws; ++i) ora_rasterize_mesh(t, &draws[i], stats3);
    return 0;
}

/* ---- PassShadowMap (passes/pass_shadow_map.hpp:44-206) -------------------------------------- */
/* Depth pass of one caster with the light camera's viewproj (:144-204); shadow cleared by the caller. */
static void shadow_caster(float *sm, int SW, int SH, const float *light_vp, const ora_shadow_caster *cst) {
    const ora_mesh *m = &cst->mesh;
    const int64_t tri_count = mesh_tris(m);
    for (int64_t ti = 0; ti < tri_count; ++ti) {
        uint32_t id[3];
        for (int k = 0; k < 3; ++k) id[k] = m->indices ? m->indices[ti * 3 + k] : (uint32_t)(ti * 3 + k);
        if ((int64_t)id[0] >= m->n_verts || (int64_t)id[1] >= m->n_verts || (int64_t)id[2] >= m->n_verts) continue;
        v3 n[3];
        int skip = 0;
        for (int k = 0; k < 3; ++k) {
            const float *p = m->positions + 3 * (size_t)id[k];
            const v4 w4 = m4v4(cst->model, (v4){p[0], p[1], p[2], 1.0f});
            const v4 c = m4v4(light_vp, (v4){w4.x, w4.y, w4.z, 1.0f});
            if (fabsf(c.w) < 1e-8f) skip = 1;
            n[k] = V3(c.x / c.w, c.y / c.w, c.z / c.w);
        }
        if (skip) continue;
        if ((n[0].x < -1.0f && n[1].x < -1.0f && n[2].x < -1.0f) || (n[0].x > 1.0f && n[1].x > 1.0f && n[2].x > 1.0f)) continue;
        if ((n[0].y < -1.0f && n[1].y < -1.0f && n[2].y < -1.0f) || (n[0].y > 1.0f && n[1].y > 1.0f && n[2].y > 1.0f)) continue;
        if ((n[0].z < -1.0f && n[1].z < -1.0f && n[2].z < -1.0f) || (n[0].z > 1.0f && n[1].z > 1.0f && n[2].z > 1.0f)) continue;
        v2 s[3];
        for (int k = 0; k < 3; ++k) {
            s[k].x = (n[k].x * 0.5f + 0.5f) * (float)(SW - 1);
            s[k].y = (n[k].y * 0.5f + 0.5f) * (float)(SH - 1);
        }
        int minx = (int)floorf(s_min(s_min(s[0].x, s[1].x), s[2].x)); if (minx < 0) minx = 0;
        int maxx = (int)ceilf(s_max(s_max(s[0].x, s[1].x), s[2].x)); if (maxx > SW - 1) maxx = SW - 1;
        int miny = (int)floorf(s_min(s_min(s[0].y, s[1].y), s[2].y)); if (miny < 0) miny = 0;
        int maxy = (int)ceilf(s_max(s_max(s[0].y, s[1].y), s[2].y)); if (maxy > SH - 1) maxy = SH - 1;
        if (minx > maxx || miny > maxy) continue;
        for (int y = miny; y <= maxy; ++y)
            for (int x = minx; x <= maxx; ++x) {
                const v2 p = {(float)x + 0.5f, (float)y + 0.5f};
                const v3 bc = barycentric_2d(p, s[0], s[1], s[2]);
                if (bc.x < 0.0f || bc.y < 0.0f || bc.z < 0.0f) continue;
                const float z_ndc = (bc.x * n[0].z + bc.y * n[1].z) + bc.z * n[2].z;
                const float z01 = s_clamp(z_ndc * 0.5f + 0.5f, 0.0f, 1.0f);
                float *zb = &sm[(size_t)y * SW + x];
                if (z01 < *zb) *zb = z01;
            }
    }
}

/* AABB helpers (geometry/aabb.hpp:17-28) */
static void aabb_expand(v3 *mn, v3 *mx, v3 p) {
    *mn = V3(g_min(mn->x, p.x), g_min(mn->y, p.y), g_min(mn->z, p.z));
    *mx = V3(g_max(mx->x, p.x), g_max(mx->y, p.y), g_max(mx->z, p.z));
}

/* glm::lookAtLH / glm::orthoLH_NO (matrix_transform.inl, matrix_clip_space.inl) */
static inline v3 cross3(v3 x, v3 y) { return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
void ora_look_at_lh(const float *eye3, const float *center3, const float *up3, float *m) {
    const v3 eye = V3(eye3[0], eye3[1], eye3[2]), center = V3(center3[0], center3[1], center3[2]), up = V3(up3[0], up3[1], up3[2]);
    const v3 f = normalize3(v3sub(center, eye));
    const v3 s = normalize3(cross3(up, f));
    const v3 uu = cross3(f, s);
    memset(m, 0, 16 * sizeof(float));
    m[15] = 1.0f;
    m[0] = s.x; m[4] = s.y; m[8] = s.z;
    m[1] = uu.x; m[5] = uu.y; m[9] = uu.z;
    m[2] = f.x; m[6] = f.y; m[10] = f.z;
    m[12] = -dot3(s, eye); m[13] = -dot3(uu, eye); m[14] = -dot3(f, eye);
}
static void ortho_lh_no(float l, float r, float b, float t, float zn, float zf, float *m) {
    memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
    m[0] = 2.0f / (r - l);
    m[5] = 2.0f / (t - b);
    m[12] = -(r + l) / (r - l);
    m[13] = -(t + b) / (t - b);
    m[10] = 2.0f / (zf - zn);
    m[14] = -(zf + zn) / (zf - zn);
}

/* build_dir_light_camera_aabb (camera/light_camera.hpp:33-98) */
void ora_dir_light_camera_aabb(const float *sun_dir3, const float *mn3, const float *mx3, float extra_margin,
                               uint32_t res, float *view, float *proj, float *viewproj) {
    const v3 dir = normalize3(V3(sun_dir3[0], sun_dir3[1], sun_dir3[2]));
    const float up[3] = {0.0f, fabsf(dir.y) > 0.95f ? 0.0f : 1.0f, fabsf(dir.y) > 0.95f ? 1.0f : 0.0f};
    const v3 mn = V3(mn3[0], mn3[1], mn3[2]), mx = V3(mx3[0], mx3[1], mx3[2]);
    const v3 c = v3s(v3add(mn, mx), 0.5f);
    const v3 ext = v3s(v3sub(mx, mn), 0.5f);
    const float scene_radius = sqrtf(dot3(ext, ext)) + extra_margin;
    const v3 pos = v3sub(c, v3s(dir, scene_radius * 2.0f));
    const float pos3[3] = {pos.x, pos.y, pos.z}, c3[3] = {c.x, c.y, c.z};
    ora_look_at_lh(pos3, c3, up, view);
    const v3 corners[8] = {{mn.x, mn.y, mn.z}, {mx.x, mn.y, mn.z}, {mn.x, mx.y, mn.z}, {mx.x, mx.y, mn.z},
                           {mn.x, mn.y, mx.z}, {mx.x, mn.y, mx.z}, {mn.x, mx.y, mx.z}, {mx.x, mx.y, mx.z}};
    float l = 1e30f, r = -1e30f, b = 1e30f, t = -1e30f, n = 1e30f, f = -1e30f;
    for (int i = 0; i < 8; ++i) {
        const v4 p = m4v4(view, (v4){corners[i].x, corners[i].y, corners[i].z, 1.0f});
        l = s_min(l, p.x); r = s_max(r, p.x);
        b = s_min(b, p.y); t = s_max(t, p.y);
        n = s_min(n, p.z); f = s_max(f, p.z);
    }
    const float m = extra_margin;
    l -= m; r += m; b -= m; t += m;
    n -= m; f += m;
    if (res > 0u) {
        const float span_x = s_max(r - l, 1e-5f), span_y = s_max(t - b, 1e-5f);
        const float inv_res = 1.0f / (float)res;
        const float texel_x = span_x * inv_res, texel_y = span_y * inv_res;
        float cx = 0.5f * (l + r), cy = 0.5f * (b + t);
        if (texel_x > 1e-6f) cx = floorf(cx / texel_x + 0.5f) * texel_x;
        if (texel_y > 1e-6f) cy = floorf(cy / texel_y + 0.5f) * texel_y;
        const float hx = 0.5f * span_x, hy = 0.5f * span_y;
        l = cx - hx; r = cx + hx; b = cy - hy; t = cy + hy;
    }
    ortho_lh_no(l, r, b, t, n, f, proj);
    ora_mat4_mul(proj, view, viewproj);
}

/* PassShadowMap::execute: clear(1), scene AABB of the casters' model-space mesh bounds (:80-131),
 * light camera (:133-137), depth pass (:144-204).  light_viewproj_out receives the light camera's
 * viewproj (ctx.shadow.light_viewproj). */
int ora_shadow_map(int SW, int SH, const float *sun_dir3, const ora_shadow_caster *casters, int n_casters, float *sm,
                   float *light_viewproj_out) {
    if (SW <= 0 || SH <= 0 || !sm || (n_casters > 0 && !casters)) return -1;
    for (size_t i = 0; i < (size_t)SW * SH; ++i) sm[i] = 1.0f;
    v3 smn = V3(1e30f, 1e30f, 1e30f), smx = V3(-1e30f, -1e30f, -1e30f);
    int any = 0;
    for (int i = 0; i < n_casters; ++i) {
        const ora_mesh *m = &casters[i].mesh;
        if (m->n_verts <= 0) continue;
        v3 bmn = V3(FLT_MAX, FLT_MAX, FLT_MAX), bmx = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        for (int32_t k = 0; k < m->n_verts; ++k) aabb_expand(&bmn, &bmx, V3(m->positions[3 * k], m->positions[3 * k + 1], m->positions[3 * k + 2]));
        const v3 c[8] = {{bmn.x, bmn.y, bmn.z}, {bmx.x, bmn.y, bmn.z}, {bmn.x, bmx.y, bmn.z}, {bmx.x, bmx.y, bmn.z},
                         {bmn.x, bmn.y, bmx.z}, {bmx.x, bmn.y, bmx.z}, {bmn.x, bmx.y, bmx.z}, {bmx.x, bmx.y, bmx.z}};
        for (int j = 0; j < 8; ++j) {
            const v4 w = m4v4(casters[i].model, (v4){c[j].x, c[j].y, c[j].z, 1.0f});
            aabb_expand(&smn, &smx, V3(w.x, w.y, w.z));
        }
        any = 1;
    }
    if (!any) {
        aabb_expand(&smn, &smx, V3(-1.0f, -1.0f, -1.0f));
        aabb_expand(&smn, &smx, V3(1.0f, 1.0f, 1.0f));
    }
    float view[16], proj[16], vp[16];
    const float mn3[3] = {smn.x, smn.y, smn.z}, mx3[3] = {smx.x, smx.y, smx.z};
    ora_dir_light_camera_aabb(sun_dir3, mn3, mx3, 10.0f, (uint32_t)(SW > 1 ? SW : 1), view, proj, vp);
    if (light_viewproj_out) memcpy(light_viewproj_out, vp, sizeof vp);
    for (int i = 0; i < n_casters; ++i)
        if (casters[i].mesh.n_verts > 0) shadow_caster(sm, SW, SH, vp, &casters[i]);
    return 0;
}
