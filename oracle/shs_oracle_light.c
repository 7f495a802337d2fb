/*
 * shs_oracle_light.c -- CPU restatement (oracle) of the shs-renderer-lib light-list binning and
 * per-light shading used by the Forward+ configuration:
 *   - per-tile depth range   shaders/vulkan/fp_stress_depth_reduce.comp:31-82
 *   - tile / cluster lists    shaders/vulkan/fp_stress_light_cull.comp:47-266
 *   - point-light sample      include/shs/lighting/light_runtime.hpp:182-237, 321-333
 *   - per-pixel combination   exp-plumbing/hello_light_types_culling_sw.cpp:404-416 (ambient
 *                             hemisphere + sum of base*diffuse + specular, clamped), evaluated per
 *                             pixel with the tile list selection rule of fp_stress_scene.frag:644-685.
 *
 * TEST INFRASTRUCTURE ONLY (see shs_oracle.h).  PARITY UNPINNED: the GLSL shaders cannot run here
 * and the CPU light binning of the reference needs Jolt (absent); GLSL expressions are evaluated
 * with the GLM operation order used everywhere else in this oracle.  Paths relative to
 * /root/reference/cpp-folders/src/shs-renderer-lib/ (and src/exp-plumbing/ for the demo).
 */
#include "shs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline float fmaxg(float a, float b) { return (a < b) ? b : a; }   /* GLSL / std max */
static inline float fming(float a, float b) { return (b < a) ? b : a; }
static inline float fclampg(float x, float lo, float hi) { return fming(fmaxg(x, lo), hi); }
static inline uint32_t umax(uint32_t a, uint32_t b) { return a < b ? b : a; }
static inline uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

/* mat4 * vec4 in GLM order */
static inline void m4v(const float *m, const float *v, float *o) {
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * v[0] + m[4 + r] * v[1]) + (m[8 + r] * v[2] + m[12 + r] * v[3]);
}

/* resolve_cull_sphere (fp_stress_light_cull.comp:47-96), point / spot branch + AABB fallback */
static void resolve_cull_sphere(const ora_culling_light *L, float *s) {
    memcpy(s, L->cull_sphere, 4 * sizeof(float));
    const uint32_t type = L->type_shape_flags[0];
    const float shading_range = fmaxg(L->position_range[3], 0.0f);
    if (type == 2u || type == 1u) {
        if (s[3] <= 0.0f || s[3] < shading_range) {
            s[0] = L->position_range[0]; s[1] = L->position_range[1]; s[2] = L->position_range[2]; s[3] = shading_range;
        }
    }
    if (s[3] > 0.0f) return;
    float ext[3];
    for (int k = 0; k < 3; ++k) ext[k] = fmaxg((L->cull_aabb_max[k] - L->cull_aabb_min[k]) * 0.5f, 0.0f);
    const float r = sqrtf((ext[0] * ext[0] + ext[1] * ext[1]) + ext[2] * ext[2]);
    if (r > 0.0f) {
        for (int k = 0; k < 3; ++k) s[k] = (L->cull_aabb_min[k] + L->cull_aabb_max[k]) * 0.5f;
        s[3] = r;
        return;
    }
    s[0] = L->position_range[0]; s[1] = L->position_range[1]; s[2] = L->position_range[2];
    s[3] = fmaxg(L->position_range[3], 0.0f);
}

/* project_light_screen (:98-127); tile-independent, so evaluated once per light */
static int project_light_screen(const ora_light_cull_desc *d, const float *pos, float r, float *cx, float *cy, float *rpx,
                                float *view_depth) {
    const float p4[4] = {pos[0], pos[1], pos[2], 1.0f};
    float view4[4], clip[4];
    m4v(d->view, p4, view4);
    const float near_z = fmaxg(d->zn, 0.001f);
    if (view4[2] + r <= near_z) return 0;
    *view_depth = fmaxg(near_z, view4[2]);
    m4v(d->proj, view4, clip);
    const float W = (float)umax((uint32_t)d->width, 1u), H = (float)umax((uint32_t)d->height, 1u);
    if (clip[3] <= 1e-6f || (view4[2] - r) <= near_z) {
        *cx = W * 0.5f; *cy = H * 0.5f;
        *rpx = (float)umax((uint32_t)d->width, (uint32_t)d->height);
        return 1;
    }
    const float nx = clip[0] / clip[3], ny = clip[1] / clip[3];
    *cx = (nx * 0.5f + 0.5f) * W;
    *cy = (0.5f - ny * 0.5f) * H;
    float rp = fabsf(((r * d->proj[5]) * H) / *view_depth);
    const float inflate = 1.0f + fclampg(r / fmaxg(*view_depth, near_z), 0.0f, 2.5f) * 0.65f;
    *rpx = rp * inflate + 4.0f;
    return 1;
}

void ora_light_project(const ora_light_cull_desc *d, const ora_culling_light *lights, int n, float *out8) {
    for (int i = 0; i < n; ++i) {
        float *o = out8 + 8 * (size_t)i;
        memset(o, 0, 8 * sizeof(float));
        if ((lights[i].type_shape_flags[2] & 1u) == 0u) continue;   /* SHS_LIGHT_FLAG_ENABLED */
        float s[4], cx, cy, rpx, vd;
        resolve_cull_sphere(&lights[i], s);
        if (!project_light_screen(d, s, s[3], &cx, &cy, &rpx, &vd)) continue;
        o[0] = cx; o[1] = cy; o[2] = rpx; o[3] = vd; o[4] = s[3];
        o[7] = 1.0f;   /* valid */
    }
}

/* depth01 -> linear view z.  fp_stress_depth_reduce.comp:29-36 reconstructs from a perspective
 * (LH_NO) depth; the software library's depth buffer holds linear view depth
 * (rasterizer.hpp:354-357: (view_z - zn) / (zf - zn)), inverted here as zn + d * (zf - zn). */
static float depth_to_view(const ora_light_cull_desc *d, float depth01) {
    const float near_z = fmaxg(d->zn, 0.001f);
    const float far_z = fmaxg(d->zf, near_z + 0.01f);
    const float dd = fclampg(depth01, 0.0f, 1.0f);
    if (d->depth_linear) return d->zn + dd * (d->zf - d->zn);
    const float denom = fmaxg(far_z - dd * (far_z - near_z), 1e-5f);
    return (near_z * far_z) / denom;
}

/* fp_stress_depth_reduce.comp main (:38-82).  depth rows are y-up (RT_ColorDepthMotion); tiles and
 * gl_FragCoord-style pixel rows are y-down, row_down = H - 1 - y_up. */
void ora_depth_reduce(const ora_light_cull_desc *d, const float *depth, float *ranges2) {
    const uint32_t W = umax((uint32_t)d->width, 1u), H = umax((uint32_t)d->height, 1u), ts = umax(d->tile_size, 1u);
    const uint32_t tx_n = (W + ts - 1) / ts, ty_n = (H + ts - 1) / ts;
    for (uint32_t ty = 0; ty < ty_n; ++ty)
        for (uint32_t tx = 0; tx < tx_n; ++tx) {
            float mn = 1e30f, mx = 0.0f;
            int any = 0;
            for (uint32_t py = ty * ts; py < umin((ty + 1) * ts, H); ++py)
                for (uint32_t px = tx * ts; px < umin((tx + 1) * ts, W); ++px) {
                    const float dv = depth[(size_t)(H - 1 - py) * W + px];
                    if (dv >= 1.0f) continue;
                    const float vz = depth_to_view(d, dv);
                    mn = fming(mn, vz); mx = fmaxg(mx, vz);
                    any = 1;
                }
            float *r = ranges2 + 2 * ((size_t)ty * tx_n + tx);
            r[0] = any ? mn : 0.0f;
            r[1] = any ? mx : 0.0f;
        }
}

/* fp_stress_light_cull.comp main (:148-266) for every tile (and cluster slice).  counts: one per
 * list; indices: max_per_tile per list, ascending light index. */
void ora_light_cull(const ora_light_cull_desc *d, const ora_culling_light *lights, int n, const float *ranges2,
                    uint32_t *counts, uint32_t *indices) {
    const uint32_t W = umax((uint32_t)d->width, 1u), H = umax((uint32_t)d->height, 1u), ts = umax(d->tile_size, 1u);
    const uint32_t tx_n = (W + ts - 1) / ts, ty_n = (H + ts - 1) / ts;
    const uint32_t maxp = umax(d->max_per_tile, 1u), zs = umax(d->z_slices, 1u), mode = d->mode;
    const uint32_t tz_n = mode == 3u ? zs : 1u;
    float proj8[8 * 256 + 8];
    float *proj = n <= 256 ? proj8 : NULL;
    float *heap = NULL;
    if (!proj) { heap = (float *)calloc((size_t)n * 8, sizeof(float)); proj = heap; }
    ora_light_project(d, lights, n, proj);
    const float near_z = fmaxg(d->zn, 0.001f), far_z = fmaxg(d->zf, near_z + 0.01f);
    for (uint32_t tz = 0; tz < tz_n; ++tz)
        for (uint32_t ty = 0; ty < ty_n; ++ty)
            for (uint32_t tx = 0; tx < tx_n; ++tx) {
                const uint32_t list = mode == 3u ? (tz * ty_n + ty) * tx_n + tx : ty * tx_n + tx;
                const float tminx = (float)(tx * ts), tminy = (float)(ty * ts);
                const float tmaxx = (float)umin((tx + 1) * ts, W), tmaxy = (float)umin((ty + 1) * ts, H);
                float c_near = 0.0f, c_far = 0.0f;
                if (mode == 3u) {
                    const float s0 = (float)tz / (float)zs, s1 = (float)(tz + 1) / (float)zs;
                    c_near = near_z * powf(far_z / near_z, s0);
                    c_far = near_z * powf(far_z / near_z, s1);
                }
                float r0 = 0.0f, r1 = 0.0f;
                if (mode == 2u) {
                    const float *rg = ranges2 + 2 * ((size_t)ty * tx_n + tx);
                    r0 = rg[0]; r1 = rg[1];
                    if (r0 <= 0.0f && r1 <= 0.0f) { r0 = near_z; r1 = far_z; }
                    r0 = fclampg(r0, near_z, far_z);
                    r1 = fclampg(r1, near_z, far_z);
                    const float expand = fmaxg(0.05f, r1 * 0.0015f);
                    r0 = fclampg(r0 - expand, near_z, far_z);
                    r1 = fclampg(r1 + expand, near_z, far_z);
                    if (r1 < r0) r1 = r0;
                    r1 = fming(far_z, fmaxg(r1, r0 + fmaxg(0.02f, r0 * 0.0005f)));
                }
                uint32_t count = 0;
                for (int i = 0; i < n && mode != 0u; ++i) {
                    const float *p = proj + 8 * (size_t)i;
                    if (p[7] == 0.0f) continue;
                    const float cx = p[0], cy = p[1], rpx = p[2], vd = p[3], rad = p[4];
                    if (((cx + rpx) + 16.0f) < tminx) continue;
                    if (((cy + rpx) + 16.0f) < tminy) continue;
                    if (((cx - rpx) - 16.0f) > tmaxx) continue;
                    if (((cy - rpx) - 16.0f) > tmaxy) continue;
                    if (mode == 2u || mode == 3u) {
                        const float pad = mode == 2u ? fmaxg(1.0f, fmaxg(rad * 0.35f, vd * 0.03f))
                                                     : fmaxg(0.8f, fmaxg(rad * 0.25f, vd * 0.02f));
                        const float lmin = (vd - rad) - pad, lmax = (vd + rad) + pad;
                        const float zlo = mode == 2u ? r0 : c_near, zhi = mode == 2u ? r1 : c_far;
                        if (lmax < zlo || lmin > zhi)
                            if (rpx < (float)ts * 4.0f) continue;
                    }
                    if (count < maxp) indices[(size_t)list * maxp + count++] = (uint32_t)i;
                }
                counts[list] = count;
            }
    free(heap);
}

/* eval_distance_attenuation (light_runtime.hpp:182-210) */
static float distance_attenuation(const ora_culling_light *L, float distance) {
    const float range = fmaxg(L->position_range[3], 0.001f);
    if (distance >= range) return 0.0f;
    const float norm = fclampg(1.0f - distance / range, 0.0f, 1.0f);
    float falloff = 0.0f;
    switch (L->type_shape_flags[3]) {
        case 0u: falloff = norm; break;
        case 1u: falloff = (norm * norm) * (3.0f - 2.0f * norm); break;
        case 2u: {
            const float denom = fmaxg(distance * distance, L->shape_attenuation[2]);
            const float inv = 1.0f / denom;
            const float range_norm = range * range;
            falloff = fming(1.0f, inv * range_norm) * (norm * norm);
            break;
        }
        default: break;
    }
    falloff = powf(fmaxg(falloff, 0.0f), fmaxg(L->shape_attenuation[1], 0.001f));
    if (L->shape_attenuation[3] > 0.0f && falloff < L->shape_attenuation[3]) return 0.0f;
    return fmaxg(falloff, 0.0f);
}

/* PointLightModel::sample + eval_local_light_brdf (light_runtime.hpp:212-237, 321-333), accumulated
 * as lit += base * diffuse + specular (hello_light_types_culling_sw.cpp:414). */
void ora_point_light_accumulate(const ora_culling_light *L, const float *world, const float *N, const float *V,
                                const float *base, float *lit) {
    const float tl[3] = {L->position_range[0] - world[0], L->position_range[1] - world[1], L->position_range[2] - world[2]};
    const float dist = sqrtf((tl[0] * tl[0] + tl[1] * tl[1]) + tl[2] * tl[2]);
    if (dist <= 1e-4f || dist > L->position_range[3]) return;
    const float Ld[3] = {tl[0] / dist, tl[1] / dist, tl[2] / dist};
    const float ndotl = fmaxg((N[0] * Ld[0] + N[1] * Ld[1]) + N[2] * Ld[2], 0.0f);
    if (ndotl <= 0.0f) return;
    const float att = distance_attenuation(L, dist) * fmaxg(1.0f, 0.0f);
    if (att <= 0.0f) return;
    float rad[3];
    for (int k = 0; k < 3; ++k) rad[k] = (fmaxg(L->color_intensity[k], 0.0f) * fmaxg(L->color_intensity[3], 0.0f)) * att;
    float h[3] = {Ld[0] + V[0], Ld[1] + V[1], Ld[2] + V[2]};
    const float len2 = (h[0] * h[0] + h[1] * h[1]) + h[2] * h[2];
    if (len2 <= 1e-10f) { h[0] = Ld[0]; h[1] = Ld[1]; h[2] = Ld[2]; }
    else { const float inv = 1.0f / sqrtf(len2); h[0] *= inv; h[1] *= inv; h[2] *= inv; }
    const float ndoth = fmaxg((N[0] * h[0] + N[1] * h[1]) + N[2] * h[2], 0.0f);
    const float spec = 0.30f * powf(ndoth, 36.0f);
    for (int k = 0; k < 3; ++k) lit[k] = lit[k] + (base[k] * (rad[k] * ndotl) + rad[k] * spec);
}
