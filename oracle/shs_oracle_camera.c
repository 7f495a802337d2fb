/* shs_oracle_camera.c -- TEST INFRASTRUCTURE ONLY (the oracle).  An independent CPU restatement of
 * the reference host's camera and model matrices, the uniforms every legacy frame is built from:
 *
 *   Camera3D::update           cpp-folders/src/hello-shs-renderer/shs_renderer.hpp:1224-1236
 *     direction from yaw / pitch, right = normalize(cross(world_up, dir)),
 *     up = normalize(cross(dir, right)), projection = glm::perspectiveLH(radians(fov), 4/3, zn, zf)
 *     (aspect hard-coded), view = glm::lookAtLH(pos, pos + dir, up)
 *   Viewer(pos, speed, w, h)   shs_renderer.hpp:1323-1337 (fov 60, zn 0.1, zf 1000)
 *   MonkeyObject::get_world_matrix
 *                              hello-3d-primitives/hello_pipeline_blinn_phong_shading.cpp:122-128
 *     translate(I, pos) * rotate(I, radians(rot), (0,1,0)) * scale(I, scl)
 *   Uniforms::mvp              blinn_phong_shading.cpp:277-279: (projection * view) * model
 *
 * GLM is not in this container and the reference pins no GLM version, so this file
 * restates GLM 0.9.9/1.0's published scalar code paths (no GLM_FORCE_* in the hot-path targets):
 *   glm::radians        deg * 0.01745329251994329576923690768489f       (trigonometric.inl)
 *   glm::dot(vec3)      (x*x' + y*y') + z*z'                            (func_geometric.inl compute_dot)
 *   glm::normalize      v * (1 / sqrt(dot(v, v)))                       (compute_normalize, inversesqrt)
 *   glm::cross          (a.y*b.z - b.y*a.z, a.z*b.x - b.z*a.x, a.x*b.y - b.x*a.y)
 *   glm::perspectiveLH_NO  tanHalf = tan(fovy / 2); [0][0] = 1 / (aspect * tanHalf);
 *                       [1][1] = 1 / tanHalf; [2][2] = (f + n) / (f - n); [2][3] = 1;
 *                       [3][2] = -((2 * f) * n) / (f - n)               (matrix_clip_space.inl)
 *   glm::lookAtLH       f = normalize(c - e); s = normalize(cross(up, f)); u = cross(f, s);
 *                       rows s / u / f, translation -dot(s|u|f, e)     (matrix_transform.inl)
 *   glm::translate / rotate / scale and mat4 * mat4 (left-to-right sums of column products).
 * Trigonometry: the reference calls unqualified cos / sin on float arguments inside namespace shs
 * with <cmath> and SDL's <math.h> included, i.e. the float overloads (cosf / sinf); tan inside GLM
 * is std::tan(float).  This is the one assumption outside GLM's text -- "parity unpinned" as the
 * whole oracle is.
 *
 * Nothing here is shared with the product's host helpers (leisure-software-renderer_amd/csrc/
 * shs_glm.hpp): tests/test_camera_oracle.py compares the two bitwise.  Matrices are column-major
 * float[16] (m[4 * col + row], glm's storage). */
#include <math.h>
#include <string.h>

#include "shs_oracle.h"

typedef struct { float v[3]; } ovec3;
typedef struct { float c[4][4]; } omat4;   /* c[col][row] */

static float o_radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

static float o_dot(ovec3 a, ovec3 b) {
    const float x = a.v[0] * b.v[0];
    const float y = a.v[1] * b.v[1];
    const float z = a.v[2] * b.v[2];
    return (x + y) + z;
}

static ovec3 o_normalize(ovec3 a) {
    const float inv = 1.0f / sqrtf(o_dot(a, a));
    ovec3 r = {{a.v[0] * inv, a.v[1] * inv, a.v[2] * inv}};
    return r;
}

static ovec3 o_cross(ovec3 a, ovec3 b) {
    ovec3 r = {{a.v[1] * b.v[2] - b.v[1] * a.v[2], a.v[2] * b.v[0] - b.v[2] * a.v[0], a.v[0] * b.v[1] - b.v[0] * a.v[1]}};
    return r;
}

static omat4 o_identity(void) {
    omat4 m;
    memset(&m, 0, sizeof m);
    for (int i = 0; i < 4; ++i) m.c[i][i] = 1.0f;
    return m;
}

static void o_store(const omat4 *m, float *out16) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out16[4 * c + r] = m->c[c][r];
}

static omat4 o_load(const float *m16) {
    omat4 m;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) m.c[c][r] = m16[4 * c + r];
    return m;
}

/* mat4 * mat4: Result[j] = ((A[0] * B[j][0] + A[1] * B[j][1]) + A[2] * B[j][2]) + A[3] * B[j][3] */
static omat4 o_mul(const omat4 *a, const omat4 *b) {
    omat4 o;
    for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 4; ++r) {
            float acc = a->c[0][r] * b->c[j][0];
            acc = acc + a->c[1][r] * b->c[j][1];
            acc = acc + a->c[2][r] * b->c[j][2];
            acc = acc + a->c[3][r] * b->c[j][3];
            o.c[j][r] = acc;
        }
    return o;
}

static omat4 o_perspective_lh_no(float fovy, float aspect, float zn, float zf) {
    const float tan_half = tanf(fovy / 2.0f);
    omat4 m;
    memset(&m, 0, sizeof m);
    m.c[0][0] = 1.0f / (aspect * tan_half);
    m.c[1][1] = 1.0f / tan_half;
    m.c[2][2] = (zf + zn) / (zf - zn);
    m.c[2][3] = 1.0f;
    m.c[3][2] = -((2.0f * zf) * zn) / (zf - zn);
    return m;
}

static omat4 o_look_at_lh(ovec3 eye, ovec3 center, ovec3 up) {
    ovec3 d = {{center.v[0] - eye.v[0], center.v[1] - eye.v[1], center.v[2] - eye.v[2]}};
    const ovec3 f = o_normalize(d);
    const ovec3 s = o_normalize(o_cross(up, f));
    const ovec3 u = o_cross(f, s);
    omat4 m = o_identity();
    for (int k = 0; k < 3; ++k) {
        m.c[k][0] = s.v[k];
        m.c[k][1] = u.v[k];
        m.c[k][2] = f.v[k];
    }
    m.c[3][0] = -o_dot(s, eye);
    m.c[3][1] = -o_dot(u, eye);
    m.c[3][2] = -o_dot(f, eye);
    return m;
}

/* glm::translate(m, v): Result[3] = ((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] */
static omat4 o_translate(const omat4 *m, ovec3 t) {
    omat4 o = *m;
    for (int r = 0; r < 4; ++r) o.c[3][r] = ((m->c[0][r] * t.v[0] + m->c[1][r] * t.v[1]) + m->c[2][r] * t.v[2]) + m->c[3][r];
    return o;
}

/* glm::rotate(m, angle, axis) */
static omat4 o_rotate(const omat4 *m, float angle, ovec3 v) {
    const float c = cosf(angle), s = sinf(angle);
    const ovec3 a = o_normalize(v);
    const ovec3 t = {{(1.0f - c) * a.v[0], (1.0f - c) * a.v[1], (1.0f - c) * a.v[2]}};
    float R[3][3];
    R[0][0] = c + t.v[0] * a.v[0];
    R[0][1] = t.v[0] * a.v[1] + s * a.v[2];
    R[0][2] = t.v[0] * a.v[2] - s * a.v[1];
    R[1][0] = t.v[1] * a.v[0] - s * a.v[2];
    R[1][1] = c + t.v[1] * a.v[1];
    R[1][2] = t.v[1] * a.v[2] + s * a.v[0];
    R[2][0] = t.v[2] * a.v[0] + s * a.v[1];
    R[2][1] = t.v[2] * a.v[1] - s * a.v[0];
    R[2][2] = c + t.v[2] * a.v[2];
    omat4 o;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r) o.c[j][r] = (m->c[0][r] * R[j][0] + m->c[1][r] * R[j][1]) + m->c[2][r] * R[j][2];
    for (int r = 0; r < 4; ++r) o.c[3][r] = m->c[3][r];
    return o;
}

/* glm::scale(m, v): Result[k] = m[k] * v[k] (k < 3), Result[3] = m[3] */
static omat4 o_scale(const omat4 *m, ovec3 sv) {
    omat4 o = *m;
    for (int k = 0; k < 3; ++k)
        for (int r = 0; r < 4; ++r) o.c[k][r] = m->c[k][r] * sv.v[k];
    return o;
}

void ora_camera3d(const float pos[3], float horizontal_angle, float vertical_angle, float fov, float zn, float zf,
                  float view16[16], float proj16[16]) {
    const float va = o_radians(vertical_angle), ha = o_radians(horizontal_angle);
    ovec3 dir = {{cosf(va) * sinf(ha), sinf(va), cosf(va) * cosf(ha)}};
    dir = o_normalize(dir);
    const ovec3 world_up = {{0.0f, 1.0f, 0.0f}};
    const ovec3 right = o_normalize(o_cross(world_up, dir));
    const ovec3 up = o_normalize(o_cross(dir, right));
    const omat4 proj = o_perspective_lh_no(o_radians(fov), 4.0f / 3.0f, zn, zf);
    const ovec3 eye = {{pos[0], pos[1], pos[2]}};
    const ovec3 center = {{eye.v[0] + dir.v[0], eye.v[1] + dir.v[1], eye.v[2] + dir.v[2]}};
    const omat4 view = o_look_at_lh(eye, center, up);
    o_store(&view, view16);
    o_store(&proj, proj16);
}

void ora_model_trs(const float pos[3], float rot_deg_y, const float scl[3], float out16[16]) {
    const omat4 I = o_identity();
    const ovec3 p = {{pos[0], pos[1], pos[2]}}, s = {{scl[0], scl[1], scl[2]}}, yaxis = {{0.0f, 1.0f, 0.0f}};
    const omat4 T = o_translate(&I, p);
    const omat4 R = o_rotate(&I, o_radians(rot_deg_y), yaxis);
    const omat4 S = o_scale(&I, s);
    const omat4 TR = o_mul(&T, &R);
    const omat4 M = o_mul(&TR, &S);
    o_store(&M, out16);
}

void ora_perspective_lh_no(float fovy, float aspect, float zn, float zf, float out16[16]) {
    const omat4 m = o_perspective_lh_no(fovy, aspect, zn, zf);
    o_store(&m, out16);
}

/* The legacy draw's uniforms as RendererSystem::process builds them (blinn_phong_shading.cpp:
 * 272-282): mvp = (projection * view) * model.  For the Flat pipeline (flat_shading.cpp:282-286)
 * mv = view * model and mvp = projection * mv. */
void ora_legacy_mvp(const float view16[16], const float proj16[16], const float model16[16], int flat, float mvp16[16],
                    float mv16[16]) {
    const omat4 V = o_load(view16), P = o_load(proj16), M = o_load(model16);
    if (flat) {
        const omat4 MV = o_mul(&V, &M);
        const omat4 MVP = o_mul(&P, &MV);
        o_store(&MVP, mvp16);
        o_store(&MV, mv16);
    } else {
        const omat4 PV = o_mul(&P, &V);
        const omat4 MVP = o_mul(&PV, &M);
        o_store(&MVP, mvp16);
        if (mv16) o_store(&M, mv16);
    }
}
