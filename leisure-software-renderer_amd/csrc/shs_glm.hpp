// shs_glm.hpp -- host-side restatement of the GLM operations the reference host code uses to
// build per-draw uniforms (camera, model, MVP, normal matrix).  Operation order follows GLM's
// published headers (glm/ext/matrix_transform.inl, matrix_clip_space.inl, detail/type_mat4x4.inl,
// detail/func_matrix.inl); GLM is unversioned in the reference build (vcpkg classic mode), so
// bit-equality with a particular GLM release is unpinned -- see DESIGN.md "Parity".
//
// Matrices are column-major float[16]: m[c*4 + r] == glm::mat4[c][r].
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace shs_host {

struct vec3 { float x, y, z; };

inline float gdot(vec3 a, vec3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
inline vec3 gscale(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 gadd(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 gsub(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 gneg(vec3 a) { return {-a.x, -a.y, -a.z}; }
// glm::normalize = v * inversesqrt(dot(v, v)), inversesqrt(x) = 1 / sqrt(x)
inline vec3 gnormalize(vec3 v) { float inv = 1.0f / std::sqrt(gdot(v, v)); return gscale(v, inv); }
// glm::cross
inline vec3 gcross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline float gradians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }

inline void identity(float *m) {
    std::memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
}

// mat4 * mat4 (type_mat4x4.inl): Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
inline void mul(const float *a, const float *b, float *out) {
    float t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) + a[2 * 4 + r] * b[c * 4 + 2]) +
                           a[3 * 4 + r] * b[c * 4 + 3];
    std::memcpy(out, t, sizeof t);
}

// glm::inverse(mat4) (detail/func_matrix.inl compute_inverse<4,4>)
inline void inverse(const float *mm, float *out) {
    auto M = [&](int c, int r) { return mm[c * 4 + r]; };
    const float c00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    const float c02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    const float c03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    const float c04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    const float c06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    const float c07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    const float c08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    const float c10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    const float c11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    const float c12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    const float c14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    const float c15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    const float c16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    const float c18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    const float c19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    const float c20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    const float c22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    const float c23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    const float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    const float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    const float v0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)};
    const float v1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    const float v2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)};
    const float v3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    const float sa[4] = {+1.f, -1.f, +1.f, -1.f}, sb[4] = {-1.f, +1.f, -1.f, +1.f};
    float inv[4][4];
    for (int i = 0; i < 4; ++i) {
        inv[0][i] = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3[i] * f2[i]) * sa[i];
        inv[1][i] = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3[i] * f4[i]) * sb[i];
        inv[2][i] = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3[i] * f5[i]) * sa[i];
        inv[3][i] = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb[i];
    }
    const float d0 = M(0, 0) * inv[0][0], d1 = M(0, 1) * inv[1][0], d2 = M(0, 2) * inv[2][0], d3 = M(0, 3) * inv[3][0];
    const float det = (d0 + d1) + (d2 + d3);
    const float one_over = 1.0f / det;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = inv[c][r] * one_over;
}

// mat3(transpose(inverse(model))) -- the legacy VS normal matrix (blinn_phong_shading.cpp:54),
// column-major 3x3: n3[c*3 + r] = inverse(model)[r][c].
inline void normal_matrix(const float *model, float *n3) {
    float inv[16];
    inverse(model, inv);
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) n3[c * 3 + r] = inv[r * 4 + c];
}

// glm::perspectiveLH_NO (matrix_clip_space.inl)
inline void perspective_lh_no(float fovy, float aspect, float zn, float zf, float *m) {
    const float tan_half = std::tan(fovy / 2.0f);
    std::memset(m, 0, 16 * sizeof(float));
    m[0 * 4 + 0] = 1.0f / (aspect * tan_half);
    m[1 * 4 + 1] = 1.0f / tan_half;
    m[2 * 4 + 3] = 1.0f;
    m[2 * 4 + 2] = (zf + zn) / (zf - zn);
    m[3 * 4 + 2] = -(2.0f * zf * zn) / (zf - zn);
}

// glm::lookAtLH (matrix_transform.inl)
inline void look_at_lh(vec3 eye, vec3 center, vec3 up, float *m) {
    const vec3 f = gnormalize(gsub(center, eye));
    const vec3 s = gnormalize(gcross(up, f));
    const vec3 u = gcross(f, s);
    identity(m);
    m[0 * 4 + 0] = s.x; m[1 * 4 + 0] = s.y; m[2 * 4 + 0] = s.z;
    m[0 * 4 + 1] = u.x; m[1 * 4 + 1] = u.y; m[2 * 4 + 1] = u.z;
    m[0 * 4 + 2] = f.x; m[1 * 4 + 2] = f.y; m[2 * 4 + 2] = f.z;
    m[3 * 4 + 0] = -gdot(s, eye);
    m[3 * 4 + 1] = -gdot(u, eye);
    m[3 * 4 + 2] = -gdot(f, eye);
}

// glm::translate(mat4(1), v): Result[3] = ((m0*v0 + m1*v1) + m2*v2) + m3
inline void translate(const float *m, vec3 v, float *out) {
    float t[16];
    std::memcpy(t, m, sizeof t);
    for (int r = 0; r < 4; ++r) t[12 + r] = ((m[0 + r] * v.x + m[4 + r] * v.y) + m[8 + r] * v.z) + m[12 + r];
    std::memcpy(out, t, sizeof t);
}

// glm::rotate(m, angle, axis)
inline void rotate(const float *m, float angle, vec3 v, float *out) {
    const float c = std::cos(angle), s = std::sin(angle);
    const vec3 axis = gnormalize(v);
    const vec3 temp = gscale(axis, 1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = temp.x * axis.y + s * axis.z;
    R[0][2] = temp.x * axis.z - s * axis.y;
    R[1][0] = temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = temp.y * axis.z + s * axis.x;
    R[2][0] = temp.z * axis.x + s * axis.y;
    R[2][1] = temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    float t[16];
    for (int k = 0; k < 3; ++k)
        for (int r = 0; r < 4; ++r)
            t[k * 4 + r] = (m[0 + r] * R[k][0] + m[4 + r] * R[k][1]) + m[8 + r] * R[k][2];
    for (int r = 0; r < 4; ++r) t[12 + r] = m[12 + r];
    std::memcpy(out, t, sizeof t);
}

// glm::scale(m, v)
inline void scale(const float *m, vec3 v, float *out) {
    float t[16];
    for (int r = 0; r < 4; ++r) {
        t[0 + r] = m[0 + r] * v.x;
        t[4 + r] = m[4 + r] * v.y;
        t[8 + r] = m[8 + r] * v.z;
        t[12 + r] = m[12 + r];
    }
    std::memcpy(out, t, sizeof t);
}

// Camera3D::update (shs_renderer.hpp:1224-1236); aspect is hard-coded 4/3 in the reference.
inline void camera3d(vec3 position, float horizontal_angle, float vertical_angle, float fov, float zn, float zf,
                     float *view, float *proj) {
    vec3 dir = {std::cos(gradians(vertical_angle)) * std::sin(gradians(horizontal_angle)),
                std::sin(gradians(vertical_angle)),
                std::cos(gradians(vertical_angle)) * std::cos(gradians(horizontal_angle))};
    dir = gnormalize(dir);
    const vec3 world_up = {0.0f, 1.0f, 0.0f};
    const vec3 right = gnormalize(gcross(world_up, dir));
    const vec3 up = gnormalize(gcross(dir, right));
    perspective_lh_no(gradians(fov), 4.0f / 3.0f, zn, zf, proj);
    look_at_lh(position, gadd(position, dir), up, view);
}

// ---- library-path helpers (shs-renderer-lib) ---------------------------------------------
// glm::determinant(mat3) (func_matrix.inl compute_determinant<3,3>), m column-major [9]
inline float det3(const float *m) {
    auto M = [&](int c, int r) { return m[c * 3 + r]; };
    return (M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2))) +
           M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
}

// glm::inverse(mat3) (func_matrix.inl compute_inverse<3,3>)
inline void inverse3(const float *m, float *o) {
    auto M = [&](int c, int r) { return m[c * 3 + r]; };
    const float one_over = 1.0f / det3(m);
    o[0] = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * one_over;
    o[3] = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * one_over;
    o[6] = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * one_over;
    o[1] = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * one_over;
    o[4] = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * one_over;
    o[7] = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * one_over;
    o[2] = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * one_over;
    o[5] = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * one_over;
    o[8] = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * one_over;
}

// glm::determinant(mat4) (func_matrix.inl compute_determinant<4,4>)
inline float det4(const float *mm) {
    auto M = [&](int c, int r) { return mm[c * 4 + r]; };
    const float s00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    const float s01 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    const float s02 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    const float s03 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    const float s04 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    const float s05 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    const float c0 = +((M(1, 1) * s00 - M(1, 2) * s01) + M(1, 3) * s02);
    const float c1 = -((M(1, 0) * s00 - M(1, 2) * s03) + M(1, 3) * s04);
    const float c2 = +((M(1, 0) * s01 - M(1, 1) * s03) + M(1, 3) * s05);
    const float c3 = -((M(1, 0) * s02 - M(1, 1) * s04) + M(1, 2) * s05);
    return ((M(0, 0) * c0 + M(0, 1) * c1) + M(0, 2) * c2) + M(0, 3) * c3;
}

// make_default_vertex_out's normal matrix (builtin_shaders.hpp:93-95): mat3(model), replaced by
// transpose(inverse(.)) when |det| > 1e-8; n3 column-major [9]
inline void lib_normal_matrix(const float *model, float *n3) {
    float m3[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) m3[c * 3 + r] = model[c * 4 + r];
    if (std::fabs(det3(m3)) > 1e-8f) {
        float inv[9];
        inverse3(m3, inv);
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) n3[c * 3 + r] = inv[r * 3 + c];
    } else {
        std::memcpy(n3, m3, sizeof m3);
    }
}

// glm::orthoLH_NO (matrix_clip_space.inl)
inline void ortho_lh_no(float l, float r, float b, float t, float zn, float zf, float *m) {
    identity(m);
    m[0] = 2.0f / (r - l);
    m[5] = 2.0f / (t - b);
    m[12] = -(r + l) / (r - l);
    m[13] = -(t + b) / (t - b);
    m[10] = 2.0f / (zf - zn);
    m[14] = -(zf + zn) / (zf - zn);
}

// RenderItem model matrix (pass_pbr_forward.hpp:136-141, pass_shadow_map.hpp:56-64):
// translate * rotate(x) * rotate(y) * rotate(z) * scale, each applied to the running matrix
inline void model_euler(vec3 pos, vec3 rot, vec3 scl, float *out) {
    float m[16], t[16];
    identity(m);
    translate(m, pos, t); std::memcpy(m, t, sizeof m);
    rotate(m, rot.x, vec3{1.0f, 0.0f, 0.0f}, t); std::memcpy(m, t, sizeof m);
    rotate(m, rot.y, vec3{0.0f, 1.0f, 0.0f}, t); std::memcpy(m, t, sizeof m);
    rotate(m, rot.z, vec3{0.0f, 0.0f, 1.0f}, t); std::memcpy(m, t, sizeof m);
    scale(m, scl, out);
}

// build_dir_light_camera_aabb (camera/light_camera.hpp:33-98)
inline void dir_light_camera_aabb(vec3 sun_dir, vec3 mn, vec3 mx, float margin, uint32_t res, float *view, float *proj,
                                  float *viewproj) {
    auto smin = [](float a, float b) { return (b < a) ? b : a; };   // std::min
    auto smax = [](float a, float b) { return (a < b) ? b : a; };   // std::max
    const vec3 dir = gnormalize(sun_dir);
    const vec3 up = (std::fabs(dir.y) > 0.95f) ? vec3{0.0f, 0.0f, 1.0f} : vec3{0.0f, 1.0f, 0.0f};
    const vec3 c = gscale(gadd(mn, mx), 0.5f);
    const vec3 ext = gscale(gsub(mx, mn), 0.5f);
    const float scene_radius = std::sqrt(gdot(ext, ext)) + margin;
    const vec3 pos = gsub(c, gscale(dir, scene_radius * 2.0f));
    look_at_lh(pos, c, up, view);
    const vec3 corners[8] = {{mn.x, mn.y, mn.z}, {mx.x, mn.y, mn.z}, {mn.x, mx.y, mn.z}, {mx.x, mx.y, mn.z},
                             {mn.x, mn.y, mx.z}, {mx.x, mn.y, mx.z}, {mn.x, mx.y, mx.z}, {mx.x, mx.y, mx.z}};
    float l = 1e30f, r = -1e30f, b = 1e30f, t = -1e30f, n = 1e30f, f = -1e30f;
    for (const vec3 &p : corners) {
        // view * vec4(p, 1): (m0*x + m1*y) + (m2*z + m3*1)
        const float px = (view[0] * p.x + view[4] * p.y) + (view[8] * p.z + view[12] * 1.0f);
        const float py = (view[1] * p.x + view[5] * p.y) + (view[9] * p.z + view[13] * 1.0f);
        const float pz = (view[2] * p.x + view[6] * p.y) + (view[10] * p.z + view[14] * 1.0f);
        l = smin(l, px); r = smax(r, px);
        b = smin(b, py); t = smax(t, py);
        n = smin(n, pz); f = smax(f, pz);
    }
    l -= margin; r += margin; b -= margin; t += margin;
    n -= margin; f += margin;
    if (res > 0u) {
        const float span_x = smax(r - l, 1e-5f), span_y = smax(t - b, 1e-5f);
        const float inv_res = 1.0f / static_cast<float>(res);
        const float texel_x = span_x * inv_res, texel_y = span_y * inv_res;
        float cx = 0.5f * (l + r), cy = 0.5f * (b + t);
        if (texel_x > 1e-6f) cx = std::floor(cx / texel_x + 0.5f) * texel_x;
        if (texel_y > 1e-6f) cy = std::floor(cy / texel_y + 0.5f) * texel_y;
        const float hx = 0.5f * span_x, hy = 0.5f * span_y;
        l = cx - hx; r = cx + hx; b = cy - hy; t = cy + hy;
    }
    ortho_lh_no(l, r, b, t, n, f, proj);
    mul(proj, view, viewproj);
}

// MonkeyObject::get_world_matrix (blinn_phong_shading.cpp:122-128): T * R * S
inline void model_trs(vec3 position, float rotation_deg_y, vec3 scl, float *out) {
    float I[16], T[16], R[16], S[16], TR[16];
    identity(I);
    translate(I, position, T);
    rotate(I, gradians(rotation_deg_y), vec3{0.0f, 1.0f, 0.0f}, R);
    scale(I, scl, S);
    mul(T, R, TR);
    mul(TR, S, out);
}

}  // namespace shs_host
