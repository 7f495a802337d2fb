// shs_canvas_post.hip -- the Canvas-API multi-pass extras on gfx950 (paths
// relative to /root/reference/cpp-folders/src/hello-render-target/):
//   k_canvas_motion_blur   combined_motion_blur_pass (hello_pbr.cpp:1128-1252): per pixel the camera
//                          velocity from depth + matrices (:1051-1109), the object / camera mix, the
//                          soft knee (:1111-1122) and the clamp, then `samples` tent-weighted taps;
//   k_canvas_gaussian      gaussian_blur_pass (hello_depth_of_field.cpp:175-251), 5 taps, one axis;
//   k_canvas_autofocus     autofocus_depth_median_center (:257-285): the nth_element median of the
//                          window's finite depths as a rank selection in one workgroup;
//   k_canvas_dof_composite dof_composite_pass (:287-343).
// One thread per pixel; every float expression keeps the reference's operation order
// (-ffp-contract=off, correctly rounded '/' and sqrt), so the output bytes are the reference's.
#include <float.h>

#include "shs_canvas_post_internal.hpp"

namespace shs_dev {

namespace {

__device__ __forceinline__ void m4v(const float *m, float x, float y, float z, float w, float (&o)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return (v < lo) ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return (v < lo) ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ float glength(float x, float y) { return sqrtf(x * x + y * y); }
// std::round then (int): half away from zero; NaN -> 0 (x86's INT_MIN clamps to the same 0)
__device__ __forceinline__ int round_i(float v) { return (int)roundf(v); }

// compute_camera_velocity_canvas_fast (hello_pbr.cpp:1077-1109)
__device__ __forceinline__ void camera_velocity(const CanvasMBParams &p, int x, int y, float view_z, float &vx, float &vy) {
    vx = 0.0f;
    vy = 0.0f;
    if (view_z == FLT_MAX) return;
    // canvas_to_ndc_xy (:1058-1068)
    const int py_screen = (p.H - 1) - y;
    const float fx = ((float)x + 0.5f) / (float)p.W;
    const float fy = ((float)py_screen + 0.5f) / (float)p.H;
    const float ndc_x = fx * 2.0f - 1.0f;
    const float ndc_y = 1.0f - fy * 2.0f;
    // viewz_to_ndcz (:1051-1056)
    float c[4];
    m4v(p.curr_proj, 0.0f, 0.0f, view_z, 1.0f, c);
    const float ndc_z = (fabsf(c[3]) < 1e-6f) ? 0.0f : c[2] / c[3];
    float wh[4];
    m4v(p.inv_curr_vp, ndc_x, ndc_y, ndc_z, 1.0f, wh);
    if (fabsf(wh[3]) < 1e-6f) return;
    const float wx = wh[0] / wh[3], wy = wh[1] / wh[3], wz = wh[2] / wh[3];
    float pc[4];
    m4v(p.prev_vp, wx, wy, wz, 1.0f, pc);
    if (fabsf(pc[3]) < 1e-6f) return;
    const float pnx = pc[0] / pc[3], pny = pc[1] / pc[3];
    // ndc_to_screen_xy (:1070-1075)
    const float psx = (pnx * 0.5f + 0.5f) * (float)(p.W - 1);
    const float psy = (1.0f - (pny * 0.5f + 0.5f)) * (float)(p.H - 1);
    vx = (float)x - psx;
    vy = -((float)py_screen - psy);
}

__device__ __forceinline__ uint32_t pack(int r, int g, int b, int a) {
    return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16) | ((uint32_t)a << 24);
}

}  // namespace

__global__ __launch_bounds__(256) void k_canvas_motion_blur(CanvasMBParams p) {
    const int x = (int)(blockIdx.x * 64u + (threadIdx.x & 63u));
    const int y = (int)(blockIdx.y * 4u + (threadIdx.x >> 6));
    if (x >= p.W || y >= p.H) return;
    const size_t i = (size_t)y * p.W + x;
    float cvx, cvy;
    camera_velocity(p, x, y, p.depth[i], cvx, cvy);
    const float2 vf = p.velocity[i];
    const float ox = vf.x - cvx, oy = vf.y - cvy;
    float vx = (p.w_obj * ox + p.w_cam * cvx) * p.strength;
    float vy = (p.w_obj * oy + p.w_cam * cvy) * p.strength;
    if (p.soft_knee) {   // apply_soft_knee (:1111-1122)
        const float len = glength(vx, vy);
        if (!(len <= 1e-6f) && !(len <= p.knee)) {
            const float den = p.max_px - p.knee;
            const float t = (len - p.knee) / ((1e-6f < den) ? den : 1e-6f);
            const float t2 = t / (1.0f + t);
            const float new_len = p.knee + (p.max_px - p.knee) * t2;
            const float s = new_len / len;
            vx *= s;
            vy *= s;
        }
    }
    float len = glength(vx, vy);
    if (len > p.max_px && len > 1e-6f) {
        const float s = p.max_px / len;
        vx *= s;
        vy *= s;
        len = p.max_px;
    }
    if (len < 0.001f || p.samples <= 1) {
        p.dst[i] = p.src[i];
        return;
    }
    const float dx = vx / len, dy = vy / len;
    float r = 0.0f, g = 0.0f, b = 0.0f, wsum = 0.0f;
    for (int k = 0; k < p.samples; ++k) {
        const float t = (float)k / (float)(p.samples - 1);
        const float a = (t - 0.5f) * 2.0f;
        const float al = a * len;
        const int sx = clampi(round_i((float)x + dx * al), 0, p.W - 1);
        const int sy = clampi(round_i((float)y + dy * al), 0, p.H - 1);
        const float wgt = 1.0f - fabsf(a);
        const uint32_t c = p.src[(size_t)sy * p.W + sx];
        r += wgt * (float)(c & 0xffu);
        g += wgt * (float)((c >> 8) & 0xffu);
        b += wgt * (float)((c >> 16) & 0xffu);
        wsum += wgt;
    }
    if (wsum < 0.0001f) wsum = 1.0f;
    p.dst[i] = pack(clampi((int)(r / wsum), 0, 255), clampi((int)(g / wsum), 0, 255), clampi((int)(b / wsum), 0, 255), 255);
}

// gaussian_blur_pass: r = w0 c0 + w1 c1 + w2 c2 + w1 c3 + w0 c4 (left to right), then color_from_rgbaf
__global__ __launch_bounds__(256) void k_canvas_gaussian(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst, int W,
                                                         int H, int horizontal) {
    const int x = (int)(blockIdx.x * 64u + (threadIdx.x & 63u));
    const int y = (int)(blockIdx.y * 4u + (threadIdx.x >> 6));
    if (x >= W || y >= H) return;
    const float w0 = 0.06136f, w1 = 0.24477f, w2 = 0.38774f;
    uint32_t c[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int sx = horizontal ? clampi(x + k - 2, 0, W - 1) : x;
        const int sy = horizontal ? y : clampi(y + k - 2, 0, H - 1);
        c[k] = src[(size_t)sy * W + sx];
    }
    uint32_t out = 0;
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
        const int sh = 8 * ch;
        float v = w0 * (float)((c[0] >> sh) & 0xffu) + w1 * (float)((c[1] >> sh) & 0xffu);
        v = v + w2 * (float)((c[2] >> sh) & 0xffu);
        v = v + w1 * (float)((c[3] >> sh) & 0xffu);
        v = v + w0 * (float)((c[4] >> sh) & 0xffu);
        const float m = (0.0f < v) ? v : 0.0f;        // std::max(0.0f, v)
        const float q = (m < 255.0f) ? m : 255.0f;    // std::min(255.0f, .)
        out |= (uint32_t)(uint8_t)q << sh;
    }
    dst[(size_t)y * W + x] = out;
}

// autofocus_depth_median_center: the window's depths that are not FLT_MAX (out-of-bounds reads are
// FLT_MAX), the element nth_element places at size / 2 == the value of rank size / 2.
constexpr int AF_MAX_RADIUS = 32;
constexpr int AF_MAX = (2 * AF_MAX_RADIUS + 1) * (2 * AF_MAX_RADIUS + 1);

__global__ __launch_bounds__(1024) void k_canvas_autofocus(CanvasDofParams p) {
    __shared__ float s_v[AF_MAX];
    __shared__ int s_n;
    const int tid = (int)threadIdx.x, side = 2 * p.radius + 1, total = side * side;
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int k = tid; k < total; k += 1024) {
        const int x = p.cx + (k % side) - p.radius, y = p.cy + (k / side) - p.radius;
        const float d = (x >= 0 && x < p.W && y >= 0 && y < p.H) ? p.depth[(size_t)y * p.W + x] : FLT_MAX;
        if (d != FLT_MAX) s_v[atomicAdd(&s_n, 1)] = d;
    }
    __syncthreads();
    const int n = s_n;
    if (n == 0) {
        if (tid == 0) {
            const bool in = p.cx >= 0 && p.cx < p.W && p.cy >= 0 && p.cy < p.H;
            const float d = in ? p.depth[(size_t)p.cy * p.W + p.cx] : FLT_MAX;
            *p.focus = (d == FLT_MAX) ? 15.0f : d;
        }
        return;
    }
    const int mid = n / 2;
    for (int k = tid; k < n; k += 1024) {
        const float v = s_v[k];
        int less = 0, equal = 0;
        for (int j = 0; j < n; ++j) {
            const float u = s_v[j];
            less += u < v;
            equal += u == v;
        }
        if (less <= mid && mid < less + equal) *p.focus = v;   // every such value compares equal
    }
}

// dof_composite_pass
__global__ __launch_bounds__(256) void k_canvas_dof_composite(CanvasDofParams p) {
    const int x = (int)(blockIdx.x * 64u + (threadIdx.x & 63u));
    const int y = (int)(blockIdx.y * 4u + (threadIdx.x >> 6));
    if (x >= p.W || y >= p.H) return;
    const size_t i = (size_t)y * p.W + x;
    const float focus = *p.focus;
    float d = p.depth[i];
    if (d == FLT_MAX) d = focus + p.range;
    const float coc = fabsf(d - focus) / p.range;
    float t = clampf(coc, 0.0f, 1.0f);            // smoothstep01
    t = t * t * (3.0f - 2.0f * t);
    t = clampf(t * p.max_blur, 0.0f, 1.0f);
    t = clampf(t, 0.0f, 1.0f);                    // lerp_color
    const float ia = 1.0f - t;
    const uint32_t a = p.sharp[i], b = p.blur[i];
    uint32_t out = 255u << 24;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const int sh = 8 * ch;
        const float v = ia * (float)((a >> sh) & 0xffu) + t * (float)((b >> sh) & 0xffu);
        out |= (uint32_t)(uint8_t)(int)v << sh;   // x86's float -> uint8_t: cvttss2si, low byte
    }
    p.out[i] = out;
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

static dim3 px_grid(int W, int H) { return dim3((unsigned)((W + 63) / 64), (unsigned)((H + 3) / 4)); }

hipError_t launch_canvas_motion_blur(const CanvasMBParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_canvas_motion_blur, px_grid(p.W, p.H), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_canvas_gaussian(const uint32_t *src, uint32_t *dst, int W, int H, bool horizontal, hipStream_t s) {
    hipLaunchKernelGGL(k_canvas_gaussian, px_grid(W, H), dim3(256), 0, s, src, dst, W, H, horizontal ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_canvas_autofocus(const CanvasDofParams &p, hipStream_t s) {
    if (p.radius < 0 || p.radius > AF_MAX_RADIUS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_canvas_autofocus, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_canvas_dof_composite(const CanvasDofParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_canvas_dof_composite, px_grid(p.W, p.H), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace shs_internal
