// shs_debugdraw.hip -- the software library's debug_draw colour + depth raster on gfx950 (SURVEY.md
// 8f row 2; shs-renderer-lib/include/shs/sw_render/debug_draw.hpp, paths relative to
// /root/reference/cpp-folders/src/):
//   draw_mesh_blinn_phong_transformed (:158-205)  k_dd_setup: one thread per triangle -- model and
//       project_world_to_screen (:38-58) of its corners, the flat Blinn-Phong colour, edge_fn area
//   draw_filled_triangle (:60-109)               k_dd_raster (a wave per triangle) / k_dd_raster_big
//       (bboxes above DD_BIG pixels, chunked over every workgroup): (triangle, pixel) over the clamped bbox,
//       edge functions, the ccw / cw inside test, depth in [0, 1], then the strict `depth < buffer`
//       test run in submission order == the lexicographic minimum of (depth, triangle) among the
//       candidates below the initial depth: a 64-bit atomicMin per pixel;
//                                                 k_dd_resolve: the winner's colour and depth (the
//       depth recomputed by the same operations, so -0 keeps its sign as the reference stores it).
// -ffp-contract=off and correctly rounded division / sqrt; GLM restated (dot (x + y) + z, normalize
// v * (1 / sqrt(dot)), mat4 * vec4 (m0 x + m1 y) + (m2 z + m3 w)).
#include <float.h>

#include "shs_debugdraw_internal.hpp"
#include "shs_wave.hpp"

namespace shs_dev {

namespace {
struct v3 { float x, y, z; };
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 mul(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(v3 a, v3 b) { const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
__device__ __forceinline__ v3 normalize(v3 a) { return mul(a, 1.0f / sqrtf(dot(a, a))); }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }   // std::max
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }   // std::min
__device__ __forceinline__ float sclamp(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }
__device__ __forceinline__ float gclamp01(float x) { const float m = (x < 0.0f) ? 0.0f : x; return (1.0f < m) ? 1.0f : m; }

__device__ __forceinline__ void m4v(const float *m, float x, float y, float z, float w, float (&o)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w);
}

// project_world_to_screen (:38-58)
__device__ __forceinline__ bool project(const DDParams &p, v3 w, float &sx, float &sy, float &z) {
    float c[4];
    m4v(p.vp, w.x, w.y, w.z, 1.0f, c);
    if (c[3] <= 0.001f) return false;
    const float nx = c[0] / c[3], ny = c[1] / c[3], nz = c[2] / c[3];
    if (nz < -1.0f || nz > 1.0f) return false;
    sx = (nx + 1.0f) * 0.5f * (float)p.W;
    sy = (ny + 1.0f) * 0.5f * (float)p.H;
    z = nz * 0.5f + 0.5f;
    return true;
}

// edge_fn (:35-37)
__device__ __forceinline__ float edge_fn(float ax, float ay, float bx, float by, float px, float py) {
    return (px - ax) * (by - ay) - (py - ay) * (bx - ax);
}

// x^32 by five squarings in double (<= 31 double ulps from the exact power: the reference's powf
// result up to float rounding ties, far inside the 1e-5 shaded-float tolerance)
__device__ __forceinline__ float pow32(float x) {
    double d = (double)x;
#pragma unroll
    for (int i = 0; i < 5; ++i) d = d * d;
    return (float)d;
}

// draw_filled_triangle's per-triangle part (:69-83): area, the clamped integer bbox
__device__ __forceinline__ void finish_tri(const DDParams &p, DDTri &t, int g) {
    t.area = edge_fn(t.x0, t.y0, t.x1, t.y1, t.x2, t.y2);
    t.flags = 0u;
    if (fabsf(t.area) <= 1e-6f) return;
    t.flags = 2u;                          // reaches the bbox (tri_lit's flag)
    if (!(t.area == t.area)) return;       // NaN area (non-finite screen points): nothing drawn
    const float min_xf = smin(t.x0, smin(t.x1, t.x2)), min_yf = smin(t.y0, smin(t.y1, t.y2));
    const float max_xf = smax(t.x0, smax(t.x1, t.x2)), max_yf = smax(t.y0, smax(t.y1, t.y2));
    // std::min / std::max of ints after the float floor / ceil (clamped into int range first)
    const float lo = -2147483648.0f, hi = 2147483520.0f;
    const int min_x = max(0, (int)sclamp(floorf(min_xf), lo, hi)), min_y = max(0, (int)sclamp(floorf(min_yf), lo, hi));
    const int max_x = min(p.W - 1, (int)sclamp(ceilf(max_xf), lo, hi)), max_y = min(p.H - 1, (int)sclamp(ceilf(max_yf), lo, hi));
    if (min_x > max_x || min_y > max_y) return;
    t.bmin = (uint32_t)min_x | ((uint32_t)min_y << 16);
    t.bmax = (uint32_t)max_x | ((uint32_t)max_y << 16);
    t.flags = 3u;
    if ((max_x - min_x + 1) * (max_y - min_y + 1) > DD_BIG) p.big_list[atomicAdd(p.big_count, 1u)] = (uint32_t)g;
}
}  // namespace

__global__ __launch_bounds__(256) void k_dd_setup(DDParams p) {
    const int g = (int)(blockIdx.x * 256u + threadIdx.x);
    if (g >= p.n_tris) return;
    int lo = 0, hi = p.n_objects - 1;   // the object of triangle g
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)p.objects[mid].tri_base <= g) lo = mid; else hi = mid - 1;
    }
    const DDObject &o = p.objects[lo];
    const int i = g - (int)o.tri_base;
    DDTri t{};
    t.flags = 0u;
    uint32_t id[3];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        id[k] = o.idx[3 * i + k];
        ok = ok && id[k] < (uint32_t)o.n_verts;
    }
    float lit_r = 0.f, lit_g = 0.f, lit_b = 0.f;
    if (ok) {
        v3 w[3];
        float sx[3], sy[3], sz[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float *P = o.pos + 3 * (size_t)id[k];
            float c[4];
            m4v(o.model, P[0], P[1], P[2], 1.0f, c);
            w[k] = {c[0], c[1], c[2]};
            ok = ok && project(p, w[k], sx[k], sy[k], sz[k]);
        }
        if (ok) {
            // face normal (LH + clockwise front faces: cross(p2 - p0, p1 - p0)), flat Blinn-Phong (:176-200)
            v3 n = cross(sub(w[2], w[0]), sub(w[1], w[0]));
            ok = !(dot(n, n) <= 1e-10f);
            if (ok) {
                n = normalize(n);
                const v3 centroid = mul(add(add(w[0], w[1]), w[2]), 1.0f / 3.0f);
                const v3 L = {p.L[0], p.L[1], p.L[2]};
                const v3 V = normalize(sub(v3{p.cam[0], p.cam[1], p.cam[2]}, centroid));
                const v3 H = normalize(add(L, V));
                const float ndotl = smax(0.0f, dot(n, L));
                const float ndoth = smax(0.0f, dot(n, H));
                const float ambient = 0.18f;
                const float diffuse = 0.72f * ndotl;
                const float specular = (ndotl > 0.0f) ? (0.35f * pow32(ndoth)) : 0.0f;
                const float a_d = ambient + diffuse;
                lit_r = gclamp01(o.base[0] * a_d + specular);
                lit_g = gclamp01(o.base[1] * a_d + specular);
                lit_b = gclamp01(o.base[2] * a_d + specular);
                const uint32_t r = (uint32_t)(uint8_t)sclamp(lit_r * 255.0f, 0.0f, 255.0f);
                const uint32_t gg = (uint32_t)(uint8_t)sclamp(lit_g * 255.0f, 0.0f, 255.0f);
                const uint32_t b = (uint32_t)(uint8_t)sclamp(lit_b * 255.0f, 0.0f, 255.0f);
                t.rgba = r | (gg << 8) | (b << 16) | (255u << 24);
                t.x0 = sx[0]; t.y0 = sy[0]; t.x1 = sx[1]; t.y1 = sy[1]; t.x2 = sx[2]; t.y2 = sy[2];
                t.z0 = sz[0]; t.z1 = sz[1]; t.z2 = sz[2];
                finish_tri(p, t, g);
            }
        }
    }
    t.lit[0] = lit_r;
    t.lit[1] = lit_g;
    p.tris[g] = t;
    if (p.lit_b) p.lit_b[g] = lit_b;
}

// Triangles given directly (draw_filled_triangle's own arguments): area and bbox only.
__global__ __launch_bounds__(256) void k_dd_prepare(DDParams p) {
    const int g = (int)(blockIdx.x * 256u + threadIdx.x);
    if (g >= p.n_tris) return;
    DDTri t = p.tris[g];
    finish_tri(p, t, g);
    p.tris[g] = t;
}

__global__ __launch_bounds__(256) void k_dd_init(DDParams p) {
    const size_t n = (size_t)p.W * p.H;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) p.keys[i] = KEY_EMPTY;
}

// The inside test and depth of draw_filled_triangle's pixel loop (:85-107)
__device__ __forceinline__ bool dd_pixel(const DDTri &t, int x, int y, float &depth) {
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;
    const float w0 = edge_fn(t.x1, t.y1, t.x2, t.y2, px, py);
    const float w1 = edge_fn(t.x2, t.y2, t.x0, t.y0, px, py);
    const float w2 = edge_fn(t.x0, t.y0, t.x1, t.y1, px, py);
    const bool ccw = t.area > 0.0f;
    const bool inside = ccw ? (w0 >= 0.0f && w1 >= 0.0f && w2 >= 0.0f) : (w0 <= 0.0f && w1 <= 0.0f && w2 <= 0.0f);
    if (!inside) return false;
    const float iw0 = w0 / t.area, iw1 = w1 / t.area, iw2 = w2 / t.area;
    depth = (iw0 * t.z0 + iw1 * t.z1) + iw2 * t.z2;
    return !(depth < 0.0f || depth > 1.0f);
}

__device__ __forceinline__ void dd_test(const DDParams &p, const DDTri &t, int x, int y, uint32_t g) {
    float depth;
    if (!dd_pixel(t, x, y, depth)) return;
    const size_t di = (size_t)y * p.W + x;
    if (!(depth < p.depth0[di])) return;   // the strict test against the buffer as it was
    atomicMin(&p.keys[di], z_key(depth, g));
}

// One wave per triangle of at most DD_BIG bbox pixels: the lanes walk the bbox row-major.
__global__ __launch_bounds__(256) void k_dd_raster(DDParams p) {
    const int g = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4u + (threadIdx.x >> 6)));
    if (g >= p.n_tris) return;
    const int lane = (int)(threadIdx.x & 63u);
    const DDTri t = p.tris[g];
    if (!(t.flags & 1u)) return;
    const int min_x = (int)(t.bmin & 0xffffu), min_y = (int)(t.bmin >> 16);
    const int bw = (int)(t.bmax & 0xffffu) - min_x + 1, bh = (int)(t.bmax >> 16) - min_y + 1;
    const int n = bw * bh;
    if (n > DD_BIG) return;                  // k_dd_raster_big
    for (int k = lane; k < n; k += 64) {
        const int ry = k / bw;
        dd_test(p, t, min_x + (k - ry * bw), min_y + ry, (uint32_t)g);
    }
}

// The big triangles: their bboxes concatenated in 256-pixel chunks, chunk c to workgroup c % G.  Each
// workgroup stages a round of DD_ROUND big triangles in LDS (triangle, inclusive chunk prefix) with one
// parallel load, then finds the triangle of each chunk it owns by a binary search in LDS.
constexpr int DD_BIG_GRID = 2048;
constexpr int DD_ROUND = 1024;

__global__ __launch_bounds__(256) void k_dd_raster_big(DDParams p) {
    __shared__ uint32_t s_g[DD_ROUND], s_end[DD_ROUND], s_wave[4];
    const uint32_t nb = *p.big_count;
    const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t base = 0;   // chunks of the rounds before
    for (uint32_t r0 = 0; r0 < nb; r0 += DD_ROUND) {
        const uint32_t m = min((uint32_t)DD_ROUND, nb - r0);
        uint32_t cnt[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = (uint32_t)tid * 4u + (uint32_t)j;
            cnt[j] = 0;
            if (i < m) {
                const uint32_t g = p.big_list[r0 + i];
                const uint32_t bmin = p.tris[g].bmin, bmax = p.tris[g].bmax;
                const uint32_t n = ((bmax & 0xffffu) - (bmin & 0xffffu) + 1u) * ((bmax >> 16) - (bmin >> 16) + 1u);
                cnt[j] = (n + 255u) / 256u;
                s_g[i] = g;
            }
            sum += cnt[j];
        }
        uint32_t incl = sum;   // wave inclusive scan of the per-thread sums
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= d) incl += v;
        }
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        uint32_t run = incl - sum;
        for (int w = 0; w < wave; ++w) run += s_wave[w];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = (uint32_t)tid * 4u + (uint32_t)j;
            run += cnt[j];
            if (i < m) s_end[i] = run;
        }
        __syncthreads();
        const uint32_t total = s_end[m - 1];
        for (uint32_t c = (blockIdx.x + DD_BIG_GRID - base % DD_BIG_GRID) % DD_BIG_GRID; c < total; c += DD_BIG_GRID) {
            uint32_t lo = 0, hi = m - 1;   // the first entry with s_end > c
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_end[mid] > c) hi = mid; else lo = mid + 1;
            }
            const uint32_t g = s_g[lo];
            const uint32_t first = lo ? s_end[lo - 1] : 0u;
            const DDTri t = p.tris[g];
            const int min_x = (int)(t.bmin & 0xffffu), min_y = (int)(t.bmin >> 16);
            const int bw = (int)(t.bmax & 0xffffu) - min_x + 1, bh = (int)(t.bmax >> 16) - min_y + 1;
            const uint32_t k = (c - first) * 256u + (uint32_t)tid;
            if (k < (uint32_t)bw * (uint32_t)bh) {
                const int ry = (int)(k / (uint32_t)bw);
                dd_test(p, t, min_x + ((int)k - ry * bw), min_y + ry, g);
            }
        }
        base += total;
        __syncthreads();   // s_g / s_end are rewritten by the next round
    }
}

__global__ __launch_bounds__(256) void k_dd_resolve(DDParams p) {
    const size_t n = (size_t)p.W * p.H;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) {
        const unsigned long long k = p.keys[i];
        if (k == KEY_EMPTY) continue;
        const uint32_t g = (uint32_t)k;
        const DDTri t = p.tris[g];
        float depth = 0.0f;
        dd_pixel(t, (int)(i % (size_t)p.W), (int)(i / (size_t)p.W), depth);   // the winner's own value
        p.depth[i] = depth;
        p.rgba[i] = t.rgba;
    }
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_dd_mesh_setup(const DDParams &p, hipStream_t s) {
    if (p.n_tris > 0) hipLaunchKernelGGL(k_dd_setup, dim3((unsigned)((p.n_tris + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_dd_fill(const DDParams &p, hipStream_t s) {
    if (!p.objects && p.n_tris > 0)
        hipLaunchKernelGGL(k_dd_prepare, dim3((unsigned)((p.n_tris + 255) / 256)), dim3(256), 0, s, p);
    const size_t n = (size_t)p.W * p.H;
    const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_dd_init, dim3(grid), dim3(256), 0, s, p);
    if (p.n_tris > 0) {
        hipLaunchKernelGGL(k_dd_raster, dim3((unsigned)((p.n_tris + 3) / 4)), dim3(256), 0, s, p);
        hipLaunchKernelGGL(k_dd_raster_big, dim3(DD_BIG_GRID), dim3(256), 0, s, p);
    }
    hipLaunchKernelGGL(k_dd_resolve, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace shs_internal
