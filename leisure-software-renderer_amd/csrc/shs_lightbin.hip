// shs_lightbin.hip -- the shs-renderer-lib CPU light binning on gfx950:
//   build_light_bin_culling   shs-renderer-lib/include/shs/lighting/light_culling_runtime.hpp:266-371
//   cull_lights_tiled / _tiled_view_depth_range / _clustered   lighting/jolt_light_culling.hpp:135-412
//   make_screen_tile_cell (6 oriented planes from 8 unprojected corners)                       :95-133
//   classify_vs_cell (bounding sphere, then the AABB's p / n vertices, tolerance 1e-5)
//                                                               geometry/jolt_culling.hpp:129-257
// (paths relative to /root/reference/cpp-folders/src/).  One thread per bin (screen tile, or tile x
// depth slice): it builds its cell and walks the frustum-visible lights, staged in LDS in ascending
// local order, appending every light not classified Outside -- the reference's per-bin loop, so the
// lists come out in the same (ascending) order.  The host prepares what is per call, not per bin:
// inverse(view_proj), the camera-frustum pre-pass, the lights' Jolt bounding spheres and the slice
// depths (std::log / std::exp of the host libm, as the reference computes them).  Arithmetic restates
// GLM's operation order; -ffp-contract=off and correctly rounded division / sqrt keep it bit-exact.
#include <float.h>

#include "shs_lightbin_internal.hpp"

namespace shs_dev {

namespace {
struct v3 { float x, y, z; };
struct Plane { float nx, ny, nz, d; };

__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ float dot(v3 a, v3 b) { const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }

// unproject_ndc: inv_vp * vec4(ndc, 1) ((m0 x + m1 y) + (m2 z + m3 w)), then xyz / w
__device__ __forceinline__ v3 unproject(const float *m, float x, float y, float z) {
    float c[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * 1.0f);
    return {c[0] / c[3], c[1] / c[3], c[2] / c[3]};
}

// make_oriented_plane_from_points: normalize(cross(b - a, c - a)), d = -dot(n, a), flipped so that the
// inside point is on the positive side
__device__ __forceinline__ Plane oriented(v3 a, v3 b, v3 c, v3 inside) {
    v3 n = cross(sub(b, a), sub(c, a));
    const float inv = 1.0f / sqrtf(dot(n, n));
    n = {n.x * inv, n.y * inv, n.z * inv};
    float d = -dot(n, a);
    if (dot(n, inside) + d < 0.0f) {
        n = {-n.x, -n.y, -n.z};
        d = -d;
    }
    return {n.x, n.y, n.z, d};
}

__device__ __forceinline__ float sdist(const Plane &p, float x, float y, float z) {
    const float a = p.nx * x, b = p.ny * y, c = p.nz * z;
    return ((a + b) + c) + p.d;
}
}  // namespace

__global__ __launch_bounds__(256) void k_light_bin(LightBinParams p) {
    constexpr int CHUNK = 512;
    __shared__ BinLight sl[CHUNK];
    const uint32_t n_bins = p.bx * p.by * p.slices;
    const uint32_t bin = blockIdx.x * 256u + threadIdx.x;
    const bool live = bin < n_bins;
    Plane pl[6];
    if (live) {
        const uint32_t per_slice = p.bx * p.by;
        const uint32_t cz = bin / per_slice, tile = bin - cz * per_slice;
        const uint32_t ty = tile / p.bx, tx = tile - ty * p.bx;
        float zn = -1.0f, zf = 1.0f;
        if (p.ndc_range) {
            const float2 r = p.ndc_range[p.ndc_per_tile ? tile : cz];
            zn = r.x;
            zf = r.y;
        }
        // make_screen_tile_cell: tile coordinates top-origin in screen space
        const float x0 = (float)(tx * p.ts) / (float)p.W * 2.0f - 1.0f;
        const float x1 = (float)min((tx + 1u) * p.ts, (uint32_t)p.W) / (float)p.W * 2.0f - 1.0f;
        const float y_top = 1.0f - (float)(ty * p.ts) / (float)p.H * 2.0f;
        const float y_bottom = 1.0f - (float)min((ty + 1u) * p.ts, (uint32_t)p.H) / (float)p.H * 2.0f;
        const v3 nbl = unproject(p.inv_vp, x0, y_bottom, zn), nbr = unproject(p.inv_vp, x1, y_bottom, zn);
        const v3 ntl = unproject(p.inv_vp, x0, y_top, zn), ntr = unproject(p.inv_vp, x1, y_top, zn);
        const v3 fbl = unproject(p.inv_vp, x0, y_bottom, zf), fbr = unproject(p.inv_vp, x1, y_bottom, zf);
        const v3 ftl = unproject(p.inv_vp, x0, y_top, zf), ftr = unproject(p.inv_vp, x1, y_top, zf);
        const v3 s = add(add(add(nbl, ntr), fbl), ftr);
        const v3 inside = {s.x * 0.25f, s.y * 0.25f, s.z * 0.25f};
        pl[0] = oriented(nbl, nbr, ntr, inside);   // near
        pl[1] = oriented(fbr, fbl, ftl, inside);   // far
        pl[2] = oriented(nbl, ntl, ftl, inside);   // left
        pl[3] = oriented(nbr, fbr, ftr, inside);   // right
        pl[4] = oriented(nbl, fbl, fbr, inside);   // bottom
        pl[5] = oriented(ntl, ntr, ftr, inside);   // top
    }
    uint32_t k = 0;
    for (uint32_t base = 0; base < p.n_vis; base += CHUNK) {
        const uint32_t m = min((uint32_t)CHUNK, p.n_vis - base);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += 256) sl[i] = p.lights[base + i];
        __syncthreads();
        if (!live) continue;
        for (uint32_t i = 0; i < m; ++i) {
            const BinLight L = sl[i];
            // classify_sphere_vs_cell (r = max(radius, 0), tolerance 1e-5)
            const float r = (L.r < 0.0f) ? 0.0f : L.r;
            bool outside = false, inside_all = true;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const float dist = sdist(pl[j], L.cx, L.cy, L.cz);
                outside = outside || dist < -(r + 1e-5f);
                inside_all = inside_all && !(dist < (r + 1e-5f));
            }
            bool hit = !outside;
            if (hit && !inside_all) {
                // classify_aabb_vs_cell: the p-vertex of each plane decides Outside
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const float px = pl[j].nx >= 0.0f ? L.mxx : L.mnx;
                    const float py = pl[j].ny >= 0.0f ? L.mxy : L.mny;
                    const float pz = pl[j].nz >= 0.0f ? L.mxz : L.mnz;
                    hit = hit && !(sdist(pl[j], px, py, pz) < -1e-5f);
                }
            }
            if (hit) {
                if (k < p.cap) p.indices[(size_t)bin * p.cap + k] = __float_as_uint(L.index_f);
                ++k;
            }
        }
    }
    if (live) p.counts[bin] = k;
}

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_light_bin(const shs_dev::LightBinParams &p, hipStream_t s) {
    const uint32_t n_bins = p.bx * p.by * p.slices;
    if (n_bins == 0) return hipSuccess;
    hipLaunchKernelGGL(shs_dev::k_light_bin, dim3((n_bins + 255u) / 256u), dim3(256), 0, s, p);
    return hipGetLastError();
}
}  // namespace shs_internal
