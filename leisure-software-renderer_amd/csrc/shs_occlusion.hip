// shs_occlusion.hip -- gfx950 kernel for the software occlusion pass:
//   culling_sw::run_software_occlusion_pass   shs-renderer-lib/include/shs/geometry/culling_software.hpp:229-331
//   project_aabb_to_screen_rect / is_rect_occluded                                    :137-218
//   rasterize_mesh_depth_transformed / rasterize_depth_triangle / project_world_to_screen :44-135
// The pass is sequential by definition: an object's test sees the depth of every visible object
// before it in view-depth order.  One 1024-thread workgroup walks the objects in that order and
// parallelises inside each step: the rect test over its pixels, the raster over (triangle, pixel)
// pairs.  The occlusion buffer (300x225 in the reference demo) stays in L2 between steps; the depth
// min is an atomicMin on the float bits (every stored value is in [0, 1]), so the buffer after each
// object equals the reference's whatever order the pairs run in.
#include <float.h>

#include "shs_glm.hpp"
#include "shs_occlusion_internal.hpp"

namespace shs_dev {

constexpr int OCC_T = 1024;

struct OccShared {
    float px[3][OCC_T], py[3][OCC_T], pz[3][OCC_T];   // projected corners of the chunk's triangles
    float area[OCC_T];
    int bx0[OCC_T], by0[OCC_T], bw[OCC_T];
    uint32_t incl[OCC_T];                              // inclusive prefix of the pixel counts
    uint32_t wtot[OCC_T / 64];
    int rect[4];
    float z_near;
    int valid, not_occ;
    uint32_t n_vis;
};

__device__ __forceinline__ float occ_min(float a, float b) { return (b < a) ? b : a; }   // std::min
__device__ __forceinline__ float occ_max(float a, float b) { return (a < b) ? b : a; }   // std::max

__device__ __forceinline__ void m4v_occ(const float *m, const float (&v)[4], float (&o)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * v[0] + m[4 + r] * v[1]) + (m[8 + r] * v[2] + m[12 + r] * v[3]);
}

__device__ __forceinline__ float edge_fn(float ax, float ay, float bx, float by, float px, float py) {
    return (px - ax) * (by - ay) - (py - ay) * (bx - ax);
}

__device__ __forceinline__ float load_depth(const uint32_t *d) {
    return __uint_as_float(__hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(OCC_T) void k_occlusion(OccParams p) {
    __shared__ OccShared sh;
    const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npx = p.W * p.H;
    for (int i = tid; i < npx; i += OCC_T) p.depth[i] = __float_as_uint(1.0f);
    if (tid == 0) sh.n_vis = 0;
    __threadfence();
    __syncthreads();
    for (int s = 0; s < p.n; ++s) {
        const OccObject &o = p.objs[s];
        // project_aabb_to_screen_rect (one lane)
        if (tid == 0) {
            float mnx = (float)p.W, mny = (float)p.H, mxx = -1.0f, mxy = -1.0f, near_depth = 1.0f;
            bool any = false;
            for (int c = 0; c < 8; ++c) {
                const float v[4] = {(c & 1) ? o.aabb_max[0] : o.aabb_min[0], (c & 2) ? o.aabb_max[1] : o.aabb_min[1],
                                    (c & 4) ? o.aabb_max[2] : o.aabb_min[2], 1.0f};
                float clip[4];
                m4v_occ(p.vp, v, clip);
                if (clip[3] <= 0.001f) continue;
                const float nx = clip[0] / clip[3], ny = clip[1] / clip[3], nz = clip[2] / clip[3];
                const float z01 = nz * 0.5f + 0.5f;
                if (z01 < 0.0f || z01 > 1.0f) continue;
                const float sx = (nx + 1.0f) * 0.5f * (float)p.W, sy = (ny + 1.0f) * 0.5f * (float)p.H;
                mnx = occ_min(mnx, sx); mny = occ_min(mny, sy);
                mxx = occ_max(mxx, sx); mxy = occ_max(mxy, sy);
                near_depth = occ_min(near_depth, z01);
                any = true;
            }
            int x0 = 0, y0 = 0, x1 = -1, y1 = -1;
            if (any) {
                x0 = max(0, (int)floorf(mnx)); y0 = max(0, (int)floorf(mny));
                x1 = min(p.W - 1, (int)ceilf(mxx)); y1 = min(p.H - 1, (int)ceilf(mxy));
            }
            sh.rect[0] = x0; sh.rect[1] = y0; sh.rect[2] = x1; sh.rect[3] = y1;
            sh.z_near = (near_depth < 0.0f) ? 0.0f : ((1.0f < near_depth) ? 1.0f : near_depth);   // std::clamp
            sh.valid = any && x0 <= x1 && y0 <= y1;
            sh.not_occ = sh.valid ? 0 : 1;   // an invalid rect is never occluded
        }
        __syncthreads();
        // is_rect_occluded: visible as soon as one pixel has z_near <= depth + eps
        if (sh.valid) {
            const int rw = sh.rect[2] - sh.rect[0] + 1, rh = sh.rect[3] - sh.rect[1] + 1;
            const float zn = sh.z_near;
            for (int k = tid; k < rw * rh; k += OCC_T) {
                if (*(volatile int *)&sh.not_occ) break;   // another lane found a visible pixel
                const int y = sh.rect[1] + k / rw, x = sh.rect[0] + k % rw;
                if (zn <= load_depth(&p.depth[(size_t)y * p.W + x]) + p.eps) sh.not_occ = 1;
            }
        }
        __syncthreads();
        const bool visible = sh.not_occ != 0;
        if (tid == 0) {
            p.occluded[o.index] = visible ? 0 : 1;
            if (visible) p.visible[sh.n_vis++] = o.index;
        }
        if (visible) {
            // rasterize_mesh_depth_transformed: (triangle, pixel) pairs of up to 1024 triangles at a time
            const int n_tris = o.n_idx / 3;
            for (int c0 = 0; c0 < n_tris; c0 += OCC_T) {
                const int t = c0 + tid;
                uint32_t cnt = 0;
                if (t < n_tris) {
                    float sx[3], sy[3], sz[3];
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t vi = o.idx[3 * t + k];
                        if (!ok || vi >= (uint32_t)o.n_verts) { ok = false; continue; }
                        const float lp[4] = {o.pos[3 * vi], o.pos[3 * vi + 1], o.pos[3 * vi + 2], 1.0f};
                        float wp[4], clip[4];
                        m4v_occ(o.model, lp, wp);
                        const float w4[4] = {wp[0], wp[1], wp[2], 1.0f};
                        m4v_occ(p.vp, w4, clip);
                        if (clip[3] <= 0.001f) { ok = false; continue; }
                        const float nx = clip[0] / clip[3], ny = clip[1] / clip[3], nz = clip[2] / clip[3];
                        if (nz < -1.0f || nz > 1.0f) { ok = false; continue; }
                        sx[k] = (nx + 1.0f) * 0.5f * (float)p.W;
                        sy[k] = (ny + 1.0f) * 0.5f * (float)p.H;
                        sz[k] = nz * 0.5f + 0.5f;
                    }
                    if (ok) {
                        const float area = edge_fn(sx[0], sy[0], sx[1], sy[1], sx[2], sy[2]);
                        if (!(fabsf(area) <= 1e-6f)) {
                            const int x0 = max(0, (int)floorf(occ_min(sx[0], occ_min(sx[1], sx[2]))));
                            const int y0 = max(0, (int)floorf(occ_min(sy[0], occ_min(sy[1], sy[2]))));
                            const int x1 = min(p.W - 1, (int)ceilf(occ_max(sx[0], occ_max(sx[1], sx[2]))));
                            const int y1 = min(p.H - 1, (int)ceilf(occ_max(sy[0], occ_max(sy[1], sy[2]))));
                            if (x0 <= x1 && y0 <= y1) {
#pragma unroll
                                for (int k = 0; k < 3; ++k) { sh.px[k][tid] = sx[k]; sh.py[k][tid] = sy[k]; sh.pz[k][tid] = sz[k]; }
                                sh.area[tid] = area;
                                sh.bx0[tid] = x0; sh.by0[tid] = y0; sh.bw[tid] = x1 - x0 + 1;
                                cnt = (uint32_t)((x1 - x0 + 1) * (y1 - y0 + 1));
                            }
                        }
                    }
                }
                // block inclusive scan of the pixel counts
                uint32_t incl = cnt;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t v = (uint32_t)__shfl_up((int)incl, off);
                    if (lane >= off) incl += v;
                }
                if (lane == 63) sh.wtot[wave] = incl;
                __syncthreads();
                uint32_t wb = 0, total = 0;
                for (int w2 = 0; w2 < OCC_T / 64; ++w2) {
                    const uint32_t v = sh.wtot[w2];
                    wb += w2 < wave ? v : 0u;
                    total += v;
                }
                sh.incl[tid] = wb + incl;
                __syncthreads();
                for (uint32_t k = (uint32_t)tid; k < total; k += OCC_T) {
                    int lo = 0, hi = OCC_T - 1;   // the first triangle whose inclusive end exceeds k
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (sh.incl[mid] > k) hi = mid; else lo = mid + 1;
                    }
                    const int q = lo;
                    const uint32_t local = k - (q > 0 ? sh.incl[q - 1] : 0u);
                    const int w = sh.bw[q];
                    const int x = sh.bx0[q] + (int)(local % (uint32_t)w), y = sh.by0[q] + (int)(local / (uint32_t)w);
                    const float qx = (float)x + 0.5f, qy = (float)y + 0.5f;
                    const float ax = sh.px[0][q], ay = sh.py[0][q], bx = sh.px[1][q], by = sh.py[1][q];
                    const float cx = sh.px[2][q], cy = sh.py[2][q];
                    const float w0 = edge_fn(bx, by, cx, cy, qx, qy);
                    const float w1 = edge_fn(cx, cy, ax, ay, qx, qy);
                    const float w2 = edge_fn(ax, ay, bx, by, qx, qy);
                    const float area = sh.area[q];
                    const bool inside = area > 0.0f ? (w0 >= 0.0f && w1 >= 0.0f && w2 >= 0.0f)
                                                    : (w0 <= 0.0f && w1 <= 0.0f && w2 <= 0.0f);
                    if (!inside) continue;
                    const float d = (w0 / area) * sh.pz[0][q] + (w1 / area) * sh.pz[1][q] + (w2 / area) * sh.pz[2][q];
                    if (d < 0.0f || d > 1.0f) continue;
                    // -0 stores as +0 (they compare equal in every later test)
                    atomicMin(&p.depth[(size_t)y * p.W + x], d == 0.0f ? 0u : __float_as_uint(d));
                }
                __syncthreads();
            }
        }
        __threadfence();
        __syncthreads();
    }
    if (tid == 0) *p.n_visible = sh.n_vis;
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_occlusion(const OccParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_occlusion, dim3(1), dim3(OCC_T), 0, s, p);
    return hipGetLastError();
}

}  // namespace shs_internal
