// shs_occlusion.hip -- gfx950 kernels for the software occlusion pass:
//   culling_sw::run_software_occlusion_pass   shs-renderer-lib/include/shs/geometry/culling_software.hpp:229-331
//   project_aabb_to_screen_rect / is_rect_occluded                                    :137-218
//   rasterize_mesh_depth_transformed / rasterize_depth_triangle / project_world_to_screen :44-135
// The pass is sequential by definition: an object's test sees the depth of every visible object
// before it in view-depth order.  What does not depend on the buffer runs first, in parallel over
// the whole chip: k_occ_setup projects every object's AABB rect and sets up every triangle
// (project_world_to_screen x3, area, clamped bbox) into records.  k_occlusion then walks the
// objects in visit order in one 1024-thread workgroup, the next objects' records prefetched a step
// ahead, and parallelises inside each step: the rect test over its pixels, the raster over
// (triangle, pixel) pairs.  The occlusion buffer (300x225 in the reference demo) stays in L2; the
// depth min is an atomicMin on the float bits (every stored value is in [0, 1]), so the buffer
// after each object equals the reference's whatever order the pairs run in.
#include <float.h>

#include "shs_glm.hpp"
#include "shs_occlusion_internal.hpp"

namespace shs_dev {

constexpr int OCC_T = 1024;
constexpr int OCC_SETUP_T = 256;
constexpr int OCC_WIN = 1 << 17;                       // pairs per bitmap window
constexpr int OCC_WORDS = OCC_WIN / 64;

struct OccShared {
    // the chunk's rasterized triangles, compacted (slots 0 .. m-1 in triangle order)
    float4 ta[OCC_T], tb[OCC_T], tc[OCC_T];
    uint32_t start[OCC_T];                             // first pair of the slot
    unsigned long long bits[OCC_WORDS];                // bit k: a slot's pairs start at window pair k (16 KB)
    uint16_t wown[OCC_WORDS];                          // slot owning each word's first pair
    uint32_t wtot[OCC_T / 64][2];
    int not_occ;
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

// ---- k_occ_setup: one block per object (visit order) ----------------------------------------
__global__ __launch_bounds__(OCC_SETUP_T) void k_occ_setup(OccParams p) {
    const int s = (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63;
    const OccObject &o = p.objs[s];
    const int n_tris = o.n_idx / 3;
    // project_aabb_to_screen_rect: lanes 0-7 project one corner each, lane 0 folds them in the
    // reference's corner order (std::min / std::max are order-sensitive only for NaN)
    if (tid < 64) {
        float sx = 0.0f, sy = 0.0f, z01 = 0.0f;
        bool ok = false;
        if (lane < 8) {
            const int c = lane;
            const float v[4] = {(c & 1) ? o.aabb_max[0] : o.aabb_min[0], (c & 2) ? o.aabb_max[1] : o.aabb_min[1],
                                (c & 4) ? o.aabb_max[2] : o.aabb_min[2], 1.0f};
            float clip[4];
            m4v_occ(p.vp, v, clip);
            if (!(clip[3] <= 0.001f)) {
                const float nx = clip[0] / clip[3], ny = clip[1] / clip[3], nz = clip[2] / clip[3];
                z01 = nz * 0.5f + 0.5f;
                ok = !(z01 < 0.0f || z01 > 1.0f);
                sx = (nx + 1.0f) * 0.5f * (float)p.W;
                sy = (ny + 1.0f) * 0.5f * (float)p.H;
            }
        }
        float mnx = (float)p.W, mny = (float)p.H, mxx = -1.0f, mxy = -1.0f, near_depth = 1.0f;
        bool any = false;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const bool okc = __shfl((int)ok, c) != 0;
            const float cx = __shfl(sx, c), cy = __shfl(sy, c), cz = __shfl(z01, c);
            if (!okc) continue;
            mnx = occ_min(mnx, cx); mny = occ_min(mny, cy);
            mxx = occ_max(mxx, cx); mxy = occ_max(mxy, cy);
            near_depth = occ_min(near_depth, cz);
            any = true;
        }
        if (lane == 0) {
            OccRect r{};
            r.x0 = 0; r.y0 = 0; r.x1 = -1; r.y1 = -1;
            if (any) {
                r.x0 = max(0, (int)floorf(mnx)); r.y0 = max(0, (int)floorf(mny));
                r.x1 = min(p.W - 1, (int)ceilf(mxx)); r.y1 = min(p.H - 1, (int)ceilf(mxy));
            }
            r.z_near = (near_depth < 0.0f) ? 0.0f : ((1.0f < near_depth) ? 1.0f : near_depth);   // std::clamp
            r.valid = any && r.x0 <= r.x1 && r.y0 <= r.y1;
            r.tri_base = o.tri_base;
            r.n_tris = (uint32_t)n_tris;
            r.index = o.index;
            p.rects[s] = r;
        }
    }
    // rasterize_depth_triangle's setup per triangle; cnt = 0 when the reference would skip it
    for (int t = tid; t < n_tris; t += OCC_SETUP_T) {
        float sx[3] = {0, 0, 0}, sy[3] = {0, 0, 0}, sz[3] = {0, 0, 0};
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
        float area = 0.0f;
        uint32_t x0 = 0, y0 = 0, bw = 0, bh = 0;
        if (ok) {
            area = edge_fn(sx[0], sy[0], sx[1], sy[1], sx[2], sy[2]);
            if (!(fabsf(area) <= 1e-6f)) {
                const int ix0 = max(0, (int)floorf(occ_min(sx[0], occ_min(sx[1], sx[2]))));
                const int iy0 = max(0, (int)floorf(occ_min(sy[0], occ_min(sy[1], sy[2]))));
                const int ix1 = min(p.W - 1, (int)ceilf(occ_max(sx[0], occ_max(sx[1], sx[2]))));
                const int iy1 = min(p.H - 1, (int)ceilf(occ_max(sy[0], occ_max(sy[1], sy[2]))));
                if (ix0 <= ix1 && iy0 <= iy1) {
                    x0 = (uint32_t)ix0; y0 = (uint32_t)iy0;
                    bw = (uint32_t)(ix1 - ix0 + 1); bh = (uint32_t)(iy1 - iy0 + 1);
                }
            }
        }
        OccTri r;
        r.a = make_float4(sx[0], sy[0], sz[0], sx[1]);
        r.b = make_float4(sy[1], sz[1], sx[2], sy[2]);
        r.c = make_float4(sz[2], area, __uint_as_float(x0 | y0 << 16), __uint_as_float(bw | bh << 16));
        p.tris[o.tri_base + t] = r;
    }
}

// ---- k_occlusion: the sequential walk -----------------------------------------------------------
struct RectU {   // wave-uniform copy of an OccRect
    int x0, y0, x1, y1, valid;
    float z_near;
    uint32_t tri_base, n_tris, index;
};

struct RectRaw {  // an OccRect in flight (vector registers; made uniform once it has arrived)
    int4 a, b;
    int idx;
};

__device__ __forceinline__ RectRaw fetch_rect(const OccRect *r) {
    return RectRaw{*(const int4 *)r, *((const int4 *)r + 1), *((const int *)r + 8)};
}

__device__ __forceinline__ RectU uniform_rect(const RectRaw &raw) {
    const int4 a = raw.a, b = raw.b;
    const int idx = raw.idx;
    RectU u;
    u.x0 = __builtin_amdgcn_readfirstlane(a.x); u.y0 = __builtin_amdgcn_readfirstlane(a.y);
    u.x1 = __builtin_amdgcn_readfirstlane(a.z); u.y1 = __builtin_amdgcn_readfirstlane(a.w);
    u.z_near = __int_as_float(__builtin_amdgcn_readfirstlane(b.x));
    u.valid = __builtin_amdgcn_readfirstlane(b.y);
    u.tri_base = (uint32_t)__builtin_amdgcn_readfirstlane(b.z);
    u.n_tris = (uint32_t)__builtin_amdgcn_readfirstlane(b.w);
    u.index = (uint32_t)__builtin_amdgcn_readfirstlane(idx);
    return u;
}

// waits for this thread's outstanding memory operations (the depth atomics: vmcnt counts them on
// gfx9) and joins the workgroup, so that the next step's L2 loads see every lane's atomicMin
__device__ __forceinline__ void step_barrier() {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
}

__global__ __launch_bounds__(OCC_T) void k_occlusion(OccParams p) {
    __shared__ OccShared sh;
    const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npx = p.W * p.H;
    for (int i = tid; i < npx; i += OCC_T) p.depth[i] = __float_as_uint(1.0f);
    if (tid == 0) sh.n_vis = 0;
    unsigned long long tacc[3] = {0, 0, 0}, tprev = wall_clock64();
    auto tmark = [&](int k) {
        if (p.prof) { const unsigned long long t = wall_clock64(); tacc[k] += t - tprev; tprev = t; }
    };
    auto load_tri = [&](const RectU &r, uint32_t t) {
        OccTri v;
        if (t < r.n_tris) {
            v = p.tris[r.tri_base + t];
        } else {
            v.a = v.b = v.c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        return v;
    };
    // prefetched a step ahead: the rects of s + 1 and s + 2, the first triangle chunk of s + 1
    RectU cur = uniform_rect(fetch_rect(&p.rects[0]));
    RectU nxt = uniform_rect(fetch_rect(&p.rects[1]));   // p.rects holds n + 2 records (the last two zeroed)
    const uint32_t chunk = (uint32_t)p.chunk, ct = (uint32_t)tid < chunk ? (uint32_t)tid : 0xffffffffu;
    OccTri cur_t = load_tri(cur, ct);
    if (tid == 0) sh.not_occ = cur.valid ? 0 : 1;
    step_barrier();
    const unsigned long long upto = ((2ull << lane) - 1ull) & ~1ull;
    for (int s = 0; s < p.n; ++s) {
        const RectRaw nn = fetch_rect(&p.rects[s + 2]);
        const OccTri nxt_t = load_tri(nxt, ct);
        // is_rect_occluded: visible as soon as one pixel has z_near <= depth + eps (sh.not_occ was
        // initialised before the previous step's barrier, so nothing waits ahead of the depth loads)
        if (cur.valid) {
            const int rw = cur.x1 - cur.x0 + 1, n = rw * (cur.y1 - cur.y0 + 1);
            // 8 loads in flight per lane, then the compares; stop once any lane found a visible pixel
            constexpr int U = 8;
            for (int k0 = tid; k0 < n; k0 += U * OCC_T) {
                if (k0 != tid && __hip_atomic_load(&sh.not_occ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                float d[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = k0 + u * OCC_T;
                    d[u] = 0.0f;
                    if (k < n) {
                        const int y = cur.y0 + k / rw, x = cur.x0 + k % rw;
                        d[u] = load_depth(&p.depth[(size_t)y * p.W + x]);
                    }
                }
                bool vis = false;
#pragma unroll
                for (int u = 0; u < U; ++u) vis = vis || (k0 + u * OCC_T < n && cur.z_near <= d[u] + p.eps);
                if (vis) sh.not_occ = 1;
            }
        }
        __syncthreads();
        tmark(0);
        const bool visible = sh.not_occ != 0;
        if (tid == 0) {
            p.occluded[cur.index] = visible ? 0 : 1;
            if (visible) p.visible[sh.n_vis++] = cur.index;
        }
        if (visible) {
            // rasterize_mesh_depth_transformed: (triangle, pixel) pairs of up to p.chunk triangles at a time
            for (uint32_t c0 = 0; c0 < cur.n_tris; c0 += chunk) {
                const OccTri ts = c0 == 0 ? cur_t : load_tri(cur, ct == 0xffffffffu ? ct : c0 + ct);
                const uint32_t wh = __float_as_uint(ts.c.w), cnt = (wh & 0xffffu) * (wh >> 16);
                // compacted slot and first pair: block scans of (cnt > 0) and cnt
                uint32_t is = cnt ? 1u : 0u, ic = cnt;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t vs = (uint32_t)__shfl_up((int)is, off), vc = (uint32_t)__shfl_up((int)ic, off);
                    if (lane >= off) { is += vs; ic += vc; }
                }
                if (lane == 63) { sh.wtot[wave][0] = is; sh.wtot[wave][1] = ic; }
                __syncthreads();
                uint32_t sb = 0, cb = 0, total = 0;
#pragma unroll
                for (int w2 = 0; w2 < OCC_T / 64; ++w2) {
                    if (w2 < wave) { sb += sh.wtot[w2][0]; cb += sh.wtot[w2][1]; }
                    total += sh.wtot[w2][1];
                }
                const int slot = (int)(sb + is) - 1;
                const uint32_t first_pair = cb + ic - cnt;
                if (cnt) {
                    sh.ta[slot] = ts.a; sh.tb[slot] = ts.b; sh.tc[slot] = ts.c;
                    sh.start[slot] = first_pair;
                }
                // pairs in windows of OCC_WIN: a start bitmap + each word's owner; a pair's slot is
                // its word's owner plus the starts up to it (k % 64 == lane: the stride is 1024)
                for (uint32_t w0 = 0; w0 < total; w0 += OCC_WIN) {
                    const uint32_t wend = min(total, w0 + OCC_WIN);
                    const int nwords = (int)((wend - w0 + 63) >> 6);
                    if (w0) __syncthreads();
                    for (int i = tid; i < nwords; i += OCC_T) sh.bits[i] = 0ull;
                    __syncthreads();
                    if (cnt) {
                        const uint32_t a = first_pair, e = first_pair + cnt;   // [a, e)
                        if (a >= w0 && a < wend) atomicOr(&sh.bits[(a - w0) >> 6], 1ull << ((a - w0) & 63));
                        const uint32_t lo = max(a, w0), hi = min(e, wend);
                        if (lo < hi)
                            for (uint32_t wd = (lo - w0 + 63) >> 6; w0 + wd * 64 < hi; ++wd) sh.wown[wd] = (uint16_t)slot;
                    }
                    __syncthreads();
                    for (uint32_t k = w0 + (uint32_t)tid; k < wend; k += OCC_T) {
                        const uint32_t wd = (k - w0) >> 6;
                        const int q = (int)sh.wown[wd] + __popcll(sh.bits[wd] & upto);
                        const int local = (int)(k - sh.start[q]);
                        const float4 A = sh.ta[q], B = sh.tb[q], C = sh.tc[q];
                        const uint32_t xy0 = __float_as_uint(C.z);
                        const int w = (int)(__float_as_uint(C.w) & 0xffffu);
                        // local / w and local % w: a float quotient, then exact integer corrections
                        int yy = (int)((float)local * __frcp_rn((float)w));
                        int xx = local - yy * w;
                        while (xx < 0) { --yy; xx += w; }
                        while (xx >= w) { ++yy; xx -= w; }
                        const int x = (int)(xy0 & 0xffffu) + xx, y = (int)(xy0 >> 16) + yy;
                        const float qx = (float)x + 0.5f, qy = (float)y + 0.5f;
                        // corners (A.x, A.y, A.z), (A.w, B.x, B.y), (B.z, B.w, C.x); signed area C.y
                        const float w0e = edge_fn(A.w, B.x, B.z, B.w, qx, qy);
                        const float w1e = edge_fn(B.z, B.w, A.x, A.y, qx, qy);
                        const float w2e = edge_fn(A.x, A.y, A.w, B.x, qx, qy);
                        const float area = C.y;
                        const bool inside = area > 0.0f ? (w0e >= 0.0f && w1e >= 0.0f && w2e >= 0.0f)
                                                        : (w0e <= 0.0f && w1e <= 0.0f && w2e <= 0.0f);
                        if (!inside) continue;
                        const float d = (w0e / area) * A.z + (w1e / area) * B.y + (w2e / area) * C.x;
                        if (d < 0.0f || d > 1.0f) continue;
                        // -0 stores as +0 (they compare equal in every later test)
                        atomicMin(&p.depth[(size_t)y * p.W + x], d == 0.0f ? 0u : __float_as_uint(d));
                    }
                }
                __syncthreads();
            }
        }
        tmark(1);
        __syncthreads();   // every lane has read sh.not_occ
        if (tid == 0) sh.not_occ = nxt.valid ? 0 : 1;
        step_barrier();
        tmark(2);
        cur = nxt;
        nxt = uniform_rect(nn);
        cur_t = nxt_t;
    }
    if (tid == 0) *p.n_visible = sh.n_vis;
    if (p.prof && tid == 0)
        printf("occ prof (10ns ticks): test %llu raster %llu barrier %llu n %d\n", tacc[0], tacc[1], tacc[2], p.n);
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

hipError_t launch_occlusion(const OccParams &p, hipStream_t s) {
    if (p.n > 0) hipLaunchKernelGGL(k_occ_setup, dim3(p.n), dim3(OCC_SETUP_T), 0, s, p);
    hipLaunchKernelGGL(k_occlusion, dim3(1), dim3(OCC_T), 0, s, p);
    return hipGetLastError();
}

}  // namespace shs_internal
