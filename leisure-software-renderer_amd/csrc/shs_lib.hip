// shs_lib.hip -- gfx950 kernels for the shs-renderer-lib software raster path.
//
// Replaces rasterize_mesh (sw_render/rasterizer.hpp:181-442) with the builtin PBR / Blinn-Phong /
// debug programs (shader/builtin_shaders.hpp:25-245) as PassPBRForward runs it
// (passes/pass_pbr_forward.hpp:49-214), and the depth pass of PassShadowMap
// (passes/pass_shadow_map.hpp:144-204).  Paths are relative to
// /root/reference/cpp-folders/src/shs-renderer-lib/include/shs/.
//
// Launches per pass, on one HIP stream:
//   k_lib_blocks  (region-sharded camera pass) the setup sub-blocks whose projected chunk boxes can
//                 reach the rank's rectangle, listed for k_lib_setup.
//   k_lib_setup   one thread per input triangle: VS x3, trivial accept (or a queue entry for the
//                 clipper), NDC -> screen (rows y-up), area / cull / bbox rejects, the per-primitive
//                 half of barycentric_2d and the 1/w terms (a 64-B LibRec + an 80-B LibShade of
//                 varyings premultiplied by 1/w per primitive), "busy" marks on the 32x8 raster tiles
//                 of its bbox and, for large scenes, per-32x32-tile bin appends (block-aggregated in
//                 LDS); primitives over many tiles go to a pass-wide queue with their task prefix.
//   k_lib_clip    (camera pass) the queued triangles: Sutherland-Hodgman against the six clip planes
//                 by 16-lane groups with the polygon in registers, then the fans as above.
//   k_lib_bigmark the queued large primitives' (primitive, tile) marks / appends over the whole chip.
//   k_lib_dyn     (camera pass) the raster's dynamic work items compacted per ticket queue, heavy
//                 tiles first.
//   k_lib_raster  persistent over the owned raster tiles: busy tiles stage their candidates'
//                 records in LDS and deal every (primitive, pixel) pair to one lane; each passing
//                 pair atomic-mins a 64-bit key (z01 bits, submission order) into LDS -- identical
//                 to the reference's in-order strict-less test on a cleared buffer.  The shadow pass
//                 writes each texel's depth here (idle tiles get the clear depth); the camera pass
//                 hands each 16x4 block's winners to k_lib_resolve as 4-B words, with a flag per block
//                 that holds one.
//   k_lib_resolve (camera pass) every owned pixel: the winner re-evaluated, its varyings interpolated,
//                 the fragment program run (+ the fused PassTonemap), HDR colour, depth, motion written;
//                 pixels without a winner get the clear values, so every output byte is written exactly
//                 once per pass.
// Primitive order: input triangle t's fan triangle k has submission index t*16 + k (a clipped
// triangle yields at most 7 fans in exact arithmetic, MAX_POLY - 2 with rounding); fan 0 lives in
// slot t, fans >= 1 in extra slots from xbase[t].  t is the submission index (draw base + MeshData
// index); a spatially ordered mesh stores triangle t at another slot, which the setup records in s2s.
#include <float.h>

#include <algorithm>
#include <climits>
#include <type_traits>

#include "shs_device.hpp"
#include "shs_lib_device.hpp"
#include "shs_lib_internal.hpp"
#include "shs_post_internal.hpp"
#include "shs_wave.hpp"

namespace shs_dev {

constexpr float PI_F = 3.14159265358979323846264338327950288f;   // glm::pi<float>()

// ---- std:: scalar semantics used by the builtin programs -------------------------------------
__device__ __forceinline__ float s_max(float a, float b) { return (a < b) ? b : a; }        // std::max
__device__ __forceinline__ float s_min(float a, float b) { return (b < a) ? b : a; }        // std::min
__device__ __forceinline__ float s_clamp(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }
__device__ __forceinline__ int s_clampi(int v, int lo, int hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }
__device__ __forceinline__ float g_clamp(float x, float lo, float hi) { return g_min(g_max(x, lo), hi); }  // glm::clamp
__device__ __forceinline__ float g_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }      // glm::mix
__device__ __forceinline__ f3 mix3(f3 a, f3 b, float t) { return {g_mix(a.x, b.x, t), g_mix(a.y, b.y, t), g_mix(a.z, b.z, t)}; }
__device__ __forceinline__ f3 mul3(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 gmax3(f3 a, f3 b) { return {g_max(a.x, b.x), g_max(a.y, b.y), g_max(a.z, b.z)}; }
__device__ __forceinline__ f3 neg3(f3 a) { return {-a.x, -a.y, -a.z}; }

struct f4 { float x, y, z, w; };
// glm mat4 * vec4: (m0*x + m1*y) + (m2*z + m3*w)
__device__ __forceinline__ f4 m4v(const float *m, f4 v) {
    return {(m[0] * v.x + m[4] * v.y) + (m[8] * v.z + m[12] * v.w), (m[1] * v.x + m[5] * v.y) + (m[9] * v.z + m[13] * v.w),
            (m[2] * v.x + m[6] * v.y) + (m[10] * v.z + m[14] * v.w), (m[3] * v.x + m[7] * v.y) + (m[11] * v.z + m[15] * v.w)};
}

constexpr int LIB_RTW = 32, LIB_RTH = 8;   // raster tile (one 256-thread workgroup, one pixel per lane)
// Candidate ids gathered per round: k_lib_raster comes in two sizes.  1024 (3 workgroups per CU by
// LDS, 119 VGPRs): deep per-tile lists (C4: up to ~6K candidates per bin tile, depth-sorted per round).
// 256 (24 KB LDS, 80 VGPRs: 6 workgroups per CU): passes whose fullest bin tile fits one round (C5's
// 62), chosen from the previous frame's statistics (LibWork::st_maxbin).
constexpr int LIB_CAND_DEEP = 1024, LIB_CAND_SHALLOW = 256;
static_assert(LIB_HSORT_MIN == (uint32_t)LIB_CAND_DEEP, "k_lib_hsort sorts the lists of more than one deep round");
constexpr int LIB_CHUNK = 128;             // records staged in LDS per pass
#ifndef SHS_HIZ_BOX
#define SHS_HIZ_BOX 16                     // deep raster: boxes up to this many pixels are tested against their pixels' keys
#endif
#ifndef SHS_HSORT_GRID
#define SHS_HSORT_GRID 256                 // k_lib_hsort workgroups (one per CU)
#endif
constexpr int MAX_POLY = 16;               // clipped polygon capacity (3 + 6 planes x up to 2 crossings)

// A footprint shadow pass's row spans (shs_footprint.hpp footprint_rows): a bin tile of the rectangle
// outside its row's span is never read by the camera pass, so nothing is binned to or rasterised on it
// (its raster tiles are only cleared).  span_rows 0: the whole rectangle.
__device__ __forceinline__ bool lib_in_span(const LibFrameParams &fp, int bx, int by) {
    if (fp.span_rows == 0) return true;
    if (by < 0 || by >= fp.span_rows) return false;
    const uint32_t s = fp.span[by];
    return bx >= (int)(s & 0xffffu) && bx <= (int)(s >> 16);
}

__device__ __forceinline__ bool lib_owned(const LibFrameParams &fp, int bx, int by) {
    return shard_owned(fp.rank, fp.count, fp.reg, bx, by, fp.tiles_x) && lib_in_span(fp, bx, by);
}

// Does the bin-tile rectangle [tx0, tx1] x [ty0, ty1] hold a tile this pass renders?  The span test
// walks the rows (a kernel-argument load each): a rectangle over more than max_rows rows is kept
// (conservative; its bin appends still test each tile).
__device__ inline bool lib_owns_any(const LibFrameParams &fp, int tx0, int tx1, int ty0, int ty1, int max_rows = LIB_SPAN_ROWS) {
    if (!shard_owns_any(fp.rank, fp.count, fp.reg, tx0, tx1, ty0, ty1, fp.tiles_x)) return false;
    if (fp.span_rows == 0) return true;
    const int xa = max(tx0, fp.reg.x0), xb = min(tx1, fp.reg.x1);
    const int ya = max(ty0, fp.reg.y0), yb = min(ty1, min(fp.reg.y1, fp.span_rows - 1));
    if (yb - ya >= max_rows) return true;
    for (int y = ya; y <= yb; ++y) {
        const uint32_t s = fp.span[y];
        if (max(xa, (int)(s & 0xffffu)) <= min(xb, (int)(s >> 16))) return true;
    }
    return false;
}

// Orderable key bits (z_key's high word) of a conservative lower bound of the depth lib_test can
// produce anywhere on the primitive.  The camera pass's 1/w depth is a weighted mean of the corners'
// clip z (weights bc_k / w_k >= 0) or, linear, 1 / sum(bc_k / w_k) with sum(bc) = 1 +- 2 ulp -- both
// bounded below by the corner minimum; the shadow pass's affine NDC z likewise.  The margin (1e-5
// of the magnitudes, ~170 ulp) covers every rounding on the way.  Non-finite inputs never cull (0).
template <bool SHADOW>
__device__ __forceinline__ uint32_t lib_zmin_ord(const LibFrameParams &fp, const LibRec &r) {
    float z01;
    if (SHADOW) {
        if (!(isfinite(r.z0) && isfinite(r.z1) && isfinite(r.z2))) return 0u;
        const float lo = fminf(fminf(r.z0, r.z1), r.z2);
        const float mag = fmaxf(fmaxf(fabsf(r.z0), fabsf(r.z1)), fabsf(r.z2));
        z01 = s_clamp((lo - 1e-5f * (1.0f + mag)) * 0.5f + 0.5f, 0.0f, 1.0f);
    } else {
        if (!(r.iw0 > 0.0f && r.iw1 > 0.0f && r.iw2 > 0.0f && isfinite(r.iw0) && isfinite(r.iw1) && isfinite(r.iw2)))
            return 0u;
        if (fp.flags & LF_LINZ) {
            const float lo = fminf(fminf(1.0f / r.iw0, 1.0f / r.iw1), 1.0f / r.iw2);
            z01 = g_clamp((lo * (1.0f - 1e-5f) - fp.zn) / fp.zspan, 0.0f, 1.0f);
        } else {
            const float c0 = r.z0 / r.iw0, c1 = r.z1 / r.iw1, c2 = r.z2 / r.iw2;
            if (!(isfinite(c0) && isfinite(c1) && isfinite(c2))) return 0u;
            const float lo = fminf(fminf(c0, c1), c2);
            const float mag = fmaxf(fmaxf(fabsf(c0), fabsf(c1)), fabsf(c2));
            z01 = g_clamp((lo - 1e-5f * (1.0f + mag)) * 0.5f + 0.5f, 0.0f, 1.0f);
        }
    }
    if (!isfinite(z01)) return 0u;
    return (uint32_t)(z_key(z01, 0u) >> 32);
}

__device__ __forceinline__ uint64_t tl_now() { return __builtin_amdgcn_s_memrealtime(); }

// The depth bucket of a bound z over a sorted list's range (lo, hi): 256 buckets, monotone in z (the
// float subtraction, product and truncation all are) -- k_lib_hsort sorts by it and k_lib_raster stops
// a tile's candidate rounds by it, with the identical arithmetic.
__device__ __forceinline__ uint32_t hs_bucket(uint2 range, uint32_t z) {
    const float scale = range.y > range.x ? 255.0f / (float)(range.y - range.x) : 0.0f;
    return z <= range.x ? 0u : min(255u, (uint32_t)((float)(z - range.x) * scale));
}


// ---- k_lib_setup ------------------------------------------------------------------------------

// A clip-space vertex with the varyings the builtin VS sets (make_default_vertex_out,
// builtin_shaders.hpp:87-103): WorldPos, NormalWS, UV0 (Color0 is never read by the programs).
struct LVert {
    float cx, cy, cz, cw;
    float wx, wy, wz;
    float nx, ny, nz;
    float u, v;
};

// The normal and UV0 varyings of a vertex (the half of make_default_vertex_out that only surviving
// primitives need; UV0 only for draws that sample a base_color_tex).
__device__ __forceinline__ void vertex_attrs(const LibDrawGPU &dr, uint32_t id, LVert &o) {
    const float *N = dr.nrm + 3 * (size_t)id;
    const f3 n = normalize3(m3v(dr.nmat, f3{N[0], N[1], N[2]}));
    o.nx = n.x; o.ny = n.y; o.nz = n.z;
    if (dr.tex) {
        const float2 t = *reinterpret_cast<const float2 *>(dr.uv + 2 * (size_t)id);
        o.u = t.x; o.v = t.y;
    }
}

// Clip and world position (the varyings are left 0 until vertex_attrs).
__device__ __forceinline__ LVert vertex_pos(const LibDrawGPU &dr, uint32_t id) {
    const float *P = dr.pos + 3 * (size_t)id;
    LVert o;
    const f4 wp = m4v(dr.model, f4{P[0], P[1], P[2], 1.0f});
    const f4 c = m4v(dr.viewproj, wp);
    o.cx = c.x; o.cy = c.y; o.cz = c.z; o.cw = c.w;
    o.wx = wp.x; o.wy = wp.y; o.wz = wp.z;
    o.nx = o.ny = o.nz = 0.0f;
    o.u = o.v = 0.0f;
    return o;
}

__device__ __forceinline__ LVert vertex_pos_xyz(const LibDrawGPU &dr, float x, float y, float z) {
    LVert o;
    const f4 wp = m4v(dr.model, f4{x, y, z, 1.0f});
    const f4 c = m4v(dr.viewproj, wp);
    o.cx = c.x; o.cy = c.y; o.cz = c.z; o.cw = c.w;
    o.wx = wp.x; o.wy = wp.y; o.wz = wp.z;
    o.nx = o.ny = o.nz = 0.0f;
    o.u = o.v = 0.0f;
    return o;
}

__device__ __forceinline__ LVert vertex_out(const LibDrawGPU &dr, uint32_t id) {
    LVert o = vertex_pos(dr, id);
    vertex_attrs(dr, id, o);
    return o;
}

__device__ __forceinline__ bool fully_inside(const LVert &v) {   // rasterizer.hpp:232-240
    if (!(v.cw > 0.0f)) return false;
    return (v.cx >= -v.cw && v.cx <= v.cw) && (v.cy >= -v.cw && v.cy <= v.cw) && (v.cz >= -v.cw && v.cz <= v.cw);
}

// detail::lerp_rv on the varyings the FS reads (rasterizer.hpp:69-79): every component glm::mix'ed
// (the NormalWS varying is NOT renormalised -- only the unused RasterVertex::normal_ws is).
__device__ __forceinline__ LVert lerp_v(const LVert &a, const LVert &b, float t) {
    LVert o;
    const float *pa = &a.cx, *pb = &b.cx;
    float *po = &o.cx;
#pragma unroll
    for (int i = 0; i < 12; ++i) po[i] = g_mix(pa[i], pb[i], t);
    return o;
}

__device__ __forceinline__ float plane_dist(const LVert &v, int p) {   // plane_dist_left .. far (:81-109)
    switch (p) {
        case 0: return v.cx + v.cw;
        case 1: return v.cw - v.cx;
        case 2: return v.cy + v.cw;
        case 3: return v.cw - v.cy;
        case 4: return v.cz + v.cw;
        default: return v.cw - v.cz;
    }
}

// detail::clip_polygon_frustum (:111-164) for the triangles k_lib_setup queues (not trivially inside),
// run by a group of CLIP_G = 16 lanes per triangle with the polygon in registers: lane L holds polygon
// buffer entry L (polygon vertex j is lane (j + rot) % n).  Per plane every lane evaluates the edge
// that starts at its vertex (clip_polygon_plane's loop body: 0, 1 or 2 outputs), a scan over the edges
// in polygon order gives each edge's output position, and every output lane pulls its vertex from the
// edge that produced it -- the reference's sequential output, vertex for vertex, with no LDS and no
// scratch.  A plane every vertex is inside of only rotates the polygon by one (each edge emits its end
// vertex), kept as an index rotation.  Capacity MAX_POLY = CLIP_G: edges whose output position exceeds
// MAX_POLY - 2 emit nothing (unreachable for a convex polygon: <= 1 vertex added per plane).
constexpr int CLIP_G = 16;

__device__ __forceinline__ float grp_shfl(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ int grp_shfl(int v, int src) { return __shfl(v, src, 64); }

__device__ __forceinline__ LVert grp_shfl_v(const LVert &v, int src) {
    LVert o;
    const float *pv = &v.cx;
    float *po = &o.cx;
#pragma unroll
    for (int c = 0; c < 12; ++c) po[c] = grp_shfl(pv[c], src);
    return o;
}

// Returns the polygon size (<= MAX_POLY); v = this lane's buffer vertex, rot as above.  Every lane of
// the 16-lane group (lanes seg .. seg + 15 of the wave, li = lane - seg) calls it: group-uniform
// control flow.
__device__ __forceinline__ int clip_frustum_group(LVert &v, int li, int seg, int &rot) {
    static_assert(MAX_POLY == CLIP_G, "one polygon vertex per group lane");
    int n = 3;
    rot = 0;
    for (int p = 0; p < 6 && n > 0; ++p) {
        const bool has = li < n;
        const float da = has ? plane_dist(v, p) : 0.0f;
        const bool cin = da >= 0.0f;
        const uint32_t out_mask = (uint32_t)(__ballot(has && !cin) >> seg) & 0xFFFFu;
        if (out_mask == 0u) {
            rot = rot + 1 == n ? 0 : rot + 1;
            continue;
        }
        // the edge (this vertex -> its successor) of clip_polygon_plane
        const int succ = li + 1 >= n ? 0 : li + 1;
        const LVert x = grp_shfl_v(v, seg + succ);
        const float db = grp_shfl(da, seg + succ);
        const bool xin = db >= 0.0f;
        int cnt = 0;
        LVert outA = x;
        if (has) {
            if (cin && xin) {
                cnt = 1;
            } else if (cin != xin) {
                const float denom = da - db;
                const bool ok = fabsf(denom) > 1e-8f;
                if (ok) outA = lerp_v(v, x, da / denom);
                cnt = (ok ? 1 : 0) + (xin ? 1 : 0);
            }
        }
        // edges in polygon order: logical edge i starts at lane (i + rot) % n
        const int phys_of = has ? (li + rot >= n ? li + rot - n : li + rot) : li;
        const int cl_raw = grp_shfl(cnt, seg + phys_of);
        const int cl = has ? cl_raw : 0;
        int incl = cl;
#pragma unroll
        for (int o = 1; o < CLIP_G; o <<= 1) {
            const int u = __shfl_up(incl, o, CLIP_G);
            if (li >= o) incl += u;
        }
        const int excl = incl - cl;
        const int emit = (has && excl <= MAX_POLY - 2) ? cl : 0;   // the sequential loop's capacity break
        int m = emit ? excl + emit : 0;
#pragma unroll
        for (int o = 1; o < CLIP_G; o <<= 1) m = max(m, __shfl_xor(m, o, CLIP_G));
        // output k = li: the last logical edge i with excl_i <= k (binary lifting over the monotone
        // excl; an edge that emits nothing shares its excl with the next one)
        int src = 0;
#pragma unroll
        for (int step = CLIP_G / 2; step >= 1; step >>= 1) {
            const int cand = src + step;
            const int e = grp_shfl(excl, seg + (cand < CLIP_G ? cand : CLIP_G - 1));
            if (cand < n && e <= li) src = cand;
        }
        const int e_src = grp_shfl(excl, seg + src);
        const int p_src = src + rot >= n ? src + rot - n : src + rot;   // the edge's start vertex lane
        const int p_nxt = p_src + 1 >= n ? 0 : p_src + 1;              // its end vertex lane
        const LVert a_src = grp_shfl_v(outA, seg + p_src);
        const LVert x_src = grp_shfl_v(v, seg + p_nxt);
        if (li < m) v = (li == e_src) ? a_src : x_src;
        n = m;
        rot = 0;
    }
    return n;
}

// A bin entry carries the primitive's box and depth bound beside its slot (e = slot, box x, box y,
// zord), so the raster's gather reads its candidates' boxes and bounds from the tile's contiguous list
// instead of one scattered 8-B and 4-B load per candidate.  (Spilled entries keep the slot only.)
__device__ __forceinline__ void lib_append_bin(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, int t,
                                               uint32_t pos, uint4 e) {
    if (pos < fp.bin_cap) {
        fb.bins[(size_t)t * fp.bin_cap + pos] = e;
    } else {
        const uint32_t sp = atomicAdd(&cnt[LC_SPILL], 1u);
        if (sp < fp.spill_cap) fb.spill[sp] = make_uint2((uint32_t)t, e.x);
        else raise_overflow(&cnt[LC_OVERFLOW], LOV_SPILL, fb.ov_host);
    }
}

// Busy marks on the owned raster tiles of [x0,x1] x [y0,y1] and (bin mode) per-bin-tile appends,
// tiles k0, k0 + dk, ... of the box (one thread: k0 = 0, dk = 1; a whole block: k0 = tid, dk = 256).
__device__ __forceinline__ void lib_mark_range(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, int x0, int x1, int y0, int y1,
                               uint32_t slot, int k0, int dk, uint32_t zk) {
    const bool sharded = fp.count > 1;
    {
        const int rx0 = x0 / LIB_RTW, ry0 = y0 / LIB_RTH, nx = x1 / LIB_RTW - rx0 + 1, n = nx * (y1 / LIB_RTH - ry0 + 1);
        for (int k = k0; k < n; k += dk) {
            const int rx = rx0 + k % nx, ry = ry0 + k / nx;
            if (!sharded || lib_owned(fp, rx, ry / (TILE / LIB_RTH))) fb.busy[ry * fp.tiles_x + rx] = 1u;
        }
    }
    if (fp.scan_mode) return;
    uint32_t *tcount = fb.tile_count + (size_t)fp.parity * fp.tiles_x * fp.tiles_y;
    const int bx0 = x0 / TILE, by0 = y0 / TILE, nx = x1 / TILE - bx0 + 1, n = nx * (y1 / TILE - by0 + 1);
    for (int k = k0; k < n; k += dk) {
        const int bx = bx0 + k % nx, by = by0 + k / nx;
        if (sharded && !lib_owned(fp, bx, by)) continue;
        const int t = by * fp.tiles_x + bx;
        lib_append_bin(fp, fb, cnt, t, atomicAdd(&tcount[t], 1u), make_uint4(slot, pack16(x0, x1), pack16(y0, y1), zk));
    }
}

// The (primitive, tile) tasks of a large primitive: its owned-or-not raster tiles (busy marks) then, in
// bin mode, its bin tiles (appends).
__device__ __forceinline__ uint32_t big_tasks(const LibFrameParams &fp, uint4 e, uint32_t &n_busy) {
    const int x0 = (int)lo16(e.y), x1 = (int)hi16(e.y), y0 = (int)lo16(e.z), y1 = (int)hi16(e.z);
    n_busy = (uint32_t)((x1 / LIB_RTW - x0 / LIB_RTW + 1) * (y1 / LIB_RTH - y0 / LIB_RTH + 1));
    const uint32_t n_bin = fp.scan_mode ? 0u : (uint32_t)((x1 / TILE - x0 / TILE + 1) * (y1 / TILE - y0 / TILE + 1));
    return n_busy + n_bin;
}

// Appends n entries with `tasks` tasks in all to the large-primitive queue: -> (first entry, its task
// prefix).  One 64-bit atomic: entries and tasks are handed out in the same order.
__device__ __forceinline__ uint2 bigq_reserve(uint32_t *cnt, uint32_t n, uint32_t tasks) {
    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long *>(&cnt[LC_BIGT]),
                                             ((unsigned long long)n << 32) | (unsigned long long)tasks);
    return make_uint2((uint32_t)(old >> 32), (uint32_t)old);
}

// Primitives covering more than SMALL_MARK raster tiles are queued in LDS and marked by the whole
// setup block after its triangles are done (a floor triangle at 4K spans thousands of tiles).
constexpr int SMALL_MARK = 8;
constexpr int BIG_CAP = 512;
// Block-aggregated marks: every thread may defer one primitive of <= 2x2 bin tiles; the block then
// counts its appends per bin tile in LDS over the union of the deferred boxes and takes one global
// atomicAdd per touched bin tile (a block's triangles are neighbours in the mesh, so the union is
// small; C4's 1M triangles otherwise hit each bin counter ~120 times).  List order inside a bin does
// not matter: the raster resolves by (z, submission index) keys.
constexpr int AGG_BINS = 256;             // union capacity in bin tiles (else the per-primitive path)
#ifndef SHS_DEFER_BT
#define SHS_DEFER_BT 2
#endif
constexpr int DEFER_BT = SHS_DEFER_BT;    // deferred primitives span at most DEFER_BT x DEFER_BT bin tiles
struct Pend {
    uint32_t slot = 0, zk = 0;
    int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
    bool valid = false;
};
struct SetupShared {
    uint4 big[BIG_CAP];       // (slot, bx, by, 0)
    uint32_t pre[2][BIG_CAP + 1]; // large primitives: task prefix; [1]: queue bases, wave sums
    uint32_t nbig;
    uint32_t stat[2];
    int ub[4];                // union of deferred bin rects: bx0, by0, bx1, by1
    uint32_t bcnt[AGG_BINS];  // per union bin tile: deferred appends, then their base in the bin list
    uint32_t rbusy[AGG_BINS]; // per union bin tile: bit r = raster row r of it is busy
};

__device__ __forceinline__ void lib_mark(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, int x0, int x1, int y0, int y1,
                         uint32_t slot, SetupShared &ss, Pend &pend, uint32_t zk) {
    if (!pend.valid && (x1 / TILE - x0 / TILE) < DEFER_BT && (y1 / TILE - y0 / TILE) < DEFER_BT) {
        pend.slot = slot; pend.zk = zk; pend.x0 = x0; pend.x1 = x1; pend.y0 = y0; pend.y1 = y1; pend.valid = true;
        return;
    }
    const int n_rt = (x1 / LIB_RTW - x0 / LIB_RTW + 1) * (y1 / LIB_RTH - y0 / LIB_RTH + 1);
    if (n_rt > SMALL_MARK) {
        const uint32_t q = atomicAdd(&ss.nbig, 1u);
        if (q < BIG_CAP) {
            ss.big[q] = make_uint4(slot, pack16(x0, x1), pack16(y0, y1), zk);
            return;
        }
    }
    lib_mark_range(fp, fb, cnt, x0, x1, y0, y1, slot, 0, 1, zk);   // small, or the queue is full
}

__device__ __forceinline__ void store_box(const LibBuffers &fb, uint32_t slot, int x0, int x1, int y0, int y1) {
    fb.boxes[slot] = make_uint2(pack16(x0, x1), pack16(y0, y1));
}

// One fan triangle of rasterize_mesh (rasterizer.hpp:255-328): NDC, screen (y-up), the area /
// cull / bbox rejects; writes the primitive's record, varyings and box into slot.  Counts
// tri_after_clip / tri_raster like the reference.
// lazy_ids (trivially inside triangles): a, b, c hold positions only; the normal / UV varyings are
// loaded and transformed for primitives that survive the culls.
// direct (k_lib_clip): marks without the block aggregation -- small boxes marked by the thread, large
// ones queued for k_lib_bigmark (ss / pend unused).
// The screen-space half of a fan triangle (rasterizer.hpp:255-292): NDC -> screen, the area / cull /
// bbox rejects (n_rast counts a non-empty bbox) and barycentric_2d's den; in a tile-sharded pass a
// primitive of <= 2x2 bin tiles on none of this rank's is dropped too.  -> live.
__device__ __forceinline__ bool fan_screen(const LibFrameParams &fp, const LibDrawGPU &dr, const LVert &a, const LVert &b,
                                           const LVert &c, float (&sx)[3], float (&sy)[3], int &x0, int &x1, int &y0,
                                           int &y1, float &den, uint32_t &n_rast) {
    const LVert *v[3] = {&a, &b, &c};
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float nx = v[k]->cx / v[k]->cw, ny = v[k]->cy / v[k]->cw, nz = v[k]->cz / v[k]->cw;
        finite = finite && isfinite(nx) && isfinite(ny) && isfinite(nz);
        sx[k] = (nx * 0.5f + 0.5f) * (float)(fp.W - 1);
        sy[k] = (ny * 0.5f + 0.5f) * (float)(fp.H - 1);
    }
    x0 = 0; x1 = -1; y0 = 0; y1 = -1;
    bool live = false;
    den = 0.0f;
    if (finite) {
        const float e0x = sx[1] - sx[0], e0y = sy[1] - sy[0], e1x = sx[2] - sx[0], e1y = sy[2] - sy[0];
        const float area2 = e0x * e1y - e0y * e1x;
        const bool is_front = (area2 > 0.0f) == (dr.front_ccw != 0);
        const bool culled = (dr.cull_mode == 1 && !is_front) || (dr.cull_mode == 2 && is_front);
        if (!(fabsf(area2) < 1e-10f) && !culled) {
            x0 = max(0, (int)floorf(s_min(s_min(sx[0], sx[1]), sx[2])));
            x1 = min(fp.W - 1, (int)ceilf(s_max(s_max(sx[0], sx[1]), sx[2])));
            y0 = max(0, (int)floorf(s_min(s_min(sy[0], sy[1]), sy[2])));
            y1 = min(fp.H - 1, (int)ceilf(s_max(s_max(sy[0], sy[1]), sy[2])));
            if (x0 <= x1 && y0 <= y1) {
                ++n_rast;
                // barycentric_2d's den (== area2) returns bc = -1 at every pixel below 1e-8
                den = e0x * e1y - e1x * e0y;
                live = !(fabsf(den) < 1e-8f);
            }
        }
    }
    if (live && fp.count > 1) {
        // tile-sharded pass: a small primitive (any primitive, region ownership) on no owned 32x32 tile
        // is not needed on this rank (its record, varyings and marks are skipped; the frame counters
        // still count it)
        const int tx0 = x0 / TILE, tx1 = x1 / TILE, ty0 = y0 / TILE, ty1 = y1 / TILE;
        if (fp.reg.on) {
            live = lib_owns_any(fp, tx0, tx1, ty0, ty1, 2);   // per primitive: at most two rows walked
        } else if ((tx1 - tx0) < 2 && (ty1 - ty0) < 2) {
            bool mine = false;
            for (int ty = ty0; ty <= ty1; ++ty)
                for (int tx = tx0; tx <= tx1; ++tx) mine = mine || lib_owned(fp, tx, ty);
            live = mine;
        }
    }
    return live;
}

template <bool DIRECT = false>
__device__ __forceinline__ void emit_fan(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, const LibDrawGPU &dr, int d,
                         uint32_t seq, uint32_t slot, LVert a, LVert b, LVert c, uint32_t &n_clip,
                         uint32_t &n_rast, SetupShared &ss, Pend &pend, const uint32_t *lazy_ids = nullptr) {
    ++n_clip;
    LVert *v[3] = {&a, &b, &c};
    float sx[3], sy[3], den;
    int x0, x1, y0, y1;
    if (!fan_screen(fp, dr, a, b, c, sx, sy, x0, x1, y0, y1, den, n_rast)) {
        store_box(fb, slot, 0, -1, 0, -1);
        return;
    }
    if (lazy_ids) {
#pragma unroll
        for (int k = 0; k < 3; ++k) vertex_attrs(dr, lazy_ids[k], *v[k]);
    }
    LibRec r;
    r.ax = sx[0]; r.ay = sy[0];
    r.v0x = sx[1] - sx[0]; r.v0y = sy[1] - sy[0];
    r.v1x = sx[2] - sx[0]; r.v1y = sy[2] - sy[0];
    r.inv_den = 1.0f / den;
    const float iw0 = 1.0f / a.cw, iw1 = 1.0f / b.cw, iw2 = 1.0f / c.cw;
    r.iw0 = iw0; r.iw1 = iw1; r.iw2 = iw2;
    r.z0 = a.cz * iw0; r.z1 = b.cz * iw1; r.z2 = c.cz * iw2;
    r.seq = seq;
    r.bx = pack16(x0, x1); r.by = pack16(y0, y1);
    if (!SHS_LIB_EXP(fp, 4u)) fb.recs[slot] = r;
    const uint32_t zk = (fp.flags & LF_DEPTH) ? lib_zmin_ord<false>(fp, r) : 0u;
    fb.zord[slot] = zk;
    LibShade s;
    const float iw[3] = {iw0, iw1, iw2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s.wp[3 * k] = v[k]->wx * iw[k]; s.wp[3 * k + 1] = v[k]->wy * iw[k]; s.wp[3 * k + 2] = v[k]->wz * iw[k];
        s.n[3 * k] = v[k]->nx * iw[k]; s.n[3 * k + 1] = v[k]->ny * iw[k]; s.n[3 * k + 2] = v[k]->nz * iw[k];
    }
    s.draw = d;
    s.pad = 0;
    // (plain stores: non-temporal 16-B stores measured 0.7 % faster per C4 frame but wrote every 80-B
    // record as partial sectors, 207 -> 303 MB per frame; profiles/r06_shade_nt_ab.txt)
    if (!SHS_LIB_EXP(fp, 1u)) fb.shade[slot] = s;
    if (dr.tex) {   // UV0 varying * 1/w (varw, rasterizer.hpp:319-326)
        fb.uvw[2 * (size_t)slot] = make_float4(a.u * iw0, a.v * iw0, b.u * iw1, b.v * iw1);
        fb.uvw[2 * (size_t)slot + 1] = make_float4(c.u * iw2, c.v * iw2, 0.0f, 0.0f);
    }
    store_box(fb, slot, x0, x1, y0, y1);
    if (SHS_LIB_EXP(fp, 2u)) return;
    if (DIRECT) {
        const int n_rt = (x1 / LIB_RTW - x0 / LIB_RTW + 1) * (y1 / LIB_RTH - y0 / LIB_RTH + 1);
        if (n_rt > SMALL_MARK) {
            const uint4 e = make_uint4(slot, pack16(x0, x1), pack16(y0, y1), zk);
            uint32_t nb;
            const uint2 at = bigq_reserve(cnt, 1u, big_tasks(fp, e, nb));
            fb.bigq[at.x] = e;
            fb.bigpre[at.x] = at.y;
        } else {
            lib_mark_range(fp, fb, cnt, x0, x1, y0, y1, slot, 0, 1, zk);
        }
    } else {
        lib_mark(fp, fb, cnt, x0, x1, y0, y1, slot, ss, pend, zk);
    }
}

// The draw of pass triangle gid: a binary search over the compact tri_base array (4 B per draw, one or
// two cache lines for hundreds of draws) instead of the 400-B draw records.
__device__ __forceinline__ int lib_find_draw(const int32_t *dbase, int n_draws, int gid) {
    int lo = 0, hi = n_draws - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (dbase[mid] <= gid) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// The submission index of pass triangle `tri` (its slot): the draw's base + the triangle's MeshData index
// (a spatially ordered mesh stores its triangles in another order, LibDrawGPU::orig).
__device__ __forceinline__ uint32_t lib_sub_tri(const LibDrawGPU &dr, int tri) {
    return dr.orig ? (uint32_t)dr.tri_base + dr.orig[tri - dr.tri_base] : (uint32_t)tri;
}

__device__ __forceinline__ bool read_tri(const LibDrawGPU &dr, int local, uint32_t (&id)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) id[k] = dr.idx ? dr.idx[3 * (size_t)local + k] : (uint32_t)(3 * local + k);
    return id[0] < (uint32_t)dr.n_verts && id[1] < (uint32_t)dr.n_verts && id[2] < (uint32_t)dr.n_verts;
}

// Can the clipped fans of a triangle that is not trivially inside land on the screen (and, tile-sharded,
// on one of this rank's 32x32 tiles)?  With every corner in front of the eye (w > 0) the clipped
// polygon lies inside the triangle, whose projection is the 2D triangle of the projected corners: its
// bbox (2 px of margin for the clipper's rounding), clamped to the screen, bounds every fan.  A bbox
// more than 2 px off one screen edge puts every corner outside that edge's plane (margin 4 / (W - 1)
// in NDC), so the reference's clipper returns an empty polygon and counts nothing.  A corner behind
// the eye gives no such bound (true).
__device__ __forceinline__ bool clip_reaches_rank(const LibFrameParams &fp, const LVert (&t)[3]) {
    if (!(t[0].cw > 0.0f && t[1].cw > 0.0f && t[2].cw > 0.0f)) return true;
    float x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float sx = (t[k].cx / t[k].cw * 0.5f + 0.5f) * (float)(fp.W - 1);
        const float sy = (t[k].cy / t[k].cw * 0.5f + 0.5f) * (float)(fp.H - 1);
        x0 = fminf(x0, sx); x1 = fmaxf(x1, sx); y0 = fminf(y0, sy); y1 = fmaxf(y1, sy);
    }
    if (!(x1 >= -2.0f && y1 >= -2.0f && x0 <= (float)fp.W + 1.0f && y0 <= (float)fp.H + 1.0f)) return false;  // off screen (NaN: kept)
    const int tx0 = max(0, (int)fmaxf(x0 - 2.0f, 0.0f) / TILE), tx1 = min(fp.tiles_x - 1, (int)fminf(x1 + 2.0f, (float)(fp.W - 1)) / TILE);
    const int ty0 = max(0, (int)fmaxf(y0 - 2.0f, 0.0f) / TILE), ty1 = min(fp.tiles_y - 1, (int)fminf(y1 + 2.0f, (float)(fp.H - 1)) / TILE);
    if (!fp.reg.on && ty1 - ty0 >= 64) return true;
    return lib_owns_any(fp, tx0, tx1, ty0, ty1);
}

// Camera pass: one input triangle of rasterize_mesh.  A triangle that is not trivially inside the
// frustum is queued for k_lib_clip (returns true): the clipper's polygon buffers live in scratch, and
// running it here would stall every wave that holds one such triangle and give the whole setup
// kernel a scratch allocation.
__device__ __forceinline__ bool setup_camera_tri(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, int tri, uint32_t &n_clip,
                                 uint32_t &n_rast, SetupShared &ss, Pend &pend, int d_uni) {
    const int d = d_uni >= 0 ? d_uni : lib_find_draw(fb.dbase, fp.n_draws, tri);
    const LibDrawGPU &dr = fb.draws[d];
    const int local = tri - dr.tri_base;
    uint32_t id[3];
    if (!read_tri(dr, local, id)) {
        store_box(fb, (uint32_t)tri, 0, -1, 0, -1);
        return false;
    }
    LVert t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = vertex_pos(dr, id[k]);
    const uint32_t sub = lib_sub_tri(dr, tri);
    if (fp.flags & LF_PERM) fb.s2s[sub] = (uint32_t)tri;   // the resolve's winner -> slot map
    const uint32_t seq0 = sub * 16u;
    if (fully_inside(t[0]) && fully_inside(t[1]) && fully_inside(t[2])) {
        emit_fan(fp, fb, cnt, dr, d, seq0, (uint32_t)tri, t[0], t[1], t[2], n_clip, n_rast, ss, pend, id);
        return false;
    }
    if (!clip_reaches_rank(fp, t)) {   // off screen, or (tile-sharded) no fan can land on an owned tile
        store_box(fb, (uint32_t)tri, 0, -1, 0, -1);
        return false;
    }
    return true;
}

// Shadow pass: one caster triangle of PassShadowMap (pass_shadow_map.hpp:155-203), draws[d].viewproj
// holding the light camera's viewproj.  n_rast counts the triangles with a non-empty bbox.
__device__ __forceinline__ void setup_shadow_tri(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, int tri, uint32_t &n_rast,
                                 SetupShared &ss, Pend &pend, int d_uni) {
    const int d = d_uni >= 0 ? d_uni : lib_find_draw(fb.dbase, fp.n_draws, tri);
    const LibDrawGPU &dr = fb.draws[d];
    const int local = tri - dr.tri_base;
    uint32_t id[3];
    float nx[3], ny[3], nz[3];
    bool ok = read_tri(dr, local, id);
    if (ok) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float *P = dr.pos + 3 * (size_t)id[k];
            const f4 w = m4v(dr.model, f4{P[0], P[1], P[2], 1.0f});
            const f4 c = m4v(dr.viewproj, f4{w.x, w.y, w.z, 1.0f});
            ok = ok && !(fabsf(c.w) < 1e-8f);
            nx[k] = c.x / c.w; ny[k] = c.y / c.w; nz[k] = c.z / c.w;
        }
    }
    if (ok) {   // all corners beyond one side of the NDC cube: early reject (:174-177)
        ok = !((nx[0] < -1.0f && nx[1] < -1.0f && nx[2] < -1.0f) || (nx[0] > 1.0f && nx[1] > 1.0f && nx[2] > 1.0f)) &&
             !((ny[0] < -1.0f && ny[1] < -1.0f && ny[2] < -1.0f) || (ny[0] > 1.0f && ny[1] > 1.0f && ny[2] > 1.0f)) &&
             !((nz[0] < -1.0f && nz[1] < -1.0f && nz[2] < -1.0f) || (nz[0] > 1.0f && nz[1] > 1.0f && nz[2] > 1.0f));
    }
    int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
    float sx[3], sy[3], den = 0.0f;
    if (ok) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            sx[k] = (nx[k] * 0.5f + 0.5f) * (float)(fp.W - 1);
            sy[k] = (ny[k] * 0.5f + 0.5f) * (float)(fp.H - 1);
        }
        x0 = max(0, (int)floorf(s_min(s_min(sx[0], sx[1]), sx[2])));
        x1 = min(fp.W - 1, (int)ceilf(s_max(s_max(sx[0], sx[1]), sx[2])));
        y0 = max(0, (int)floorf(s_min(s_min(sy[0], sy[1]), sy[2])));
        y1 = min(fp.H - 1, (int)ceilf(s_max(s_max(sy[0], sy[1]), sy[2])));
        ok = x0 <= x1 && y0 <= y1;
        if (ok) {
            ++n_rast;
            den = (sx[1] - sx[0]) * (sy[2] - sy[0]) - (sx[2] - sx[0]) * (sy[1] - sy[0]);
            ok = !(fabsf(den) < 1e-8f);
        }
    }
    if (!ok) {
        store_box(fb, (uint32_t)tri, 0, -1, 0, -1);
        return;
    }
    LibRec r;
    r.ax = sx[0]; r.ay = sy[0];
    r.v0x = sx[1] - sx[0]; r.v0y = sy[1] - sy[0];
    r.v1x = sx[2] - sx[0]; r.v1y = sy[2] - sy[0];
    r.inv_den = 1.0f / den;
    r.z0 = nz[0]; r.z1 = nz[1]; r.z2 = nz[2];
    r.iw0 = r.iw1 = r.iw2 = 0.0f;
    r.seq = (uint32_t)tri * 16u;
    r.bx = pack16(x0, x1); r.by = pack16(y0, y1);
    fb.recs[tri] = r;
    const uint32_t zk = lib_zmin_ord<true>(fp, r);
    fb.zord[tri] = zk;
    store_box(fb, (uint32_t)tri, x0, x1, y0, y1);
    lib_mark(fp, fb, cnt, x0, x1, y0, y1, (uint32_t)tri, ss, pend, zk);
}

__device__ __forceinline__ void setup_shared_init(SetupShared &ss, int tid) {
    if (tid < 2) ss.stat[tid] = 0u;
    if (tid == 0) ss.nbig = 0u;
    if (tid < 4) ss.ub[tid] = tid < 2 ? INT_MAX : -1;
    static_assert(AGG_BINS == 256, "one union bin tile per thread");
    ss.bcnt[tid] = 0u;
    ss.rbusy[tid] = 0u;
}

// Per-thread pass statistics into the block's ss.stat, and the thread's deferred box into the union.
__device__ __forceinline__ void setup_gather(SetupShared &ss, const Pend &pend, uint32_t n_clip, uint32_t n_rast) {
    if (pend.valid) {
        atomicMin(&ss.ub[0], pend.x0 / TILE);
        atomicMin(&ss.ub[1], pend.y0 / TILE);
        atomicMax(&ss.ub[2], pend.x1 / TILE);
        atomicMax(&ss.ub[3], pend.y1 / TILE);
    }
    for (int o = 32; o > 0; o >>= 1) {
        n_clip += __shfl_down(n_clip, o);
        n_rast += __shfl_down(n_rast, o);
    }
    if (__lane_id() == 0) {
        atomicAdd(&ss.stat[0], n_clip);
        atomicAdd(&ss.stat[1], n_rast);
    }
}

// The deferred primitives (<= 2x2 bin tiles each): busy rows and bin appends through LDS (after a
// barrier that follows setup_gather).  Returns the union's w * h (timeline).
__device__ int setup_deferred(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt, SetupShared &ss, const Pend &pend, int tid) {
    const int ubx0 = ss.ub[0], uby0 = ss.ub[1], uw = ss.ub[2] - ubx0 + 1, uh = ss.ub[3] - uby0 + 1;
    const bool agg = uw > 0 && uh > 0 && uw * uh <= AGG_BINS;   // block-uniform
    const bool sharded = fp.count > 1;
    constexpr int RPB = TILE / LIB_RTH;                        // raster rows per bin tile
    const int bx0 = pend.x0 / TILE, by0 = pend.y0 / TILE, bx1 = pend.x1 / TILE, by1 = pend.y1 / TILE;
    uint32_t pos[DEFER_BT][DEFER_BT] = {};
    if (pend.valid) {
        if (!agg) {
            lib_mark_range(fp, fb, cnt, pend.x0, pend.x1, pend.y0, pend.y1, pend.slot, 0, 1, pend.zk);
        } else {
            for (int ry = pend.y0 / LIB_RTH; ry <= pend.y1 / LIB_RTH; ++ry) {
                const int by = ry / RPB;
                for (int rx = pend.x0 / LIB_RTW; rx <= pend.x1 / LIB_RTW; ++rx)
                    if (!sharded || lib_owned(fp, rx, by))
                        atomicOr(&ss.rbusy[(by - uby0) * uw + (rx - ubx0)], 1u << (ry % RPB));
            }
            if (!fp.scan_mode) {
#pragma unroll
                for (int j = 0; j < DEFER_BT; ++j)
#pragma unroll
                    for (int i = 0; i < DEFER_BT; ++i)
                        if (bx0 + i <= bx1 && by0 + j <= by1 && (!sharded || lib_owned(fp, bx0 + i, by0 + j)))
                            pos[j][i] = atomicAdd(&ss.bcnt[(by0 + j - uby0) * uw + (bx0 + i - ubx0)], 1u);
            }
        }
    }
    if (agg) {
        __syncthreads();
        if (tid < uw * uh) {
            const int bx = ubx0 + tid % uw, by = uby0 + tid / uw;
            const uint32_t rb = ss.rbusy[tid];
            for (int r = 0; r < RPB; ++r)
                if ((rb >> r) & 1u) fb.busy[(by * RPB + r) * fp.tiles_x + bx] = 1u;
            const uint32_t n = ss.bcnt[tid];
            if (!fp.scan_mode && n) {
                uint32_t *tcount = fb.tile_count + (size_t)fp.parity * fp.tiles_x * fp.tiles_y;
                ss.bcnt[tid] = atomicAdd(&tcount[by * fp.tiles_x + bx], n);
            }
        }
        __syncthreads();
        if (pend.valid && !fp.scan_mode) {
#pragma unroll
            for (int j = 0; j < DEFER_BT; ++j)
#pragma unroll
                for (int i = 0; i < DEFER_BT; ++i)
                    if (bx0 + i <= bx1 && by0 + j <= by1 && (!sharded || lib_owned(fp, bx0 + i, by0 + j))) {
                        const int u = (by0 + j - uby0) * uw + (bx0 + i - ubx0);
                        lib_append_bin(fp, fb, cnt, (by0 + j) * fp.tiles_x + bx0 + i, ss.bcnt[u] + pos[j][i],
                                       make_uint4(pend.slot, pack16(pend.x0, pend.x1), pack16(pend.y0, pend.y1), pend.zk));
                    }
        }
    }
    return max(uw, 0) * max(uh, 0);
}

// The block's large primitives go to the pass-wide queue that k_lib_bigmark spreads over the chip
// (a floor triangle at 4K spans thousands of raster tiles; a few blocks holding all of them were the
// setup's critical path).  Block-uniform; one atomic per block.
__device__ __forceinline__ uint32_t setup_flush_big(const LibFrameParams &fp, const LibBuffers &fb, uint32_t *cnt,
                                                    SetupShared &ss, int tid) {
    const uint32_t nbig = min(ss.nbig, (uint32_t)BIG_CAP);
    if (nbig > 0) {   // block-uniform: the entries' task prefix in LDS, then one reservation
        static_assert(BIG_CAP == 2 * 256, "two queue entries per thread");
        uint32_t nb;
        const uint32_t i0 = 2u * (uint32_t)tid;
        const uint32_t t0 = i0 < nbig ? big_tasks(fp, ss.big[i0], nb) : 0u;
        const uint32_t t1 = i0 + 1 < nbig ? big_tasks(fp, ss.big[i0 + 1], nb) : 0u;
        const int lane = tid & 63, wave = tid >> 6;
        uint32_t incl = t0 + t1;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) ss.pre[1][2 + wave] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int w = 0; w < wave; ++w) off += ss.pre[1][2 + w];
        const uint32_t ex = off + incl - (t0 + t1);
        if (i0 < nbig) ss.pre[0][i0] = ex;
        if (i0 + 1 < nbig) ss.pre[0][i0 + 1] = ex + t0;
        if (tid == 255) {
            const uint2 at = bigq_reserve(cnt, nbig, off + incl);
            ss.pre[1][0] = at.x;
            ss.pre[1][1] = at.y;
        }
        __syncthreads();
        const uint32_t base = ss.pre[1][0], tbase = ss.pre[1][1];
        for (uint32_t i = (uint32_t)tid; i < nbig; i += 256) {
            fb.bigq[base + i] = ss.big[i];
            fb.bigpre[base + i] = tbase + ss.pre[0][i];
        }
    }
    return nbig;
}

// Appends the lanes with `pred` to a queue: one atomic per wave; every lane of the wave calls it.
template <typename T>
__device__ __forceinline__ void wave_append(uint32_t *counter, T *queue, bool pred, T value) {
    const uint64_t m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = __lane_id();
    uint32_t base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (pred) queue[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = value;
}

// Setup workgroup start: LDS state, and the next frame's counter set, raster queues and bin counts zeroed.
__device__ __forceinline__ void setup_zero_next(const LibFrameParams &fp, const LibBuffers &fb, int b, int tid) {
    if (b == 0 && tid < LC_N) fb.counters[(fp.parity ^ 1u) * LC_N + tid] = 0u;
    if (b == 0 && tid < LIB_NQW) fb.rqueue[((fp.parity ^ 1u) * LIB_NQW + tid) * LIB_QSTRIDE] = 0u;
    {
        const int n_bt = fp.tiles_x * fp.tiles_y;
        uint32_t *next_count = fb.tile_count + (size_t)(fp.parity ^ 1u) * n_bt;
        for (int t = b * 256 + tid; t < n_bt; t += (int)gridDim.x * 256) next_count[t] = 0u;
    }
}

__device__ __forceinline__ void setup_prologue(const LibFrameParams &fp, const LibBuffers &fb, SetupShared &ss, int b, int tid) {
    setup_shared_init(ss, tid);
    setup_zero_next(fp, fb, b, tid);
    __syncthreads();
}

// A minimum of six waves per SIMD for k_lib_setup (80 VGPRs, 8 spilled in the camera instance): C4
// 0.569 -> 0.563 ms per frame, C5 -0.5 %, the 8-way C4 split's worst rank -0.5 %, where eight waves (64
// VGPRs, 71 spilled) were 4 % slower (profiles/r06_resolve_waves_ab.txt).  The tile-sharded (LISTED)
// instance keeps the compiler's choice: at six waves it would spill 153 VGPRs.  SHS_SETUP_WAVES
// (timing experiments) overrides the bound.
#ifndef SHS_SETUP_WAVES
#define SHS_SETUP_WAVES 6
#endif
#define SHS_SETUP_BOUNDS __launch_bounds__(256, LISTED ? 1 : SHS_SETUP_WAVES)
// Tile-sharded camera pass (LISTED): a setup workgroup first reads the positions of CULL_PER x 256
// consecutive input triangles and keeps in LDS those k_lib_setup would not drop -- a trivially inside
// triangle whose fan_screen is live (on screen, not culled, on one of this rank's tiles), a triangle
// that needs clipping and can reach the rank (clip_reaches_rank) -- then sets up only the kept ones,
// 256 per round.  The same functions decide, so the kept set is exactly the triangles whose records,
// marks or clip-queue entries this rank needs; at 8 shards C4 drops 7 in 8 triangles after a
// positions-only transform.  No global list and no same-address atomics (the counts of the dropped
// trivially inside triangles go into the block's blk_stat slot): a separate pre-pass kernel with a
// global list reservation and per-wave statistic atomics took 114 us for C4's 1M triangles.
constexpr int CULL_PER = 4;

// The tile-sharded front end's decision for one input triangle (clip-space corners t): would k_lib_setup
// keep it on this rank?  The dropped trivially inside ones count like emit_fan's fan 0.
__device__ __forceinline__ bool cull_keep(const LibFrameParams &fp, const LibDrawGPU &dr, const LVert (&t)[3],
                                          uint32_t &pre_clip, uint32_t &pre_rast) {
    if (fully_inside(t[0]) && fully_inside(t[1]) && fully_inside(t[2])) {
        float sx[3], sy[3], den;
        int x0, x1, y0, y1;
        uint32_t nr = 0u;
        const bool keep = fan_screen(fp, dr, t[0], t[1], t[2], sx, sy, x0, x1, y0, y1, den, nr);
        if (!keep) { ++pre_clip; pre_rast += nr; }
        return keep;
    }
    return clip_reaches_rank(fp, t);
}

// Region-sharded camera pass, before k_lib_setup (BLK_G lanes per setup block): the screen bounds of
// block b's triangles from their 256-triangle chunks' model-space boxes (LibDrawGPU::cbox, 8 corners
// each).  Every point of a box whose corners are all in front of the eye projects inside the hull of
// the projected corners, so the bin tiles of that bbox (2 px of margin for the rounding of the
// per-vertex transforms, as clip_reaches_rank) bound every fan of every triangle of the block
// ("bounded").  A box with corners behind the eye gets an estimate instead: the hull of the part of the
// box with clip w >= 1e-3 of its largest |w| (corners there and box edges cut at that w) -- what a floor
// reaching behind the camera covers -- used as a cost estimate only, never to skip.  The bounds go to
// fb.blkrect (the region balancer's input, shs_abi_shard.cpp; w: 1 bounded, 2 estimate, 0 none -- a
// block straddling draws).  A block whose bounded bounds miss the rank's rectangle needs no setup (its
// statistics are zero; scan mode: its slots read as not rasterised); the others are listed in
// fb.blist, and k_lib_setup's workgroup i sets up listed block i -- the rank's setup grid holds no
// workgroup that only finds it has nothing to do (C4 rank 3 of 8: 2,100 of its 3,907 workgroups were
// such, ~4.6 us of a workgroup slot each, a quarter of the kernel).
// BLK_G lanes per block: lane j transforms corner j & 7 of chunk j >> 3, the bounds are reduced across
// the group with shuffles (fminf / fmaxf: the same bounds as a serial walk over the corners and edge
// cuts); one thread per block took ~11 us per rank frame at C4 (16 workgroups, a 16-corner chain each).
constexpr int BLK_G = 16;
__global__ __launch_bounds__(256) void k_lib_blocks(LibFrameParams fp, LibBuffers fb) {
    const int gid = (int)(blockIdx.x * 256 + threadIdx.x);
    const int b = gid / BLK_G, j = gid % BLK_G;
    const int ci = j >> 3, k = j & 7;
    uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const bool valid = b < fp.setup_blocks;   // uniform over the group
    int t0 = 0, t1 = -1;
    bool have = false;
    f4 p{0.0f, 0.0f, 0.0f, 1.0f};
    if (valid) {
        t0 = b * 256;
        t1 = min(t0 + 255, fp.n_tris - 1);
        const int d = fb.bdraw[b];
        const LibDrawGPU &dr = fb.draws[d];
        have = t0 <= t1 && (d + 1 >= fp.n_draws || fb.dbase[d + 1] > t1) && dr.cbox != nullptr;
        if (have) {
            const int c0 = (t0 - dr.tri_base) >> 8, c1 = (t1 - dr.tri_base) >> 8;   // at most two chunks
            const int c = min(c0 + ci, c1);
            const float4 mn = dr.cbox[2 * c], mx = dr.cbox[2 * c + 1];
            p = m4v(dr.viewproj, m4v(dr.model, f4{(k & 1) ? mx.x : mn.x, (k & 2) ? mx.y : mn.y, (k & 4) ? mx.z : mn.z, 1.0f}));
        }
    }
    // group reductions (every lane of the wave takes part in the shuffles)
    const int gsh = (int)(__lane_id() & ~(BLK_G - 1));
    const uint64_t fin_m = __ballot(isfinite(p.x) && isfinite(p.y) && isfinite(p.w));
    const uint64_t pos_m = __ballot(p.w > 0.0f);
    const uint32_t gmask = (1u << BLK_G) - 1u;
    const bool finite = have && ((uint32_t)(fin_m >> gsh) & gmask) == gmask;
    const bool bounded = finite && ((uint32_t)(pos_m >> gsh) & gmask) == gmask;
    float wmax = fabsf(p.w);
#pragma unroll
    for (int o = 1; o < BLK_G; o <<= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, o, BLK_G));
    const float eps = bounded ? 0.0f : 1e-3f * wmax;
    float x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    auto add = [&](float cx, float cy, float cw) {
        const float sx = (cx / cw * 0.5f + 0.5f) * (float)(fp.W - 1);
        const float sy = (cy / cw * 0.5f + 0.5f) * (float)(fp.H - 1);
        x0 = fminf(x0, sx); x1 = fmaxf(x1, sx); y0 = fminf(y0, sy); y1 = fmaxf(y1, sy);
    };
    if (finite && p.w > eps) add(p.x, p.y, p.w);
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {   // the box edges from this corner, cut at w = eps
        const f4 n{__shfl_xor(p.x, m, BLK_G), __shfl_xor(p.y, m, BLK_G), 0.0f, __shfl_xor(p.w, m, BLK_G)};
        if (finite && !bounded && (p.w - eps) * (n.w - eps) < 0.0f) {
            const float t = (eps - p.w) / (n.w - p.w);
            add(p.x + (n.x - p.x) * t, p.y + (n.y - p.y) * t, eps);
        }
    }
#pragma unroll
    for (int o = 1; o < BLK_G; o <<= 1) {
        x0 = fminf(x0, __shfl_xor(x0, o, BLK_G)); x1 = fmaxf(x1, __shfl_xor(x1, o, BLK_G));
        y0 = fminf(y0, __shfl_xor(y0, o, BLK_G)); y1 = fmaxf(y1, __shfl_xor(y1, o, BLK_G));
    }
    bool keep = false;
    if (valid) {
        int bx0 = 0, bx1 = fp.tiles_x - 1, by0 = 0, by1 = fp.tiles_y - 1;
        const bool est = finite && !(x1 < x0);   // some point in front of the eye
        if (finite && (bounded || est)) {
            if (!(x1 >= -2.0f && y1 >= -2.0f && x0 <= (float)fp.W + 1.0f && y0 <= (float)fp.H + 1.0f)) {
                bx0 = 1; bx1 = 0; by0 = 1; by1 = 0;   // off screen: no fan reaches a pixel
            } else {
                bx0 = max(0, (int)fmaxf(x0 - 2.0f, 0.0f) / TILE);
                bx1 = min(fp.tiles_x - 1, (int)fminf(x1 + 2.0f, (float)(fp.W - 1)) / TILE);
                by0 = max(0, (int)fmaxf(y0 - 2.0f, 0.0f) / TILE);
                by1 = min(fp.tiles_y - 1, (int)fminf(y1 + 2.0f, (float)(fp.H - 1)) / TILE);
            }
        }
        if (j == 0)
            fb.blkrect[b] = make_uint4((uint32_t)bx0 | ((uint32_t)bx1 << 16), (uint32_t)by0 | ((uint32_t)by1 << 16),
                                       (uint32_t)max(0, t1 - t0 + 1), bounded ? 1u : (finite && est) ? 2u : 0u);
        const bool need = !(bounded && !lib_owns_any(fp, bx0, bx1, by0, by1));
        if (!need) {   // no triangle of the block reaches this rank
            if (j == 0) fb.blk_stat[b] = make_uint2(0u, 0u);
            if (fp.scan_mode)
                for (int t = t0 + j; t <= t1; t += BLK_G) store_box(fb, (uint32_t)t, 0, -1, 0, -1);
        }
        keep = need && j == 0;
    }
    wave_append(&cnt[LC_BLOCKS], fb.blist, keep, (uint32_t)b);
}

template <bool SHADOW, bool LISTED = false>
__global__ SHS_SETUP_BOUNDS void k_lib_setup(LibFrameParams fp, LibBuffers fb) {
    __shared__ SetupShared ss;
    constexpr bool listed = !SHADOW && LISTED;
    __shared__ uint2 s_kept[listed ? 256 * CULL_PER : 1];   // (triangle, draw)
    __shared__ uint32_t s_nkept;
    int b = (int)blockIdx.x;   // the setup block (triangles b * 256 ...)
    const int tid = (int)threadIdx.x;
    uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const bool stl = fb.stimeline != nullptr && tid == 0;
    const uint64_t st0 = stl ? tl_now() : 0ull;
    if (listed && tid == 0) s_nkept = 0u;
    // region-sharded camera pass: workgroup i sets up k_lib_blocks' listed block i; the workgroups past
    // the list only do their share of the next frame's zeroing
    const int wg = b;
    if constexpr (!SHADOW && !listed) {
        if (fb.blist != nullptr) {
            const uint32_t n_listed = cnt[LC_BLOCKS];
            if ((uint32_t)wg >= n_listed) {
                setup_zero_next(fp, fb, wg, tid);
                if (fb.stimeline && tid == 0) {
                    uint64_t *o = fb.stimeline + (size_t)wg * STL_STRIDE;
                    o[0] = st0; o[1] = o[2] = o[3] = tl_now(); o[4] = o[5] = o[6] = o[7] = 0ull;
                }
                return;
            }
            b = (int)fb.blist[wg];
        }
    }
    setup_prologue(fp, fb, ss, wg, tid);
    // the triangles: b * 256 + tid (one chunk per block), or (tile-sharded camera pass) the block's kept
    // triangles of its CULL_PER x 256 inputs, 256 per round
    uint32_t pre_clip = 0u, pre_rast = 0u;
    uint64_t stf = 0ull;
    int n_items = 256;
    if constexpr (listed) {
        const int lane = tid & 63;
        const int base = b * 256 * CULL_PER;
        const int t_end = min(base + 256 * CULL_PER, fp.n_tris) - 1;
        bool keep_k[CULL_PER];
        int d_k[CULL_PER];
        const int d_first = fb.bdraw[base >> 8];
        if (d_first + 1 >= fp.n_draws || fb.dbase[d_first + 1] > t_end) {   // block-uniform: one draw
            // scalar draw uniforms; every index load of the CULL_PER triangles issued, then every
            // position load, then the math (two memory round trips instead of one chain per triangle)
            const LibDrawGPU &dr = fb.draws[d_first];
            uint32_t id[CULL_PER][3];
            bool ok[CULL_PER];
#pragma unroll
            for (int k = 0; k < CULL_PER; ++k) {
                const int tri = base + 256 * k + tid;
                ok[k] = read_tri(dr, min(tri, t_end) - dr.tri_base, id[k]) && tri <= t_end;
            }
            float P[CULL_PER][3][3];
#pragma unroll
            for (int k = 0; k < CULL_PER; ++k)
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const float *pp = dr.pos + 3 * (size_t)(ok[k] ? id[k][q] : 0u);
                    P[k][q][0] = pp[0]; P[k][q][1] = pp[1]; P[k][q][2] = pp[2];
                }
#pragma unroll
            for (int k = 0; k < CULL_PER; ++k) {
                LVert t[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) t[q] = vertex_pos_xyz(dr, P[k][q][0], P[k][q][1], P[k][q][2]);
                keep_k[k] = ok[k] && cull_keep(fp, dr, t, pre_clip, pre_rast);
                d_k[k] = d_first;
            }
        } else {   // the span straddles draws: per-lane draw search
#pragma unroll
            for (int k = 0; k < CULL_PER; ++k) {
                const int tri = base + 256 * k + tid;
                bool keep = false;
                int d = 0;
                if (tri <= t_end) {
                    d = lib_find_draw(fb.dbase, fp.n_draws, tri);
                    const LibDrawGPU &dr = fb.draws[d];
                    uint32_t id[3];
                    if (read_tri(dr, tri - dr.tri_base, id)) {
                        LVert t[3];
#pragma unroll
                        for (int q = 0; q < 3; ++q) t[q] = vertex_pos(dr, id[q]);
                        keep = cull_keep(fp, dr, t, pre_clip, pre_rast);
                    }
                }
                keep_k[k] = keep;
                d_k[k] = d;
            }
        }
#pragma unroll
        for (int k = 0; k < CULL_PER; ++k) {   // one LDS atomic per wave and triangle round
            const uint64_t m = __ballot(keep_k[k]);
            if (m == 0ull) continue;
            const int first = __ffsll((long long)m) - 1;
            uint32_t at = 0u;
            if (lane == first) at = atomicAdd(&s_nkept, (uint32_t)__popcll(m));
            at = (uint32_t)__shfl((int)at, first);
            if (keep_k[k]) s_kept[at + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = make_uint2((uint32_t)(base + 256 * k + tid), (uint32_t)d_k[k]);
        }
        __syncthreads();
        n_items = (int)s_nkept;
        if (stl) stf = tl_now();
        if (SHS_LIB_EXP(fp, 8u)) n_items = 0;
    }
    uint32_t acc_clip = 0u, acc_rast = 0u, nbig = 0u;
    uint64_t st1 = 0ull, st2 = 0ull;
    int uwh = 0;
    for (int round = 0; round == 0 || round * 256 < n_items; ++round) {   // block-uniform
        if (round != 0) {
            __syncthreads();   // the previous round's LDS state is consumed
            setup_shared_init(ss, tid);
            __syncthreads();
        }
        int tri = b * 256 + tid;
        uint32_t n_clip = round == 0 ? pre_clip : 0u, n_rast = round == 0 ? pre_rast : 0u;
        Pend pend;
        bool need_clip = false;
        if constexpr (listed) {
            const int i = round * 256 + tid;
            const bool act = i < n_items;
            uint2 e = make_uint2(0u, 0u);
            if (act) e = s_kept[i];
            tri = act ? (int)e.x : -1;
            const int d = (int)e.y;
            const int d0 = __builtin_amdgcn_readfirstlane(d);
            if (__ballot(act && d != d0) == 0ull) {   // wave-uniform draw: scalar uniform loads
                if (act) need_clip = setup_camera_tri(fp, fb, cnt, tri, n_clip, n_rast, ss, pend, d0);
            } else if (act) {
                need_clip = setup_camera_tri(fp, fb, cnt, tri, n_clip, n_rast, ss, pend, d);
            }
        } else if (tri < fp.n_tris) {
            // the block's draw when all its triangles share one (block-uniform: its uniforms come in
            // through scalar loads), else -1 and a per-thread search
            const int t_last = min(b * 256 + 255, fp.n_tris - 1);
            const int d_first = fb.bdraw[b];
            const int d_uni = (d_first + 1 >= fp.n_draws || fb.dbase[d_first + 1] > t_last) ? d_first : -1;
            if (d_uni >= 0) {   // two inlined copies: this one sees d_uni as the (scalar) draw
                if (SHADOW) setup_shadow_tri(fp, fb, cnt, tri, n_rast, ss, pend, d_uni);
                else need_clip = setup_camera_tri(fp, fb, cnt, tri, n_clip, n_rast, ss, pend, d_uni);
            } else {
                if (SHADOW) setup_shadow_tri(fp, fb, cnt, tri, n_rast, ss, pend, -1);
                else need_clip = setup_camera_tri(fp, fb, cnt, tri, n_clip, n_rast, ss, pend, -1);
            }
        }
        if (!SHADOW) wave_append(&cnt[LC_CLIPQ], fb.clipq, need_clip, (uint32_t)tri);
        setup_gather(ss, pend, n_clip, n_rast);
        __syncthreads();
        if (stl) st1 = tl_now();
        uwh = setup_deferred(fp, fb, cnt, ss, pend, tid);
        if (stl) st2 = tl_now();
        nbig += setup_flush_big(fp, fb, cnt, ss, tid);
        if (tid == 0) { acc_clip += ss.stat[0]; acc_rast += ss.stat[1]; }
        if (!listed) break;
    }
    if (tid == 0 && b < fp.setup_blocks) fb.blk_stat[b] = make_uint2(acc_clip, acc_rast);
    if (fb.stimeline) {
        __syncthreads();
        if (tid == 0) {
            uint64_t *o = fb.stimeline + (size_t)wg * STL_STRIDE;
            o[0] = st0; o[1] = st1; o[2] = st2; o[3] = tl_now(); o[4] = nbig; o[5] = (uint64_t)uwh;
            o[6] = stf; o[7] = listed ? (uint64_t)n_items : 0ull;
        }
    }
}

// The camera pass's queued triangles (k_lib_setup: not trivially inside): Sutherland-Hodgman against
// the 6 planes and the fans (rasterizer.hpp:241-328), one 16-lane group per triangle striding the
// queue, the fans emitted in parallel (lane k: fan k).  Same slots, submission order (tri * 16 + fan),
// marks and counters as the reference's per-triangle clip.
// six waves per SIMD (80 VGPRs, 19 spilled, instead of 103 at four): C4 0.564 -> 0.561, C5 0.340 -> 0.337 ms
// per frame in two A/B pairs (profiles/r06_resolve_waves_ab.txt); SHS_CLIP_WAVES overrides (experiments)
#ifndef SHS_CLIP_WAVES
#define SHS_CLIP_WAVES 6
#endif
__global__ __launch_bounds__(256, SHS_CLIP_WAVES) void k_lib_clip(LibFrameParams fp, LibBuffers fb) {
    __shared__ SetupShared ss_unused;   // emit_fan<true> marks directly
    const int lane = __lane_id(), li = lane & (CLIP_G - 1), seg = lane & ~(CLIP_G - 1);
    uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const uint32_t n = cnt[LC_CLIPQ];
    uint32_t n_clip = 0, n_rast = 0;
    Pend pend;
    const uint32_t groups = gridDim.x * (256 / CLIP_G);
    for (uint32_t q = blockIdx.x * (256 / CLIP_G) + threadIdx.x / CLIP_G; q < n; q += groups) {   // group-uniform
        const int tri = (int)fb.clipq[q];
        const int d = lib_find_draw(fb.dbase, fp.n_draws, tri);
        const LibDrawGPU &dr = fb.draws[d];
        uint32_t id[3];
        (void)read_tri(dr, tri - dr.tri_base, id);   // in range: checked by k_lib_setup
        LVert v{};
        if (li < 3) v = vertex_out(dr, id[li]);
        int rot = 0;
        const int m = clip_frustum_group(v, li, seg, rot);
        if (m < 3) {
            if (li == 0) store_box(fb, (uint32_t)tri, 0, -1, 0, -1);
            continue;
        }
        uint32_t xb = 0;
        if (m > 3) {   // fans 1 .. m-3 take consecutive extra slots
            int e = 0;
            if (li == 0) e = (int)atomicAdd(&cnt[LC_EXTRA], (uint32_t)(m - 3));
            e = grp_shfl(e, seg);
            if ((uint32_t)e + (uint32_t)(m - 3) > fp.extra_cap) {
                if (li == 0) {
                    raise_overflow(&cnt[LC_OVERFLOW], LOV_EXTRA, fb.ov_host);
                    store_box(fb, (uint32_t)tri, 0, -1, 0, -1);
                }
                continue;
            }
            xb = (uint32_t)fp.n_tris + (uint32_t)e;
            if (li == 0) fb.xbase[tri] = xb;
        }
        // fan k = (p0, p_k, p_k+1) on lane k; polygon vertex j is lane (j + rot) % m
        const int k = li;
        const int l1 = k + rot >= m ? k + rot - m : k + rot;
        const int l2 = l1 + 1 >= m ? 0 : l1 + 1;
        const LVert p0 = grp_shfl_v(v, seg + rot);
        const LVert pk = grp_shfl_v(v, seg + (k < m ? l1 : 0));
        const LVert pk1 = grp_shfl_v(v, seg + (k < m ? l2 : 0));
        if (k >= 1 && k + 1 < m) {
            const uint32_t slot = k == 1 ? (uint32_t)tri : xb + (uint32_t)(k - 2);
            emit_fan<true>(fp, fb, cnt, dr, d, lib_sub_tri(dr, tri) * 16u + (uint32_t)(k - 1), slot, p0, pk, pk1, n_clip, n_rast,
                           ss_unused, pend);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        n_clip += __shfl_down(n_clip, o);
        n_rast += __shfl_down(n_rast, o);
    }
    if (lane == 0 && (n_clip | n_rast)) {
        atomicAdd(&fb.blk_stat[0].x, n_clip);
        atomicAdd(&fb.blk_stat[0].y, n_rast);
    }
}

// The large primitives' (primitive, tile) tasks, a contiguous range per workgroup: busy marks on the
// owned raster tiles, then bin appends on the owned bin tiles.  Each workgroup stages the queue
// window its range touches in LDS and finds a task's primitive by binary search there.
constexpr int BIG_WIN = 1024;

__global__ __launch_bounds__(256) void k_lib_bigmark(LibFrameParams fp, LibBuffers fb) {
    __shared__ uint32_t s_pre[BIG_WIN + 1];
    __shared__ uint4 s_e[BIG_WIN];
    __shared__ uint32_t s_lo;
    uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const uint32_t n = cnt[LC_BIGQ];
    if (n == 0u) return;
    const uint32_t total = cnt[LC_BIGT];
    const uint32_t per = (total + gridDim.x - 1u) / gridDim.x;
    const uint32_t t0 = blockIdx.x * per, t1 = min(total, t0 + per);
    const int tid = (int)threadIdx.x;
    const bool sharded = fp.count > 1;
    uint32_t *tcount = fb.tile_count + (size_t)fp.parity * fp.tiles_x * fp.tiles_y;
    for (uint32_t w0 = t0; w0 < t1;) {   // block-uniform: windows of at most BIG_WIN primitives
        if (tid == 0) {   // the primitive holding task w0: last i with bigpre[i] <= w0
            uint32_t lo = 0, hi = n - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (fb.bigpre[mid] <= w0) lo = mid; else hi = mid - 1;
            }
            s_lo = lo;
        }
        __syncthreads();
        const uint32_t e0 = s_lo, m = min((uint32_t)BIG_WIN, n - e0);
        for (uint32_t i = (uint32_t)tid; i <= m; i += 256) s_pre[i] = e0 + i < n ? fb.bigpre[e0 + i] : total;
        for (uint32_t i = (uint32_t)tid; i < m; i += 256) s_e[i] = fb.bigq[e0 + i];
        __syncthreads();
        const uint32_t w1 = min(t1, s_pre[m]);   // the tasks this window covers
        for (uint32_t t = w0 + (uint32_t)tid; t < w1; t += 256) {
            uint32_t lo = 0, hi = m - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (s_pre[mid] <= t) lo = mid; else hi = mid - 1;
            }
            const uint4 e = s_e[lo];
            uint32_t nb;
            (void)big_tasks(fp, e, nb);
            const int k = (int)(t - s_pre[lo]);
            const int x0 = (int)lo16(e.y), x1 = (int)hi16(e.y), y0 = (int)lo16(e.z);
            if ((uint32_t)k < nb) {
                const int nx = x1 / LIB_RTW - x0 / LIB_RTW + 1;
                const int cx = x0 / LIB_RTW + k % nx, cy = y0 / LIB_RTH + k / nx;
                if (!sharded || lib_owned(fp, cx, cy / (TILE / LIB_RTH))) fb.busy[cy * fp.tiles_x + cx] = 1u;
            } else {
                const int kb = k - (int)nb;
                const int nx = x1 / TILE - x0 / TILE + 1;
                const int cx = x0 / TILE + kb % nx, cy = y0 / TILE + kb / nx;
                if (!sharded || lib_owned(fp, cx, cy)) {
                    const int bt = cy * fp.tiles_x + cx;
                    lib_append_bin(fp, fb, cnt, bt, atomicAdd(&tcount[bt], 1u), e);
                }
            }
        }
        w0 = w1;
        __syncthreads();
    }
}

// ---- k_lib_raster -----------------------------------------------------------------------------

// One (primitive, pixel) test: barycentric_2d (rasterizer.hpp:167-179), the inside test (:338),
// then the camera pass's 1/w depth (:341-361) or the shadow pass's NDC depth (pass_shadow_map.hpp
// :193-200).  Returns whether the fragment passes the depth test against the clear value.
template <bool SHADOW>
__device__ __forceinline__ bool lib_test(const LibFrameParams &fp, const LibRec &r, int px, int py, float &z01, float &u,
                                         float &v, float &w, float &inv_denom) {
    const float vpx = ((float)px + 0.5f) - r.ax, vpy = ((float)py + 0.5f) - r.ay;
    v = (vpx * r.v1y - r.v1x * vpy) * r.inv_den;
    w = (r.v0x * vpy - vpx * r.v0y) * r.inv_den;
    u = (1.0f - v) - w;
    if (u < 0.0f || v < 0.0f || w < 0.0f) return false;
    if (SHADOW) {
        const float z_ndc = (u * r.z0 + v * r.z1) + w * r.z2;
        z01 = s_clamp(z_ndc * 0.5f + 0.5f, 0.0f, 1.0f);
        return z01 < 1.0f;   // RT_ShadowDepth cleared to 1, `if (z01 < zbuf)`
    }
    const float denom = (u * r.iw0 + v * r.iw1) + w * r.iw2;
    if (denom <= 1e-10f) return false;
    inv_denom = 1.0f / denom;
    if ((fp.flags & (LF_DEPTH | LF_LINZ)) == (LF_DEPTH | LF_LINZ)) {   // linear view depth replaces z01
        z01 = g_clamp((inv_denom - fp.zn) / fp.zspan, 0.0f, 1.0f);
        return z01 < 1.0f;
    }
    const float z_clip = (u * r.z0 + v * r.z1) + w * r.z2;
    z01 = g_clamp((z_clip * inv_denom) * 0.5f + 0.5f, 0.0f, 1.0f);
    if (!(fp.flags & LF_DEPTH)) return true;   // no depth_motion target: every fragment writes
    return z01 < 1.0f;                         // depth cleared to 1, `if (z01 >= zbuf) continue`
}

// Without a depth target the last fragment in submission order wins: its key is the smallest.
__device__ __forceinline__ unsigned long long lib_key(const LibFrameParams &fp, float z01, uint32_t seq, bool shadow) {
    return (shadow || (fp.flags & LF_DEPTH)) ? z_key(z01, seq) : (unsigned long long)(0xffffffffu - seq);
}

// The camera pass hands each pixel's winner to k_lib_resolve as 4 B: lib_resolve reads only the key's
// low word (the submission sequence, painter's order inverted) and whether it is empty, and recomputes
// z from the record.  Word = sequence + 1 (sequences are < 2^31), 0 = no winner.
__device__ __forceinline__ uint32_t lib_winner_word(const LibFrameParams &fp, unsigned long long key) {
    if (key == KEY_EMPTY) return 0u;
    const uint32_t seq = (fp.flags & LF_DEPTH) ? (uint32_t)key : 0xffffffffu - (uint32_t)key;
    return seq + 1u;
}
// The key lib_resolve decodes for a word: its low word and emptiness are the original key's.
__device__ __forceinline__ unsigned long long lib_winner_key(const LibFrameParams &fp, uint32_t w) {
    if (w == 0u) return KEY_EMPTY;
    const uint32_t seq = w - 1u;
    return (fp.flags & LF_DEPTH) ? (unsigned long long)seq : (unsigned long long)(0xffffffffu - seq);
}

// (2R+1)^2 PCF taps with every fetch issued before the first compare (one memory round trip).
template <int R>
__device__ __forceinline__ float pcf_fixed(const LibFrameParams &fp, const LibBuffers &fb, int cx, int cy, int step, float z_test) {
    constexpr int N = 2 * R + 1;
    float ref[N * N];
#pragma unroll
    for (int oy = -R; oy <= R; oy++) {
        const size_t row = (size_t)s_clampi(cy + oy * step, 0, fp.sm_h - 1) * fp.sm_w;
#pragma unroll
        for (int ox = -R; ox <= R; ox++) ref[(oy + R) * N + ox + R] = fb.shadow_map[row + s_clampi(cx + ox * step, 0, fp.sm_w - 1)];
    }
    int lit = 0;
#pragma unroll
    for (int i = 0; i < N * N; ++i) lit += (z_test <= ref[i]) ? 1 : 0;
    return (float)lit / (float)(N * N);
}

// shadow_visibility_dir (lighting/shadow_sample.hpp:65-104) with the FS's ShadowParams.
__device__ float shadow_visibility(const LibFrameParams &fp, const LibBuffers &fb, const LibDrawGPU &dr, f3 pos, float ndotl) {
    const f4 p = m4v(dr.light_vp, f4{pos.x, pos.y, pos.z, 1.0f});
    if (fabsf(p.w) < 1e-8f) return 1.0f;
    const float su = (p.x / p.w) * 0.5f + 0.5f, sv = (p.y / p.w) * 0.5f + 0.5f, sz = (p.z / p.w) * 0.5f + 0.5f;
    if (su < 0.0f || su > 1.0f || sv < 0.0f || sv > 1.0f) return 1.0f;
    const float slope = 1.0f - s_clamp(ndotl, 0.0f, 1.0f);
    const float z_test = sz - (dr.shp[0] + dr.shp[1] * slope);
    const int cx = (int)roundf(su * (float)(fp.sm_w - 1)), cy = (int)roundf(sv * (float)(fp.sm_h - 1));
    const int rad = __float_as_int(dr.shp[2]);
    if (rad == 0) {
        const float z_ref = fb.shadow_map[(size_t)s_clampi(cy, 0, fp.sm_h - 1) * fp.sm_w + s_clampi(cx, 0, fp.sm_w - 1)];
        return (z_test <= z_ref) ? 1.0f : 0.0f;
    }
    const int step = max(1, (int)roundf(dr.shp[3]));
    if (rad == 2 && step == 1 && cx >= 2 && cx + 2 < fp.sm_w && cy >= 2 && cy + 2 < fp.sm_h) {
        // the reference default (5x5, step 1) away from the map's edges: each row's five texels as one
        // dword-aligned 16-B load and one 4-B load (10 loads instead of 25), compared in the same order
        typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
        f4u q[5];
        float e[5];
#pragma unroll
        for (int oy = 0; oy < 5; ++oy) {
            const float *p = fb.shadow_map + (size_t)(cy - 2 + oy) * fp.sm_w + (cx - 2);
            q[oy] = *reinterpret_cast<const f4u *>(p);
            e[oy] = p[4];
        }
        int lit = 0;
#pragma unroll
        for (int oy = 0; oy < 5; ++oy)
            lit += ((z_test <= q[oy].x) ? 1 : 0) + ((z_test <= q[oy].y) ? 1 : 0) + ((z_test <= q[oy].z) ? 1 : 0) +
                   ((z_test <= q[oy].w) ? 1 : 0) + ((z_test <= e[oy]) ? 1 : 0);
        return (float)lit / 25.0f;
    }
    if (rad == 1) return pcf_fixed<1>(fp, fb, cx, cy, step, z_test);
    if (rad == 2) return pcf_fixed<2>(fp, fb, cx, cy, step, z_test);   // the reference default (5x5)
    int count = 0, lit = 0;
    for (int oy = -rad; oy <= rad; oy++) {
        const size_t row = (size_t)s_clampi(cy + oy * step, 0, fp.sm_h - 1) * fp.sm_w;
        for (int ox = -rad; ox <= rad; ox++) {
            lit += (z_test <= fb.shadow_map[row + s_clampi(cx + ox * step, 0, fp.sm_w - 1)]) ? 1 : 0;
            count++;
        }
    }
    return (float)lit / (float)count;
}

// x^5 by (x^2)^2 x in double, narrowed to float: x^2 is exact and the two other products carry 2^-53
// each, so the float result is the correctly rounded power (libm's powf(x, 5.0f)) except within ~1e-15
// relative of a float rounding boundary -- at a few multiplications instead of a general powf's log / exp
// evaluation (the device powf itself is not correctly rounded).
__device__ __forceinline__ float pow5(float x) {
    const double d = (double)x, d2 = d * d;
    return (float)((d2 * d2) * d);
}

// eval_fake_ibl (builtin_shaders.hpp:57-85)
__device__ f3 fake_ibl(f3 N, f3 V, f3 base, float metallic, float roughness, float ao) {
    const f3 n = normalize3(N), v = normalize3(V);
    const f3 I = neg3(v);
    const f3 r = sub3(I, sc3(sc3(n, dot3(n, I)), 2.0f));
    const f3 zen = {0.32f, 0.46f, 0.72f}, hor = {0.62f, 0.66f, 0.72f}, gnd = {0.16f, 0.15f, 0.14f};
    const float up_n = s_clamp(n.y * 0.5f + 0.5f, 0.0f, 1.0f);
    const float up_r = s_clamp(r.y * 0.5f + 0.5f, 0.0f, 1.0f);
    const f3 env_n = mix3(gnd, mix3(hor, zen, up_n), up_n);
    const f3 env_r = mix3(gnd, mix3(hor, zen, up_r), up_r);
    const float m = s_clamp(metallic, 0.0f, 1.0f), rgh = s_clamp(roughness, 0.0f, 1.0f);
    const f3 F0 = mix3(f3{0.04f, 0.04f, 0.04f}, gmax3(base, f3{0.0f, 0.0f, 0.0f}), m);
    const float fres = pow5(1.0f - s_max(0.0f, dot3(n, v)));
    const f3 F = add3(F0, sc3(sub3(f3{1.0f, 1.0f, 1.0f}, F0), fres));
    const f3 kd = sc3(sub3(f3{1.0f, 1.0f, 1.0f}, F), 1.0f - m);
    const f3 diffuse_ibl = sc3(mul3(mul3(kd, base), env_n), 0.12f);
    const float spec_strength = 0.02f + (1.0f - rgh) * 0.18f;
    const f3 spec_ibl = sc3(mul3(env_r, F), spec_strength);
    return sc3(add3(diffuse_ibl, spec_ibl), s_clamp(ao, 0.0f, 1.0f));
}

// The CullingLightGPU fields the point-light program reads (64 B; staged in LDS per workgroup).
struct PLight {
    float4 pr;        // position_range
    float4 ci;        // color_intensity
    float4 sa;        // shape_attenuation
    uint32_t model;   // type_shape_flags[3]: attenuation model
};
constexpr int LIB_LDS_LIGHTS = 256;                  // lights staged in LDS by the camera pass
__shared__ float4 lib_lds_lights[LIB_LDS_LIGHTS * 4];  // per light: pr, ci, sa, (model bits, 0, 0, 0)

__device__ __forceinline__ PLight plight_global(const CullLight &L) {
    PLight p;
    p.pr = *reinterpret_cast<const float4 *>(L.position_range);
    p.ci = *reinterpret_cast<const float4 *>(L.color_intensity);
    p.sa = *reinterpret_cast<const float4 *>(L.shape_attenuation);
    p.model = L.type_shape_flags[3];
    return p;
}

// A light at a wave-uniform index through the constant address space: scalar loads into SGPRs (the
// light table is read-only while a pass runs), so the uniform-list loop holds no light in VGPRs and
// reads no LDS.
typedef const __attribute__((address_space(4))) float ConstF;
__device__ __forceinline__ PLight plight_uniform(const CullLight *lights, uint32_t idx) {
    ConstF *p = (ConstF *)(lights + idx);   // 40 floats: position_range at 0, color_intensity 4,
    PLight o;                               // shape_attenuation 20, type_shape_flags 24
    o.pr = make_float4(p[0], p[1], p[2], p[3]);
    o.ci = make_float4(p[4], p[5], p[6], p[7]);
    o.sa = make_float4(p[20], p[21], p[22], p[23]);
    o.model = __float_as_uint(p[27]);
    return o;
}

__device__ __forceinline__ PLight plight_lds(uint32_t i) {
    PLight p;
    p.pr = lib_lds_lights[4 * i];
    p.ci = lib_lds_lights[4 * i + 1];
    p.sa = lib_lds_lights[4 * i + 2];
    p.model = __float_as_uint(lib_lds_lights[4 * i + 3].x);
    return p;
}

// eval_distance_attenuation (lighting/light_runtime.hpp:182-210) on a CullingLightGPU
__device__ __forceinline__ float distance_attenuation(const PLight &L, float distance) {
    const float range = s_max(L.pr.w, 0.001f);
    if (distance >= range) return 0.0f;
    const float norm = s_clamp(1.0f - distance / range, 0.0f, 1.0f);
    float falloff = 0.0f;
    const uint32_t model = L.model;
    if (model == 0u) {
        falloff = norm;
    } else if (model == 1u) {
        falloff = (norm * norm) * (3.0f - 2.0f * norm);
    } else if (model == 2u) {
        const float inv = 1.0f / s_max(distance * distance, L.sa.z);
        falloff = s_min(1.0f, inv * (range * range)) * (norm * norm);
    }
    const float fpow = s_max(L.sa.y, 0.001f);
    falloff = fpow == 1.0f ? s_max(falloff, 0.0f) : powf(s_max(falloff, 0.0f), fpow);   // pow(x, 1) == x exactly
    if (L.sa.w > 0.0f && falloff < L.sa.w) return 0.0f;
    return s_max(falloff, 0.0f);
}

// PointLightModel::sample + eval_local_light_brdf (light_runtime.hpp:212-237, 321-333), accumulated
// as lit += base * diffuse + specular (exp-plumbing/hello_light_types_culling_sw.cpp:414).
__device__ __forceinline__ void point_light(const PLight &L, f3 world, f3 N, f3 V, f3 base, f3 &lit) {
    const f3 tl = {L.pr.x - world.x, L.pr.y - world.y, L.pr.z - world.z};
    const float d2 = dot3(tl, tl);
    // out of range without the square root: d2 > range^2 (1 + 2^-20) implies the correctly rounded
    // sqrt(d2) > range (NaN / overflow fall through to the exact test)
    if (d2 > (L.pr.w * L.pr.w) * (1.0f + 0x1p-20f)) return;
    const float dist = sqrtf(d2);
    if (dist <= 1e-4f || dist > L.pr.w) return;
    const f3 Ld = {tl.x / dist, tl.y / dist, tl.z / dist};
    const float ndotl = s_max(dot3(N, Ld), 0.0f);
    if (ndotl <= 0.0f) return;
    const float att = distance_attenuation(L, dist) * s_max(1.0f, 0.0f);
    if (att <= 0.0f) return;
    const float ci = s_max(L.ci.w, 0.0f);
    const f3 rad = {(s_max(L.ci.x, 0.0f) * ci) * att, (s_max(L.ci.y, 0.0f) * ci) * att,
                    (s_max(L.ci.z, 0.0f) * ci) * att};
    f3 h = add3(Ld, V);
    const float len2 = dot3(h, h);
    h = len2 <= 1e-10f ? Ld : sc3(h, 1.0f / sqrtf(len2));                     // normalize_or(L + V, L)
    // pow(x, 36) by squaring (x^32 * x^4, <= 6 ulp): well inside the shaded-float tolerance
    const float x1 = s_max(dot3(N, h), 0.0f), x2 = x1 * x1, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8, x32 = x16 * x16;
    const float spec = 0.30f * (x32 * x4);
    lit = add3(lit, add3(mul3(base, sc3(rad, ndotl)), sc3(rad, spec)));
}

// The Forward+ list of one resolve wave's 16x4 pixel block when every lane of the wave reads the same
// list (tiled modes, light tiles a multiple of 16 x 4 px): its count and indices copied into the
// wave's own LDS slice (<= 128 entries) by the whole wave, so the shading loop reads one broadcast
// index per light -- no workgroup barrier (a wave's LDS accesses are in order).  (Not v_readlane of
// per-lane registers: inside the shading branch the compiler may copy such a register for the active
// lanes only, leaving the other lanes' entries stale.)  list = ~0: per-lane lists.
struct LtWave {
    uint32_t list = 0xffffffffu;
    uint32_t count = 0;
    const uint32_t *ids = nullptr;   // LDS
    uint32_t *fids = nullptr;        // LDS, 128 entries: the list culled by the wave's world box
    uint32_t *box = nullptr;         // LDS, 6 words: the wave's world box (orderable bits)
};

// float <-> unsigned with the same order (box reductions through LDS unsigned atomics)
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o); }

// The wave's light list culled by the box of its shading lanes' world positions (the active lanes;
// a wave-uniform list, LtWave): point_light adds exactly nothing for a light whose range sphere the
// pixel lies outside -- it returns before touching `lit` when its float d2 > range^2 (1 + 2^-20) or
// sqrt(d2) > range -- and the float d2 of any pixel in the box is at least the box's exact squared
// distance to the light times (1 - 2^-21) (three roundings of the differences, squares and sums).
// The box distance here, computed in float (a few roundings, relative 2^-22), is compared with
// range^2 * (1 + 2^-10): a culled light is out of every lane's range with a wide margin, so the
// survivors in list order give bit-identical sums.  Lanes with a non-finite world position keep the
// whole list (their sums depend on every light).  Returns the culled count; ids -> lw.fids.
__device__ __forceinline__ uint32_t cull_wave_list(const LibFrameParams &fp, const LibBuffers &fb, const LtWave &lw, f3 world,
                                                   bool lds) {
    const uint64_t ex = __ballot(1);
    const bool fin = isfinite(world.x) && isfinite(world.y) && isfinite(world.z);
    if (!lds || __ballot(!fin) != 0ull) return 0xffffffffu;   // (lights staged in LDS: <= LIB_LDS_LIGHTS)
    const int lane = __lane_id();
    const int first = __ffsll((unsigned long long)ex) - 1;
    uint32_t *bx = lw.box;
    __builtin_amdgcn_wave_barrier();   // the previous call's reads of the box are issued
    if (lane == first) {
        bx[0] = bx[1] = bx[2] = 0xffffffffu;
        bx[3] = bx[4] = bx[5] = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    atomicMin(&bx[0], f2ord(world.x)); atomicMin(&bx[1], f2ord(world.y)); atomicMin(&bx[2], f2ord(world.z));
    atomicMax(&bx[3], f2ord(world.x)); atomicMax(&bx[4], f2ord(world.y)); atomicMax(&bx[5], f2ord(world.z));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const float lx = ord2f(bx[0]), ly = ord2f(bx[1]), lz = ord2f(bx[2]);
    const float hx = ord2f(bx[3]), hy = ord2f(bx[4]), hz = ord2f(bx[5]);
    const uint32_t n_act = (uint32_t)__popcll(ex);
    const uint32_t rank = (uint32_t)__popcll(ex & ((1ull << lane) - 1ull));
    uint32_t w = 0u;
    for (uint32_t base = 0; base < lw.count; base += n_act) {
        const uint32_t i = base + rank;
        bool keep = false;
        uint32_t idx = 0u;
        if (i < lw.count) {
            idx = lw.ids[i];
            if (idx < fp.n_lights) {
                const float4 pr = lib_lds_lights[4 * idx];
                // (fmaxf, not s_max: ROCm 7.2's instruction selection crashes on the select form here;
                // a NaN difference gives gap 0 -- kept -- and an infinite light position an infinite gap,
                // which point_light's d2 test rejects as well)
                const float gx = fmaxf(0.0f, fmaxf(lx - pr.x, pr.x - hx));
                const float gy = fmaxf(0.0f, fmaxf(ly - pr.y, pr.y - hy));
                const float gz = fmaxf(0.0f, fmaxf(lz - pr.z, pr.z - hz));
                const float d2 = (gx * gx + gy * gy) + gz * gz;
                keep = !(d2 > (pr.w * pr.w) * (1.0f + 0x1p-10f));   // NaN / inf ranges: kept
            }
        }
        const uint64_t m = __ballot(keep);
        if (keep) lw.fids[w + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = idx;
        w += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return w;
}

// The pixel's tile list (tiled modes; fp_stress_scene.frag:644-652 tile index).
__device__ __forceinline__ uint32_t lt_tile_list(const LibFrameParams &fp, int px, int py) {
    const uint32_t ts = fp.lt_size;
    const uint32_t tx = min((uint32_t)px / ts, fp.lt_tx - 1u), ty = min((uint32_t)(fp.H - 1 - py) / ts, fp.lt_ty - 1u);
    return ty * fp.lt_tx + tx;
}

// Forward+ program: the pixel's light list (fp_stress_scene.frag:644-685 selection: a saturated list
// falls back to every light) through PointLightModel::sample, combined as the software light-culling
// demo does (hello_light_types_culling_sw.cpp:404-416): ambient hemisphere + sum, clamped to [0,1].
template <bool CULL>
__device__ f3 forward_plus(const LibFrameParams &fp, const LibBuffers &fb, const LibDrawGPU &dr, f3 world, f3 nrm, int px, int py,
                           const LtWave &lw) {
    const f3 N = normalize3(nrm);
    f3 V = sub3(f3{dr.cam[0], dr.cam[1], dr.cam[2]}, world);
    const float vl2 = dot3(V, V);
    V = vl2 <= 1e-10f ? f3{0.0f, 0.0f, 1.0f} : sc3(V, 1.0f / sqrtf(vl2));        // normalize_or
    const float hemi = 0.5f + 0.5f * s_clamp(N.y, -1.0f, 1.0f);
    const float amb = 0.22f + 0.12f * hemi;                                     // kAmbientBase / kAmbientHemi
    const f3 base = {dr.base[0], dr.base[1], dr.base[2]};
    f3 lit = sc3(base, amb);
    const uint32_t ts = fp.lt_size, maxp = fp.lt_maxp;
    const uint32_t tx = min((uint32_t)px / ts, fp.lt_tx - 1u), ty = min((uint32_t)(fp.H - 1 - py) / ts, fp.lt_ty - 1u);
    uint32_t list = lt_tile_list(fp, px, py);
    if (fp.lt_mode == 3u) {   // cluster_slice_from_view_depth (fp_stress_scene.frag:525-533)
        const float vz = (fp.lt_view_z[0] * world.x + fp.lt_view_z[1] * world.y) + (fp.lt_view_z[2] * world.z + fp.lt_view_z[3] * 1.0f);
        const float near_z = s_max(fp.lt_zn, 0.001f), far_z = s_max(fp.lt_zf, near_z + 0.01f);
        const float d = g_clamp(s_max(0.001f, vz), near_z, far_z);
        const float t = logf(d / near_z) / s_max(logf(far_z / near_z), 1e-6f);
        const float zi = g_clamp(floorf(t * (float)fp.lt_zs), 0.0f, (float)(fp.lt_zs - 1u));
        list = ((uint32_t)zi * fp.lt_ty + ty) * fp.lt_tx + tx;
    }
    const bool lds = fp.n_lights <= (uint32_t)LIB_LDS_LIGHTS;   // k_lib_resolve staged them
    const bool uni = lw.list != 0xffffffffu;   // wave-uniform: every lane's list is lw.list
    const uint32_t count = uni ? lw.count : fp.lt_mode == 0u ? maxp : min(fb.tile_counts[list], maxp);
    if (count >= maxp) {
        for (uint32_t i = 0; i < fp.n_lights; ++i)
            point_light(lds ? plight_lds(i) : plight_global(fb.lights[i]), world, N, V, base, lit);
    } else if (uni) {   // the list in the wave's LDS slice: one broadcast index per light
        const uint32_t *ids = lw.ids;
        uint32_t n = count;
        if (CULL && lw.fids) {   // culled by the wave's world box (exact: cull_wave_list)
            const uint32_t nc = (uint32_t)__builtin_amdgcn_readfirstlane((int)cull_wave_list(fp, fb, lw, world, lds));
            if (nc != 0xffffffffu) { ids = lw.fids; n = nc; }
        }
        for (uint32_t i = 0; i < n; ++i) {   // C4 0.828 -> 0.815 ms against LDS-staged lights
            const uint32_t idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)ids[i]);   // uniform
            if (idx < fp.n_lights) point_light(plight_uniform(fb.lights, idx), world, N, V, base, lit);
        }
    } else {
        // the next index is loaded while the current light is evaluated
        const uint32_t *ids = fb.tile_indices + (size_t)list * maxp;
        uint32_t next = count > 0 ? ids[0] : 0u;
        for (uint32_t i = 0; i < count; ++i) {
            const uint32_t idx = next;
            if (i + 1 < count) next = ids[i + 1];
            if (idx < fp.n_lights) point_light(lds ? plight_lds(idx) : plight_global(fb.lights[idx]), world, N, V, base, lit);
        }
    }
    return f3{g_clamp(lit.x, 0.0f, 1.0f), g_clamp(lit.y, 0.0f, 1.0f), g_clamp(lit.z, 0.0f, 1.0f)};
}

// sample_texture2d_bilinear_repeat_linear (builtin_shaders.hpp:33-55): repeat wrap, bilinear over
// srgb_to_linear_rgb (:25-31) texels; the sRGB decode is the host-computed table of the reference's
// own std::pow values (bit-identical), the lerps glm::mix's x * (1 - a) + y * a.  Indices are clamped
// into the texture, which only changes non-finite UVs (where the reference reads out of bounds).
__device__ __forceinline__ f3 srgb_texel(const LibBuffers &fb, uint32_t c) {
    return f3{fb.srgb_lut[c & 0xffu], fb.srgb_lut[(c >> 8) & 0xffu], fb.srgb_lut[(c >> 16) & 0xffu]};
}

__device__ __noinline__ f3 sample_base_color(const LibBuffers &fb, const LibDrawGPU &dr, float uvx, float uvy) {
    const float u = uvx - floorf(uvx);
    const float v = uvy - floorf(uvy);
    const float fx = u * (float)(dr.tex_w - 1);
    const float fy = v * (float)(dr.tex_h - 1);
    const int x0 = min(max((int)floorf(fx), 0), dr.tex_w - 1);
    const int y0 = min(max((int)floorf(fy), 0), dr.tex_h - 1);
    const int x1 = min(x0 + 1, dr.tex_w - 1);
    const int y1 = min(y0 + 1, dr.tex_h - 1);
    const float tx = fx - (float)x0;
    const float ty = fy - (float)y0;
    const uint32_t *row0 = dr.tex + (size_t)y0 * dr.tex_w, *row1 = dr.tex + (size_t)y1 * dr.tex_w;
    const f3 c00 = srgb_texel(fb, row0[x0]), c10 = srgb_texel(fb, row0[x1]);
    const f3 c01 = srgb_texel(fb, row1[x0]), c11 = srgb_texel(fb, row1[x1]);
    return mix3(mix3(c00, c10, tx), mix3(c01, c11, tx), ty);
}

// The builtin fragment programs (builtin_shaders.hpp:105-245); tex = the base_color_tex sample
// (vec3(1) without a texture, :35).
// PROG >= 0: every draw of the pass runs that program (k_lib_resolve specialisations: only its
// registers are live); -1: per draw.
template <int PROG>
__device__ f3 lib_fragment(const LibFrameParams &fp, const LibBuffers &fb, const LibDrawGPU &dr, f3 world, f3 nrm, float depth01,
                           int px, int py, const LtWave &st, f3 tex = f3{1.0f, 1.0f, 1.0f}) {
    const f3 bc = {dr.base[0], dr.base[1], dr.base[2]};
    const int program = PROG >= 0 ? PROG : dr.program;
    if (program == 5) return forward_plus<true>(fp, fb, dr, world, nrm, px, py, st);
    if (program == 2) return bc;                                                   // debug albedo
    if (program == 3) return add3(sc3(normalize3(nrm), 0.5f), f3{0.5f, 0.5f, 0.5f});  // debug normal
    if (program == 4) {                                                            // debug depth
        const float dd = s_clamp(depth01, 0.0f, 1.0f);
        return f3{dd, dd, dd};
    }
    const f3 L = {dr.L[0], dr.L[1], dr.L[2]};
    const f3 cam = {dr.cam[0], dr.cam[1], dr.cam[2]};
    const f3 lcol = {dr.lcol[0], dr.lcol[1], dr.lcol[2]};
    const f3 albedo = gmax3(mul3(bc, tex), f3{0.0f, 0.0f, 0.0f});   // max(base_color * albedo_tex, 0)
    const f3 N = normalize3(nrm);
    const f3 V = normalize3(sub3(cam, world));
    if (program == 1) {   // make_blinn_phong_program (:111-150)
        const f3 H = normalize3(add3(L, V));
        const float NdotL = s_max(0.0f, dot3(N, L));
        const float NdotH = s_max(0.0f, dot3(N, H));
        const float rough = s_clamp(dr.mat[0], 0.0f, 1.0f);
        const float metal = s_clamp(dr.base[3], 0.0f, 1.0f);
        const float spec_pow = s_max(4.0f, 8.0f + (1.0f - rough) * 120.0f);
        const float spec_norm = (spec_pow + 2.0f) / (2.0f * PI_F);
        const float spec_f0 = 0.04f + 0.96f * metal;
        const float spec = ((powf(NdotH, spec_pow) * spec_norm) * spec_f0) * NdotL;
        const float kd = 1.0f - metal;
        const f3 diffuse = sc3(mul3(f3{kd, kd, kd}, albedo), NdotL / PI_F);
        float vis = 1.0f;
        if (dr.shadow && NdotL > 0.0f) vis = g_mix(1.0f, shadow_visibility(fp, fb, dr, world, NdotL), s_clamp(dr.mat[2], 0.0f, 1.0f));
        const f3 direct = sc3(sc3(mul3(add3(diffuse, f3{spec, spec, spec}), lcol), dr.lcol[3]), vis);
        return add3(direct, fake_ibl(N, V, albedo, dr.base[3], dr.mat[0], dr.mat[1]));
    }
    // make_pbr_mr_program (:160-212)
    const f3 H = normalize3(add3(V, L));
    const float NdotL = s_max(0.0f, dot3(N, L));
    const float NdotV = s_max(0.0f, dot3(N, V));
    const float NdotH = s_max(0.0f, dot3(N, H));
    const float VdotH = s_max(0.0f, dot3(V, H));
    const float rough = s_clamp(dr.mat[0], 0.04f, 1.0f);
    const float metal = s_clamp(dr.base[3], 0.0f, 1.0f);
    const f3 F0 = mix3(f3{0.04f, 0.04f, 0.04f}, albedo, metal);
    const float a = rough * rough;
    const float a2 = a * a;
    const float denomD = (NdotH * NdotH) * (a2 - 1.0f) + 1.0f;
    const float D = a2 / ((PI_F * denomD) * denomD + 1e-7f);
    const float k = ((a + 1.0f) * (a + 1.0f)) * 0.125f;
    const float G = (NdotV / ((NdotV * (1.0f - k) + k) + 1e-7f)) * (NdotL / ((NdotL * (1.0f - k) + k) + 1e-7f));
    const f3 F = add3(F0, sc3(sub3(f3{1.0f, 1.0f, 1.0f}, F0), pow5(1.0f - VdotH)));
    const float sden = s_max((4.0f * NdotL) * NdotV, 1e-6f);
    const f3 dgf = sc3(F, D * G);
    const f3 spec = {dgf.x / sden, dgf.y / sden, dgf.z / sden};
    const f3 kd = sc3(sub3(f3{1.0f, 1.0f, 1.0f}, F), 1.0f - metal);
    const f3 diff = sc3(mul3(kd, albedo), 1.0f / PI_F);
    const f3 radiance = sc3(lcol, dr.lcol[3]);
    float vis = 1.0f;
    if (dr.shadow && NdotL > 0.0f) vis = g_mix(1.0f, shadow_visibility(fp, fb, dr, world, NdotL), s_clamp(dr.mat[2], 0.0f, 1.0f));
    const f3 direct = (NdotL > 0.0f && NdotV > 0.0f) ? sc3(sc3(mul3(add3(diff, spec), radiance), NdotL), vis) : f3{0.0f, 0.0f, 0.0f};
    return add3(direct, fake_ibl(N, V, albedo, metal, rough, dr.mat[1]));
}

__device__ __forceinline__ float4 bg_color(const LibFrameParams &fp, int y) {
    if (!(fp.flags & LF_GRADIENT)) return make_float4(fp.clear[0], fp.clear[1], fp.clear[2], fp.clear[3]);
    const float t = (float)y / (float)max(1, fp.H - 1);   // pass_pbr_forward.hpp:75-81
    return make_float4(0.06f + 0.08f * t, 0.08f + 0.10f * t, 0.12f + 0.12f * t, 1.0f);
}

constexpr int LIB_PAIR_WORDS = LIB_CHUNK * LIB_RTW * LIB_RTH / 64;   // pair-start bitmap words
constexpr int LIB_MAX_STATIC = 256;                                  // static work items per raster workgroup

template <int LIB_CAND>
struct LibShared {
    float4 rec[LIB_CHUNK * 4];            // staged records (8 KB)
    unsigned long long key[LIB_RTH * LIB_RTW];
    unsigned long long bits[LIB_PAIR_WORDS]; // bit k: a surviving candidate's pairs start at pair k (4 KB)
    // deep raster: per nonempty row span (segment) first pair | x0 << 16 | row << 21 | slot << 24;
    // shallow: per staged box (uint4 pinfo) first pair, x0 | y0 << 16, width | slot << 16, 2^16/width
    alignas(16) uint32_t seg[LIB_CAND == LIB_CAND_DEEP ? LIB_CHUNK * LIB_RTH : LIB_CHUNK * 4];
    uint32_t zord[LIB_CHUNK];             // per staged candidate: its depth bound (0: never skipped)
    uint2 lbox[LIB_CAND];                 // the tile's candidate list, front to back: boxes,
    uint32_t lid[LIB_CAND];               //   slots
    uint32_t lkey[LIB_CAND];              //   and depth bounds (lib_zmin_ord; 0 without a depth test)
    uint32_t sel[LIB_CHUNK];              // list positions staged by the current pass
    uint32_t hist[256];                   // depth buckets: counts, then first positions (the sort)
    uint32_t zlo, zhi;
    uint32_t wtot[4][2];                  // per wave: surviving candidates, pairs
    uint32_t wmax[4];                     // deep camera raster: per wave, the largest key z of its pixels after a pass
    uint32_t last;                        // split tile: this part finished last (it writes the merged keys)
    uint32_t colmax[2][LIB_RTW];          // per pixel column: max key z (orderable bits) over its rows, by chunk parity
    uint32_t nc, nbusy, cov, maxbin, npairs;
    int next[4];                          // the workgroup's next item: any, queue, queues tried, its word
    uint32_t qlen[2 * LIB_NQ];            // camera pass: k_lib_dyn's light, then heavy list lengths
    uint32_t sitem[LIB_MAX_STATIC];       // the workgroup's static work items (k_lib_raster)
    uint64_t tl[LTL_STRIDE];              // SHS_OPT_TIMELINE accumulators (thread 0)
    uint32_t tl_staged;                   // SHS_OPT_TIMELINE: candidates staged in the current tile
    // segment (deep) or staged box (shallow) owning each bitmap word's first pair
    typename std::conditional<LIB_CAND == LIB_CAND_DEEP, uint16_t, uint8_t>::type wown[LIB_PAIR_WORDS];
};


__device__ __forceinline__ LibRec lib_rec_from(const float4 *s) {
    LibRec r;
    float4 *d = reinterpret_cast<float4 *>(&r);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = s[j];
    return r;
}

template <int PROG>
__device__ __forceinline__ void shade_px(const LibFrameParams &fp, const LibBuffers &fb, const LibDrawGPU &dr, const LibRec &r,
                                         const LibShade &s, uint32_t slot, int px, int py, float4 &color, float &depth,
                                         float2 &mv, const LtWave &st);

// Resolve one pixel of a tile (one thread): the winner of the key array is re-evaluated with the
// identical arithmetic, shaded and written; pixels without a winner get the clear values.
template <bool SHADOW, int PROG = -1>
__device__ __forceinline__ float4 lib_resolve(const LibFrameParams &fp, const LibBuffers &fb, unsigned long long key, int px,
                                              int py, bool &covered, const LtWave &st = LtWave{}) {
    covered = key != KEY_EMPTY && px < fp.W && py < fp.H;
    if (px >= fp.W || py >= fp.H) return make_float4(0.f, 0.f, 0.f, 0.f);
    const size_t o = (size_t)py * fp.W + px;
    if (SHADOW) {
        fb.depth[o] = covered ? __uint_as_float((uint32_t)(key >> 32) & 0x7fffffffu) : 1.0f;
        return make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 color = bg_color(fp, py);
    float depth = 1.0f;
    float2 mv = make_float2(0.0f, 0.0f);
    if (covered) {
        const uint32_t seq = (fp.flags & LF_DEPTH) ? (uint32_t)key : 0xffffffffu - (uint32_t)key;
        const uint32_t k = seq & 15u;
        const uint32_t tri = (fp.flags & LF_PERM) ? fb.s2s[seq >> 4] : seq >> 4;   // submission -> stored order
        const uint32_t slot = k == 0 ? tri : fb.xbase[tri] + k - 1u;
        const LibRec r = fb.recs[slot];
        const LibShade s = fb.shade[slot];
        // a wave whose covered pixels share one draw reads its uniforms with scalar loads
        const int d0 = __builtin_amdgcn_readfirstlane(s.draw);
        if (__ballot(s.draw != d0) == 0) shade_px<PROG>(fp, fb, fb.draws[d0], r, s, slot, px, py, color, depth, mv, st);
        else shade_px<PROG>(fp, fb, fb.draws[s.draw], r, s, slot, px, py, color, depth, mv, st);
    }
#ifdef SHS_EXP_RESOLVE_STORES   // timing experiments (wrong images): bit 1 no HDR, 2 no depth, 4 no motion
    if (!(SHS_EXP_RESOLVE_STORES & 1)) fb.hdr[o] = color;
    if (fp.flags & LF_DEPTH) {
        if (!(SHS_EXP_RESOLVE_STORES & 2)) fb.depth[o] = depth;
        if (!(SHS_EXP_RESOLVE_STORES & 4)) fb.motion[o] = mv;
    }
    if (color.x == -1234.5f && depth == -2.0f && mv.x == -3.0f) fb.hdr[o] = color;   // keeps the shading live
#else
    // non-temporal, like the fused tonemap's stores: no later kernel of the frame reads these targets, and
    // 232 MB of them per 4K frame would otherwise cycle through the L2 under the other frames in flight
    // (C4 0.574 -> 0.564, C5 0.372 -> 0.351 ms per frame in three A/B pairs, profiles/r06_resolve_nt_ab.txt)
    {
        typedef float v4f __attribute__((ext_vector_type(4)));
        typedef float v2f __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(v4f{color.x, color.y, color.z, color.w}, reinterpret_cast<v4f *>(&fb.hdr[o]));
        if (fp.flags & LF_DEPTH) {
            __builtin_nontemporal_store(depth, &fb.depth[o]);
            __builtin_nontemporal_store(v2f{mv.x, mv.y}, reinterpret_cast<v2f *>(&fb.motion[o]));
        }
    }
#endif
    return color;
}

// The winner of one pixel: identical re-evaluation of the pixel test, the varyings, motion and the
// fragment program (rasterizer.hpp:341-419).
template <int PROG>
__device__ __forceinline__ void shade_px(const LibFrameParams &fp, const LibBuffers &fb, const LibDrawGPU &dr, const LibRec &r,
                                         const LibShade &s, uint32_t slot, int px, int py, float4 &color, float &depth,
                                         float2 &mv, const LtWave &st) {
    {
        float z01, u, v, w, idn;
        lib_test<false>(fp, r, px, py, z01, u, v, w, idn);
        depth = z01;
        // FragmentIn from the varyings (rasterizer.hpp:365-387): (bc.x*varw0 + bc.y*varw1 + bc.z*varw2) * inv_denom
        const f3 world = {((u * s.wp[0] + v * s.wp[3]) + w * s.wp[6]) * idn, ((u * s.wp[1] + v * s.wp[4]) + w * s.wp[7]) * idn,
                          ((u * s.wp[2] + v * s.wp[5]) + w * s.wp[8]) * idn};
        const f3 nv = {((u * s.n[0] + v * s.n[3]) + w * s.n[6]) * idn, ((u * s.n[1] + v * s.n[4]) + w * s.n[7]) * idn,
                       ((u * s.n[2] + v * s.n[5]) + w * s.n[8]) * idn};
        const f3 nrm = normalize3(nv);
        if ((fp.flags & LF_MOTION) && dr.motion) {   // rasterizer.hpp:388-411
            const f4 cw = {world.x, world.y, world.z, 1.0f};
            const f4 pw = m4v(dr.c2p, cw);
            const f4 cc = m4v(dr.viewproj, cw);
            const f4 pc = m4v(dr.prev_vp, pw);
            if (fabsf(cc.w) > 1e-8f && fabsf(pc.w) > 1e-8f) {
                float vx = ((cc.x / cc.w - pc.x / pc.w) * 0.5f) * (float)fp.W;
                float vy = ((cc.y / cc.w - pc.y / pc.w) * 0.5f) * (float)fp.H;
                const float len = sqrtf(vx * vx + vy * vy);
                if (len > 96.0f && len > 1e-6f) {
                    const float sc = 96.0f / len;
                    vx *= sc; vy *= sc;
                }
                mv = make_float2(vx, vy);
            }
        }
        f3 tex = {1.0f, 1.0f, 1.0f};
        if (PROG != 5 && dr.tex) {   // fin.uv from the UV0 varying (rasterizer.hpp:383-387)
            const size_t slot2 = 2 * (size_t)slot;
            const float4 a = fb.uvw[slot2], b = fb.uvw[slot2 + 1];
            const float uvx = ((u * a.x + v * a.z) + w * b.x) * idn;
            const float uvy = ((u * a.y + v * a.w) + w * b.y) * idn;
            tex = sample_base_color(fb, dr, uvx, uvy);
        }
        const f3 c = lib_fragment<PROG>(fp, fb, dr, world, nrm, z01, px, py, st, tex);
        color = make_float4(c.x, c.y, c.z, 1.0f);
    }
}

// Conservative row span of a staged primitive inside its clipped box [bx0, bx1]: the pixels of row py
// that can pass lib_test's inside test.  With t = px + 0.5 - ax, dy = py + 0.5 - ay the exact
// barycentrics of the record's float values are linear in t:
//   v = av t + cv dy,  w = aw t + cw dy,  u = 1 + au t + cu dy,
//   av = id v1y, cv = -id v1x, aw = -id v0y, cw = id v0x, au = id (v0y - v1y), cu = id (v1x - v0x).
// lib_test's float evaluation (no contraction) is within 4 u Mv of v, Mv = |id| (|v1y t| + |v1x dy|)
// (u = 2^-24; likewise w), and u's within 4 u (1 + 2 Mv + 2 Mw); a pixel can pass only where every
// exact barycentric is >= minus its bound.  Each half-line a t >= -e - c is solved here in float with
// e = E (...) at E = 2^-18, 16x the bound: the slack absorbs this computation's own roundings (a few
// ulps of |e| + |c|, divided by a), and 2^-12 px more covers the conversion to pixel indices.
// Non-finite inputs keep the whole box row.
__device__ __forceinline__ void lib_row_span(const float4 r0, const float4 r1, int py, int bx0, int bx1, int &x0, int &x1) {
    x0 = bx0; x1 = bx1;
    // r0, r1: the record's first two float4s, ax ay v0x v0y | v1x v1y inv_den z0
    const float ax = r0.x, ay = r0.y, v0x = r0.z, v0y = r0.w, v1x = r1.x, v1y = r1.y, id = r1.z;
    if (!(isfinite(ax) && isfinite(ay) && isfinite(v0x) && isfinite(v0y) && isfinite(v1x) && isfinite(v1y) && isfinite(id)))
        return;
    constexpr float E = 0x1p-18f;
    const float dy = ((float)py + 0.5f) - ay, ady = fabsf(dy);
    const float T = fmaxf(fabsf(((float)bx0 + 0.5f) - ax), fabsf(((float)bx1 + 0.5f) - ax));
    const float aid = fabsf(id);
    const float mv = aid * (fabsf(v1y) * T + fabsf(v1x) * ady), mw = aid * (fabsf(v0y) * T + fabsf(v0x) * ady);
    float lo = -1e30f, hi = 1e30f;
    // a t + c >= -e: a > 0: t >= (-e - c) / a; a < 0: t <= (-e - c) / a; a == 0: all or none
    auto edge = [&](float a, float c, float e) {
        const float b = -e - c;
        if (a > 0.0f) lo = fmaxf(lo, b / a);
        else if (a < 0.0f) hi = fminf(hi, b / a);
        else if (b > 0.0f) { lo = 1e30f; hi = -1e30f; }
    };
    edge(id * v1y, -id * v1x * dy, E * mv);
    edge(-id * v0y, id * v0x * dy, E * mw);
    edge(id * (v0y - v1y), 1.0f + id * (v1x - v0x) * dy, E * (1.0f + 2.0f * (mv + mw)));
    // pixels with px + 0.5 - ax in [lo, hi]
    const float flo = (lo + ax) - 0.5f, fhi = (hi + ax) - 0.5f;
    const float slo = 0x1p-12f * (fabsf(lo) + fabsf(ax) + 1.0f), shi = 0x1p-12f * (fabsf(hi) + fabsf(ax) + 1.0f);
    x0 = max(bx0, (int)ceilf(fmaxf(fminf(flo - slo, 1e9f), -1e9f)));
    x1 = min(bx1, (int)floorf(fmaxf(fminf(fhi + shi, 1e9f), -1e9f)));
}

// One work item: raster tile rt, or (k_lib_plan, camera pass) part `part` of `parts` of it: the list
// positions [part n / parts, (part + 1) n / parts) over the whole tile, its keys merged with the other
// parts' in fb.pkeys[sid] (plan_parts).  T0 = the tile origin (LDS key layout); X0..Y1 = the tile.
template <bool SHADOW, int LIB_CAND>
__device__ void lib_raster_tile(const LibFrameParams &fp, const LibBuffers &fb, const uint32_t *cnt, int rt, LibShared<LIB_CAND> &sh,
                                uint32_t &chunk, uint32_t part = 0u, uint32_t parts = 1u, uint32_t sid = 0u) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool hiz = SHADOW || (fp.flags & LF_DEPTH);   // painter's order (no depth target): never
    const int col = rt % fp.tiles_x, row = rt / fp.tiles_x;
    const int TX0 = col * LIB_RTW, TY0 = row * LIB_RTH;
    const int X0 = TX0, Y0 = TY0, X1 = TX0 + LIB_RTW - 1, Y1 = TY0 + LIB_RTH - 1;
    // this thread's pixel (tile layout: wave w = 16x4 block w)
    const int my_lx = 16 * (wave & 1) + (lane & 15), my_ly = 4 * (wave >> 1) + (lane >> 4);
    const int bt = (row / (TILE / LIB_RTH)) * fp.tiles_x + col;
    // (no barrier here: the previous tile ended with each thread resetting its own pixel's key, and
    // every round below starts with one before any shared state is touched)
    const bool tlon = fb.timeline != nullptr && tid == 0;
    const uint64_t t_tile = tlon ? tl_now() : 0ull;
    uint64_t t_gather = 0ull;
    const uint32_t chunk0 = chunk;
    uint32_t t_rounds = 0u, t_pairs = 0u, t_breaks = 0u;   // (timeline, thread 0: this tile's counts)
    if (tlon) sh.tl_staged = 0u;

    uint32_t n_bin = 0, n_spill = 0, n_items;
    bool gsorted = false;   // the bin list is depth-sorted whole (k_lib_hsort) over hsr's range
    uint2 hsr = make_uint2(0u, 0u);
    if (fp.scan_mode) {
        n_items = (uint32_t)fp.n_tris + (SHADOW ? 0u : min(cnt[LC_EXTRA], fp.extra_cap));
    } else {
        const uint32_t n_bin_total = fb.tile_count[(size_t)fp.parity * fp.tiles_x * fp.tiles_y + bt];
        n_bin = min(n_bin_total, fp.bin_cap);
        if (n_bin_total > fp.bin_cap) n_spill = min(cnt[LC_SPILL], fp.spill_cap);
        n_items = n_bin + n_spill;
        if (tid == 0) sh.maxbin = max(sh.maxbin, n_bin_total);
        // (the predicate k_lib_dyn listed the tile's bin list by; this tile is busy, so it was listed)
        gsorted = !SHADOW && LIB_CAND == LIB_CAND_DEEP && hiz && fp.hsort && parts == 1u && n_bin_total > fp.hsort_min &&
                  n_bin_total <= min(fp.bin_cap, (uint32_t)LIB_HSORT_MAX);
        if (gsorted) hsr = fb.hsr[bt];
    }
    const uint4 *bin = fb.bins + (size_t)bt * fp.bin_cap;
    // a part's share of the list (positions [lo, n_items))
    const uint32_t lo = (uint32_t)(((uint64_t)n_items * part) / parts);
    n_items = (uint32_t)(((uint64_t)n_items * (part + 1u)) / parts);

    const uint32_t tl_items = n_items;
    for (uint32_t base = lo; base < n_items; base += LIB_CAND) {
        __syncthreads();
        if (gsorted && base > lo && chunk != chunk0) {
            // a sorted list: every entry from `base` on lies in hsr bucket >= the one of bin[base]; once the
            // tile's largest key z (the waves' maxima after the last pass, stale only upwards) sorts into a
            // lower bucket, or below the whole range, no later entry can beat any pixel -- the tile is done
            const uint32_t om = max(max(sh.wmax[0], sh.wmax[1]), max(sh.wmax[2], sh.wmax[3]));
            if (om < hsr.x || hs_bucket(hsr, om) < hs_bucket(hsr, bin[base].w)) break;
        }
        ++t_rounds;
        if (tid == 0) { sh.nc = 0; sh.zlo = 0xffffffffu; sh.zhi = 0u; }
        sh.hist[tid] = 0u;
        __syncthreads();
        const uint64_t t_g0 = tlon ? tl_now() : 0ull;
        // (1) gather up to LIB_CAND candidates (bin list or every primitive), their boxes and depth
        //     bounds in one round trip; a candidate's box overlaps the tile
        constexpr int NG = LIB_CAND / 256;
        uint32_t ids[NG], zk[NG];
        uint2 bx[NG];
        bool hit[NG];
        if (fp.scan_mode) {
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const uint32_t item = base + tid + 256u * k;
                ids[k] = item < n_items ? item : 0xffffffffu;
            }
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                bx[k] = ids[k] != 0xffffffffu ? fb.boxes[ids[k]] : make_uint2(0u, 0u);
                zk[k] = hiz && ids[k] != 0xffffffffu ? fb.zord[ids[k]] : 0u;
            }
        } else {
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const uint32_t item = base + tid + 256u * k;
                uint4 e = make_uint4(0xffffffffu, 0u, 0u, 0u);
                if (item < n_bin) {   // the entry carries the box and the depth bound
                    e = bin[item];
                } else if (item < n_items) {   // spilled entries hold the slot only (rare)
                    const uint2 sp = fb.spill[item - n_bin];
                    if ((int)sp.x == bt) {
                        const uint2 b = fb.boxes[sp.y];
                        e = make_uint4(sp.y, b.x, b.y, fb.zord[sp.y]);
                    }
                }
                ids[k] = e.x;
                bx[k] = e.x != 0xffffffffu ? make_uint2(e.y, e.z) : make_uint2(0u, 0u);
                zk[k] = hiz && e.x != 0xffffffffu ? e.w : 0u;
            }
        }
        uint32_t zlo = 0xffffffffu, zhi = 0u, nhit = 0u;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int gx0 = lo16(bx[k].x), gx1 = hi16(bx[k].x), gy0 = lo16(bx[k].y), gy1 = hi16(bx[k].y);
            hit[k] = ids[k] != 0xffffffffu && gx0 <= gx1 && gy0 <= gy1 && gx1 >= X0 && gx0 <= X1 && gy1 >= Y0 && gy0 <= Y1;
            if (hit[k]) { zlo = min(zlo, zk[k]); zhi = max(zhi, zk[k]); }
            nhit += (uint32_t)__popcll(__ballot(hit[k]));
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            zlo = min(zlo, (uint32_t)__shfl_xor((int)zlo, off));
            zhi = max(zhi, (uint32_t)__shfl_xor((int)zhi, off));
        }
        uint32_t basew = 0;   // this wave's first position in gather order
        if (lane == 0 && nhit) { basew = atomicAdd(&sh.nc, nhit); atomicMin(&sh.zlo, zlo); atomicMax(&sh.zhi, zhi); }
        basew = (uint32_t)__shfl((int)basew, 0);
        __syncthreads();
        const uint32_t nc = sh.nc;
        // one staging pass holds every candidate (or painter's order): gather order, no sort
        const bool sorted = hiz && nc > (uint32_t)LIB_CHUNK;
        if (!sorted) {
            uint32_t run = 0;
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const uint64_t hm = __ballot(hit[k]);
                if (hit[k]) {
                    const uint32_t pos = basew + run + lanes_below(hm);
                    sh.lid[pos] = ids[k];
                    sh.lkey[pos] = zk[k];
                    sh.lbox[pos] = bx[k];
                }
                run += (uint32_t)__popcll(hm);
            }
        }
        // (2) the list, front to back: a 256-bucket counting sort by depth bound.  bucket(z) is
        //     monotone in z, so the entries from position p on lie in buckets >= bucket(lkey[p]).
        //     Order inside a tile is otherwise free -- the resolve is by (z, submission index) keys.
        const uint32_t s_lo = sh.zlo, s_span = sh.zhi - sh.zlo;
        const float s_scale = (hiz && s_span) ? 255.0f / (float)s_span : 0.0f;
        auto bucket = [&](uint32_t z) { return min(255u, (uint32_t)((float)(z - s_lo) * s_scale)); };
        uint32_t bk[NG], rk[NG];
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            bk[k] = 0u; rk[k] = 0u;
            if (sorted && hit[k]) { bk[k] = bucket(zk[k]); rk[k] = atomicAdd(&sh.hist[bk[k]], 1u); }
        }
        if (sorted) {
            __syncthreads();
            const uint32_t cntb = sh.hist[tid];
            uint32_t incl = cntb;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t vv = (uint32_t)__shfl_up((int)incl, o);
                if (lane >= o) incl += vv;
            }
            if (lane == 63) sh.wtot[wave][0] = incl;
            __syncthreads();
            uint32_t wbase = 0;
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) wbase += w2 < wave ? sh.wtot[w2][0] : 0u;
            sh.hist[tid] = wbase + incl - cntb;   // first position of bucket tid
            __syncthreads();
#pragma unroll
            for (int k = 0; k < NG; ++k)
                if (hit[k]) {
                    const uint32_t pos = sh.hist[bk[k]] + rk[k];
                    sh.lid[pos] = ids[k];
                    sh.lkey[pos] = zk[k];
                    sh.lbox[pos] = bx[k];
                }
        }
        __syncthreads();
        if (tlon) { t_gather += tl_now() - t_g0; sh.tl[LTL_NCAND] += nc; }

        if constexpr (LIB_CAND == LIB_CAND_DEEP && !SHADOW) {
            // (3) deep camera raster: passes over LIB_CHUNK list positions, a pair of threads per position
            //     (position c = tid / 2; half h = tid & 1 takes the tile rows 4h .. 4h + 3), three barriers
            //     per pass.  A position is staged when its depth bound can still beat the key z of some
            //     pixel of its box (hierarchical z against the keys themselves: exact, never drops a
            //     possible winner); its pair of threads loads the record, solves its row spans in
            //     registers and lays its segments out after one block prefix.  In a sorted list, once the
            //     item's largest key z (a per-wave maximum read after the previous pass, stale only
            //     upwards) sorts into a lower bucket than the next position's bound, the rest is skipped.
            static_assert(2 * LIB_CHUNK == 256 && LIB_PAIR_WORDS == 512, "a thread pair per staged position");
            const int c = tid >> 1, h = tid & 1;
            const uint32_t *keyhi = reinterpret_cast<const uint32_t *>(sh.key);   // [2 * pixel + 1]: key z
            uint32_t p = 0;
            while (p < nc) {
                __syncthreads();   // [A] the previous pass's pairs are resolved; its bits, segments, records free
                const uint64_t t_a = tlon ? tl_now() : 0ull;
                const bool first = chunk == chunk0;   // no key of the tile written yet
                const uint32_t ordmax = first ? 0xffffffffu : max(max(sh.wmax[0], sh.wmax[1]), max(sh.wmax[2], sh.wmax[3]));
                // (the list is front to back only when sorted; the per-position test below holds either way)
                if (sorted && ordmax != 0xffffffffu && (ordmax < s_lo || bucket(ordmax) < bucket(sh.lkey[p]))) {
                    ++t_breaks;
                    break;
                }
                ++chunk;
                sh.bits[tid] = 0ull;
                sh.bits[tid + 256] = 0ull;
                const uint32_t q = p + (uint32_t)c;
                bool alive = false;
                int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1;
                uint32_t zk = 0u;
                if (q < nc) {
                    const uint2 b = sh.lbox[q];
                    bx0 = max(lo16(b.x), X0); bx1 = min(hi16(b.x), X1);
                    by0 = max(lo16(b.y), Y0); by1 = min(hi16(b.y), Y1);
                    zk = sh.lkey[q];
                    alive = bx0 <= bx1 && by0 <= by1;
                    if (alive && hiz && !first) {
                        if (zk > ordmax) {
                            alive = false;
                        } else if ((bx1 - bx0 + 1) * (by1 - by0 + 1) <= SHS_HIZ_BOX) {
                            uint32_t mx = 0u;
                            for (int y = by0; y <= by1; ++y)
                                for (int x = bx0; x <= bx1; ++x) mx = max(mx, keyhi[2 * ((y - TY0) * LIB_RTW + (x - TX0)) + 1]);
                            alive = zk <= mx;
                        }
                    }
                }
                if (fb.timeline) {   // (uniform) staged candidates of this tile
                    const uint64_t am = __ballot(alive && h == 0);
                    if (lane == 0 && am) atomicAdd(&sh.tl_staged, (uint32_t)__popcll(am));
                }
                // the record: half h loads and stages its two float4s; both need the first two (the spans)
                float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
                if (alive) {
                    const float4 *src = reinterpret_cast<const float4 *>(&fb.recs[sh.lid[q]]) + 2 * h;
                    ra = src[0];
                    rb = src[1];
                    sh.rec[c * 4 + 2 * h] = ra;
                    sh.rec[c * 4 + 2 * h + 1] = rb;
                    if (h == 0) sh.zord[c] = zk;
                }
                const float4 oa = make_float4(__shfl_xor(ra.x, 1), __shfl_xor(ra.y, 1), __shfl_xor(ra.z, 1), __shfl_xor(ra.w, 1));
                const float4 ob = make_float4(__shfl_xor(rb.x, 1), __shfl_xor(rb.y, 1), __shfl_xor(rb.z, 1), __shfl_xor(rb.w, 1));
                const float4 r0 = h ? oa : ra, r1 = h ? ob : rb;
                // this half's four row spans (tile-relative x0 | x1 << 8; 0x1f: empty)
                uint32_t spw[4];
                uint32_t pk = 0u;   // pairs << 11 | segments
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int py = TY0 + 4 * h + k;
                    int s0 = 1, s1 = 0;
                    if (alive && py >= by0 && py <= by1) lib_row_span(r0, r1, py, bx0, bx1, s0, s1);
                    spw[k] = s1 >= s0 ? (uint32_t)(s0 - TX0) | ((uint32_t)(s1 - TX0) << 8) : 0x1fu;
                    if (s1 >= s0) pk += ((uint32_t)(s1 - s0 + 1) << 11) + 1u;
                }
                uint32_t incl = pk;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t vv = (uint32_t)__shfl_up((int)incl, o);
                    if (lane >= o) incl += vv;
                }
                if (lane == 63) sh.wtot[wave][1] = incl;
                __syncthreads();   // [B] every wave's total, the zeroed bits
                const uint64_t t_b = tlon ? tl_now() : 0ull;
                uint32_t pbase = 0, ptot = 0;
#pragma unroll
                for (int w2 = 0; w2 < 4; ++w2) {
                    const uint32_t p2 = sh.wtot[w2][1];
                    if (w2 < wave) pbase += p2;
                    ptot += p2;
                }
                if (pk) {
                    const uint32_t ex = pbase + incl - pk;
                    uint32_t ps = ex >> 11, sg = ex & 2047u;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int s0 = (int)(spw[k] & 0xffu), s1 = (int)(spw[k] >> 8);
                        if (s1 < s0) continue;
                        const uint32_t wdt = (uint32_t)(s1 - s0 + 1);
                        sh.seg[sg] = ps | ((uint32_t)s0 << 16) | ((uint32_t)(4 * h + k) << 21) | ((uint32_t)c << 24);
                        atomicOr(&sh.bits[ps >> 6], 1ull << (ps & 63u));
                        for (uint32_t wd = (ps + 63u) >> 6; wd * 64u < ps + wdt; ++wd) sh.wown[wd] = (uint16_t)sg;
                        ps += wdt;
                        ++sg;
                    }
                }
                __syncthreads();   // [C] segments, starts and staged records complete
                const int total = (int)(ptot >> 11);
                if (tlon) {
                    const uint64_t t_c = tl_now();
                    t_pairs += (uint32_t)total;
                    sh.tl[LTL_NPAIRS] += (uint32_t)total;
                    sh.tl[LTL_STAGE] += t_b - t_a;
                    sh.tl[LTL_SEG] += t_c - t_b;
                }
                const unsigned long long upto = ((2ull << lane) - 1ull) & ~1ull;   // bits 1..lane
                for (int k0 = 64 * wave; k0 < total; k0 += 256) {
                    const int k = k0 + lane;
                    if (k >= total) continue;
                    const unsigned long long wb = sh.bits[k0 >> 6];
                    const int o = (int)sh.wown[k0 >> 6] + __popcll(wb & upto);
                    const uint32_t sgi = sh.seg[o];
                    const int lx = (int)((sgi >> 16) & 31u) + (k - (int)(sgi & 0xffffu)), ly = (int)((sgi >> 21) & 7u);
                    const int slot = (int)(sgi >> 24);
                    const int kp = ly * LIB_RTW + lx;
                    // per-pixel hierarchical z: the pixel's current key already beats the primitive's
                    // depth bound (a stale, higher key only skips less)
                    if (sh.zord[slot] > keyhi[2 * kp + 1]) continue;
                    const LibRec r = lib_rec_from(&sh.rec[slot * 4]);
                    float z01, u, v, w, idn;
                    if (lib_test<SHADOW>(fp, r, TX0 + lx, TY0 + ly, z01, u, v, w, idn))
                        atomicMin(&sh.key[kp], lib_key(fp, z01, r.seq, SHADOW));
                }
                // this wave's largest key z for the next pass (read under the other waves' atomics: stale
                // only upwards, which selects more, never less); a part counts its own pixels only
                {
                    uint32_t o = keyhi[2 * tid + 1];
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) o = max(o, (uint32_t)__shfl_xor((int)o, off));
                    if (lane == 0) sh.wmax[wave] = o;
                }
                p += LIB_CHUNK;
            }
            continue;   // the next candidate round
        }
        // (3) staging passes.  Each selects, in list order, the entries that can still win a pixel
        //     -- depth bound <= the largest current key z over the pixel columns their box covers
        //     (hierarchical z; 0xffffffff = an uncovered pixel) -- stages up to LIB_CHUNK of them and
        //     expands their (primitive, pixel) pairs.  Once the whole tile's largest key z sorts into
        //     a lower bucket than the next entry, the rest of the list is skipped.
        uint32_t p = 0;
        while (p < nc) {
            if (p > 0) __syncthreads();   // the previous pass's pairs are resolved
            uint32_t m = 0;
            if (!sorted) {   // list order, LIB_CHUNK at a time (one pass unless painter's order)
                m = min((uint32_t)LIB_CHUNK, nc - p);
                for (int i = tid; i < (int)m; i += 256) sh.sel[i] = p + (uint32_t)i;
                p += m;
                ++chunk;
                __syncthreads();
            } else {
                if (hiz) {   // per pixel column, the largest key z so far
                    uint32_t o = (uint32_t)(sh.key[tid] >> 32);
                    o = max(o, (uint32_t)__shfl_xor((int)o, 32));   // a wave holds two rows of the column
                    if (lane < LIB_RTW) atomicMax(&sh.colmax[chunk & 1u][lane], o);
                }
                __syncthreads();
                const uint32_t *colmax = sh.colmax[chunk & 1u];
                uint32_t ordmax = colmax[lane & (LIB_RTW - 1)];   // the whole tile's max (every wave alike)
#pragma unroll
                for (int off = LIB_RTW / 2; off > 0; off >>= 1) ordmax = max(ordmax, (uint32_t)__shfl_xor((int)ordmax, off));
                if (tid < LIB_RTW) sh.colmax[(chunk + 1u) & 1u][tid] = 0u;   // next pass's maxima start here
                ++chunk;
                auto done_after = [&](uint32_t q) {   // nothing from list position q on can win (uniform)
                    return hiz && ordmax != 0xffffffffu && (ordmax < s_lo || bucket(ordmax) < bucket(sh.lkey[q]));
                };
                if (done_after(p)) break;
                // select the next survivors (at most LIB_CHUNK), skipping rejected runs
                while (p < nc) {
                    const uint32_t q = p + (uint32_t)tid;
                    bool alive = false;
                    if (tid < LIB_CHUNK && q < nc) {
                        alive = true;
                        if (hiz) {
                            const uint2 b = sh.lbox[q];
                            const int x0 = max(lo16(b.x), X0) - TX0, x1 = min(hi16(b.x), X1) - TX0;
                            uint32_t cm = 0u;
                            for (int x = x0; x <= x1; ++x) cm = max(cm, colmax[x]);
                            alive = sh.lkey[q] <= cm;
                        }
                    }
                    const uint64_t am = __ballot(alive);
                    if (lane == 0) sh.wtot[wave][0] = (uint32_t)__popcll(am);
                    __syncthreads();
                    uint32_t wb = 0;
#pragma unroll
                    for (int w2 = 0; w2 < 4; ++w2) {
                        const uint32_t c2 = sh.wtot[w2][0];
                        wb += w2 < wave ? c2 : 0u;
                        m += c2;
                    }
                    if (alive) sh.sel[wb + lanes_below(am)] = q;
                    p += LIB_CHUNK;
                    __syncthreads();   // sel complete; wtot reusable
                    if (m > 0 || p >= nc || done_after(p)) break;
                }
                if (m == 0) break;
            }
            // stage the survivors' records (consecutive lanes: consecutive float4s of one record)
            for (int i = tid; i < (int)m * (LIB_RTW * LIB_RTH / 64); i += 256) sh.bits[i] = 0ull;
            {
                constexpr int NQ = LIB_CHUNK * 4 / 256;
                float4 q4[NQ];
#pragma unroll
                for (int k = 0; k < NQ; ++k) {
                    const int f = tid + 256 * k;
                    const int ci = f >> 2;
                    q4[k] = f < 4 * (int)m ? reinterpret_cast<const float4 *>(&fb.recs[sh.lid[sh.sel[min(ci, (int)m - 1)]]])[f & 3]
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
                }
#pragma unroll
                for (int k = 0; k < NQ; ++k) {
                    const int f = tid + 256 * k;
                    if (f < 4 * (int)m) sh.rec[f] = q4[k];
                }
            }
            __syncthreads();
            // Pair tasks (shallow raster and shadow pass -- the deep camera raster takes its own passes
            // above): the staged boxes laid end to end (C5: few, mostly large primitives; the span
            // arithmetic would spill the shallow raster's 80 registers, and measured 10 % slower on C5's
            // shadow map).  Every (primitive, pixel) pair is dealt to one lane, 64-pair windows
            // round-robin over the waves (start bitmap + word owners, as in shs_legacy.hip).
            {
                uint4 *pinfo = reinterpret_cast<uint4 *>(sh.seg);   // per staged box: first pair, x0 | y0 << 16, width | slot << 16, 2^16/width
                int area = 0, bx0 = 0, by0 = 0, bw = 1;
                uint32_t zord = 0u;
                if (tid < (int)m) {
                    const uint32_t q = sh.sel[tid];
                    const uint2 b = sh.lbox[q];
                    const int x0 = max(lo16(b.x), X0), x1 = min(hi16(b.x), X1);
                    const int y0 = max(lo16(b.y), Y0), y1 = min(hi16(b.y), Y1);
                    area = (x1 - x0 + 1) * (y1 - y0 + 1); bx0 = x0; by0 = y0; bw = x1 - x0 + 1;
                    zord = sh.lkey[q];
                }
                int incl = area;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int vv = __shfl_up(incl, o);
                    if (lane >= o) incl += vv;
                }
                if (lane == 63) sh.wtot[wave][1] = (uint32_t)incl;
                __syncthreads();
                uint32_t pbase = 0, ptot = 0;
#pragma unroll
                for (int w2 = 0; w2 < 4; ++w2) {
                    const uint32_t p2 = sh.wtot[w2][1];
                    if (w2 < wave) pbase += p2;
                    ptot += p2;
                }
                if (area > 0) {
                    const int start = (int)pbase + incl - area;
                    pinfo[tid] = make_uint4((uint32_t)start, (uint32_t)bx0 | ((uint32_t)by0 << 16),
                                               (uint32_t)bw | ((uint32_t)tid << 16), (65536u + (uint32_t)bw - 1u) / (uint32_t)bw);
                    sh.zord[tid] = zord;
                    atomicOr(&sh.bits[start >> 6], 1ull << (start & 63));
                    for (int wd = (start + 63) >> 6; wd * 64 < start + area; ++wd) sh.wown[wd] = (uint8_t)tid;
                }
                __syncthreads();
                const int total = (int)ptot;
                if (tlon) sh.tl[LTL_NPAIRS] += ptot;
                const unsigned long long upto = ((2ull << lane) - 1ull) & ~1ull;   // bits 1..lane
                // one pair: its owner (word's first owner + starts up to it), pixel, then the test
                auto pair = [&](int k0) {
                    const int k = k0 + lane;
                    if (k >= total) return;
                    const unsigned long long wb = sh.bits[k0 >> 6];
                    const int o = (int)sh.wown[k0 >> 6] + __popcll(wb & upto);
                    const uint4 pi = pinfo[o];
                    const int local = k - (int)pi.x, ow = (int)(pi.z & 0xffffu);
                    const int ly = (int)(((uint32_t)local * pi.w) >> 16), lx = local - ly * ow;
                    const int px = (int)(pi.y & 0xffffu) + lx, py = (int)(pi.y >> 16) + ly;
                    const int kp = (py - TY0) * LIB_RTW + (px - TX0);
                    // per-pixel hierarchical z: the pixel's current key already beats the
                    // primitive's depth bound (a stale, higher key only skips less)
                    if (sh.zord[o] > reinterpret_cast<const uint32_t *>(sh.key)[2 * kp + 1]) return;
                    const LibRec r = lib_rec_from(&sh.rec[(pi.z >> 16) * 4]);
                    float z01, u, v, w, idn;
                    if (lib_test<SHADOW>(fp, r, px, py, z01, u, v, w, idn))
                        atomicMin(&sh.key[kp], lib_key(fp, z01, r.seq, SHADOW));
                };
                for (int k0 = 64 * wave; k0 < total; k0 += 256) pair(k0);
            }
        }
    }
    __syncthreads();
    const uint64_t t_res = tlon ? tl_now() : 0ull;
    // a wave takes a 16x4 block of the tile (rows are 128-B key / 256-B HDR segments); the shadow pass
    // resolves here, the camera pass hands its keys to k_lib_resolve
    const int lx = my_lx, ly = my_ly;
    const int px = TX0 + lx, py = TY0 + ly;
    unsigned long long key = sh.key[ly * LIB_RTW + lx];
    sh.key[ly * LIB_RTW + lx] = KEY_EMPTY;   // this thread's pixel only: clean for the next tile
    bool covered = false;
    bool write = true;
    if (!SHADOW && parts > 1u) {
        // a split tile: merge this part's keys into the tile's pkeys slot; the part that finishes last
        // takes the merged keys (resetting the slot for the next pass) and writes the winners
        unsigned long long *pk = fb.pkeys + (size_t)sid * (LIB_RTH * LIB_RTW) + ly * LIB_RTW + lx;
        if (key != KEY_EMPTY) atomicMin(pk, key);
        __threadfence();
        __syncthreads();
        if (tid == 0) sh.last = atomicAdd(&fb.pcount[sid], 1u) == parts - 1u ? 1u : 0u;
        __syncthreads();
        write = sh.last != 0u;   // block-uniform
        if (write) {
            __threadfence();
            key = atomicExch(pk, KEY_EMPTY);   // (device-scope: never a stale L1 line)
            if (tid == 0) fb.pcount[sid] = 0u;
        }
    }
    if (SHADOW) {
        lib_resolve<SHADOW>(fp, fb, key, px, py, covered);
    } else if (write) {
        // keys only for 16x4 blocks holding a winner; the block's flag tells k_lib_resolve which
        // (the wave's block is sub-block `wave` of the tile, k_lib_resolve's numbering)
        covered = key != KEY_EMPTY && px < fp.W && py < fp.H;
        const bool any = __ballot(covered) != 0ull;
        if (any && px < fp.W && py < fp.H) fb.keys[(size_t)py * fp.W + px] = lib_winner_word(fp, key);
        if (lane == 0) fb.blkcov[(size_t)rt * 4 + wave] = any ? 1u : 0u;
    }
    const uint64_t cm = __ballot(covered);
    if (lane == 0 && cm) atomicAdd(&sh.cov, (uint32_t)__popcll(cm));
    if (SHADOW && tid == 0) fb.busy[rt] = 0u;   // camera pass: k_lib_resolve resets it (split tiles' parts)
    if (tlon) {
        const uint64_t t_end = tl_now();
        sh.tl[LTL_GATHER] += t_gather;
        sh.tl[LTL_PAIRS] += (t_res - t_tile) - t_gather;
        sh.tl[LTL_SHADE] += t_end - t_res;
        sh.tl[LTL_NBUSY] += 1;
        sh.tl[LTL_CHUNKS] += chunk - chunk0;
        if (t_end - t_tile > sh.tl[LTL_MAXTILE]) {   // this workgroup's longest tile so far
            sh.tl[LTL_MT_RT] = (uint64_t)rt; sh.tl[LTL_MT_ITEMS] = tl_items; sh.tl[LTL_MT_ROUNDS] = t_rounds;
            sh.tl[LTL_MT_PASSES] = chunk - chunk0; sh.tl[LTL_MT_STAGED] = sh.tl_staged; sh.tl[LTL_MT_PAIRS] = t_pairs;
            sh.tl[LTL_MT_GATHER] = t_gather; sh.tl[LTL_MT_BREAKS] = t_breaks;
        }
        sh.tl[LTL_MAXTILE] = max(sh.tl[LTL_MAXTILE], t_end - t_tile);
        sh.tl[LTL_TILES] += t_end - t_tile;
        sh.tl[LTL_LAST] = t_end;
    }
}

// A shadow-map raster tile no primitive touches: its texels get the clear depth.
__device__ __forceinline__ void lib_clear_shadow_tile(const LibFrameParams &fp, const LibBuffers &fb, int rt) {
    const int tid = threadIdx.x;
    const int col = rt % fp.tiles_x, row = rt / fp.tiles_x;
    const int px = col * LIB_RTW + (tid & 31), py = row * LIB_RTH + (tid >> 5);
    bool covered;
    lib_resolve<true>(fp, fb, KEY_EMPTY, px, py, covered);
}

// The camera pass's raster work plan, after the marks are final (one thread per owned raster tile):
// a busy tile whose candidate list holds more than fp.part entries is split into ceil(n / fp.part)
// parts (at most LIB_MAXK), part j taking list positions [j n / k, (j + 1) n / k) over the whole tile.
// Each part resolves its own candidates' keys in LDS and merges them into the tile's slot of
// fb.pkeys with 64-bit atomicMin -- min is order-free, so the merged keys are the tile's keys -- and
// the part that finishes last writes the winners.  The parts (cnt[LC_ITEMS] of them, in fb.items) are
// the first work items, rendered by any workgroups at once, then the owned tiles in order with the
// split ones skipped.  The densest tiles no longer bound a sharded rank's raster (C4 rank 3 of 8: a
// ~2,800-candidate tile took one workgroup 72-84 us of a 119-us raster).
__device__ __forceinline__ uint32_t plan_parts(const LibFrameParams &fp, const LibBuffers &fb, const uint32_t *cnt, int rt) {
    if (!fb.busy[rt]) return 1u;
    const int col = rt % fp.tiles_x, row = rt / fp.tiles_x;
    const uint32_t total = fb.tile_count[(size_t)fp.parity * fp.tiles_x * fp.tiles_y + (row / (TILE / LIB_RTH)) * fp.tiles_x + col];
    const uint32_t n = min(total, fp.bin_cap) + (total > fp.bin_cap ? min(cnt[LC_SPILL], fp.spill_cap) : 0u);
    return min((uint32_t)LIB_MAXK, (n + fp.part - 1u) / fp.part);
}

// k_lib_raster's work items: position j < n_split is k_lib_plan's part j (word 0x80000000 | j), the rest
// the owned raster tiles in rt_order (word rt | min(busy, 3) << 28, | LIB_HEAVY for a heavy camera-pass
// tile: its bin list holds >= fp.heavy_min entries).  Workgroup b takes positions b + i * G, i < S
// (static), the rest (from dyn0 = S * G on) come from LIB_NQ ticket queues, position p in queue
// (p - dyn0) % LIB_NQ.
constexpr uint32_t LIB_HEAVY = 0x40000000u;
__device__ __forceinline__ int lib_static_items(int n_work, int G, int div) { return min(max(1, n_work / (max(div, 1) * G)), LIB_MAX_STATIC); }
__device__ __forceinline__ uint32_t lib_item_word(const LibFrameParams &fp, const LibBuffers &fb, int n_split, int j) {
    if (j < n_split) return 0x80000000u | (uint32_t)j;
    const int rt = fb.rt_order[j - n_split];
    const uint32_t busy = min(fb.busy[rt], 3u);
    uint32_t w = (uint32_t)rt | (busy << 28);
    if (fp.heavy_min && busy == 1u) {
        const int bt = (rt / fp.tiles_x / (TILE / LIB_RTH)) * fp.tiles_x + rt % fp.tiles_x;
        if (fb.tile_count[(size_t)fp.parity * fp.tiles_x * fp.tiles_y + bt] >= fp.heavy_min) w |= LIB_HEAVY;
    }
    return w;
}

// Camera pass: the work items a raster ticket can hand out, compacted per queue into LibBuffers::dynq --
// the dynamic positions that have anything to render (parts, busy tiles) into the light lists, and the
// heavy tiles of every position, static ones included, into the heavy lists that the tickets serve first
// (the longest tiles start early instead of ending the pass; a static workgroup skips its heavy items).
// A ticket never lands on a tile nothing touches: each such ticket cost a workgroup an atomic and two
// dependent loads, and at the end of the pass, when only those were left, ~25 us of every workgroup's
// life.  Order inside a list: per wave (the waves' appends race), which the raster does not depend on.
__global__ __launch_bounds__(256) void k_lib_dyn(LibFrameParams fp, LibBuffers fb) {
    const uint32_t *cnt = fb.counters + fp.parity * LC_N;
    uint32_t *rq = fb.rqueue + (size_t)fp.parity * LIB_NQW * LIB_QSTRIDE;
    const int n_split = fp.part ? (int)cnt[LC_ITEMS] : 0;
    const int n_work = n_split + fp.n_owned_rt;
    const int dyn0 = lib_static_items(n_work, fp.raster_grid, fp.static_div) * fp.raster_grid;
    const int p = (int)(blockIdx.x * 256 + threadIdx.x);
    uint32_t w = 0u;
    bool keep = false, heavy = false;
    int q = 0;
    if (p < n_work && (p >= dyn0 || fp.heavy_min)) {
        w = lib_item_word(fp, fb, n_split, p);
        heavy = (w & LIB_HEAVY) != 0u;
        keep = heavy || (p >= dyn0 && ((w & 0x80000000u) || ((w >> 28) & 3u) == 1u));
        q = (p >= dyn0 ? p - dyn0 : p) & (LIB_NQ - 1);
    }
    const int lane = __lane_id();
    if (fp.hsort) {
        // a bin list k_lib_hsort sorts: longer than one candidate round, held whole in its bin (no spill),
        // listed once -- by its first busy raster row (every raster tile of an owned bin tile is owned)
        bool hs = false;
        uint32_t hbt = 0u;
        if (p >= n_split && p < n_work) {
            const int rt = fb.rt_order[p - n_split];
            if (fb.busy[rt] == 1u) {
                constexpr int RPB = TILE / LIB_RTH;
                const int col = rt % fp.tiles_x, row = rt / fp.tiles_x, r = row % RPB;
                hbt = (uint32_t)((row / RPB) * fp.tiles_x + col);
                const uint32_t n = fb.tile_count[(size_t)fp.parity * fp.tiles_x * fp.tiles_y + hbt];
                if (n > fp.hsort_min && n <= min(fp.bin_cap, (uint32_t)LIB_HSORT_MAX)) {
                    hs = true;
                    for (int k = 1; k <= r; ++k) hs = hs && fb.busy[rt - k * fp.tiles_x] == 0u;
                }
            }
        }
        wave_append(const_cast<uint32_t *>(&cnt[LC_HSORT]), fb.hsq, hs, hbt);
    }
    for (int qq = 0; qq < LIB_NQ; ++qq)
        for (int hv = 0; hv < 2; ++hv) {
            const bool me = keep && q == qq && heavy == (hv == 1);
            const uint64_t m = __ballot(me);
            if (m == 0ull) continue;   // wave-uniform
            const int lead = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0u;
            if (lane == lead) base = atomicAdd(&rq[((hv ? 2 : 1) * LIB_NQ + qq) * LIB_QSTRIDE], (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, lead);
            if (me) fb.dynq[(size_t)(2 * qq + (hv ? 0 : 1)) * fp.dyn_cap + base + lanes_below(m)] = w;
        }
}

// Camera pass: each listed bin tile's list (k_lib_dyn: more than one candidate round of entries) sorted in
// place by depth bound -- a counting sort over 256 buckets of its range, order inside a bucket free.
// k_lib_raster's rounds over such a list then run front to back over the whole list, not over each
// 1024-entry window of it: the first round sets the tile's keys from the list's true front, and a later
// round whose first entry's bucket lies beyond the tile's largest key z is not gathered at all (C4's hot
// tiles: ~5,000 entries in five rounds, each round's own front near the list's front).  The order of a
// tile's list is free: the raster resolves by (z, submission) keys.
__global__ __launch_bounds__(LIB_HSORT_T) void k_lib_hsort(LibFrameParams fp, LibBuffers fb) {
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_lo, s_hi, s_wsum[4];
    const uint32_t n_list = fb.counters[fp.parity * LC_N + LC_HSORT];
    const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t *tcount = fb.tile_count + (size_t)fp.parity * fp.tiles_x * fp.tiles_y;
    for (uint32_t li = blockIdx.x; li < n_list; li += gridDim.x) {   // block-uniform
        const uint32_t bt = fb.hsq[li];
        const uint32_t n = tcount[bt];   // (hsort_min < n <= min(bin_cap, LIB_HSORT_MAX): k_lib_dyn)
        uint4 *bin = fb.bins + (size_t)bt * fp.bin_cap;
        if (tid < 256) s_hist[tid] = 0u;
        if (tid == 0) { s_lo = 0xffffffffu; s_hi = 0u; }
        __syncthreads();
        uint4 e[LIB_HSORT_PER];
        uint32_t zlo = 0xffffffffu, zhi = 0u;
#pragma unroll
        for (int k = 0; k < LIB_HSORT_PER; ++k) {
            const uint32_t j = (uint32_t)(tid + LIB_HSORT_T * k);
            e[k] = j < n ? bin[j] : make_uint4(0u, 0u, 0u, 0u);
            if (j < n) { zlo = min(zlo, e[k].w); zhi = max(zhi, e[k].w); }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            zlo = min(zlo, (uint32_t)__shfl_xor((int)zlo, off));
            zhi = max(zhi, (uint32_t)__shfl_xor((int)zhi, off));
        }
        if (lane == 0) { atomicMin(&s_lo, zlo); atomicMax(&s_hi, zhi); }
        __syncthreads();
        const uint2 range = make_uint2(s_lo, s_hi);
        uint32_t br[LIB_HSORT_PER];   // bucket | rank in bucket << 8
#pragma unroll
        for (int k = 0; k < LIB_HSORT_PER; ++k) {
            const uint32_t j = (uint32_t)(tid + LIB_HSORT_T * k);
            br[k] = 0u;
            if (j < n) {
                const uint32_t b = hs_bucket(range, e[k].w);
                br[k] = b | (atomicAdd(&s_hist[b], 1u) << 8);
            }
        }
        __syncthreads();
        uint32_t c = 0u, incl = 0u;
        if (tid < 256) {   // exclusive prefix of the bucket counts (waves 0..3)
            c = s_hist[tid];
            incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
                if (lane >= o) incl += v;
            }
            if (lane == 63) s_wsum[wave] = incl;
        }
        __syncthreads();
        if (tid < 256) {
            uint32_t base = 0u;
            for (int w2 = 0; w2 < wave; ++w2) base += s_wsum[w2];
            s_hist[tid] = base + incl - c;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LIB_HSORT_PER; ++k) {
            const uint32_t j = (uint32_t)(tid + LIB_HSORT_T * k);
            if (j < n) bin[s_hist[br[k] & 255u] + (br[k] >> 8)] = e[k];
        }
        if (tid == 0) fb.hsr[bt] = range;
        __syncthreads();   // LDS reused by the next listed tile
    }
}

__global__ __launch_bounds__(256) void k_lib_plan(LibFrameParams fp, LibBuffers fb) {
    uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const int j = (int)(blockIdx.x * 256 + threadIdx.x);
    const int rt = j < fp.n_owned_rt ? fb.rt_order[j] : 0;
    uint32_t k = j < fp.n_owned_rt ? plan_parts(fp, fb, cnt, rt) : 1u;
    const int lane = __lane_id();
    // a pkeys slot per split tile (wave-aggregated); past fp.split_cap the tile stays whole
    const uint64_t sm = __ballot(k > 1u);
    uint32_t sid = 0u;
    if (sm) {
        const int lead = __ffsll((unsigned long long)sm) - 1;
        if (lane == lead) sid = atomicAdd(&cnt[LC_SPLITS], (uint32_t)__popcll(sm));
        sid = (uint32_t)__shfl((int)sid, lead) + lanes_below(sm);
        if (k > 1u && sid >= fp.split_cap) k = 1u;
    }
    const uint32_t kk = k > 1u ? k : 0u;
    // wave-aggregated reservation of this wave's parts
    uint32_t incl = kk;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += a;
    }
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
    uint32_t base = 0u;
    if (lane == 63 && tot) base = atomicAdd(&cnt[LC_ITEMS], tot);
    base = (uint32_t)__shfl((int)base, 63) + incl - kk;
    for (uint32_t p = 0; p < kk; ++p) fb.items[base + p] = make_uint2((uint32_t)rt, p | (k << 8) | (sid << 16));
    if (kk) fb.busy[rt] = 2u;   // split: the in-order pass skips it (k_lib_resolve resets the flag)
}

#ifndef SHS_RASTER_SHALLOW_WAVES
#define SHS_RASTER_SHALLOW_WAVES 6
#endif
#ifndef SHS_RASTER_DEEP_WAVES
#define SHS_RASTER_DEEP_WAVES 3
#endif
template <bool SHADOW, int LIB_CAND>
__global__ __launch_bounds__(256, LIB_CAND == LIB_CAND_SHALLOW ? SHS_RASTER_SHALLOW_WAVES : SHS_RASTER_DEEP_WAVES)
void k_lib_raster(LibFrameParams fp, LibBuffers fb) {
    __shared__ LibShared<LIB_CAND> sh;
    const int tid = threadIdx.x;
    const uint32_t *cnt = fb.counters + fp.parity * LC_N;
    const int G = (int)gridDim.x;
    if (tid == 0) { sh.cov = 0; sh.maxbin = 0; }
    if (tid < 2 * LIB_RTW) sh.colmax[tid / LIB_RTW][tid % LIB_RTW] = 0u;
    sh.key[tid] = KEY_EMPTY;
    uint32_t chunk = 0;   // staging passes so far (selects the colmax slot)
    if (fb.timeline && tid < LTL_STRIDE) sh.tl[tid] = tid == LTL_START ? tl_now() : 0ull;
    // Owned raster tiles: the first S * G statically interleaved (tile b + i * G, i < S), the rest
    // from LIB_NQ ticket queues (the next ticket requested while the current tile renders; an
    // exhausted queue sends the workgroup on to the others).  S covers about half of the tiles, so the
    // dense tiles that end up late in some workgroup's static list are balanced by the dynamic half;
    // one tile per ticket keeps a dense bin tile's 4 rows on different workgroups.  The static items'
    // tiles and busy flags come in one round trip at the start, so a tile nothing touches costs the
    // workgroup nothing: the camera pass has no pixel to write there (k_lib_resolve writes the clear
    // values and resets the block flags it read), the shadow pass clears its depth.
    uint32_t *rq = fb.rqueue + (size_t)fp.parity * LIB_NQW * LIB_QSTRIDE;
    // work items: the owned raster tiles, or k_lib_plan's list (split tiles' parts first)
    const int n_split = (!SHADOW && fp.part) ? (int)cnt[LC_ITEMS] : 0;
    const int n_work = n_split + fp.n_owned_rt;
    const int S = lib_static_items(n_work, G, fp.static_div);
    const int dyn0 = S * G;
    // the camera pass's dynamic items come from k_lib_dyn's per-queue lists (busy tiles and parts only)
    constexpr bool listed = !SHADOW;
    if (tid < S) {
        const int jj = (int)blockIdx.x + tid * G;
        sh.sitem[tid] = jj < n_work ? lib_item_word(fp, fb, n_split, jj) : 0xffffffffu;
    }
    if (listed && tid < 2 * LIB_NQ) sh.qlen[tid] = rq[(LIB_NQ + tid) * LIB_QSTRIDE];   // light lengths, then heavy
    __syncthreads();
    // queue q's end: its two list lengths (camera pass) or its share of the positions
    auto q_end = [&](int qq) -> int {
        return listed ? (int)(sh.qlen[LIB_NQ + qq] + sh.qlen[qq]) : (n_work - dyn0 - qq + LIB_NQ - 1) / LIB_NQ;
    };
    // ticket t of queue q (camera pass): the heavy list first, then the light one
    auto q_item = [&](int qq, int t) -> uint32_t {
        const int nh = (int)sh.qlen[LIB_NQ + qq];
        return t < nh ? fb.dynq[(size_t)(2 * qq) * fp.dyn_cap + t] : fb.dynq[(size_t)(2 * qq + 1) * fp.dyn_cap + (t - nh)];
    };
    int q = (int)(blockIdx.x & (LIB_NQ - 1)), tried = 0;
    // (dyn0 <= n_work always: every static position is a work item); the camera pass's heavy static
    // items wait in the heavy lists, so its workgroups always go on to the tickets
    const bool dynamic = listed || dyn0 < n_work;
    uint32_t tk = 0;
    for (int i = 0;; ++i) {   // block-uniform; one call site of the tile raster (its code is large)
        uint32_t w;
        if (i < S) {
            w = sh.sitem[i];
            if (w == 0xffffffffu) break;
            if (i == S - 1 && dynamic && tid == 0) tk = atomicAdd(&rq[q * LIB_QSTRIDE], 1u);   // under the last static tile
        } else {
            if (!dynamic) break;
            if (tid == 0) {
                int t = (int)tk;
                while (t >= q_end(q) && ++tried < LIB_NQ) {   // this queue is exhausted: the next one
                    q = (q + 1) & (LIB_NQ - 1);
                    t = (int)atomicAdd(&rq[q * LIB_QSTRIDE], 1u);
                }
                const bool more = t < q_end(q);
                sh.next[0] = more ? 1 : 0;
                sh.next[1] = q;
                sh.next[2] = tried;
                if (more) tk = atomicAdd(&rq[q * LIB_QSTRIDE], 1u);   // the next ticket, under this tile
                sh.next[3] = !more ? 0 : listed ? (int)q_item(q, t) : (int)lib_item_word(fp, fb, n_split, dyn0 + q + LIB_NQ * t);
            }
            __syncthreads();   // (sh.next is rewritten only after a whole tile, past many barriers)
            if (!sh.next[0]) break;
            q = sh.next[1];
            tried = sh.next[2];
            w = (uint32_t)sh.next[3];
        }
        int rt;
        uint32_t part = 0u, parts = 1u, busy = 1u, sid = 0u;
        if (w & 0x80000000u) {   // a split tile's part
            const uint2 it = fb.items[w & 0x7fffffffu];
            rt = (int)it.x;
            part = it.y & 0xffu;
            parts = (it.y >> 8) & 0xffu;
            sid = it.y >> 16;
        } else {
            rt = (int)(w & 0x0fffffffu);
            busy = (w >> 28) & 3u;
            if (!SHADOW && busy == 2u) continue;   // rendered as parts (k_lib_plan)
            if (i < S && (w & LIB_HEAVY)) continue;   // static, heavy: served first from the heavy lists
        }
        if (busy) {
            lib_raster_tile<SHADOW, LIB_CAND>(fp, fb, cnt, rt, sh, chunk, part, parts, sid);
        } else {
            const uint64_t t_c = fb.timeline && tid == 0 ? tl_now() : 0ull;
            if (SHADOW) lib_clear_shadow_tile(fp, fb, rt);
            if (fb.timeline && tid == 0) { sh.tl[LTL_CLEAR] += tl_now() - t_c; sh.tl[LTL_NCLEAR] += 1ull; }
        }
    }
    __syncthreads();
    if (tid == 0) fb.rstat[blockIdx.x] = make_uint2(sh.cov, sh.maxbin);
    if (fb.timeline && tid == 0) {
        sh.tl[LTL_END] = tl_now();
        for (int i = 0; i < LTL_STRIDE; ++i) fb.timeline[(size_t)blockIdx.x * LTL_STRIDE + i] = sh.tl[i];
    }
}

// The camera pass's resolve (rasterizer.hpp:341-419 per winner): every owned raster tile's pixels,
// their winning key from k_lib_raster re-evaluated, shaded and written; pixels without a winner get
// the clear values.  Each wave independently takes 16x4 pixel blocks (4 per raster tile, tiles in
// k_lib_raster's order, block w + i * waves): no barrier after the Forward+ lights are staged in LDS
// at the start, so the waves' dependent loads (key -> record -> draw -> shadow map) and shading
// overlap freely.  A separate kernel: the shading's register and LDS footprint stays out of the
// raster's.  With fb.tm_thr the pixel's HDR value is also tonemapped (fused PassTonemap).
#ifndef SHS_RESOLVE_WAVES_FP
#define SHS_RESOLVE_WAVES_FP 4
#endif
#ifndef SHS_RESOLVE_WAVES_PBR
#define SHS_RESOLVE_WAVES_PBR 5
#endif
#ifndef SHS_RESOLVE_WAVES_FP_SHARD
#define SHS_RESOLVE_WAVES_FP_SHARD SHS_RESOLVE_WAVES_FP
#endif
#ifndef SHS_RESOLVE_WAVES_PBR_SHARD
#define SHS_RESOLVE_WAVES_PBR_SHARD 3
#endif
// Minimum waves per SIMD: 4 for the Forward+ kernel (no spills; 5 measured +2.3 % per C4 frame), 3 for
// the mixed one, and for the PBR one two builds: WIDE at 5 waves (96 VGPRs with 24 spilled) for a whole
// frame's pass -- C5 0.350 -> 0.341 ms per frame in three A/B pairs -- and 3 waves (no spills) for a
// sharded rank's, where the 5-wave build measured +4 % per rank frame at 8 ranks and the 3-wave one -4 %
// against 4 waves (profiles/r06_resolve_waves_ab.txt).  (-DSHS_RESOLVE_WAVES_FP / _PBR / _FP_SHARD / _PBR_SHARD override:
// timing experiments; the Forward+ kernel has one build unless _FP_SHARD differs.)
template <int PROG, bool WIDE = false>
__global__ __launch_bounds__(256, PROG == 5 ? (WIDE ? SHS_RESOLVE_WAVES_FP : SHS_RESOLVE_WAVES_FP_SHARD)
                                  : PROG == 0 ? (WIDE ? SHS_RESOLVE_WAVES_PBR : SHS_RESOLVE_WAVES_PBR_SHARD) : 3)
void k_lib_resolve(LibFrameParams fp, LibBuffers fb) {
    __shared__ float tm_thr[256];
    __shared__ uint32_t wlist[PROG == 0 ? 1 : 4][128];   // per wave: its block's light list (LtWave)
    __shared__ uint32_t wflist[PROG == 0 ? 1 : 4][128];  // ... culled by the wave's world box
    __shared__ uint32_t wbox[PROG == 0 ? 1 : 4][8];      // ... and that box
    __shared__ uint32_t s_cov;                            // covered pixels of this workgroup's blocks
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_cov = 0u;
    if (fb.tm_thr) tm_thr[tid] = fb.tm_thr[tid];
    if (PROG != 0 && fb.lights && fp.n_lights <= LIB_LDS_LIGHTS) {   // Forward+ lights
        for (int i = tid; i < (int)fp.n_lights; i += 256) {
            const PLight p = plight_global(fb.lights[i]);
            lib_lds_lights[4 * i] = p.pr;
            lib_lds_lights[4 * i + 1] = p.ci;
            lib_lds_lights[4 * i + 2] = p.sa;
            lib_lds_lights[4 * i + 3] = make_float4(__uint_as_float(p.model), 0.0f, 0.0f, 0.0f);
        }
    }
    __syncthreads();
    // tiled Forward+ lists can be wave-uniform (LtWave); clustered ones depend on the pixel's depth
    const bool tiled = PROG != 0 && fb.tile_counts && (fp.lt_mode == 1u || fp.lt_mode == 2u) && fp.lt_maxp <= 128u;
    const int n_blocks = 4 * fp.n_owned_rt;
    const int bstep = 4 * (int)gridDim.x;
    // the next block's raster tile is loaded a block ahead (off the block's dependent chain of loads:
    // C4 0.614 -> 0.607, C5 0.390 -> 0.387 ms per frame)
    int rt_next = 4 * (int)blockIdx.x < n_blocks ? fb.rt_order[blockIdx.x] : 0;
    for (int blk = 4 * (int)blockIdx.x + wave; blk < n_blocks; blk += bstep) {   // wave-uniform
        const int rt = rt_next, sub = blk & 3;
        if (blk + bstep < n_blocks) rt_next = fb.rt_order[(blk + bstep) >> 2];
        const int px = (rt % fp.tiles_x) * LIB_RTW + 16 * (sub & 1) + (lane & 15);
        const int py = (rt / fp.tiles_x) * LIB_RTH + 4 * (sub >> 1) + (lane >> 4);
        const bool inb = px < fp.W && py < fp.H;
        const bool any = fb.blkcov[(size_t)rt * 4 + sub] != 0u;   // wave-uniform
        if (sub == 0 && lane == 0) fb.busy[rt] = 0u;   // the raster's busy / split flag, for the next pass
        if (any && lane == 0) fb.blkcov[(size_t)rt * 4 + sub] = 0u;   // the next pass's raster sets only its busy tiles' flags
        const unsigned long long key = lib_winner_key(fp, inb && any ? fb.keys[(size_t)py * fp.W + px] : 0u);
        LtWave lw;
#ifdef SHS_RESOLVE_NO_LTWAVE
        if (false) {
#else
        if (tiled && __ballot(key != KEY_EMPTY && inb) != 0ull) {
#endif
            const uint32_t list = lt_tile_list(fp, min(px, fp.W - 1), min(py, fp.H - 1));
            const uint32_t l0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)list);
            if (__ballot(list != l0) == 0ull) {   // every lane active here: the VGPR entries are whole
                const uint32_t cnt = min(fb.tile_counts[l0], fp.lt_maxp);
                const uint32_t *ids = fb.tile_indices + (size_t)l0 * fp.lt_maxp;
                uint32_t *wl = wlist[PROG == 0 ? 0 : wave];
                lw.list = l0;
                lw.count = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt);
                lw.ids = wl;
                if (!SHS_LIB_EXP(fp, 16u)) {   // (exp bit 4: no wave culling -- timing experiments)
                    lw.fids = wflist[PROG == 0 ? 0 : wave];
                    lw.box = wbox[PROG == 0 ? 0 : wave];
                }
                __builtin_amdgcn_wave_barrier();   // the previous block's reads of the slice are issued
                if ((uint32_t)lane < lw.count) wl[lane] = ids[lane];
                if ((uint32_t)(64 + lane) < lw.count) wl[64 + lane] = ids[64 + lane];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
        bool covered;
        const float4 c = lib_resolve<false, PROG>(fp, fb, key, px, py, covered, lw);
        const uint64_t cm = __ballot(covered);
        if (lane == 0 && cm) atomicAdd(&s_cov, (uint32_t)__popcll(cm));
        if (fb.tm_thr && inb) {   // fused PassTonemap of this pixel's HDR value
            const uint32_t rgba = tonemap_byte(c.x, fp.tm_exposure, fp.tm_inv_gamma, tm_thr) |
                                  (tonemap_byte(c.y, fp.tm_exposure, fp.tm_inv_gamma, tm_thr) << 8) |
                                  (tonemap_byte(c.z, fp.tm_exposure, fp.tm_inv_gamma, tm_thr) << 16) | (255u << 24);
            if (fb.tm_ldr) __builtin_nontemporal_store(rgba, &fb.tm_ldr[(size_t)py * fp.W + px]);
#if defined(SHS_EXP_RESOLVE_STORES) && (SHS_EXP_RESOLVE_STORES & 8)
            if (fb.tm_present && rgba == 0x12345678u) __builtin_nontemporal_store(rgba, &fb.tm_present[(size_t)(fp.H - 1 - py) * fp.W + px]);
#else
            if (fb.tm_present) __builtin_nontemporal_store(rgba, &fb.tm_present[(size_t)(fp.H - 1 - py) * fp.W + px]);
#endif
        }
    }
    __syncthreads();
    if (tid == 0 && s_cov) atomicAdd(&fb.counters[fp.parity * LC_N + LC_COVERED], s_cov);
}

}  // namespace shs_dev

namespace shs_internal {
using namespace shs_dev;

// k_lib_setup, then (camera pass) k_lib_clip over the queued triangles, then the large primitives'
// marks (k_lib_bigmark).  The queue lengths stay on the device: the later kernels'
// grids are fixed and stride or split what the counters hold.
int lib_setup_grid(int n_tris, bool listed) {
    const int span = listed ? 256 * CULL_PER : 256;
    return std::max(1, (n_tris + span - 1) / span);
}

hipError_t launch_lib_setup(const LibFrameParams &fp, const LibBuffers &fb, bool shadow, bool listed, hipStream_t s) {
    const int grid = lib_setup_grid(fp.n_tris, listed && !shadow);
    // the striding kernels' grid: 1024 workgroups, a region-sharded rank's share of them
    const int wide = (fp.count > 1 && fp.reg.on) ? std::max(128, 1024 / fp.count) : 1024;
    if (shadow) {
        hipLaunchKernelGGL(k_lib_setup<true>, dim3(grid), dim3(256), 0, s, fp, fb);
    } else {
        if (fb.blist) hipLaunchKernelGGL(k_lib_blocks, dim3((fp.setup_blocks * BLK_G + 255) / 256), dim3(256), 0, s, fp, fb);
        if (listed) {   // tile-sharded: each workgroup culls CULL_PER x 256 triangles, then sets up the kept ones
            hipLaunchKernelGGL((k_lib_setup<false, true>), dim3(grid), dim3(256), 0, s, fp, fb);
        } else {
            hipLaunchKernelGGL(k_lib_setup<false>, dim3(grid), dim3(256), 0, s, fp, fb);
        }
        // one 16-lane group per queued triangle (the queue can hold every input triangle), at most
        // 1024 workgroups striding a longer queue (a region-sharded rank queues about 1 / count of them)
        hipLaunchKernelGGL(k_lib_clip, dim3(std::max(1, std::min((fp.n_tris + 15) / 16, wide))), dim3(256), 0, s, fp, fb);
    }
    hipLaunchKernelGGL(k_lib_bigmark, dim3(wide), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}

#define SHS_RASTER_KERNEL(shadow, shallow)                                                                   \
    ((shadow) ? ((shallow) ? k_lib_raster<true, LIB_CAND_SHALLOW> : k_lib_raster<true, LIB_CAND_DEEP>)         \
              : ((shallow) ? k_lib_raster<false, LIB_CAND_SHALLOW> : k_lib_raster<false, LIB_CAND_DEEP>))

int lib_raster_resident_blocks(int device, bool shadow, bool shallow) {
    // persistent grid: every workgroup resident at once (CUs x the kernel's occupancy)
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, SHS_RASTER_KERNEL(shadow, shallow), 256, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 2;
    (void)hipGetLastError();   // a failed query must not leave a sticky error for the host's next HIP user
    return cus * per_cu;
}

// k_lib_resolve per program class: 5 (Forward+ only), 0 (PBR metallic-roughness only), -1 (any mix)
#if SHS_RESOLVE_WAVES_FP_SHARD != SHS_RESOLVE_WAVES_FP
#define SHS_RESOLVE_FP(wide) ((wide) ? k_lib_resolve<5, true> : k_lib_resolve<5>)
#else
#define SHS_RESOLVE_FP(wide) k_lib_resolve<5, true>
#endif
#define SHS_RESOLVE_KERNEL(prog, wide) \
    (prog == 5 ? SHS_RESOLVE_FP(wide) : prog == 0 ? ((wide) ? k_lib_resolve<0, true> : k_lib_resolve<0>) : k_lib_resolve<-1>)

int lib_resolve_resident_blocks(int device, int prog, bool wide) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, SHS_RESOLVE_KERNEL(prog, wide), 256, 0) != hipSuccess || per_cu <= 0)
        per_cu = 2;
    (void)hipGetLastError();
    return cus * per_cu;
}

hipError_t launch_lib_resolve(const LibFrameParams &fp, const LibBuffers &fb, int prog, bool wide, int grid, hipStream_t s) {
    hipLaunchKernelGGL(SHS_RESOLVE_KERNEL(prog, wide), dim3(std::max(grid, 1)), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}

hipError_t launch_lib_raster(const LibFrameParams &fp, const LibBuffers &fb, bool shadow, bool shallow, int grid, hipStream_t s) {
    if (!shadow && fp.part) hipLaunchKernelGGL(k_lib_plan, dim3(std::max(1, (fp.n_owned_rt + 255) / 256)), dim3(256), 0, s, fp, fb);
    if (!shadow) {   // every position could be dynamic (a grid of one workgroup); threads past the end exit
        const int64_t n_max = (int64_t)fp.n_owned_rt * (fp.part ? 1 + LIB_MAXK : 1);
        hipLaunchKernelGGL(k_lib_dyn, dim3((unsigned)std::max<int64_t>(1, (n_max + 255) / 256)), dim3(256), 0, s, fp, fb);
        // the listed bin tiles (at most one per owned bin tile), a workgroup per CU striding the list
        if (fp.hsort) hipLaunchKernelGGL(k_lib_hsort, dim3(SHS_HSORT_GRID), dim3(LIB_HSORT_T), 0, s, fp, fb);
    }
    hipLaunchKernelGGL(SHS_RASTER_KERNEL(shadow, shallow), dim3(std::max(grid, 1)), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}

}  // namespace shs_internal
