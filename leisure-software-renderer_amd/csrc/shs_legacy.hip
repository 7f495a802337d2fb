// shs_legacy.hip -- gfx950 kernels for the shs_renderer legacy triangle scan-conversion path.
//
// Replaces RendererSystem::process + draw_triangle_tile + the four legacy shader pairs
// (cpp-folders/src/hello-3d-primitives/hello_pipeline_{blinn_phong,phong,gouraud,flat}_shading.cpp).
//
// Pipeline per frame: two launches on one HIP stream, no memsets, no copies for <= 6 draws.
//   k_setup   one thread per triangle: VS x3 (mvp), clip_to_screen, area/denominator culls, the
//             per-triangle half of barycentric_coordinate, a 96-B raster record, and the triangle
//             id appended straight into the per-tile bins its bin box touches (unordered; a spill
//             list past the bin capacity).
//   k_raster  one 256-thread workgroup per 32x32 tile (8x8 blocks, a column of four per wave):
//             stage the tile's records in LDS, resolve every pixel to the lexicographic minimum
//             (z, submission index) -- identical to the reference's in-order strict-less z test
//             (the first triangle with the minimal z wins) -- then shade only the winners from the
//             per-triangle varyings k_setup wrote, and write colour (canvas rows) and depth (screen
//             rows) once, with the clear fused (empty tiles take a clear-only fast path).
// The z-buffer never round-trips through HBM: HBM sees each input once and each output once.
//
// Tile-clamp semantics.  draw_triangle_tile clamps a triangle's bbox to the 80x80 tile job that
// runs it (blinn_phong_shading.cpp:208-224), so the reference also tests pixels OUTSIDE the
// triangle's bbox (the clamped edge rows/columns/corners of every other tile).  Such a pixel is
// >= 0.49 px outside the bbox, so an exact barycentric is <= -(distance)/(2*extent); k_setup
// bounds barycentric_coordinate's float error (an affine function of the distance) and proves
// those pixels rejected, except inside a small "danger box" around slivers (TRI_GHOST): k_raster
// then evaluates the reference's exact visited set there.  DESIGN.md has the derivation.
#include <float.h>

#include "shs_device.hpp"
#include "shs_internal.hpp"

namespace shs_dev {

// ---- k_setup --------------------------------------------------------------------------------

// Forward error bound of barycentric_coordinate (u, v, w) at a pixel whose centre lies rx / ry px
// outside the triangle's float bbox: E = e0 + ex*rx + ey*ry (u = 2^-24; dot products carry 2u,
// the two-product differences 6u, the divide and 1-v-w a few u more; 25 % slack).  Such a pixel
// has min exact barycentric <= -max(rx/(2Wx), ry/(2Wy)), so it is provably rejected when
// E < max(...), i.e. outside the box expanded by 2*W*m0, m0 = e0 / (1 - 2(ex*Wx + ey*Wy)).
// Returns the expansion (dgx, dgy) >= 0, or (-1, -1) if no bound exists (then every visited pixel
// is tested).
__device__ __forceinline__ double2 danger_margin(const TriRec &r) {
    const double2 none = make_double2(-1.0, -1.0);
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double a = fabs((double)r.v0x), b = fabs((double)r.v0y);
    const double c = fabs((double)r.v1x), d = fabs((double)r.v1y);
    const double Wx = (double)r.fmaxx - (double)r.fminx, Wy = (double)r.fmaxy - (double)r.fminy;
    if (!(Wx > 0.0) || !(Wy > 0.0)) return none;
    const double A00 = a * a + b * b, A11 = c * c + d * d, A01 = a * c + b * d;
    const double Dabs = fabs((double)r.denom);
    const double ED = 6.1 * u * (A00 * A11 + A01 * A01);
    const double Dlow = Dabs - ED;
    if (!(Dlow > 0.0) || !(Dabs < 1e300)) return none;
    const double K1 = 7.2 * u + ED / Dlow;
    const double p0 = Wx + 0.01, q0 = Wy + 0.01;
    const double A20 = p0 * a + q0 * b, A21 = p0 * c + q0 * d;
    const double Nv0 = A11 * A20 + A01 * A21, Nvx = A11 * a + A01 * c, Nvy = A11 * b + A01 * d;
    const double Nw0 = A00 * A21 + A01 * A20, Nwx = A00 * c + A01 * a, Nwy = A00 * d + A01 * b;
    const double s = K1 / Dabs * (2.0 + 2.0 * u);
    const double e0 = 1.25 * ((Nv0 + Nw0) * s + u * (2.0 + (2.0 * Nv0 + Nw0) / Dlow));
    const double ex = 1.25 * ((Nvx + Nwx) * s + u * (2.0 * Nvx + Nwx) / Dlow);
    const double ey = 1.25 * ((Nvy + Nwy) * s + u * (2.0 * Nvy + Nwy) / Dlow);
    const double S = ex * Wx + ey * Wy;
    if (!(S < 0.5)) return none;
    const double m0 = e0 / (1.0 - 2.0 * S);
    const double dgx = 2.0 * Wx * m0, dgy = 2.0 * Wy * m0;
    return (dgx < 1e6 && dgy < 1e6) ? make_double2(dgx, dgy) : none;
}

__device__ __forceinline__ bool finitef(float x) { return fabsf(x) <= FLT_MAX; }

__device__ __forceinline__ const DrawGPU *draw_table(const FrameParams &fp, const FrameBuffers &fb, const KArgDraws &ka) {
    return fp.n_draws <= KARG_DRAWS ? ka.d : fb.draws;
}

// floor of a finite float, clamped into [lo, hi] before the conversion
__device__ __forceinline__ int floor_clamped(float x, int lo, int hi) {
    return (int)fminf(fmaxf(floorf(x), (float)lo), (float)hi);
}

__device__ __forceinline__ TriRec rec_from(const float4 *s) {
    TriRec r;
    float4 *d = reinterpret_cast<float4 *>(&r);
#pragma unroll
    for (int j = 0; j < 6; ++j) d[j] = s[j];
    return r;
}

__device__ __forceinline__ int find_draw(const DrawGPU *draws, int n_draws, int gid) {
    int lo = 0, hi = n_draws - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (draws[mid].tri_base <= gid) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Per-triangle setup of draw_triangle_tile: VS position (mvp * vec4(p,1)), Canvas::clip_to_screen
// (shs_renderer.hpp:823-831), the area cull (blinn_phong_shading.cpp:219-220), the per-triangle
// half of barycentric_coordinate, the integer bbox and the bin box (flags/boxes as in TriRec).
__device__ __forceinline__ TriRec make_rec(const FrameParams &fp, const DrawGPU &dr, int draw, int local) {
    const float *p = dr.pos + 9 * (size_t)local;
    float sx[3], sy[3], sz[3];
    const float fw = (float)(fp.W - 1), fh = (float)(fp.H - 1);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float cx, cy, cz, cw;
        m4p(dr.mvp, p[3 * k + 0], p[3 * k + 1], p[3 * k + 2], cx, cy, cz, cw);
        const float nx = cx / cw, ny = cy / cw, nz = cz / cw;
        sx[k] = (nx + 1.0f) * 0.5f * fw;
        sy[k] = (1.0f - ny) * 0.5f * fh;
        sz[k] = nz;
    }
    TriRec r;
    r.ax = sx[0]; r.ay = sy[0];
    r.v0x = sx[1] - sx[0]; r.v0y = sy[1] - sy[0];
    r.v1x = sx[2] - sx[0]; r.v1y = sy[2] - sy[0];
    {
        const float a = r.v0x * r.v0x, b = r.v0y * r.v0y; r.d00 = a + b;
        const float c = r.v0x * r.v1x, d = r.v0y * r.v1y; r.d01 = c + d;
        const float e = r.v1x * r.v1x, f = r.v1y * r.v1y; r.d11 = e + f;
    }
    r.denom = r.d00 * r.d11 - r.d01 * r.d01;
    r.z0 = sz[0]; r.z1 = sz[1]; r.z2 = sz[2];
    r.draw = draw;
    r.local = local;
    r.fminx = g_min(g_min(sx[0], sx[1]), sx[2]);
    r.fmaxx = g_max(g_max(sx[0], sx[1]), sx[2]);
    r.fminy = g_min(g_min(sy[0], sy[1]), sy[2]);
    r.fmaxy = g_max(g_max(sy[0], sy[1]), sy[2]);

    uint32_t flags = 0;
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) finite = finite && finitef(sx[k]) && finitef(sy[k]);
    const float area = (sx[1] - sx[0]) * (sy[2] - sy[0]) - (sy[1] - sy[0]) * (sx[2] - sx[0]);
    // A non-finite corner makes denom NaN for every pixel (no write); |denom| < 1e-5 (a double
    // compare, shs_renderer.hpp:816) returns bc = -1 everywhere.
    if (!finite || area <= 0.0f || !((double)fabsf(r.denom) >= 1e-5)) flags |= TRI_CULLED;

    int ix0 = 0, ix1 = -1, iy0 = 0, iy1 = -1;     // integer bbox (empty by default)
    int gx0 = 0, gx1 = -1, gy0 = 0, gy1 = -1;     // bin box
    if (!(flags & TRI_CULLED)) {
        ix0 = floor_clamped(r.fminx, 0, fp.W);
        ix1 = floor_clamped(r.fmaxx, -1, fp.W - 1);
        iy0 = floor_clamped(r.fminy, 0, fp.H);
        iy1 = floor_clamped(r.fmaxy, -1, fp.H - 1);
        // Straight-line selects after the bound: ROCm 7.2 hipcc mis-allocated a value kept live
        // across danger_margin() on a divergent path when this was an if / else-if chain (found by
        // test_config_blinn_phong[c1]); keep this region free of values live across branches.
        const bool dfin = finitef(r.d00) && finitef(r.d01) && finitef(r.d11) && finitef(r.denom);
        const double2 dg = dfin ? danger_margin(r) : make_double2(-1.0, -1.0);
        const bool unbounded = !(dg.x >= 0.0);
        const bool ghost = unbounded || dg.x >= 0.49 || dg.y >= 0.49;
        // expansion of the bin box beyond the float bbox: 0 (the ibox) or the danger margin + 1 px;
        // unbounded slivers keep their ibox here and k_setup's ghost waves cover the rest
        const double exx = (ghost && !unbounded) ? dg.x + 1.0 : 0.0;
        const double exy = (ghost && !unbounded) ? dg.y + 1.0 : 0.0;
        gx0 = floor_clamped((float)((double)r.fminx - exx), 0, fp.W);
        gx1 = floor_clamped((float)((double)r.fmaxx + exx), -1, fp.W - 1);
        gy0 = floor_clamped((float)((double)r.fminy - exy), 0, fp.H);
        gy1 = floor_clamped((float)((double)r.fmaxy + exy), -1, fp.H - 1);
        flags |= (ghost ? TRI_GHOST : 0u) | (unbounded ? TRI_UNBOUNDED : 0u);
    }
    r.flags = flags;
    r.ibx = pack16(ix0, ix1); r.iby = pack16(iy0, iy1);
    r.gbx = pack16(gx0, gx1); r.gby = pack16(gy0, gy1);
    return r;
}

// Ghost waves: the pixels the reference's tile clamp makes an unbounded sliver visit OUTSIDE its
// integer bbox (blinn_phong_shading.cpp:208-224: per 80x80 tile job, the bbox clamped to the tile).
// One wave per GHOST_GROUP triangles recomputes their records (make_rec is deterministic); for each
// unbounded sliver the wave enumerates those pixels lane-parallel (per reference tile: a corner
// pixel, or a row / column segment) and appends every pixel whose barycentrics pass as a fragment.
constexpr int GHOST_GROUP = 32;

// LDS hand-off between lanes of ONE wave: the wave's LDS operations execute in order, so only the
// compiler must be kept from reordering (no s_barrier: the four waves of a ghost block diverge).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct GhostScratch {          // per-wave LDS
    float4 rec[6];
    int pref[64], w[64], x0[64], y0[64];
};

__device__ __forceinline__ void ghost_wave(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *draws,
                                           uint32_t *cnt, int group, int slice, GhostScratch &gs) {
    const int lane = threadIdx.x & 63;
    const int gid = group * GHOST_GROUP + lane;
    TriRec r;
    bool unb = false;
    if (lane < GHOST_GROUP && gid < fp.n_tris) {
        const int d = find_draw(draws, fp.n_draws, gid);
        r = make_rec(fp, draws[d], d, gid - draws[d].tri_base);
        unb = (r.flags & TRI_UNBOUNDED) != 0;
    }
    uint64_t todo = __ballot(unb);
    const int n_rt = fp.rt_x * fp.rt_y;
    while (todo) {
        const int src = __ffsll((unsigned long long)todo) - 1;
        todo &= todo - 1;
        if (lane == src) {
            const float4 *q = reinterpret_cast<const float4 *>(&r);
#pragma unroll
            for (int j = 0; j < 6; ++j) gs.rec[j] = q[j];
        }
        wave_lds_sync();
        const TriRec t = rec_from(gs.rec);
        const uint32_t tri = (uint32_t)(group * GHOST_GROUP + src);
        const int ix0 = lo16(t.ibx), ix1 = hi16(t.ibx), iy0 = lo16(t.iby), iy1 = hi16(t.iby);
        for (int rb = 0; rb < n_rt; rb += 64) {
            // lane -> reference tile rb + lane: its clamped visited rectangle and pixel count
            const int rt = rb + lane;
            int lx0 = 0, ly0 = 0, w = 1, npx = 0;
            if (rt < n_rt) {
                const int rx = rt % fp.rt_x, ry = rt / fp.rt_x;
                const float tminx = (float)(rx * fp.rtw), tmaxx = (float)(min(rx * fp.rtw + fp.rtw, fp.W) - 1);
                const float tminy = (float)(ry * fp.rth), tmaxy = (float)(min(ry * fp.rth + fp.rth, fp.H) - 1);
                const float bminx = g_max(tminx, g_min(tmaxx, t.fminx)), bmaxx = g_min(tmaxx, g_max(tminx, t.fmaxx));
                const float bminy = g_max(tminy, g_min(tmaxy, t.fminy)), bmaxy = g_min(tmaxy, g_max(tminy, t.fmaxy));
                if (!(bminx > bmaxx || bminy > bmaxy)) {
                    lx0 = (int)bminx; ly0 = (int)bminy;
                    const int lx1 = (int)bmaxx, ly1 = (int)bmaxy;
                    const bool inside = lx0 >= ix0 && lx1 <= ix1 && ly0 >= iy0 && ly1 <= iy1;
                    w = lx1 - lx0 + 1;
                    npx = inside ? 0 : w * (ly1 - ly0 + 1);
                }
            }
            // wave-inclusive prefix of the pixel counts (all lanes active here)
            int incl = npx;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const int total = __shfl(incl, 63);
            gs.pref[lane] = incl;
            gs.w[lane] = w;
            gs.x0[lane] = lx0;
            gs.y0[lane] = ly0;
            wave_lds_sync();
            // this wave's slice of the pixel index space (fp.ghost_slices waves share each group)
            for (int k = slice * 64 + lane; k < total; k += 64 * (int)fp.ghost_slices) {
                int lo = 0, hi = 63;                         // owner: first lane with pref > k
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (gs.pref[mid] > k) hi = mid; else lo = mid + 1;
                }
                const int off = k - (lo ? gs.pref[lo - 1] : 0);
                const int wq = gs.w[lo];
                const int px = gs.x0[lo] + off % wq, py = gs.y0[lo] + off / wq;
                if (px >= ix0 && px <= ix1 && py >= iy0 && py <= iy1) continue;   // k_raster's part
                const int tl = (py / TILE) * fp.tiles_x + px / TILE;
                if (tl % fp.count != fp.rank) continue;
                float u, v, ww;
                bary(t, (float)px + 0.5f, (float)py + 0.5f, u, v, ww);
                if (u < 0 || v < 0 || ww < 0) continue;
                const float z = (u * t.z0 + v * t.z1) + ww * t.z2;
                if (!(z < FLT_MAX)) continue;   // NaN / FLT_MAX never pass the strict z test
                const uint32_t slot = atomicAdd(&cnt[C_FRAG], 1u);
                if (slot < fp.frag_cap) {
                    GhostFrag g;
                    g.xy = (uint32_t)px | ((uint32_t)py << 16);
                    g.z = z;
                    g.id = tri;
                    g.v = v;
                    g.w = ww;
                    g.pad[0] = g.pad[1] = g.pad[2] = 0u;
                    fb.frags[slot] = g;
                } else {
                    atomicOr(&cnt[C_OVERFLOW], OV_FRAG);
                }
            }
            wave_lds_sync();   // the next reference-tile batch overwrites gs
        }
    }
}

__global__ __launch_bounds__(256) void k_setup(FrameParams fp, FrameBuffers fb, KArgDraws ka) {
    __shared__ GhostScratch s_ghost[4];
    uint32_t *cnt = fb.counters + fp.parity * C_NCOUNTERS;
    const DrawGPU *draws = draw_table(fp, fb, ka);
    const int setup_blocks = (fp.n_tris + 255) / 256;
    // zero the other parity set for the next frame (block 0 exists even for an empty frame)
    if (blockIdx.x == 0 && threadIdx.x < C_NCOUNTERS) fb.counters[(fp.parity ^ 1u) * C_NCOUNTERS + threadIdx.x] = 0u;
    if ((int)blockIdx.x >= setup_blocks) {
        const int wave = threadIdx.x >> 6;
        const int gw = ((int)blockIdx.x - setup_blocks) * 4 + wave;
        const int n_groups = (fp.n_tris + GHOST_GROUP - 1) / GHOST_GROUP;
        if (gw < n_groups * (int)fp.ghost_slices && !(fp.flags & DBG_SKIP_GHOST))
            ghost_wave(fp, fb, draws, cnt, gw / (int)fp.ghost_slices, gw % (int)fp.ghost_slices, s_ghost[wave]);
        return;
    }
    const int gid = blockIdx.x * 256 + threadIdx.x;
    if (gid >= fp.n_tris) return;
    const int lo = find_draw(draws, fp.n_draws, gid);
    const DrawGPU &dr = draws[lo];
    const int local = gid - dr.tri_base;
    const float *p = dr.pos + 9 * (size_t)local;
    TriRec r = make_rec(fp, dr, lo, local);
    const uint32_t flags = r.flags;
    {
        const float4 *src = reinterpret_cast<const float4 *>(&r);
        float4 *dst = reinterpret_cast<float4 *>(&fb.recs[gid]);
#pragma unroll
        for (int j = 0; j < 6; ++j) dst[j] = src[j];
    }
    fb.boxes[gid] = make_uint2(r.gbx, r.gby);   // culled: the empty box (0, -1)
    const int gx0 = lo16(r.gbx), gx1 = hi16(r.gbx), gy0 = lo16(r.gby), gy1 = hi16(r.gby);
    if (flags & TRI_CULLED) return;

    // Shading varyings of the three corners (the VS outputs the FS interpolates), computed once per
    // triangle instead of once per winning pixel.
    {
        ShadeRec sr;
        sr.shading = dr.shading;
        sr.draw = lo;
        const float *N = dr.nrm + 9 * (size_t)local;
        if (dr.shading == 0) {
            // Flat VS (flat_shading.cpp:54): normal = mat3(mv) * n
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const f3 n = m3v(dr.nmat, f3{N[3 * k], N[3 * k + 1], N[3 * k + 2]});
                sr.v[3 * k] = n.x; sr.v[3 * k + 1] = n.y; sr.v[3 * k + 2] = n.z;
            }
        } else {
            const f3 L = {dr.light[0], dr.light[1], dr.light[2]};
            const f3 cam = {dr.cam[0], dr.cam[1], dr.cam[2]};
            const f3 oc = {dr.ocol[0], dr.ocol[1], dr.ocol[2]};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                float x, y, z, ww;
                m4p(dr.model, p[3 * k], p[3 * k + 1], p[3 * k + 2], x, y, z, ww);
                const f3 wp = {x, y, z};
                const f3 nr = normalize3(m3v(dr.nmat, f3{N[3 * k], N[3 * k + 1], N[3 * k + 2]}));
                if (dr.shading == 1) {
                    // Gouraud VS (gouraud_shading.cpp:46-77): Blinn-Phong per vertex, shininess 32
                    const f3 viewDir = normalize3(sub3(cam, wp));
                    const float diff = g_max(dot3(nr, L), 0.0f);
                    const f3 half = normalize3(add3(L, viewDir));
                    const float spec = (float)pow((double)g_max(dot3(nr, half), 0.0f), 32.0);
                    const float sum = (0.15f + diff * 1.0f) + (0.5f * spec) * 1.0f;
                    sr.v[3 * k] = g_clamp01(sum * oc.x);
                    sr.v[3 * k + 1] = g_clamp01(sum * oc.y);
                    sr.v[3 * k + 2] = g_clamp01(sum * oc.z);
                } else {
                    // Phong / Blinn-Phong VS (blinn_phong_shading.cpp:48-57)
                    sr.v[3 * k] = wp.x; sr.v[3 * k + 1] = wp.y; sr.v[3 * k + 2] = wp.z;
                    sr.v[9 + 3 * k] = nr.x; sr.v[9 + 3 * k + 1] = nr.y; sr.v[9 + 3 * k + 2] = nr.z;
                }
            }
        }
        const float4 *src = reinterpret_cast<const float4 *>(&sr);
        float4 *dst = reinterpret_cast<float4 *>(&fb.shade[gid]);
#pragma unroll
        for (int j = 0; j < 5; ++j) dst[j] = src[j];
    }

    atomicAdd(&cnt[C_SETUP], 1u);
    if (flags & TRI_GHOST) atomicAdd(&cnt[C_GHOST], 1u);
    if (flags & TRI_UNBOUNDED) atomicAdd(&cnt[C_UNBOUNDED], 1u);
    if (fp.scan_mode) return;   // small scene: k_raster scans the bin boxes; no bins
    if (gx0 > gx1 || gy0 > gy1 || (fp.flags & DBG_SKIP_BIN)) return;
    const int tx0 = gx0 / TILE, tx1 = gx1 / TILE, ty0 = gy0 / TILE, ty1 = gy1 / TILE;
    const int ntx = tx1 - tx0 + 1, nty = ty1 - ty0 + 1;
    if (ntx * nty <= 4) {
        // common case: issue every bin append before consuming any position (one round trip)
        int t[4];
        uint32_t pos[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int kx = tx0 + (k % ntx), ky = ty0 + (k / ntx);
            t[k] = (k < ntx * nty) ? ky * fp.tiles_x + kx : -1;
            if (t[k] >= 0 && t[k] % fp.count != fp.rank) t[k] = -1;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) pos[k] = t[k] >= 0 ? atomicAdd(&fb.tile_count[t[k]], 1u) : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (t[k] < 0) continue;
            if (pos[k] < fp.bin_cap) {
                fb.bins[(size_t)t[k] * fp.bin_cap + pos[k]] = (uint32_t)gid;
            } else {
                const uint32_t sp = atomicAdd(&cnt[C_SPILL], 1u);
                if (sp < fp.spill_cap) fb.spill[sp] = make_uint2((uint32_t)t[k], (uint32_t)gid);
                else atomicOr(&cnt[C_OVERFLOW], OV_SPILL);
            }
        }
        return;
    }
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            const int t = ty * fp.tiles_x + tx;
            if (t % fp.count != fp.rank) continue;
            const uint32_t pos = atomicAdd(&fb.tile_count[t], 1u);
            if (pos < fp.bin_cap) {
                fb.bins[(size_t)t * fp.bin_cap + pos] = (uint32_t)gid;
            } else {
                const uint32_t sp = atomicAdd(&cnt[C_SPILL], 1u);
                if (sp < fp.spill_cap) fb.spill[sp] = make_uint2((uint32_t)t, (uint32_t)gid);
                else atomicOr(&cnt[C_OVERFLOW], OV_SPILL);
            }
        }
}

// ---- k_raster -------------------------------------------------------------------------------


// Fragment shaders of the four legacy pipelines for the winning triangle, from its per-corner
// varyings.  Returns the pre-truncation floats; the caller truncates to uint8 like the reference.
__device__ __forceinline__ void shade_winner(const DrawGPU &dr, const ShadeRec &sr, float u, float v, float w, float pre[3]) {
    const f3 a0 = {sr.v[0], sr.v[1], sr.v[2]}, a1 = {sr.v[3], sr.v[4], sr.v[5]}, a2 = {sr.v[6], sr.v[7], sr.v[8]};
    if (sr.shading == 0) {
        // Flat FS (flat_shading.cpp:69-98): the interpolated normal is normalised in
        // draw_triangle_tile and again in the FS; intensity = min(0.2 + max(n.l, 0), 1)
        const f3 in_n = normalize3(add3(add3(sc3(a0, u), sc3(a1, v)), sc3(a2, w)));
        const f3 nn = normalize3(in_n);
        const f3 l = {dr.light[0], dr.light[1], dr.light[2]};
        const float diffuse = g_max(dot3(nn, l), 0.0f);
        float intensity = 0.2f + diffuse;
        if (intensity > 1.0f) intensity = 1.0f;
        pre[0] = dr.colf[0] * intensity;
        pre[1] = dr.colf[1] * intensity;
        pre[2] = dr.colf[2] * intensity;
        return;
    }
    if (sr.shading == 1) {
        // Gouraud FS (gouraud_shading.cpp:80-89): interpolated colour * 255
        const f3 c = add3(add3(sc3(a0, u), sc3(a1, v)), sc3(a2, w));
        pre[0] = c.x * 255.0f;
        pre[1] = c.y * 255.0f;
        pre[2] = c.z * 255.0f;
        return;
    }
    // Phong / Blinn-Phong: normal and world position interpolated (blinn_phong_shading.cpp:235-236)
    const f3 n0 = {sr.v[9], sr.v[10], sr.v[11]}, n1 = {sr.v[12], sr.v[13], sr.v[14]}, n2 = {sr.v[15], sr.v[16], sr.v[17]};
    const f3 in_n = normalize3(add3(add3(sc3(n0, u), sc3(n1, v)), sc3(n2, w)));
    const f3 in_w = add3(add3(sc3(a0, u), sc3(a1, v)), sc3(a2, w));
    const f3 L = {dr.light[0], dr.light[1], dr.light[2]};
    const f3 cam = {dr.cam[0], dr.cam[1], dr.cam[2]};
    const f3 norm = normalize3(in_n);
    const f3 viewDir = normalize3(sub3(cam, in_w));
    const float diff = g_max(dot3(norm, L), 0.0f);
    float specular;
    if (sr.shading == 2) {
        // Phong (phong_shading.cpp:70-108): reflect(-L, N) = I - N*dot(N,I)*2, spec 0.8,
        // pow(float, int 32) resolves to std::pow(double, double)
        const f3 I = {-L.x, -L.y, -L.z};
        const float dn = dot3(norm, I);
        const f3 t = sc3(sc3(norm, dn), 2.0f);
        const f3 refl = sub3(I, t);
        const float spec = (float)pow((double)g_max(dot3(viewDir, refl), 0.0f), 32.0);
        specular = (0.8f * spec) * 1.0f;
    } else {
        // Blinn-Phong (blinn_phong_shading.cpp:63-97): powf(max(N.H,0), 64), spec 0.5
        const f3 half = normalize3(add3(L, viewDir));
        const float spec = (float)pow((double)g_max(dot3(norm, half), 0.0f), 64.0);
        specular = (0.5f * spec) * 1.0f;
    }
    const f3 oc = {dr.ocol[0], dr.ocol[1], dr.ocol[2]};
    const float s = (0.15f + diff * 1.0f) + specular;
    pre[0] = g_clamp01(s * oc.x) * 255.0f;
    pre[1] = g_clamp01(s * oc.y) * 255.0f;
    pre[2] = g_clamp01(s * oc.z) * 255.0f;
}

// Per-pixel winner state: depth, submission index and the winner's (v, w) (u is recomputed
// exactly as (1 - v) - w, shs_renderer.hpp:819).
struct Best {
    float z;
    uint32_t id;
    float v, w;
};

__device__ __forceinline__ void resolve(float z, uint32_t id, float v, float w, Best &b) {
    // In-order strict-less z test == lexicographic min of (z, submission index); NaN never wins,
    // z == FLT_MAX never beats the FLT_MAX clear (id sentinel 0 makes id < b.id false).
    if (z < b.z || (z == b.z && id < b.id)) { b.z = z; b.id = id; b.v = v; b.w = w; }
}

// One triangle against one pixel.  ibox pixels are always in the reference's visited set; outside
// it only ghost triangles can pass, and only where the tile clamp visits the pixel.
__device__ __forceinline__ void raster_px(int px, int py, float rtminx, float rtmaxx, float rtminy, float rtmaxy,
                                          const TriRec &r, uint32_t id, Best &b) {
    const bool in_ibox = px >= lo16(r.ibx) && px <= hi16(r.ibx) && py >= lo16(r.iby) && py <= hi16(r.iby);
    bool test = in_ibox;
    if (r.flags & TRI_GHOST) {
        const bool in_gbox = px >= lo16(r.gbx) && px <= hi16(r.gbx) && py >= lo16(r.gby) && py <= hi16(r.gby);
        if (!in_ibox && in_gbox) {
            // draw_triangle_tile's visited rectangle in this pixel's tile job (blinn_phong_shading.cpp:208-224)
            const float bminx = g_max(rtminx, g_min(rtmaxx, r.fminx));
            const float bmaxx = g_min(rtmaxx, g_max(rtminx, r.fmaxx));
            const float bminy = g_max(rtminy, g_min(rtmaxy, r.fminy));
            const float bmaxy = g_min(rtmaxy, g_max(rtminy, r.fmaxy));
            test = !(bminx > bmaxx || bminy > bmaxy) && px >= (int)bminx && px <= (int)bmaxx && py >= (int)bminy &&
                   py <= (int)bmaxy;
        }
    }
    if (test) {
        float u, v, w;
        bary(r, (float)px + 0.5f, (float)py + 0.5f, u, v, w);
        if (!(u < 0 || v < 0 || w < 0)) {
            const float z = (u * r.z0 + v * r.z1) + w * r.z2;
            resolve(z, id, v, w, b);
        }
    }
}

// Speed-only XCD grouping: blocks b and b+8 (dealt to the same XCD) render horizontally adjacent
// tiles, so neighbouring row segments are written through one L2.
__device__ __forceinline__ int tile_of_block(int b, int n_owned) {
    const int g = b >> 4;
    if ((g << 4) + 16 > n_owned) return b;          // ragged last group: identity
    return (g << 4) + ((b & 7) << 1) + ((b >> 3) & 1);
}

constexpr int NB = TILE / 8;   // 8x8 blocks per tile edge (4): wave w owns block column w

__global__ __launch_bounds__(256) void k_raster(FrameParams fp, FrameBuffers fb, KArgDraws ka) {
    __shared__ float4 s_rec[CHUNK * 6];
    __shared__ uint32_t s_id[CHUNK];
    __shared__ uint32_t s_cand[CAND];
    __shared__ float s_bz[TILE * TILE];
    __shared__ uint32_t s_bid[TILE * TILE];
    __shared__ uint32_t s_cov, s_nc;
    float *s_bv = reinterpret_cast<float *>(s_rec);    // reused once the raster passes are done
    float *s_bw = s_bv + TILE * TILE;

    const int n_owned = (fp.tiles_x * fp.tiles_y - fp.rank + fp.count - 1) / fp.count;
    const int tile = fp.rank + tile_of_block((int)blockIdx.x, n_owned) * fp.count;
    const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
    const int X0 = tx * TILE, Y0 = ty * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *cnt = fb.counters + fp.parity * C_NCOUNTERS;
    const DrawGPU *draws = draw_table(fp, fb, ka);
    if (tid == 0) s_cov = 0;

    // candidate sources.  scan mode: every triangle's bin box.  bin mode: the tile's bin, then the
    // spill list (entries of this tile).
    uint32_t n_bin_total = 0, n_bin = 0, n_spill = 0, n_items;
    if (fp.scan_mode) {
        n_items = (uint32_t)fp.n_tris;
    } else {
        n_bin_total = fb.tile_count[tile];
        n_bin = n_bin_total < fp.bin_cap ? n_bin_total : fp.bin_cap;
        if (n_bin_total > fp.bin_cap) n_spill = min(cnt[C_SPILL], fp.spill_cap);
        n_items = n_bin + n_spill;
    }
    if (fp.flags & DBG_CLEAR_ONLY) n_items = 0;
    const uint32_t *bin = fb.bins + (size_t)tile * fp.bin_cap;
    const int tx1 = X0 + TILE - 1, ty1 = Y0 + TILE - 1;

    // raster mapping: wave w owns the 8-px column of blocks (w, 0..3); lane -> (lane&7, lane>>3)
    const int px = X0 + wave * 8 + (lane & 7);
    const int py0 = Y0 + (lane >> 3);
    const int rxs = (px / fp.rtw) * fp.rtw;
    const float rtminx = (float)rxs, rtmaxx = (float)(min(rxs + fp.rtw, fp.W) - 1);
    const int bxl = X0 + wave * 8;
    Best best[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) { best[i].z = FLT_MAX; best[i].id = 0u; best[i].v = 0.f; best[i].w = 0.f; }

    for (uint32_t base = 0; base < n_items; base += CAND) {
        __syncthreads();
        if (tid == 0) s_nc = 0;
        __syncthreads();
        // gather up to CAND candidate ids (4 independent loads per thread, one round trip)
#pragma unroll
        for (int k = 0; k < CAND / 256; ++k) {
            const uint32_t item = base + tid + 256u * k;
            if (item >= n_items) continue;
            uint32_t id = 0xffffffffu;
            if (fp.scan_mode) {
                const uint2 bx = fb.boxes[item];
                if (!(hi16(bx.x) < X0 || lo16(bx.x) > tx1 || hi16(bx.y) < Y0 || lo16(bx.y) > ty1)) id = item;
            } else if (item < n_bin) {
                id = bin[item];
            } else {
                const uint2 e = fb.spill[item - n_bin];
                if ((int)e.x == tile) id = e.y;
            }
            if (id != 0xffffffffu) s_cand[atomicAdd(&s_nc, 1u)] = id;
        }
        __syncthreads();
        const uint32_t nc = s_nc;
        for (uint32_t c = 0; c < nc; c += CHUNK) {
            const int m = (int)min((uint32_t)CHUNK, nc - c);
            if (c > 0) __syncthreads();
            if (tid < m) {
                const uint32_t id = s_cand[c + tid];
                s_id[tid] = id;
                const float4 *src = reinterpret_cast<const float4 *>(&fb.recs[id]);
                float4 q[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) q[j] = src[j];
#pragma unroll
                for (int j = 0; j < 6; ++j) s_rec[tid * 6 + j] = q[j];
            }
            __syncthreads();
            for (int j = 0; j < m; ++j) {
                const uint4 bb = reinterpret_cast<const uint4 *>(&s_rec[j * 6])[4];   // ibx iby gbx gby
                if (hi16(bb.z) < bxl || lo16(bb.z) > bxl + 7 || hi16(bb.w) < Y0 || lo16(bb.w) > ty1) continue;
                const TriRec r = rec_from(&s_rec[j * 6]);
                const uint32_t id = s_id[j];
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    const int by = Y0 + 8 * i;
                    if (hi16(bb.w) < by || lo16(bb.w) > by + 7) continue;        // block cull (uniform)
                    const int py = py0 + 8 * i;
                    const int ry = (py / fp.rth) * fp.rth;
                    raster_px(px, py, rtminx, rtmaxx, (float)ry, (float)(min(ry + fp.rth, fp.H) - 1), r, id, best[i]);
                }
            }
        }
    }
    // tile-clamp pixels of unbounded slivers outside their bbox that passed (k_setup ghost waves)
    {
        const uint32_t n_frag = min(cnt[C_FRAG], fp.frag_cap);
        for (uint32_t f = 0; f < n_frag; ++f) {
            const GhostFrag g = fb.frags[f];
            const int gx = (int)(g.xy & 0xffffu), gy = (int)(g.xy >> 16);
            if (gx != px) continue;
#pragma unroll
            for (int i = 0; i < NB; ++i)
                if (gy == py0 + 8 * i) resolve(g.z, g.id, g.v, g.w, best[i]);
        }
    }
    __syncthreads();   // s_rec is reused below

    // hand the winners to the row-major output mapping through LDS
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int o = (py0 - Y0 + 8 * i) * TILE + (px - X0);
        s_bz[o] = best[i].z;
        s_bid[o] = best[i].id;
        s_bv[o] = best[i].v;
        s_bw[o] = best[i].w;
    }
    __syncthreads();

    // output mapping: thread -> row tid>>3, 4 consecutive pixels (16-B colour and depth stores;
    // 8 threads cover a 128-B row segment of each)
    const int oy = Y0 + (tid >> 3), ox = X0 + (tid & 7) * 4;
    uint32_t covered = 0;
    if (oy < fp.H) {
        const size_t crow = (size_t)(fp.H - 1 - oy) * fp.W, drow = (size_t)oy * fp.W;
        uint32_t rgba[4];
        float dep[4];
        float4 pq[4];
        const int lo = (tid >> 3) * TILE + (tid & 7) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            dep[j] = s_bz[lo + j];
            rgba[j] = fp.clear_rgba;
            pq[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        // shade the winners two pixels at a time: both varyings loads in flight before any math
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            ShadeRec sr[2];
            bool win[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = 2 * h + q;
                win[q] = dep[j] < FLT_MAX && ox + j < fp.W;
                if (win[q]) {
                    ++covered;
                    if (fp.flags & DBG_SKIP_SHADE) { win[q] = false; continue; }
                    const float4 *src = reinterpret_cast<const float4 *>(&fb.shade[s_bid[lo + j]]);
                    float4 *d = reinterpret_cast<float4 *>(&sr[q]);
#pragma unroll
                    for (int k = 0; k < 5; ++k) d[k] = src[k];
                }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = 2 * h + q;
                if (!win[q]) continue;
                const float v = s_bv[lo + j], w = s_bw[lo + j];
                const float u = (1.0f - v) - w;
                float pre[3];
                shade_winner(draws[sr[q].draw], sr[q], u, v, w, pre);
                const uint32_t cr = (uint32_t)(uint8_t)pre[0], cg = (uint32_t)(uint8_t)pre[1], cb = (uint32_t)(uint8_t)pre[2];
                rgba[j] = cr | (cg << 8) | (cb << 16) | (255u << 24);
                pq[j] = make_float4(pre[0], pre[1], pre[2], 1.0f);
            }
        }
        if (ox + 3 < fp.W && (fp.W & 3) == 0) {
            *reinterpret_cast<uint4 *>(fb.color + (crow + ox) * 4) = make_uint4(rgba[0], rgba[1], rgba[2], rgba[3]);
            *reinterpret_cast<float4 *>(fb.depth + drow + ox) = make_float4(dep[0], dep[1], dep[2], dep[3]);
        } else {
            for (int j = 0; j < 4; ++j)
                if (ox + j < fp.W) {
                    reinterpret_cast<uint32_t *>(fb.color)[crow + ox + j] = rgba[j];
                    fb.depth[drow + ox + j] = dep[j];
                }
        }
        if (fb.prequant)
            for (int j = 0; j < 4; ++j)
                if (ox + j < fp.W) fb.prequant[crow + ox + j] = pq[j];
    }
    // covered-pixel count: wave reduction, one LDS atomic per wave; per-tile stats go to their own
    // slot (no same-address global atomics across workgroups) and the host sums them at sync
    for (int o = 32; o > 0; o >>= 1) covered += __shfl_down(covered, o);
    if (lane == 0) atomicAdd(&s_cov, covered);
    __syncthreads();
    if (tid == 0) {
        fb.tile_stat[tile] = make_uint2(s_cov, n_bin_total);
        if (!fp.scan_mode) fb.tile_count[tile] = 0u;   // bins are empty for the next frame
    }
}

}  // namespace shs_dev

// ---- launch wrappers (called by shs_abi.cpp) -----------------------------------------------
namespace shs_internal {
using namespace shs_dev;

hipError_t launch_setup(const FrameParams &fp, const FrameBuffers &fb, const KArgDraws &ka, hipStream_t s) {
    // setup blocks (one thread per triangle) + ghost blocks (4 waves; each group of GHOST_GROUP
    // triangles is shared by fp.ghost_slices waves)
    const int setup_blocks = (fp.n_tris + 255) / 256;
    const int n_groups = (fp.n_tris + GHOST_GROUP - 1) / GHOST_GROUP;
    const int ghost_blocks = (n_groups * (int)fp.ghost_slices + 3) / 4;
    hipLaunchKernelGGL(k_setup, dim3(setup_blocks > 0 ? setup_blocks + ghost_blocks : 1), dim3(256), 0, s, fp, fb, ka);
    return hipGetLastError();
}
hipError_t launch_raster(const FrameParams &fp, const FrameBuffers &fb, const KArgDraws &ka, int n_owned_tiles,
                         hipStream_t s) {
    if (n_owned_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_raster, dim3(n_owned_tiles), dim3(256), 0, s, fp, fb, ka);
    return hipGetLastError();
}
}  // namespace shs_internal
