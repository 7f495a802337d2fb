// shs_legacy.hip -- gfx950 kernels for the shs_renderer legacy triangle scan-conversion path.
//
// Replaces RendererSystem::process + draw_triangle_tile + the four legacy shader pairs
// (cpp-folders/src/hello-3d-primitives/hello_pipeline_{blinn_phong,phong,gouraud,flat}_shading.cpp).
//
// Pipeline per frame: two launches on one HIP stream, no memsets, no copies for <= 6 draws.
//   k_setup   three block roles in one grid:
//             setup  one thread per triangle: VS x3 (mvp), clip_to_screen, area/denominator culls,
//                    the per-triangle half of barycentric_coordinate (a 96-B raster record), the
//                    per-corner shading varyings, "busy" marks on the raster tiles its bin box
//                    touches and (large scenes) appends into per-bin-tile lists;
//             ghost  the reference's tile-clamp pixels of unbounded slivers (see below);
//             clear  streaming clear of the colour / depth planes (16-B stores).
//   k_raster  persistent: each workgroup takes the busy 32x8 raster tiles of its share; a wave owns
//             an 8x8 block, one pixel per lane.  Candidates (bin box overlaps the tile) are staged
//             in LDS; each pixel resolves to the lexicographic minimum (z, submission index) --
//             identical to the reference's in-order strict-less z test (the first triangle with
//             the minimal z wins); only the winner is shaded, then colour (canvas rows) and depth
//             (screen rows) are written as whole 128-B row segments.
// The z-buffer never round-trips through HBM: each busy tile's pixels are written once more on
// top of the clear, everything else exactly once.
//
// Tile-clamp semantics.  draw_triangle_tile clamps a triangle's bbox to the 80x80 tile job that
// runs it (blinn_phong_shading.cpp:208-224), so the reference also tests pixels OUTSIDE the
// triangle's bbox (the clamped edge rows/columns/corners of every other tile).  Such a pixel is
// >= 0.49 px outside the bbox, so an exact barycentric is <= -(distance)/(2*extent); k_setup
// bounds barycentric_coordinate's float error (an affine function of the distance) and proves
// those pixels rejected, except inside a small "danger box" around slivers (TRI_GHOST): k_raster
// then evaluates the reference's exact visited set there.  Slivers with no usable bound
// (TRI_UNBOUNDED) keep their own bbox for binning; k_setup's ghost waves test every pixel the
// reference visits outside it and hand the rare passing ones to k_raster as fragments.
// DESIGN.md has the derivation.
#include <float.h>
#include <limits.h>

#include "shs_device.hpp"
#include "shs_internal.hpp"
#include "shs_wave.hpp"

// Framebuffer stores of the raster and the clears: non-temporal (streamed past the caches) unless
// -DSHS_LEGACY_PLAIN_STORES (timing experiments).
#ifdef SHS_LEGACY_PLAIN_STORES
template <typename T> __device__ __forceinline__ void LEGACY_STORE(T v, T *p) { *p = v; }
#else
#define LEGACY_STORE(v, p) __builtin_nontemporal_store(v, p)
#endif

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
    const double iDlow = 1.0 / Dlow, iDabs = 1.0 / Dabs;   // (the 1.25 slack covers the products' rounding)
    const double K1 = 7.2 * u + ED * iDlow;
    const double p0 = Wx + 0.01, q0 = Wy + 0.01;
    const double A20 = p0 * a + q0 * b, A21 = p0 * c + q0 * d;
    const double Nv0 = A11 * A20 + A01 * A21, Nvx = A11 * a + A01 * c, Nvy = A11 * b + A01 * d;
    const double Nw0 = A00 * A21 + A01 * A20, Nwx = A00 * c + A01 * a, Nwy = A00 * d + A01 * b;
    const double s = K1 * iDabs * (2.0 + 2.0 * u);
    const double e0 = 1.25 * ((Nv0 + Nw0) * s + u * (2.0 + (2.0 * Nv0 + Nw0) * iDlow));
    const double ex = 1.25 * ((Nvx + Nwx) * s + u * (2.0 * Nvx + Nwx) * iDlow);
    const double ey = 1.25 * ((Nvy + Nwy) * s + u * (2.0 * Nvy + Nwy) * iDlow);
    const double S = ex * Wx + ey * Wy;
    if (!(S < 0.5)) return none;
    const double m0 = e0 / (1.0 - 2.0 * S);
    const double dgx = 2.0 * Wx * m0, dgy = 2.0 * Wy * m0;
    return (dgx < 1e6 && dgy < 1e6) ? make_double2(dgx, dgy) : none;
}

__device__ __forceinline__ bool finitef(float x) { return fabsf(x) <= FLT_MAX; }

// x^(2^k) for the shaders' integer shininess (32, 64), by k squarings in double, narrowed to
// float.  The reference's powf / pow(double) results are the correctly rounded (or <= 1 ulp double)
// power; the squaring chain is within (2^k - 1) double ulps of the exact value, so the float
// result agrees except within ~1e-14 relative of a float rounding boundary -- far inside the
// 1e-5 shaded-float tolerance (north_star).
template <int K>
__device__ __forceinline__ float pow2k(float x) {
    double d = (double)x;
#pragma unroll
    for (int i = 0; i < K; ++i) d = d * d;
    return (float)d;
}

// The draw table: the kernel-argument copy (KARG, <= KARG_DRAWS draws) or the device table.  A
// compile-time choice, so the pointer keeps its address space (uniform indices -> scalar loads).
template <bool KARG>
__device__ __forceinline__ const DrawGPU *draw_table(const FrameBuffers &fb, const KArgDraws &ka) {
    return KARG ? ka.d : fb.draws;
}

// floor of a finite float, clamped into [lo, hi] before the conversion
__device__ __forceinline__ int floor_clamped(float x, int lo, int hi) {
    return (int)fminf(fmaxf(floorf(x), (float)lo), (float)hi);
}

// RF_NO_RECS: the per-triangle word k_setup stores -- the triangle's draw in the frame's slice and its
// record flags (TRI_*, from danger_margin's double-precision bound, which k_raster then need not redo).
__device__ __forceinline__ int32_t tdraw_word(int d, uint32_t flags) { return (int32_t)((uint32_t)d | (flags << 29)); }

__device__ __forceinline__ TriRec rec_from(const float4 *s) {
    TriRec r;
    float4 *d = reinterpret_cast<float4 *>(&r);
#pragma unroll
    for (int j = 0; j < 6; ++j) d[j] = s[j];
    return r;
}

// Bin and spill entries carry this tag on a ghost's id: k_raster stages the ghost's float bbox (the
// tile-clamp test's input, FrameBuffers::rext) beside its record, in the same round trip.
constexpr uint32_t BIN_GHOST = 0x80000000u;

// The record from its stored 64-B part h (TriHot, four float4s) and float bbox e (fminx fmaxx fminy
// fmaxy; read only when the flags say TRI_GHOST -- other triangles' e is never stored): the integer
// bbox is the clamped floor of the float bbox, as rec_from_screen computes it for a kept triangle.
__device__ __forceinline__ TriRec rec_from_hot(const FrameParams &fp, float4 h0, float4 h1, float4 h2, float4 h3, float4 e) {
    TriRec r;
    r.ax = h0.x; r.ay = h0.y; r.v0x = h0.z; r.v0y = h0.w;
    r.v1x = h1.x; r.v1y = h1.y; r.d00 = h1.z; r.d01 = h1.w;
    r.d11 = h2.x; r.denom = h2.y; r.z0 = h2.z; r.z1 = h2.w;
    r.z2 = h3.x;
    const uint32_t word = __float_as_uint(h3.y);
    r.flags = word >> 29;
    r.draw = (int32_t)(word & 0x1fffffffu);
    r.local = 0;
    r.gbx = __float_as_uint(h3.z); r.gby = __float_as_uint(h3.w);
    r.fminx = e.x; r.fmaxx = e.y; r.fminy = e.z; r.fmaxy = e.w;
    r.ibx = pack16(floor_clamped(e.x, 0, fp.W), floor_clamped(e.y, -1, fp.W - 1));
    r.iby = pack16(floor_clamped(e.z, 0, fp.H), floor_clamped(e.w, -1, fp.H - 1));
    return r;
}

__device__ __forceinline__ TriRec rec_from_hot(const FrameParams &fp, const float4 *h, const float4 *e) {
    return rec_from_hot(fp, h[0], h[1], h[2], h[3], *e);
}

// Quad: lane q stores float4 q of the triangle's 64-B TriHot, lane 0 also its float bbox when ext.
__device__ __forceinline__ void quad_store_hot(float4 *hot, float4 *bbox, const TriRec &r, bool ext) {
    const int q = __lane_id() & 3;
    const float f[16] = {r.ax, r.ay, r.v0x, r.v0y, r.v1x, r.v1y, r.d00, r.d01, r.d11, r.denom, r.z0, r.z1,
                         r.z2, __uint_as_float(r.flags << 29 | (uint32_t)r.draw), __uint_as_float(r.gbx), __uint_as_float(r.gby)};
    float x = f[0], y = f[1], z = f[2], w = f[3];
#pragma unroll
    for (int qq = 1; qq < 4; ++qq) {   // selects, not an indexed read (which would put the record in scratch)
        x = q == qq ? f[4 * qq] : x;
        y = q == qq ? f[4 * qq + 1] : y;
        z = q == qq ? f[4 * qq + 2] : z;
        w = q == qq ? f[4 * qq + 3] : w;
    }
    hot[q] = make_float4(x, y, z, w);
    if (ext && q == 0) *bbox = make_float4(r.fminx, r.fmaxx, r.fminy, r.fmaxy);
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
// Load a soup triangle's 9 floats into registers (before any store of the caller, so the compiler
// never has to re-read them behind a possibly aliasing store).
__device__ __forceinline__ void load9(const float *src, float (&v)[9]) {
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = src[k];
}

// VS position of one corner (mvp * vec4(p, 1)) and Canvas::clip_to_screen (shs_renderer.hpp:823-831).
__device__ __forceinline__ void vertex_screen(const FrameParams &fp, const float *mvp, float x, float y, float z, float &sx,
                                              float &sy, float &sz) {
    float cx, cy, cz, cw;
    m4p(mvp, x, y, z, cx, cy, cz, cw);
    const float nx = cx / cw, ny = cy / cw, nz = cz / cw;
    sx = (nx + 1.0f) * 0.5f * (float)(fp.W - 1);
    sy = (1.0f - ny) * 0.5f * (float)(fp.H - 1);
    sz = nz;
}

__device__ __forceinline__ TriRec rec_from_screen(const FrameParams &fp, int draw, int local, const float (&sx)[3],
                                                  const float (&sy)[3], const float (&sz)[3]) {
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
        // no bound, or a danger box too large to bin cheaply: the ghost waves take the pixels outside
        // the ibox (exact either way)
        const bool unbounded = !(dg.x >= 0.0) || dg.x > GHOST_MAX_EXPAND || dg.y > GHOST_MAX_EXPAND;
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

__device__ __forceinline__ TriRec make_rec(const FrameParams &fp, const DrawGPU &dr, int draw, int local, const float (&p)[9]) {
    float sx[3], sy[3], sz[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) vertex_screen(fp, dr.mvp, p[3 * k], p[3 * k + 1], p[3 * k + 2], sx[k], sy[k], sz[k]);
    return rec_from_screen(fp, draw, local, sx, sy, sz);
}

// ---- quad-lane triangle setup ---------------------------------------------------------------
// Four lanes per triangle (q = lane & 3): lanes 0..2 transform one corner each (the reference's VS
// runs per corner), the screen corners are exchanged within the quad, and every lane of the quad
// then holds the triangle's record.  Cuts the per-thread dependency chain of setup ~3x.
__device__ __forceinline__ float quad_bcast(float v, int k) {
    // DPP quad_perm(k, k, k, k)
    int r;
    switch (k) {
        case 0: r = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0x00, 0xf, 0xf, false); break;
        case 1: r = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0x55, 0xf, 0xf, false); break;
        case 2: r = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0xaa, 0xf, 0xf, false); break;
        default: r = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0xff, 0xf, 0xf, false); break;
    }
    return __int_as_float(r);
}

// Record of the quad's triangle (all four lanes return it); p3 = this lane's corner (q < 3; lane 3
// repeats corner 2).
__device__ __forceinline__ TriRec quad_make_rec(const FrameParams &fp, const DrawGPU &dr, int draw, int local,
                                                const float (&p3)[3]) {
    float vx, vy, vz;
    vertex_screen(fp, dr.mvp, p3[0], p3[1], p3[2], vx, vy, vz);
    float sx[3], sy[3], sz[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { sx[k] = quad_bcast(vx, k); sy[k] = quad_bcast(vy, k); sz[k] = quad_bcast(vz, k); }
    return rec_from_screen(fp, draw, local, sx, sy, sz);
}

// Index of the draw owning triangle gid, and whether the whole wave shares it (then the draw's
// uniforms are read with scalar loads).
__device__ __forceinline__ int wave_draw(const DrawGPU *draws, int n_draws, int gid, bool valid, bool &uniform) {
    const int lo = valid ? find_draw(draws, n_draws, gid) : 0;
    const int lo0 = __builtin_amdgcn_readfirstlane(lo);
    uniform = __ballot(valid && lo != lo0) == 0;
    return uniform ? lo0 : lo;
}

// Profiling marks (SHS_OPT_TIMELINE): thread 0 stamps phase k of its workgroup.
__device__ __forceinline__ void tl_mark(uint64_t *tl, int slot, int k) {
    if (tl && threadIdx.x == 0) tl[TL_STRIDE * slot + 2 + k] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ bool owned_bin_tile(const FrameParams &fp, int bx, int by) {
    return ((by * fp.tiles_x + bx) % fp.count) == fp.rank;
}

// ---- busy tiles --------------------------------------------------------------------------------
// A raster tile is busy in this launch when busy[rt] == fp.epoch.  The first marker of a tile (the
// atomic exchange returns another value) also enters it into the batch's busy list exactly once;
// k_raster deals the list out as work items.
__device__ __forceinline__ uint32_t busy_entry(const FrameParams &fp, int frame, int rt) {
    return (uint32_t)(frame * fp.tiles_x * fp.rtiles_y + rt);
}

// Mark and append directly (rare callers: ghost fragments).
__device__ __forceinline__ void mark_busy_direct(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, int frame,
                                                 int rt) {
    if (atomicExch(&fb.busy[rt], fp.epoch) != fp.epoch) fb.busy_list[atomicAdd(&cnt[C_BUSY], 1u)] = busy_entry(fp, frame, rt);
}

// Setup blocks collect their newly busy tiles in LDS and append them with one atomic per block.
constexpr int NEW_BUSY_CAP = 1024;
struct NewBusy {
    uint32_t n, base;
    uint32_t e[NEW_BUSY_CAP];
};

// The tile's listing once its mark found it not yet busy (old != epoch).
__device__ __forceinline__ void list_busy(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, int frame, int rt,
                                          NewBusy &nb) {
    const uint32_t k = atomicAdd(&nb.n, 1u);
    if (k < (uint32_t)NEW_BUSY_CAP) nb.e[k] = busy_entry(fp, frame, rt);
    else fb.busy_list[atomicAdd(&cnt[C_BUSY], 1u)] = busy_entry(fp, frame, rt);
}

__device__ __forceinline__ void mark_busy(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, int frame, int rt,
                                          NewBusy &nb) {
    if (atomicExch(&fb.busy[rt], fp.epoch) != fp.epoch) list_busy(fp, fb, cnt, frame, rt, nb);
}

// Bin mode: the first append to bin tile t (its counter returned 0) makes the tile's raster rows busy.
// Exactly one appender sees 0, so the flags are plain stores and no raster tile is listed twice; a
// row no primitive touches is rastered with no hits (written with the clear values), like a busy
// tile whose candidates all miss.
__device__ __forceinline__ void mark_bin_rows(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, int frame, int t,
                                              NewBusy &nb) {
    const int bx = t % fp.tiles_x, ry0 = (t / fp.tiles_x) * (TILE / RTH);
    if (fp.flags & RF_XCD_ROWS) {   // the rows as one 4-aligned group (every bin-mode append is 4 entries)
        static_assert(TILE / RTH == 4 && NEW_BUSY_CAP % 4 == 0, "row groups of four");
        const uint32_t k = atomicAdd(&nb.n, 4u);
        uint32_t *dst = k < (uint32_t)NEW_BUSY_CAP ? &nb.e[k] : &fb.busy_list[atomicAdd(&cnt[C_BUSY], 4u)];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rt = (ry0 + r) * fp.tiles_x + bx;
            if (ry0 + r < fp.rtiles_y) fb.busy[rt] = fp.epoch;
            dst[r] = ry0 + r < fp.rtiles_y ? busy_entry(fp, frame, rt) : BUSY_SKIP;
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < TILE / RTH; ++r) {
        const int ry = ry0 + r;
        if (ry >= fp.rtiles_y) break;
        const int rt = ry * fp.tiles_x + bx;
        fb.busy[rt] = fp.epoch;
        const uint32_t k = atomicAdd(&nb.n, 1u);
        if (k < (uint32_t)NEW_BUSY_CAP) nb.e[k] = busy_entry(fp, frame, rt);
        else fb.busy_list[atomicAdd(&cnt[C_BUSY], 1u)] = busy_entry(fp, frame, rt);
    }
}

// Block-wide (all threads, after the marks): append the block's collected tiles.
__device__ __forceinline__ void flush_busy(const FrameBuffers &fb, uint32_t *cnt, NewBusy &nb) {
    __syncthreads();
    const uint32_t n = min(nb.n, (uint32_t)NEW_BUSY_CAP);
    if (threadIdx.x == 0 && n) nb.base = atomicAdd(&cnt[C_BUSY], n);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) fb.busy_list[nb.base + i] = nb.e[i];
}

// ---- ghost waves ------------------------------------------------------------------------------
// The pixels the reference's tile clamp makes an unbounded sliver visit OUTSIDE its integer bbox
// (blinn_phong_shading.cpp:208-224: per 80x80 tile job, the float bbox clamped to the tile).  The
// visited set is separable: in reference-tile column c the x-range is [(int)max(tminx, min(tmaxx,
// fminx)), (int)min(tmaxx, max(tminx, fmaxx))] -- one edge column for the columns left (tmaxx <
// fminx, a prefix) or right (tminx > fmaxx, a suffix) of the bbox, the bbox's own span for the
// overlapping columns -- and likewise in y.  With Xout / Yout the edge columns / rows and Xin /
// Yin the overlapping spans, the visited pixels outside the ibox are (Xout x (Yout u Yin)) u
// (Xin x Yout): enumerated lane-parallel by index arithmetic.  One wave per (GHOST_GROUP
// triangles, slice) recomputes the group's records (quad setup, deterministic) and takes every
// fp.ghost_slices-th 64-pixel batch of each unbounded sliver in the group.
constexpr int GHOST_GROUP = 16;   // triangles per wave (a quad of lanes each)

struct SliverSpan {
    int cl, cr, ru, rd;             // edge columns left / right, edge rows above / below
    int xi0, xi1, yi0, yi1;         // overlapping spans (empty when lo > hi)
};

// Count the reference-tile columns (rows) entirely before / after [fmin, fmax]; span of the rest.
__device__ __forceinline__ void classify_axis(int n_rt, int rts, int extent, float fmin, float fmax, int &before,
                                              int &after, int &lo, int &hi) {
    before = 0; after = 0;
    for (int c0 = 0; c0 < n_rt; c0 += 64) {
        const int c = c0 + __lane_id();
        const bool valid = c < n_rt;
        const float tmin = (float)(c * rts), tmax = (float)(min(c * rts + rts, extent) - 1);
        before += __popcll(__ballot(valid && tmax < fmin));
        after += __popcll(__ballot(valid && tmin > fmax));
    }
    lo = 0; hi = -1;
    if (before + after < n_rt) {
        const int c0 = before, c1 = n_rt - 1 - after;
        lo = (int)g_max((float)(c0 * rts), fmin);
        hi = (int)g_min((float)(min(c1 * rts + rts, extent) - 1), fmax);
    }
}

// i-th edge column (row): the first `before` are the right edges of the leading tiles, the rest
// the left edges of the trailing ones.
__device__ __forceinline__ int edge_coord(int i, int before, int n_rt, int after, int rts, int extent) {
    return i < before ? min((i + 1) * rts, extent) - 1 : (n_rt - after + (i - before)) * rts;
}

struct GhostScratch {           // per-wave LDS
    float4 rec[6];
};

struct SliverRecs {             // per-wave LDS (RF_GHOST_INLINE): the records of the wave's 16 triangles' slivers
    float4 rec[16 * 6];
};

// The draw of triangle gid from its setup block's first draw d0 (FrameBuffers::bdraw): a block of 64
// triangles rarely crosses a draw boundary, so this is one tri_base load instead of a binary search.
__device__ __forceinline__ int wave_draw_from(const DrawGPU *draws, int n_draws, int gid, bool valid, int d0, bool &uniform) {
    int d = d0;
    if (valid)
        while (d + 1 < n_draws && draws[d + 1].tri_base <= gid) ++d;
    uniform = __ballot(valid && d != d0) == 0;
    return d;
}

// The quad's triangle index, draw and this lane's corner, with the wave-uniform draw fast path.
struct QuadTri {
    int tri, draw, local;
    bool valid, uniform;
};

__device__ __forceinline__ QuadTri quad_tri(const DrawGPU *draws, int n_draws, int n_tris, int tri) {
    QuadTri t;
    t.tri = tri;
    t.valid = tri < n_tris;
    t.draw = wave_draw(draws, n_draws, tri, t.valid, t.uniform);
    return t;
}

// Record of the quad's triangle through the draw's uniforms (scalar loads when wave-uniform).
__device__ __forceinline__ TriRec quad_record(const FrameParams &fp, const DrawGPU *draws, QuadTri &t) {
    const int q = __lane_id() & 3, qv = q < 3 ? q : 2;
    TriRec r;
    if (t.uniform) {
        const int d = __builtin_amdgcn_readfirstlane(t.draw);
        const DrawGPU &dr = draws[d];
        t.local = t.tri - dr.tri_base;
        const float *P = dr.pos + 9 * (size_t)t.local + 3 * qv;
        const float p3[3] = {P[0], P[1], P[2]};
        r = quad_make_rec(fp, dr, d, t.local, p3);
    } else {
        const DrawGPU &dr = draws[t.draw];
        t.local = t.tri - dr.tri_base;
        const float *P = dr.pos + 9 * (size_t)t.local + 3 * qv;
        const float p3[3] = {P[0], P[1], P[2]};
        r = quad_make_rec(fp, dr, t.draw, t.local, p3);
    }
    return r;
}

// Conservative row span of a staged candidate inside its clipped box [bx0, bx1]: the pixels of row py
// that can pass bary_pass (barycentric_coordinate, shs_renderer.hpp:802-821).  With t = px + 0.5 - ax,
// Y = py + 0.5 - ay the exact Gram-form barycentrics of the record's float values are linear in t:
//   v = av t + cv,  w = aw t + cw,  u = 1 - v - w,
//   av = (d11 v0x - d01 v1x) / denom, cv = Y (d11 v0y - d01 v1y) / denom (w: d00 / v1 and v0 swapped).
// bary_pass's float evaluation (no contraction) is within ~8 u Mv of v, Mv = (|d11| S0 + |d01| S1) /
// |denom| with S0 = |v0x| |t| + |v0y| |Y|, S1 likewise (u = 2^-24: the rounding of t, the products
// and sums of d20 / d21, the outer products, the difference and the division; likewise w), and u's
// within ~10 u (1 + Mv + Mw).  A pixel can pass only where every exact barycentric is >= minus its
// bound; each half-line a t >= -e - c is solved here in float with e = E (...) at E = 2^-18 (>= 6x the
// bound: the slack absorbs this computation's own roundings, a few u of the magnitudes), and 2^-12 px
// more covers the conversion to pixel indices.  Non-finite records keep the whole box row.  The bound
// holds outside the triangle's bbox too (the 80x80 tile clamp's ghost pixels, section 5 of DESIGN.md).
// tests/test_legacy_row_spans.py restates this in numpy and checks it against the per-pixel test.
__device__ __forceinline__ void legacy_row_span(const float4 r0, const float4 r1, const float4 r2, int py, int bx0, int bx1,
                                                int &x0, int &x1) {
    x0 = bx0; x1 = bx1;
    // r0, r1, r2: the record's first three float4s: ax ay v0x v0y | v1x v1y d00 d01 | d11 denom ...
    const float ax = r0.x, ay = r0.y, v0x = r0.z, v0y = r0.w, v1x = r1.x, v1y = r1.y, d00 = r1.z, d01 = r1.w;
    const float d11 = r2.x, den = r2.y;
    if (!(isfinite(ax) && isfinite(ay) && isfinite(v0x) && isfinite(v0y) && isfinite(v1x) && isfinite(v1y) && isfinite(d00) &&
          isfinite(d01) && isfinite(d11) && isfinite(den) && fabsf(den) > 0.0f))
        return;
    constexpr float E = 0x1p-18f;
    const float Y = ((float)py + 0.5f) - ay, aY = fabsf(Y);
    const float T = fmaxf(fabsf(((float)bx0 + 0.5f) - ax), fabsf(((float)bx1 + 0.5f) - ax));
    const float idn = 1.0f / den, aid = fabsf(idn);
    const float s0 = fabsf(v0x) * T + fabsf(v0y) * aY, s1 = fabsf(v1x) * T + fabsf(v1y) * aY;
    const float mv = aid * (fabsf(d11) * s0 + fabsf(d01) * s1), mw = aid * (fabsf(d00) * s1 + fabsf(d01) * s0);
    const float av = (d11 * v0x - d01 * v1x) * idn, cv = ((d11 * v0y - d01 * v1y) * idn) * Y;
    const float aw = (d00 * v1x - d01 * v0x) * idn, cw = ((d00 * v1y - d01 * v0y) * idn) * Y;
    float lo = -1e30f, hi = 1e30f;
    auto edge = [&](float a, float c, float e) {   // a t + c >= -e
        const float b = -e - c;
        if (a > 0.0f) lo = fmaxf(lo, b / a);
        else if (a < 0.0f) hi = fminf(hi, b / a);
        else if (b > 0.0f) { lo = 1e30f; hi = -1e30f; }
    };
    edge(av, cv, E * mv);
    edge(aw, cw, E * mw);
    edge(-(av + aw), 1.0f - (cv + cw), E * (1.0f + 2.0f * (mv + mw)));
    const float flo = (lo + ax) - 0.5f, fhi = (hi + ax) - 0.5f;
    const float slo = 0x1p-12f * ((fabsf(lo) + fabsf(ax)) + 1.0f), shi = 0x1p-12f * ((fabsf(hi) + fabsf(ax)) + 1.0f);
    x0 = max(bx0, (int)ceilf(fmaxf(fminf(flo - slo, 1e9f), -1e9f)));
    x1 = min(bx1, (int)floorf(fmaxf(fminf(fhi + shi, 1e9f), -1e9f)));
}

// Every pixel sliver `tri` (record t) visits outside its ibox in the reference's tile jobs that can
// pass: passing ones become ghost fragments.  The visited set is walked line by line -- the edge
// columns over their rows (Yout u Yin), then the edge rows over Xin -- and on each line only the
// pixels inside its conservative span (legacy_row_span: every pixel that can pass barycentric_coordinate
// lies in it, outside the bbox too; a column's span is the row span of the record with x and y
// swapped, which leaves every Gram term and every computed barycentric bit-identical).  Round 4 tested
// every visited pixel: up to the edge columns times the bbox height per sliver.  The slice-th line
// of every `stride` / 64 lines per lane.  Wave-uniform arguments, converged wave.
__device__ __forceinline__ void sliver_pixels(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, const TriRec &t,
                                              uint32_t tri, uint32_t frame, int slice, int stride) {
    const int lane = __lane_id();
    const int ix0 = lo16(t.ibx), ix1 = hi16(t.ibx), iy0 = lo16(t.iby), iy1 = hi16(t.iby);
    SliverSpan sp;
    classify_axis(fp.rt_x, fp.rtw, fp.W, t.fminx, t.fmaxx, sp.cl, sp.cr, sp.xi0, sp.xi1);
    classify_axis(fp.rt_y, fp.rth, fp.H, t.fminy, t.fmaxy, sp.ru, sp.rd, sp.yi0, sp.yi1);
    const int nxo = sp.cl + sp.cr, nyo = sp.ru + sp.rd;
    const int n_lines = nxo + nyo;
    // the rows an edge column visits span [y_lo, y_hi] (its span's distance bound)
    const int yo0 = nyo ? edge_coord(0, sp.ru, fp.rt_y, sp.rd, fp.rth, fp.H) : INT_MAX;
    const int yo1 = nyo ? edge_coord(nyo - 1, sp.ru, fp.rt_y, sp.rd, fp.rth, fp.H) : INT_MIN;
    const bool yin = sp.yi0 <= sp.yi1;
    const int y_lo = min(yo0, yin ? sp.yi0 : INT_MAX), y_hi = max(yo1, yin ? sp.yi1 : INT_MIN);
    const float4 r2 = make_float4(t.d11, t.denom, 0.0f, 0.0f);
    for (int lb = slice * 64; lb < n_lines; lb += stride) {
        const int L = lb + lane;
        // this lane's line: a column x over the Yin run [a0, a1] then the edge rows j in [0, nyo) inside
        // [s0, s1]; or a row y over the Xin run [a0, a1]
        const bool col = L < nxo;
        const int fixed = col ? edge_coord(L, sp.cl, fp.rt_x, sp.cr, fp.rtw, fp.W)
                              : edge_coord(L - nxo, sp.ru, fp.rt_y, sp.rd, fp.rth, fp.H);
        int a0 = 0, a1 = -1, s0 = 1, s1 = 0;
        if (L < n_lines && (col || sp.xi0 <= sp.xi1)) {
            const float4 q0 = col ? make_float4(t.ay, t.ax, t.v0y, t.v0x) : make_float4(t.ax, t.ay, t.v0x, t.v0y);   // x <-> y
            const float4 q1 = col ? make_float4(t.v1y, t.v1x, t.d00, t.d01) : make_float4(t.v1x, t.v1y, t.d00, t.d01);
            legacy_row_span(q0, q1, r2, fixed, col ? y_lo : sp.xi0, col ? y_hi : sp.xi1, s0, s1);
            a0 = col ? max(sp.yi0, s0) : s0;
            a1 = col ? (yin ? min(sp.yi1, s1) : -1) : s1;
        }
        int i = a0, j = 0;   // next run pixel, next edge row
        while (true) {
            bool have = false;
            int px = 0, py = 0;
            if (i <= a1) {
                have = true;
                px = col ? fixed : i;
                py = col ? i : fixed;
                ++i;
            } else if (col) {
                while (j < nyo && !have) {
                    const int y = edge_coord(j, sp.ru, fp.rt_y, sp.rd, fp.rth, fp.H);
                    ++j;
                    if (y >= s0 && y <= s1) { have = true; px = fixed; py = y; }
                }
            }
            if (__ballot(have) == 0ull) break;
            bool pass = false;
            float z = 0.f, u = 0.f, v = 0.f, w = 0.f;
            if (have) {
                const bool in_ibox = px >= ix0 && px <= ix1 && py >= iy0 && py <= iy1;   // k_raster's part
                if (!in_ibox && (fp.count == 1 || owned_bin_tile(fp, px / TILE, py / TILE)) &&
                    bary_pass(t, (float)px + 0.5f, (float)py + 0.5f, u, v, w)) {
                    z = (u * t.z0 + v * t.z1) + w * t.z2;
                    pass = z < FLT_MAX;   // NaN / FLT_MAX never pass the strict z test
                }
            }
            const uint32_t slot = wave_append1(&cnt[C_FRAG], pass);
            if (pass) {
                if (slot < fp.frag_cap) {
                    GhostFrag g;
                    g.xy = (uint32_t)px | ((uint32_t)py << 16);
                    g.z = z;
                    g.id = tri;
                    g.v = v;
                    g.w = w;
                    g.frame = frame;
                    g.pad[0] = g.pad[1] = 0u;
                    fb.frags[slot] = g;
                    mark_busy_direct(fp, fb, cnt, (int)frame, (py / RTH) * fp.tiles_x + px / RTW);
                } else {
                    raise_overflow(&cnt[C_OVERFLOW], OV_FRAG, fb.ov_host);
                }
            }
        }
    }
}

__device__ __forceinline__ void ghost_wave(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *draws,
                                           uint32_t *cnt, int frame, int group, int slice, GhostScratch &gs) {
    const int lane = __lane_id();
    QuadTri qt = quad_tri(draws, fp.n_draws, fp.n_tris, group * GHOST_GROUP + (lane >> 2));
    TriRec r;
    if (qt.valid) r = quad_record(fp, draws, qt);
    // one lane per quad votes
    uint64_t todo = __ballot(qt.valid && (lane & 3) == 0 && (r.flags & TRI_UNBOUNDED) && !(r.flags & TRI_CULLED));
    const int stride = 64 * (int)fp.ghost_slices;
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
        wave_lds_sync();   // gs.rec is rewritten by the next sliver
        sliver_pixels(fp, fb, cnt, t, (uint32_t)(group * GHOST_GROUP + (src >> 2)), (uint32_t)frame, slice, stride);
    }
}

// ---- k_setup ----------------------------------------------------------------------------------

__device__ __forceinline__ void append_bin(const FrameParams &fp, const FrameBuffers &fb, uint32_t *cnt, int frame, int t,
                                           uint32_t pos, uint32_t id) {
    if (pos < fp.bin_cap) {
        fb.bins[(size_t)t * fp.bin_cap + pos] = id;
    } else {
        const uint32_t sp = atomicAdd(&cnt[C_SPILL], 1u);
        if (sp < fp.spill_cap) fb.spill[sp] = make_uint2((uint32_t)(frame * fp.tiles_x * fp.tiles_y + t), id);
        else raise_overflow(&cnt[C_OVERFLOW], OV_SPILL, fb.ov_host);
    }
}

// This lane's corner's shading varyings (the VS outputs the FS interpolates): a = world position
// (Phong / Blinn-Phong), the clamped Gouraud colour, or the Flat view-space normal; nr = the
// normalised world normal (Phong / Blinn-Phong).
__device__ __forceinline__ void corner_varyings(const DrawGPU &dr, const float (&p3)[3], const float (&n3)[3], f3 &a, f3 &nr) {
    nr = f3{0.f, 0.f, 0.f};
    if (dr.shading == 0) {
        a = m3v(dr.nmat, f3{n3[0], n3[1], n3[2]});   // Flat VS (flat_shading.cpp:54): mat3(mv) * n
        return;
    }
    float x, y, z, ww;
    m4p(dr.model, p3[0], p3[1], p3[2], x, y, z, ww);
    const f3 wp = {x, y, z};
    const f3 n = normalize3(m3v(dr.nmat, f3{n3[0], n3[1], n3[2]}));
    if (dr.shading == 1) {
        // Gouraud VS (gouraud_shading.cpp:46-77): Blinn-Phong per vertex, shininess 32
        const f3 L = {dr.light[0], dr.light[1], dr.light[2]};
        const f3 cam = {dr.cam[0], dr.cam[1], dr.cam[2]};
        const f3 viewDir = normalize3(sub3(cam, wp));
        const float diff = g_max(dot3(n, L), 0.0f);
        const f3 half = normalize3(add3(L, viewDir));
        const float spec = pow2k<5>(g_max(dot3(n, half), 0.0f));   // glm::pow(x, 32.0f)
        const float sum = (0.15f + diff * 1.0f) + (0.5f * spec) * 1.0f;
        a = f3{g_clamp01(sum * dr.ocol[0]), g_clamp01(sum * dr.ocol[1]), g_clamp01(sum * dr.ocol[2])};
        return;
    }
    // Phong / Blinn-Phong VS (blinn_phong_shading.cpp:48-57)
    a = wp;
    nr = n;
}

// Quad: the triangle's 80-B ShadeRec (corner k's a at floats 3k.., its nr at 9 + 3k.., then shading
// and draw): lane q < 3 stores its own corner's six floats, lane 3 the two words.  (Round 4 assembled
// the record in every lane with 18 quad broadcasts, each lane storing a contiguous fifth: the
// broadcasts' registers were the bin-mode setup's register peak -- 80 VGPRs against its 64-VGPR
// bound, spilled.)
__device__ __forceinline__ void quad_store_shade_at(ShadeRec *rec, int draw, int shading, const f3 &a, const f3 &nr) {
    const int q = __lane_id() & 3;
    float *dst = reinterpret_cast<float *>(rec);
    if (q < 3) {
        dst[3 * q] = a.x; dst[3 * q + 1] = a.y; dst[3 * q + 2] = a.z;
        dst[9 + 3 * q] = nr.x; dst[9 + 3 * q + 1] = nr.y; dst[9 + 3 * q + 2] = nr.z;
    } else {
        dst[18] = __int_as_float(shading);
        dst[19] = __int_as_float(draw);
    }
}

__device__ __forceinline__ void quad_store_shade(const FrameBuffers &fb, int tri, int draw, int shading, const f3 &a,
                                                 const f3 &nr) {
    quad_store_shade_at(&fb.shade[tri], draw, shading, a, nr);
}

// Quad: lane q stores floats [6q, 6q + 6) of the 96-B record (global memory or an LDS copy).
__device__ __forceinline__ void quad_store_rec_at(TriRec *rec, const TriRec &r) {
    const int q = __lane_id() & 3;
    const float *f = reinterpret_cast<const float *>(&r);
    float2 *dst = reinterpret_cast<float2 *>(reinterpret_cast<float *>(rec) + 6 * q);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float x = f[2 * j], y = f[2 * j + 1];
#pragma unroll
        for (int qq = 1; qq < 4; ++qq) {
            x = q == qq ? f[6 * qq + 2 * j] : x;
            y = q == qq ? f[6 * qq + 2 * j + 1] : y;
        }
        dst[j] = make_float2(x, y);
    }
}

// The stored record (TriHot) and, for ghosts, the float bbox.
__device__ __forceinline__ void quad_store_rec(const FrameBuffers &fb, int tri, const TriRec &r) {
    quad_store_hot(reinterpret_cast<float4 *>(&fb.recs[tri]), &fb.rext[tri], r, (r.flags & TRI_GHOST) != 0u);
}

// Record, varyings and their stores for the quad's triangle; returns the flags and the bin box.
// vary: this frame stores the varyings (false: RF_SHARED_VARY and not frame 0 -- frame 0's are read).
// sliv: the wave's 16 record slots in LDS (RF_GHOST_INLINE), or nullptr.
__device__ __forceinline__ uint32_t setup_quad(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU &dr, int d,
                                               int dbase, int tri, uint2 &gbox, bool vary, float4 *sliv) {
    const int q = __lane_id() & 3, qv = q < 3 ? q : 2;
    const int local = tri - dr.tri_base;
    const float *P = dr.pos + 9 * (size_t)local + 3 * qv;
    const float p3[3] = {P[0], P[1], P[2]};
    const bool recs = !(fp.flags & RF_NO_RECS);
    float n3[3] = {0.0f, 0.0f, 0.0f};
    if (recs && vary) {   // issued with the position loads (their latency overlaps the record's arithmetic)
        const float *Nn = dr.nrm + 9 * (size_t)local + 3 * qv;
        n3[0] = Nn[0]; n3[1] = Nn[1]; n3[2] = Nn[2];
    }
    const TriRec r = quad_make_rec(fp, dr, d, local, p3);
    tl_mark(fb.timeline, blockIdx.x, 4);
    if (!recs) {
        // binned frame: k_raster recomputes records and varyings from the mesh; only k_ghost's
        // unbounded slivers keep their record (quad-uniform condition)
        if ((r.flags & (TRI_UNBOUNDED | TRI_CULLED)) == TRI_UNBOUNDED) quad_store_rec(fb, tri, r);
        if (q == 0) fb.tdraw[tri] = tdraw_word(d, r.flags);
    } else {
        // a culled triangle's record is never read (its bin box is empty: never binned, staged or a
        // winner); its varyings are, in the other frames, when frame 0's are shared (quad-uniform tests)
        const bool culled = r.flags & TRI_CULLED;
        if (!culled) quad_store_rec(fb, tri, r);
        if (vary && (!culled || (fp.flags & RF_SHARED_VARY))) {
            f3 a, nr;
            corner_varyings(dr, p3, n3, a, nr);
            quad_store_shade(fb, tri, dbase + d, dr.shading, a, nr);   // the draw-table index of the batch
        }
    }
    if (q == 0) fb.boxes[tri] = make_uint2(r.gbx, r.gby);   // culled: the empty box (0, -1)
    if (sliv && (r.flags & (TRI_UNBOUNDED | TRI_CULLED)) == TRI_UNBOUNDED)   // quad-uniform
        quad_store_rec_at(reinterpret_cast<TriRec *>(sliv + ((__lane_id() >> 2) & 15) * 6), r);
    gbox = make_uint2(r.gbx, r.gby);
    return r.flags;
}

constexpr int SMALL_RT = 16;  // raster tiles a quad marks by itself (4 per lane)
constexpr int SMALL_BT = 8;   // bin tiles a quad appends to by itself (2 per lane)

// One setup workgroup: 64 triangles, a quad of lanes each.
// frame / lb: the batch frame and this block's index among the frame's setup blocks; draws = the
// frame's draw slice (table entries dbase ..).  BIN: a bin-mode batch (k_setup<., true>: !fp.scan_mode,
// fp.ghost_list set, no inline slivers) -- the scan-mode marks and sliver walks are not compiled in.
template <bool BIN>
__device__ __forceinline__ void setup_block(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *draws, int dbase,
                                            int frame, int lb, uint32_t *cnt, uint32_t (&s_stat)[4], NewBusy &nb,
                                            float4 *sliv) {
    const int tid = threadIdx.x, lane = __lane_id(), q = lane & 3;
    if (tid < 4) s_stat[tid] = 0u;
    if (tid == 0) nb.n = 0u;
    __syncthreads();
    QuadTri qt;
    if (fb.bdraw) {
        qt.tri = lb * 64 + (tid >> 2);
        qt.valid = qt.tri < fp.n_tris;
        qt.draw = wave_draw_from(draws, fp.n_draws, qt.tri, qt.valid, fb.bdraw[lb], qt.uniform);
    } else {
        qt = quad_tri(draws, fp.n_draws, fp.n_tris, lb * 64 + (tid >> 2));
    }
    const int tri = qt.tri;
    const bool vary = !(fp.flags & RF_SHARED_VARY) || frame == 0;
    uint32_t flags = TRI_CULLED;
    int gx0 = 0, gx1 = -1, gy0 = 0, gy1 = -1;
    tl_mark(fb.timeline, blockIdx.x, 0);
    if (qt.valid) {
        uint2 gb;
        if (qt.uniform) {
            const int d = __builtin_amdgcn_readfirstlane(qt.draw);
            flags = setup_quad(fp, fb, draws[d], d, dbase, tri, gb, vary, sliv);
        } else {
            flags = setup_quad(fp, fb, draws[qt.draw], qt.draw, dbase, tri, gb, vary, sliv);
        }
        gx0 = lo16(gb.x); gx1 = hi16(gb.x); gy0 = lo16(gb.y); gy1 = hi16(gb.y);
    }
    tl_mark(fb.timeline, blockIdx.x, 1);
    const bool live = qt.valid && !(flags & TRI_CULLED) && gx0 <= gx1 && gy0 <= gy1;
    if (!live) { gx0 = 0; gx1 = -1; gy0 = 0; gy1 = -1; }
    const bool sharded = fp.count > 1;

    // -- scan mode: busy marks on the raster tiles (32x8) of the bin box (owned bin tiles only), the
    //    quad's four lanes taking every fourth tile (bin mode marks whole bin tiles at their first
    //    append, below)
    const int rx0 = gx0 / RTW, rx1 = live ? gx1 / RTW : -1, ry0 = gy0 / RTH, ry1 = live ? gy1 / RTH : -1;
    const int nrx = rx1 - rx0 + 1, n_rt = (live && !BIN) ? nrx * (ry1 - ry0 + 1) : 0;
    if (n_rt > 0 && n_rt <= SMALL_RT) {
        // every mark's exchange is issued before any result is used: one round trip, not one per tile
        int rts[SMALL_RT / 4];
        uint32_t old[SMALL_RT / 4];
#pragma unroll
        for (int i = 0; i < SMALL_RT / 4; ++i) {
            const int k = q + 4 * i;
            rts[i] = -1;
            old[i] = fp.epoch;
            if (k < n_rt) {
                const int rx = rx0 + k % nrx, ry = ry0 + k / nrx;
                if (!sharded || owned_bin_tile(fp, rx, ry / (TILE / RTH))) {
                    rts[i] = ry * fp.tiles_x + rx;
                    old[i] = atomicExch(&fb.busy[rts[i]], fp.epoch);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < SMALL_RT / 4; ++i)
            if (rts[i] >= 0 && old[i] != fp.epoch) list_busy(fp, fb, cnt, frame, rts[i], nb);
    }
    {
        uint64_t big = __ballot(n_rt > SMALL_RT && q == 0);
        while (big) {
            const int src = __ffsll((unsigned long long)big) - 1;
            big &= big - 1;
            const int bx0 = __shfl(rx0, src), bx1 = __shfl(rx1, src), by0 = __shfl(ry0, src), by1 = __shfl(ry1, src);
            const int nx = bx1 - bx0 + 1, n = nx * (by1 - by0 + 1);
            for (int k = lane; k < n; k += 64) {
                const int rx = bx0 + k % nx, ry = by0 + k / nx;
                if (!sharded || owned_bin_tile(fp, rx, ry / (TILE / RTH))) mark_busy(fp, fb, cnt, frame, ry * fp.tiles_x + rx, nb);
            }
        }
    }
    tl_mark(fb.timeline, blockIdx.x, 2);

    // -- bin appends (large scenes): bin tiles of the bin box, two per quad lane
    uint32_t n_bin = 0;
    if (BIN && !SHS_DBG(fp, DBG_SKIP_BIN)) {
        uint32_t *tcount = fb.tile_count;
        const int bx0 = gx0 / TILE, bx1 = live ? gx1 / TILE : -1, by0 = gy0 / TILE, by1 = live ? gy1 / TILE : -1;
        const int nbx = max(bx1 - bx0 + 1, 1), n_bt = live ? (bx1 - bx0 + 1) * (by1 - by0 + 1) : 0;
        int key[2];
        uint32_t pos[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = q + 4 * k;
            const int bx = bx0 + i % nbx, by = by0 + i / nbx;
            key[k] = (n_bt <= SMALL_BT && i < n_bt && (!sharded || owned_bin_tile(fp, bx, by))) ? by * fp.tiles_x + bx : -1;
        }
        wave_append<2>(tcount, key, pos);
        const uint32_t entry = (uint32_t)tri | ((flags & TRI_GHOST) ? BIN_GHOST : 0u);
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (key[k] >= 0) {
                append_bin(fp, fb, cnt, frame, key[k], pos[k], entry);
                ++n_bin;
                if (pos[k] == 0u) mark_bin_rows(fp, fb, cnt, frame, key[k], nb);
            }
        uint64_t big = __ballot(n_bt > SMALL_BT && q == 0);
        while (big) {
            const int src = __ffsll((unsigned long long)big) - 1;
            big &= big - 1;
            const int cx0 = __shfl(bx0, src), cx1 = __shfl(bx1, src), cy0 = __shfl(by0, src), cy1 = __shfl(by1, src);
            const uint32_t id = (uint32_t)__shfl((int)entry, src);
            const int nx = cx1 - cx0 + 1, n = nx * (cy1 - cy0 + 1);
            uint32_t mine = 0;
            for (int k = lane; k < n; k += 64) {
                const int bx = cx0 + k % nx, by = cy0 + k / nx;
                if (sharded && !owned_bin_tile(fp, bx, by)) continue;
                const int t = by * fp.tiles_x + bx;
                const uint32_t p = atomicAdd(&tcount[t], 1u);
                append_bin(fp, fb, cnt, frame, t, p, id);
                if (p == 0u) mark_bin_rows(fp, fb, cnt, frame, t, nb);
                ++mine;
            }
            for (int o = 32; o > 0; o >>= 1) mine += __shfl_down(mine, o);
            const uint32_t tot = __shfl(mine, 0);
            if (lane == src) n_bin += tot;
        }
    }
    flush_busy(fb, cnt, nb);
    tl_mark(fb.timeline, blockIdx.x, 3);

    // -- per-block statistics (no same-address global atomics); one lane per quad counts
    const bool lead = qt.valid && q == 0 && !(flags & TRI_CULLED);
    if (BIN || fp.ghost_list) {   // the unbounded slivers, listed for k_ghost (ids < n_tris: never overflows)
        const bool unb = lead && (flags & TRI_UNBOUNDED);
        const uint32_t slot = wave_append1(&cnt[C_SLIVER], unb);
        if (unb) fb.slivers[slot] = (uint32_t)(frame * fp.n_tris + tri);
    }
    const uint64_t m_setup = __ballot(lead);
    const uint64_t m_ghost = __ballot(lead && (flags & TRI_GHOST));
    const uint64_t m_unb = __ballot(lead && (flags & TRI_UNBOUNDED));
    for (int o = 32; o > 0; o >>= 1) n_bin += __shfl_down(n_bin, o);
    if (lane == 0) {
        atomicAdd(&s_stat[0], (uint32_t)__popcll(m_setup));
        atomicAdd(&s_stat[1], (uint32_t)__popcll(m_ghost));
        atomicAdd(&s_stat[2], (uint32_t)__popcll(m_unb));
        atomicAdd(&s_stat[3], n_bin);
    }
    __syncthreads();
    if (tid == 0) fb.blk_stat[frame * fp.setup_blocks + lb] = make_uint4(s_stat[0], s_stat[1], s_stat[2], s_stat[3]);
    tl_mark(fb.timeline, blockIdx.x, 5);
    if (!BIN && sliv && !SHS_DBG(fp, DBG_SKIP_GHOST)) {   // RF_GHOST_INLINE: this wave's unbounded slivers, one at a time
        uint64_t todo = m_unb;
        while (todo) {
            const int src = __ffsll((unsigned long long)todo) - 1;
            todo &= todo - 1;
            wave_lds_sync();   // the quads' record stores are complete
            const TriRec t = rec_from(sliv + (src >> 2) * 6);
            sliver_pixels(fp, fb, cnt, t, (uint32_t)__shfl(tri, src), (uint32_t)frame, 0, 64);
        }
    }
}

// One k_setup block b of the batch (setup or ghost role by its index in its frame); draw_tab = the
// batch's draw table (kernel arguments or the device table).  BIN: as setup_block's (no ghost roles).
template <bool BIN>
__device__ __forceinline__ void setup_item(const FrameParams &fp, const FrameBuffers &fb_all, const DrawGPU *draw_tab, int b,
                                           GhostScratch (&s_ghost)[4], uint32_t (&s_stat)[4], NewBusy &s_new,
                                           SliverRecs (&s_sliv)[4]) {
    uint32_t *cnt = fb_all.counters + fp.parity * CSET;
    if (b == 0)   // the next batch's counter set (its previous user, batch k - 2, has finished)
        for (int i = (int)threadIdx.x; i < CSET; i += 256) fb_all.counters[(size_t)fp.zero_set * CSET + i] = 0u;
    // frame of the batch and the block's role inside it
    const int frame = b / fp.frame_blocks, lb = b - frame * fp.frame_blocks;
    const FrameBuffers fb = frame_view(fp, fb_all, frame);
    const int dbase = frame * fp.n_draws;
    const DrawGPU *draws = draw_tab + dbase;
    const uint64_t t_start = fb.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint64_t c_start = fb.timeline ? __builtin_amdgcn_s_memtime() : 0ull;
    // (the counter set and the bin counts were zeroed on the setup stream before this launch)
    if (lb < fp.setup_blocks) {
        setup_block<BIN>(fp, fb, draws, dbase, frame, lb, cnt, s_stat, s_new,
                         (!BIN && (fp.flags & RF_GHOST_INLINE)) ? s_sliv[threadIdx.x >> 6].rec : nullptr);
    } else if (!BIN && lb < fp.setup_blocks + fp.ghost_blocks) {
        const int wave = threadIdx.x >> 6;
        const int gw = (lb - fp.setup_blocks) * 4 + wave;
        const int n_groups = (fp.n_tris + GHOST_GROUP - 1) / GHOST_GROUP;
        if (gw < n_groups * (int)fp.ghost_slices && !SHS_DBG(fp, DBG_SKIP_GHOST))
            ghost_wave(fp, fb, draws, cnt, frame, gw / (int)fp.ghost_slices, gw % (int)fp.ghost_slices, s_ghost[wave]);
    }
    if (fb.timeline) {
        __syncthreads();
        if (threadIdx.x == 0) {
            fb.timeline[TL_STRIDE * b] = t_start;
            fb.timeline[TL_STRIDE * b + 1] = __builtin_amdgcn_s_memrealtime();
            fb.timeline[TL_STRIDE * b + 10] = c_start;
            fb.timeline[TL_STRIDE * b + 11] = __builtin_amdgcn_s_memtime();
        }
    }
}

// BIN: a bin-mode batch's setup runs beside its raster, which keeps three workgroups per CU (3 waves x
// 128 VGPRs per SIMD): at 64 VGPRs two setup workgroups fit in the rest instead of one (a few spilled
// registers; C3 0.668 -> 0.646 ms per step).  Scan-mode setups run once the raster drains, where the
// spills only cost (C2 0.279 -> 0.287): they keep five waves per SIMD (96 VGPRs, none spilled; the
// span-walked slivers would take 104 unbounded, four waves).
#ifndef SHS_BIN_SETUP_WAVES
#define SHS_BIN_SETUP_WAVES 8   // (-D...: timing experiments)
#endif
#ifndef SHS_SCAN_SETUP_WAVES
#define SHS_SCAN_SETUP_WAVES 5  // (-D...: timing experiments)
#endif
template <bool KARG, bool BIN>
__global__ __launch_bounds__(256, BIN ? SHS_BIN_SETUP_WAVES : SHS_SCAN_SETUP_WAVES) void k_setup(FrameParams fp, FrameBuffers fb_all, KArgDraws ka) {
    __shared__ GhostScratch s_ghost[4];
    __shared__ uint32_t s_stat[4];
    __shared__ NewBusy s_new;
    __shared__ SliverRecs s_sliv[4];
    setup_item<BIN>(fp, fb_all, draw_table<KARG>(fb_all, ka), (int)blockIdx.x, s_ghost, s_stat, s_new, s_sliv);
}

// ---- k_ghost (ghost_list mode) -----------------------------------------------------------------
// The listed unbounded slivers' tile-clamp pixels: wave w takes items w, w + waves, ... of
// (sliver, slice); each sliver is cut into enough slices that the grid's waves stay busy.  The
// records come from k_setup's stores (identical to the ghost waves' recomputation).
#ifndef SHS_GHOST_BLOCKS
#define SHS_GHOST_BLOCKS 512
#endif
constexpr int GHOST_LIST_BLOCKS = SHS_GHOST_BLOCKS;

// A wave's items are known up front: lane j loads the sliver entry of its j-th next item in one round
// trip.
__global__ __launch_bounds__(256) void k_ghost(FrameParams fp, FrameBuffers fb_all) {
    uint32_t *cnt = fb_all.counters + fp.parity * CSET;
    const int n = (int)min(cnt[C_SLIVER], (uint32_t)fp.n_tris * (uint32_t)fp.n_frames);
    const int waves = (int)gridDim.x * 4, gw = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = __lane_id();
    const int slices = n > 0 ? max(1, min(16, waves / n)) : 1;
    const int n_items = n * slices;
    // the sliver's record is wave-uniform: scalar loads through the constant address space (the records
    // are read-only here), so it occupies SGPRs and the kernel's VGPRs stay few -- it runs beside the
    // previous batch's raster, in the VGPRs the raster leaves free
    typedef const __attribute__((address_space(4))) float ConstF;
    auto record = [&](uint32_t e) {   // e = frame * n_tris + triangle (wave-uniform)
        e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);
        const uint32_t frame = e / (uint32_t)fp.n_tris, tri = e - frame * (uint32_t)fp.n_tris;
        ConstF *src = (ConstF *)(fb_all.recs + (size_t)frame * fp.n_tris + tri);
        ConstF *ext = (ConstF *)(fb_all.rext + (size_t)frame * fp.n_tris + tri);   // stored: a sliver is a ghost
        float h[16], bb[4];
#pragma unroll
        for (int k = 0; k < 16; ++k) h[k] = src[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) bb[k] = ext[k];
        return rec_from_hot(fp, make_float4(h[0], h[1], h[2], h[3]), make_float4(h[4], h[5], h[6], h[7]),
                            make_float4(h[8], h[9], h[10], h[11]), make_float4(h[12], h[13], h[14], h[15]),
                            make_float4(bb[0], bb[1], bb[2], bb[3]));
    };
    for (int base = gw; base < n_items; base += 64 * waves) {   // wave-uniform
        const int mine = base + lane * waves;
        const uint32_t my_e = mine < n_items ? fb_all.slivers[mine / slices] : 0u;
        const int m = min(64, (n_items - base + waves - 1) / waves);
        for (int j = 0; j < m; ++j) {
            const int item = base + j * waves;
            const int s = item / slices, slice = item - s * slices;
            const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)my_e, j));
            const uint32_t frame = e / (uint32_t)fp.n_tris, tri = e - frame * (uint32_t)fp.n_tris;
            const TriRec t = record(e);
            sliver_pixels(fp, frame_view(fp, fb_all, (int)frame), cnt, t, tri, frame, slice, 64 * slices);
        }
    }
}

// ---- k_raster ---------------------------------------------------------------------------------

// Fragment shaders of the four legacy pipelines for the winning triangle, from its per-corner
// varyings.  Returns the pre-truncation floats; the caller truncates to uint8 like the reference.
// du = the draw's {light, cam, ocol, colf} float4s (DrawGPU::light.. or the LDS copy).
// The FS from the interpolated varyings: A = (a0 u + a1 v) + a2 w of the ShadeRec's first three
// vectors (world position / Gouraud colour / Flat normal), N = the same of the normals (Phong,
// Blinn-Phong).  Split from the interpolation so a winner's varyings can be accumulated corner by
// corner in the same operation order (recs_from_mesh's caller).
__device__ __forceinline__ void shade_interp(const float4 (&du)[4], int shading, f3 A, f3 N, float pre[3]) {
    const float4 dl = du[0], dc = du[1], doc = du[2], dcf = du[3];
    if (shading == 0) {
        // Flat FS (flat_shading.cpp:69-98): the interpolated normal is normalised in
        // draw_triangle_tile and again in the FS; intensity = min(0.2 + max(n.l, 0), 1)
        const f3 in_n = normalize3(A);
        const f3 nn = normalize3(in_n);
        const f3 l = {dl.x, dl.y, dl.z};
        const float diffuse = g_max(dot3(nn, l), 0.0f);
        float intensity = 0.2f + diffuse;
        if (intensity > 1.0f) intensity = 1.0f;
        pre[0] = dcf.x * intensity;
        pre[1] = dcf.y * intensity;
        pre[2] = dcf.z * intensity;
        return;
    }
    if (shading == 1) {
        // Gouraud FS (gouraud_shading.cpp:80-89): interpolated colour * 255
        const f3 c = A;
        pre[0] = c.x * 255.0f;
        pre[1] = c.y * 255.0f;
        pre[2] = c.z * 255.0f;
        return;
    }
    // Phong / Blinn-Phong: normal and world position interpolated (blinn_phong_shading.cpp:235-236)
    const f3 in_n = normalize3(N);
    const f3 in_w = A;
    const f3 L = {dl.x, dl.y, dl.z};
    const f3 cam = {dc.x, dc.y, dc.z};
    const f3 norm = normalize3(in_n);
    const f3 viewDir = normalize3(sub3(cam, in_w));
    const float diff = g_max(dot3(norm, L), 0.0f);
    float specular;
    if (shading == 2) {
        // Phong (phong_shading.cpp:70-108): reflect(-L, N) = I - N*dot(N,I)*2, spec 0.8,
        // pow(float, int 32) resolves to std::pow(double, double)
        const f3 I = {-L.x, -L.y, -L.z};
        const float dn = dot3(norm, I);
        const f3 t = sc3(sc3(norm, dn), 2.0f);
        const f3 refl = sub3(I, t);
        const float spec = pow2k<5>(g_max(dot3(viewDir, refl), 0.0f));
        specular = (0.8f * spec) * 1.0f;
    } else {
        // Blinn-Phong (blinn_phong_shading.cpp:63-97): powf(max(N.H,0), 64), spec 0.5
        const f3 half = normalize3(add3(L, viewDir));
        const float spec = pow2k<6>(g_max(dot3(norm, half), 0.0f));
        specular = (0.5f * spec) * 1.0f;
    }
    const f3 oc = {doc.x, doc.y, doc.z};
    const float s = (0.15f + diff * 1.0f) + specular;
    pre[0] = g_clamp01(s * oc.x) * 255.0f;
    pre[1] = g_clamp01(s * oc.y) * 255.0f;
    pre[2] = g_clamp01(s * oc.z) * 255.0f;
}

// The ShadeRec's varyings at barycentrics (u, v, w): A = (a0 u + a1 v) + a2 w, N likewise (Phong,
// Blinn-Phong) -- blinn_phong_shading.cpp:235-236's operation order.
__device__ __forceinline__ void interp_varyings(const ShadeRec &sr, float u, float v, float w, f3 &A, f3 &N) {
    const f3 a0 = {sr.v[0], sr.v[1], sr.v[2]}, a1 = {sr.v[3], sr.v[4], sr.v[5]}, a2 = {sr.v[6], sr.v[7], sr.v[8]};
    A = add3(add3(sc3(a0, u), sc3(a1, v)), sc3(a2, w));
    N = f3{0.0f, 0.0f, 0.0f};
    if (sr.shading >= 2) {
        const f3 n0 = {sr.v[9], sr.v[10], sr.v[11]}, n1 = {sr.v[12], sr.v[13], sr.v[14]}, n2 = {sr.v[15], sr.v[16], sr.v[17]};
        N = add3(add3(sc3(n0, u), sc3(n1, v)), sc3(n2, w));
    }
}

__device__ __forceinline__ void shade_winner(const float4 *du, const ShadeRec &sr, float u, float v, float w, float pre[3]) {
    const float4 d4[4] = {du[0], du[1], du[2], du[3]};
    f3 A, N;
    interp_varyings(sr, u, v, w, A, N);
    shade_interp(d4, sr.shading, A, N, pre);
}

// The draw's {light, cam, ocol, colf} (DrawGPU::light.., or its LDS copy) into registers.
__device__ __forceinline__ void load_du(const float4 *p, float4 (&du)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) du[k] = p[k];
}

// The z test (ZBuffer::test_and_set_depth, strict '<' in submission order) resolves through z_key
// (shs_wave.hpp); NaN and z >= FLT_MAX never pass (never written).

// One (triangle, pixel) test: the pixel is in the reference's visited set for this triangle
// (inside the ibox, or for a bounded ghost where its tile job's clamped rectangle covers it) and
// its barycentrics pass; returns z.  The caller's pixel lies in the triangle's bin box (every raster
// loop walks clipped bin boxes), which is the ibox itself unless the triangle is a ghost: only
// ghosts test the ibox.
__device__ __forceinline__ bool pixel_test(const FrameParams &fp, const TriRec &r, int px, int py, float &z) {
    const bool in_ibox = !(r.flags & TRI_GHOST) ||
                         (px >= lo16(r.ibx) && px <= hi16(r.ibx) && py >= lo16(r.iby) && py <= hi16(r.iby));
    bool test = in_ibox;
    if (!in_ibox && (r.flags & TRI_GHOST)) {
        // draw_triangle_tile's visited rectangle in this pixel's tile job (blinn_phong_shading.cpp:208-224)
        const int rxs = (px / fp.rtw) * fp.rtw, rys = (py / fp.rth) * fp.rth;
        const float rtminx = (float)rxs, rtmaxx = (float)(min(rxs + fp.rtw, fp.W) - 1);
        const float rtminy = (float)rys, rtmaxy = (float)(min(rys + fp.rth, fp.H) - 1);
        const float bminx = g_max(rtminx, g_min(rtmaxx, r.fminx));
        const float bmaxx = g_min(rtmaxx, g_max(rtminx, r.fmaxx));
        const float bminy = g_max(rtminy, g_min(rtmaxy, r.fminy));
        const float bmaxy = g_min(rtmaxy, g_max(rtminy, r.fmaxy));
        test = !(bminx > bmaxx || bminy > bmaxy) && px >= (int)bminx && px <= (int)bmaxx && py >= (int)bminy &&
               py <= (int)bmaxy;
    }
    float u, v, w;
    if (!(test && bary_pass(r, (float)px + 0.5f, (float)py + 0.5f, u, v, w))) return false;
    z = (u * r.z0 + v * r.z1) + w * r.z2;
    return z < FLT_MAX;   // NaN and FLT_MAX never beat the FLT_MAX clear
}

constexpr int RCHUNK = 64;         // candidate records staged per pass (one wave scans their areas)
constexpr int LDS_DRAWS = 64;      // draws whose shading uniforms are kept in LDS
constexpr int PAIR_WORDS = RCHUNK * RTW * RTH / 64;   // pair-start bitmap words (a box is <= 256 px)
constexpr uint32_t SLOT_NONE = 127u;                  // key slot field: winner not staged in LDS

// Candidate key: z_key with the low word (id << 7 | staging slot) when ids fit in 25 bits.  The order
// is still (z, id) -- a triangle has one slot per tile -- and the slot lets the resolve read the
// winner's records from LDS instead of HBM.  SLOT_NONE (multi-pass tiles, ghost fragments): HBM.
__device__ __forceinline__ unsigned long long cand_key(float z, uint32_t id, bool slot_keys, uint32_t slot) {
    return z_key(z, slot_keys ? (id << 7) | slot : id);
}

struct RasterShared {
    float4 rec[RCHUNK * 4];           // staged triangle records (TriHot, 4 KB)
    float4 ext[RCHUNK];               // ... their float bboxes (ghosts; every candidate in scan mode, 1 KB)
    float4 srec[RCHUNK * 5];          // staged shading records (single-pass tiles, 5 KB)
    unsigned long long key[RTH * RTW];// per-pixel (z, index) keys (2 KB)
    unsigned long long bits[PAIR_WORDS]; // bit k: a staged candidate's pairs start at pair k (2 KB)
    uint32_t seg[RCHUNK * RTH];       // spans: per nonempty row span, first pair | x0 << 14 | row << 19 | candidate << 22
    uint4 pinfo[RCHUNK];              // boxes: per staged candidate first pair, x0 | y0 << 16, box width, 2^16/width
    uint32_t wtot[4];                 // per wave: pairs << 11 | segments (the staging pass's block prefix)
    uint32_t id[RCHUNK];
    uint32_t cand[CAND];
    float4 du[LDS_DRAWS * 4];         // per-draw {light, cam, ocol, colf} (4 KB)
    uint8_t skip[512];                // clear strip: per raster tile across, 1 = not cleared (busy / not owned)
    uint32_t nc, item, cov, maxbin, npairs;
    uint16_t wown[PAIR_WORDS];        // segment (boxes: staged candidate) owning each bitmap word's first pair
};

// The record rebuilt from the screen corners with the stored flags and bin box: rec_from_screen's
// float arithmetic (the Gram terms, z, float bbox, integer bbox) without danger_margin -- its only
// outputs, the flags and the bin box, come from k_setup.  Candidates are never culled (their bin box
// is non-empty), so the integer bbox is always the clamped floor.
__device__ __forceinline__ TriRec rec_from_stored(const FrameParams &fp, int draw, int local, const float (&sx)[3],
                                                  const float (&sy)[3], const float (&sz)[3], uint32_t flags, uint2 gbox) {
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
    r.flags = flags;
    r.ibx = pack16(floor_clamped(r.fminx, 0, fp.W), floor_clamped(r.fmaxx, -1, fp.W - 1));
    r.iby = pack16(floor_clamped(r.fminy, 0, fp.H), floor_clamped(r.fmaxy, -1, fp.H - 1));
    r.gbx = gbox.x; r.gby = gbox.y;
    return r;
}

// RF_NO_RECS (binned frames): staged candidate `id`'s record -- and for single-pass tiles its shading
// varyings -- recomputed from the resident mesh by the quad of lanes 4c .. 4c + 3 exactly as k_setup's
// setup_quad computes them (same functions, same operands: identical bits), into the LDS copies.
// fdraws: the frame's draw slice (batch table entries dbase ..).
__device__ __forceinline__ void stage_from_mesh(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *fdraws, int dbase,
                                                uint32_t id, bool shade, float4 *rec, float4 *ext, float4 *srec) {
    const int q = __lane_id() & 3, qv = q < 3 ? q : 2;
    const uint32_t word = (uint32_t)fb.tdraw[id];
    const uint2 gbox = fb.boxes[id];
    const int d = (int)(word & 0x1fffffffu);
    const DrawGPU &dr = fdraws[d];
    const int local = (int)id - dr.tri_base;
    const float *P = dr.pos + 9 * (size_t)local + 3 * qv;
    const float p3[3] = {P[0], P[1], P[2]};
    float n3[3] = {0.0f, 0.0f, 0.0f};
    if (shade) {
        const float *Nn = dr.nrm + 9 * (size_t)local + 3 * qv;
        n3[0] = Nn[0]; n3[1] = Nn[1]; n3[2] = Nn[2];
    }
    float vx, vy, vz;
    vertex_screen(fp, dr.mvp, p3[0], p3[1], p3[2], vx, vy, vz);
    float sx[3], sy[3], sz[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { sx[k] = quad_bcast(vx, k); sy[k] = quad_bcast(vy, k); sz[k] = quad_bcast(vz, k); }
    const TriRec r = rec_from_stored(fp, d, local, sx, sy, sz, word >> 29, gbox);
    quad_store_hot(rec, ext, r, true);
    if (shade) {
        f3 a, nr;
        corner_varyings(dr, p3, n3, a, nr);
        quad_store_shade_at(reinterpret_cast<ShadeRec *>(srec), dbase + d, dr.shading, a, nr);
    }
}

// RF_NO_RECS: one thread's winner (tiles whose winners are not staged: several staging passes, ghost
// fragments) re-evaluated from the mesh -- the record's barycentric terms, the pixel's (u, v, w) and
// depth, then the corners' varyings accumulated one corner at a time in shade_winner's operation order
// ((a0 u + a1 v) + a2 w) -- and shaded.  draws: the batch table; dbase: the frame's slice.
__device__ __forceinline__ void resolve_from_mesh(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *draws, int dbase,
                                                  uint32_t id, int px, int py, const float4 *lds_du, bool shade, float &depth,
                                                  f3 &A, f3 &N, int &shading, float4 (&du)[4]) {
    const int d = (int)((uint32_t)fb.tdraw[id] & 0x1fffffffu);
    const DrawGPU &dr = draws[dbase + d];
    const int local = (int)id - dr.tri_base;
    const float *P = dr.pos + 9 * (size_t)local;
    float u, v, w;
    {
        float sx[3], sy[3], sz[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) vertex_screen(fp, dr.mvp, P[3 * k], P[3 * k + 1], P[3 * k + 2], sx[k], sy[k], sz[k]);
        const TriRec r = rec_from_stored(fp, d, local, sx, sy, sz, 0u, make_uint2(0u, 0u));
        bary_pass(r, (float)px + 0.5f, (float)py + 0.5f, u, v, w);   // the winner's own values
        depth = (u * r.z0 + v * r.z1) + w * r.z2;
    }
    if (!shade) return;
    const float *Nn = dr.nrm + 9 * (size_t)local;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float p3[3] = {P[3 * k], P[3 * k + 1], P[3 * k + 2]};
        const float n3[3] = {Nn[3 * k], Nn[3 * k + 1], Nn[3 * k + 2]};
        f3 a, nr;
        corner_varyings(dr, p3, n3, a, nr);
        const float b = k == 0 ? u : k == 1 ? v : w;
        A = k == 0 ? sc3(a, b) : add3(A, sc3(a, b));
        N = k == 0 ? sc3(nr, b) : add3(N, sc3(nr, b));
    }
    const int bd = dbase + d;
    if (bd < LDS_DRAWS) load_du(&lds_du[bd * 4], du);
    else load_du(reinterpret_cast<const float4 *>(dr.light), du);
    shading = dr.shading;
}

// One busy raster tile.  Candidates (bin box overlaps the tile) are staged in LDS; every (candidate,
// pixel of its clipped bin box) pair is one lane-task, dealt evenly over the workgroup by a prefix
// sum of the box areas; passing pairs atomic-min their key into the tile's LDS key array.  Then
// each thread owns one pixel: the winner's record and varyings are fetched by index, (u, v, w)
// recomputed with the identical arithmetic, the pixel shaded and written.
// fb: the frame's view (frame_view); draws: the whole batch's draw table; rt: raster tile of the frame.
// SCAN: the frame's candidate source -- 0 binned, 1 scan mode (every bin box), 2 fp.scan_mode at run
// time (the per-pixel kernels and k_pipe).
constexpr int SCAN_BINNED = 0, SCAN_ALL = 1, SCAN_RUNTIME = 2;
template <bool NO_RECS, bool SPANS, bool PIX, int SCAN>
__device__ __forceinline__ void raster_tile(const FrameParams &fp, const FrameBuffers &fb, const DrawGPU *draws,
                                            const uint32_t *cnt, uint32_t n_frag, int frame, int rt,
                                            RasterShared &sh, uint64_t *tl) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tls = fp.setup_grid + (int)blockIdx.x;
    const int col = rt % fp.tiles_x, row = rt / fp.tiles_x;
    const int X0 = col * RTW, Y0 = row * RTH;
    const int X1 = X0 + RTW - 1, Y1 = Y0 + RTH - 1;
    const int bt = (row / (TILE / RTH)) * fp.tiles_x + col;
    const int bt_spill = frame * fp.tiles_x * fp.tiles_y + bt;   // the bin tile's key in spill entries
    constexpr bool no_recs = NO_RECS;   // == (fp.flags & RF_NO_RECS): a kernel variant each
    const bool scan = SCAN == SCAN_RUNTIME ? fp.scan_mode != 0u : SCAN == SCAN_ALL;
    const int dbase = frame * fp.n_draws;                       // the frame's slice of the draw table

    // candidate sources.  scan mode: every triangle's bin box.  bin mode: the bin tile's list, then
    // the spill list (entries of this bin tile).
    uint32_t n_bin_total = 0, n_bin = 0, n_spill = 0, n_items;
    if (scan) {
        n_items = (uint32_t)fp.n_tris;
    } else {
        n_bin_total = fb.tile_count[bt];
        n_bin = n_bin_total < fp.bin_cap ? n_bin_total : fp.bin_cap;
        if (n_bin_total > fp.bin_cap) n_spill = min(cnt[C_SPILL], fp.spill_cap);
        n_items = n_bin + n_spill;
        if (tid == 0) sh.maxbin = max(sh.maxbin, n_bin_total);
    }
    // the previous tile's key resets (each thread its own pixel) precede every shared write of this
    // one: a candidate round starts with a barrier; without one, the ghost fragments below need it
    if (n_items == 0u) __syncthreads();
    const uint32_t *bin = fb.bins + (size_t)bt * fp.bin_cap;
    uint32_t seq = 0;   // candidates processed (profiling)
    int pairs = 0;      // (candidate, pixel) tasks (profiling)
    unsigned long long kmin = KEY_EMPTY;   // per-pixel loop: this thread's pixel key
    const bool slot_keys = fp.n_tris < (1 << 25);
    bool single = n_items <= (uint32_t)CAND;   // one gather round and one staging pass: winners in LDS

    for (uint32_t base = 0; base < n_items; base += CAND) {
        __syncthreads();
        if (tid == 0) sh.nc = 0;
        __syncthreads();
        // gather up to CAND candidate ids (4 independent loads per thread, one round trip)
        uint32_t ids[CAND / 256];
        uint2 bx[CAND / 256];
#pragma unroll
        for (int k = 0; k < CAND / 256; ++k) {
            const uint32_t item = base + tid + 256u * k;
            uint32_t id = 0xffffffffu;
            if (item < n_items) {
                if (scan) {
                    id = item;
                } else if (item < n_bin) {
                    id = bin[item];
                } else {
                    const uint2 e = fb.spill[item - n_bin];
                    if ((int)e.x == bt_spill) id = e.y;
                }
            }
            ids[k] = id;
        }
#pragma unroll
        for (int k = 0; k < CAND / 256; ++k) bx[k] = ids[k] != 0xffffffffu ? fb.boxes[ids[k] & ~BIN_GHOST] : make_uint2(0u, 0u);
#pragma unroll
        for (int k = 0; k < CAND / 256; ++k) {
            // non-empty bin box overlapping the tile (so its clipped box holds >= 1 pixel: the pair
            // mapping below relies on it; off-screen triangles have empty boxes like [W, W-1])
            const int gx0 = lo16(bx[k].x), gx1 = hi16(bx[k].x), gy0 = lo16(bx[k].y), gy1 = hi16(bx[k].y);
            const bool hit = ids[k] != 0xffffffffu && gx0 <= gx1 && gy0 <= gy1 && gx1 >= X0 && gx0 <= X1 && gy1 >= Y0 &&
                             gy0 <= Y1;
            const uint64_t m = __ballot(hit);
            uint32_t basew = 0;
            if (lane == 0 && m) basew = atomicAdd(&sh.nc, (uint32_t)__popcll(m));
            basew = __shfl(basew, 0);
            if (hit) sh.cand[basew + lanes_below(m)] = ids[k];
        }
        __syncthreads();
        tl_mark(tl, tls, 1);
        const uint32_t nc = sh.nc;
        single = single && nc <= (uint32_t)RCHUNK;
        for (uint32_t c = 0; c < nc; c += RCHUNK) {
            const int m = (int)min((uint32_t)RCHUNK, nc - c);
            if (c > 0) __syncthreads();
            // stage records (single-pass tiles: the shading records too, so the resolve reads no HBM):
            // consecutive lanes load consecutive float4s of one record; all loads in one round trip
            if (tid < m) sh.id[tid] = sh.cand[c + tid] & ~BIN_GHOST;
            for (int i = tid; i < m * (RTW * RTH / 64); i += 256) sh.bits[i] = 0ull;
            if constexpr (no_recs) {   // a quad of lanes per candidate (RCHUNK * 4 == 256)
                const int ci = tid >> 2;
                if (ci < m)
                    stage_from_mesh(fp, fb, draws + dbase, dbase, sh.cand[c + ci] & ~BIN_GHOST, single, &sh.rec[ci * 4], &sh.ext[ci],
                                    &sh.srec[ci * 5]);
            } else {
                // (the float bbox only for ghosts -- tagged entries -- or every candidate in scan mode)
                constexpr int NQ = (RCHUNK * 4 + 255) / 256, NS = (RCHUNK * 5 + 255) / 256;
                float4 q[NQ], s[NS], e = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int k = 0; k < NQ; ++k) {
                    const int f = tid + 256 * k;
                    const int ci = f >> 2;
                    q[k] = f < 4 * m ? reinterpret_cast<const float4 *>(&fb.recs[sh.cand[c + min(ci, m - 1)] & ~BIN_GHOST])[f & 3]
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                {
                    const uint32_t ce = tid < m ? sh.cand[c + tid] : 0u;
                    if (tid < m && (scan || (ce & BIN_GHOST))) e = fb.rext[ce & ~BIN_GHOST];
                }
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const int f = tid + 256 * k;
                    const int ci = f / 5;
                    s[k] = single && f < 5 * m ? reinterpret_cast<const float4 *>(&fb.shade[sh.cand[min(ci, m - 1)] & ~BIN_GHOST])[f - 5 * ci]
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
                }
#pragma unroll
                for (int k = 0; k < NQ; ++k) {
                    const int f = tid + 256 * k;
                    if (f < 4 * m) sh.rec[f] = q[k];
                }
                if (tid < m) sh.ext[tid] = e;
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const int f = tid + 256 * k;
                    if (single && f < 5 * m) sh.srec[f] = s[k];
                }
            }
            __syncthreads();
            tl_mark(tl, tls, 2);
            if ((PIX || NO_RECS) && (fp.flags & RF_PER_PIXEL)) {   // (PIX: the per-pixel loop compiled in)
                // Per-pixel loop: every thread tests its own pixel against the staged candidates in
                // order (LDS broadcast reads, the key min kept in a register).  A wave owns two tile
                // rows and skips a candidate whose box misses them as a whole.
                const int px = X0 + (tid & 31), py = Y0 + (tid >> 5);
                const int wy0 = Y0 + 2 * wave, wy1 = wy0 + 1;
                for (int cc = 0; cc < m; ++cc) {
                    const uint4 bb = reinterpret_cast<const uint4 *>(&sh.rec[cc * 4])[3];   // z2 word gbx gby
                    const int x0 = lo16(bb.z), x1 = hi16(bb.z), y0 = lo16(bb.w), y1 = hi16(bb.w);
                    if (y1 < wy0 || y0 > wy1) continue;                                     // wave-uniform
                    if (px < x0 || px > x1 || py < y0 || py > y1) continue;
                    const TriRec r = rec_from_hot(fp, &sh.rec[cc * 4], &sh.ext[cc]);
                    float z;
                    if (pixel_test(fp, r, px, py, z)) {
                        const unsigned long long k = cand_key(z, sh.id[cc], slot_keys, single ? (uint32_t)cc : SLOT_NONE);
                        kmin = k < kmin ? k : kmin;
                    }
                }
                seq += (uint32_t)m;
                continue;
            }
            if constexpr (SPANS) {
                // Pair tasks over conservative row spans (legacy_row_span), dealt evenly over the workgroup:
                // thread (ci = tid / 4, q = tid % 4) takes staged candidate ci's tile rows 2q and 2q + 1; their
                // spans inside its clipped bin box are laid end to end as segments after one block prefix of
                // (pairs, segments), and each segment's first pair is marked in a bitmap over the pairs, plus
                // the segment owning every bitmap word's first pair.  Wave w then takes the 64-pair windows w,
                // w + 4, ...: a pair's segment = that word's first owner + the starts in the word up to it.
                // (Whole bin boxes made ~2,600 pairs for ~42 candidates per C3 tile: thin triangles' boxes are
                // mostly empty.)
                uint32_t ptot = 0u;
                {
                    const int ci = tid >> 2, q = tid & 3;
                    uint32_t spw[2] = {0x1fu, 0x1fu};   // tile-relative x0 | x1 << 8; 0x1f: empty
                    uint32_t pk = 0u;                   // pairs << 11 | segments
                    if (ci < m) {
                        const float4 *rc = &sh.rec[ci * 4];
                        const uint4 bb = reinterpret_cast<const uint4 *>(rc)[3];   // z2 word gbx gby
                        const int x0 = max(lo16(bb.z), X0), x1 = min(hi16(bb.z), X1);
                        const int y0 = max(lo16(bb.w), Y0), y1 = min(hi16(bb.w), Y1);
                        if (x0 <= x1 && y0 <= y1) {
                            const float4 r0 = rc[0], r1 = rc[1], r2 = rc[2];
    #pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                const int py = Y0 + 2 * q + j;
                                if (py < y0 || py > y1) continue;
                                int s0, s1;
                                legacy_row_span(r0, r1, r2, py, x0, x1, s0, s1);
                                if (s1 < s0) continue;
                                spw[j] = (uint32_t)(s0 - X0) | ((uint32_t)(s1 - X0) << 8);
                                pk += ((uint32_t)(s1 - s0 + 1) << 11) + 1u;
                            }
                        }
                    }
                    uint32_t incl = pk;
    #pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const uint32_t vv = (uint32_t)__shfl_up((int)incl, o);
                        if (lane >= o) incl += vv;
                    }
                    if (lane == 63) sh.wtot[wave] = incl;
                    __syncthreads();
                    uint32_t pbase = 0u;
    #pragma unroll
                    for (int w2 = 0; w2 < 4; ++w2) {
                        const uint32_t p2 = sh.wtot[w2];
                        if (w2 < wave) pbase += p2;
                        ptot += p2;
                    }
                    if (pk) {
                        const uint32_t ex = pbase + incl - pk;
                        uint32_t ps = ex >> 11, sg = ex & 2047u;
    #pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (spw[j] == 0x1fu) continue;
                            const uint32_t s0 = spw[j] & 0xffu, wdt = (spw[j] >> 8) - s0 + 1u;
                            sh.seg[sg] = ps | (s0 << 14) | ((uint32_t)(2 * q + j) << 19) | ((uint32_t)ci << 22);
                            atomicOr(&sh.bits[ps >> 6], 1ull << (ps & 63u));
                            for (uint32_t wd = (ps + 63u) >> 6; wd * 64u < ps + wdt; ++wd) sh.wown[wd] = (uint16_t)sg;
                            ps += wdt;
                            ++sg;
                        }
                    }
                }
                __syncthreads();
                const int total = SHS_DBG(fp, DBG_SKIP_PAIRS) ? 0 : (int)(ptot >> 11);
                pairs += total;
                for (int k0 = 64 * wave; k0 < total; k0 += 256) {
                    const int k = k0 + lane;
                    if (k < total) {
                        const unsigned long long wb = sh.bits[k0 >> 6];
                        const unsigned long long upto = ((2ull << lane) - 1ull) & ~1ull;   // bits 1..lane
                        const int o = (int)sh.wown[k0 >> 6] + __popcll(wb & upto);
                        const uint32_t sgi = sh.seg[o];
                        const int cc = (int)(sgi >> 22);
                        const int px = X0 + (int)((sgi >> 14) & 31u) + (k - (int)(sgi & 0x3fffu)), py = Y0 + (int)((sgi >> 19) & 7u);
                        const TriRec r = rec_from_hot(fp, &sh.rec[cc * 4], &sh.ext[cc]);
                        float z;
                        if (pixel_test(fp, r, px, py, z))
                            atomicMin(&sh.key[(py - Y0) * RTW + (px - X0)],
                                      cand_key(z, sh.id[cc], slot_keys, single ? (uint32_t)cc : SLOT_NONE));
                    }
                }
            } else {
                // (scan-mode frames: whole clipped bin boxes -- C2's Suzanne triangles fill most of their boxes,
                // and the spans measured slower there: 0.271 -> 0.278 ms per step)
                // Pair tasks, dealt evenly over the workgroup.  Wave 0 lays the staged candidates' clipped
                // bin boxes end to end (prefix of the areas; every staged box holds >= 1 pixel of the tile,
                // so the starts are distinct) and marks each start in a bitmap over the pairs, plus the
                // owner of every bitmap word's first pair.  Wave w then takes the 64-pair windows w, w + 4,
                // ...: a pair's owner = that word's first owner + the starts in the word up to it.
                if (wave == 0) {
                    int area = 0, bx0 = 0, by0 = 0, bw = 1;
                    if (lane < m) {
                        const uint4 bb = reinterpret_cast<const uint4 *>(&sh.rec[lane * 4])[3];   // z2 word gbx gby
                        const int x0 = max(lo16(bb.z), X0), x1 = min(hi16(bb.z), X1);
                        const int y0 = max(lo16(bb.w), Y0), y1 = min(hi16(bb.w), Y1);
                        if (x0 <= x1 && y0 <= y1) { area = (x1 - x0 + 1) * (y1 - y0 + 1); bx0 = x0; by0 = y0; bw = x1 - x0 + 1; }
                    }
                    int incl = area;
    #pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int v = __shfl_up(incl, o);
                        if (lane >= o) incl += v;
                    }
                    const int start = incl - area;
                    if (area > 0) {
                        // 2^16 / width rounded up: (local * magic) >> 16 == local / width for local < 256
                        sh.pinfo[lane] = make_uint4((uint32_t)start, (uint32_t)bx0 | ((uint32_t)by0 << 16), (uint32_t)bw,
                                                    (65536u + (uint32_t)bw - 1u) / (uint32_t)bw);
                        atomicOr(&sh.bits[start >> 6], 1ull << (start & 63));
                        for (int wd = (start + 63) >> 6; wd * 64 < incl; ++wd) sh.wown[wd] = (uint16_t)lane;
                    }
                    if (lane == 63) sh.npairs = (uint32_t)incl;
                }
                __syncthreads();
                const int total = SHS_DBG(fp, DBG_SKIP_PAIRS) ? 0 : (int)sh.npairs;
                pairs += total;
                for (int k0 = 64 * wave; k0 < total; k0 += 256) {
                    const int k = k0 + lane;
                    if (k < total) {
                        const unsigned long long wb = sh.bits[k0 >> 6];
                        const unsigned long long upto = ((2ull << lane) - 1ull) & ~1ull;   // bits 1..lane
                        const int o = (int)sh.wown[k0 >> 6] + __popcll(wb & upto);
                        const uint4 pi = sh.pinfo[o];
                        const int local = k - (int)pi.x;
                        const int ly = (int)(((uint32_t)local * pi.w) >> 16), lx = local - ly * (int)pi.z;
                        const int px = (int)(pi.y & 0xffffu) + lx, py = (int)(pi.y >> 16) + ly;
                        const TriRec r = rec_from_hot(fp, &sh.rec[o * 4], &sh.ext[o]);
                        float z;
                        if (pixel_test(fp, r, px, py, z))
                            atomicMin(&sh.key[(py - Y0) * RTW + (px - X0)],
                                      cand_key(z, sh.id[o], slot_keys, single ? (uint32_t)o : SLOT_NONE));
                    }
                }
            }
            seq += (uint32_t)m;
        }
    }
    tl_mark(tl, tls, 3);
    // tile-clamp pixels of unbounded slivers outside their bbox that passed (k_setup ghost waves)
    {
        for (uint32_t f = tid; f < n_frag; f += 256) {
            const GhostFrag g = fb.frags[f];
            const int gx = (int)(g.xy & 0xffffu), gy = (int)(g.xy >> 16);
            if (g.frame == (uint32_t)frame && gx >= X0 && gx <= X1 && gy >= Y0 && gy <= Y1)
                atomicMin(&sh.key[(gy - Y0) * RTW + (gx - X0)], cand_key(g.z, g.id, slot_keys, SLOT_NONE));
        }
    }
    __syncthreads();

    // one pixel per thread: resolve, shade the winner, write (rows of 32 px: 128-B segments)
    const int px = X0 + (tid & 31), py = Y0 + (tid >> 5);
    const unsigned long long lkey = sh.key[tid];
    const unsigned long long key = lkey < kmin ? lkey : kmin;
    sh.key[tid] = KEY_EMPTY;   // clean for the next tile (read above, by this thread only)
    uint32_t rgba = fp.clear_rgba;
    float depth = FLT_MAX;
    float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool covered = key != KEY_EMPTY && px < fp.W && py < fp.H;
    if (covered) {
        const uint32_t lo = (uint32_t)key;
        const uint32_t id = slot_keys ? lo >> 7 : lo, slot = slot_keys ? lo & SLOT_NONE : SLOT_NONE;
        if constexpr (!no_recs) {   // stored records: the staged copies (single-pass tiles) or HBM
            TriRec r;
            ShadeRec sr;
            {
                float4 h4[4];   // the winner's stored record (its float bbox is not read here)
                float4 *e4 = reinterpret_cast<float4 *>(&sr);
                if (slot != SLOT_NONE) {   // only single-pass tiles encode a slot: the staged copies
#pragma unroll
                    for (int k = 0; k < 4; ++k) h4[k] = sh.rec[slot * 4 + k];
#pragma unroll
                    for (int k = 0; k < 5; ++k) e4[k] = sh.srec[slot * 5 + k];
                } else {
                    const float4 *s4 = reinterpret_cast<const float4 *>(&fb.recs[id]);
                    const float4 *g4 = reinterpret_cast<const float4 *>(&fb.shade[id]);
#pragma unroll
                    for (int k = 0; k < 4; ++k) h4[k] = s4[k];
#pragma unroll
                    for (int k = 0; k < 5; ++k) e4[k] = g4[k];
                }
                r = rec_from_hot(fp, h4[0], h4[1], h4[2], h4[3], make_float4(0.f, 0.f, 0.f, 0.f));
            }
            float u, v, w;
            bary_pass(r, (float)px + 0.5f, (float)py + 0.5f, u, v, w);   // the winner's own values
            depth = (u * r.z0 + v * r.z1) + w * r.z2;
            if (!SHS_DBG(fp, DBG_SKIP_SHADE)) {
                const int wd = dbase + r.draw;   // the frame's draw (ShadeRec::draw is frame 0's when shared)
                const float4 *du = wd < LDS_DRAWS ? &sh.du[wd * 4] : reinterpret_cast<const float4 *>(draws[wd].light);
                float pre[3];
                shade_winner(du, sr, u, v, w, pre);
                const uint32_t cr = (uint32_t)(uint8_t)pre[0], cg = (uint32_t)(uint8_t)pre[1], cb = (uint32_t)(uint8_t)pre[2];
                rgba = cr | (cg << 8) | (cb << 16) | (255u << 24);
                pq = make_float4(pre[0], pre[1], pre[2], 1.0f);
            }
        } else {
            const bool shade = !SHS_DBG(fp, DBG_SKIP_SHADE);
            f3 A = {0.f, 0.f, 0.f}, N = {0.f, 0.f, 0.f};   // interpolated varyings (shade_interp's inputs)
            int shading = 0;
            float4 du[4];
            if (no_recs && slot == SLOT_NONE) {   // binned frame, winner not staged: recomputed from the mesh
                resolve_from_mesh(fp, fb, draws, dbase, id, px, py, sh.du, shade, depth, A, N, shading, du);
            } else {
                TriRec r;
                ShadeRec sr;
                {
                    float4 h4[4];   // the winner's stored record (its float bbox is not read here)
                    float4 *e4 = reinterpret_cast<float4 *>(&sr);
                    if (slot != SLOT_NONE) {   // only single-pass tiles encode a slot: the staged copies
    #pragma unroll
                        for (int k = 0; k < 4; ++k) h4[k] = sh.rec[slot * 4 + k];
    #pragma unroll
                        for (int k = 0; k < 5; ++k) e4[k] = sh.srec[slot * 5 + k];
                    } else {
                        const float4 *s4 = reinterpret_cast<const float4 *>(&fb.recs[id]);
                        const float4 *g4 = reinterpret_cast<const float4 *>(&fb.shade[id]);
    #pragma unroll
                        for (int k = 0; k < 4; ++k) h4[k] = s4[k];
    #pragma unroll
                        for (int k = 0; k < 5; ++k) e4[k] = g4[k];
                    }
                    r = rec_from_hot(fp, h4[0], h4[1], h4[2], h4[3], make_float4(0.f, 0.f, 0.f, 0.f));
                }
                float u, v, w;
                bary_pass(r, (float)px + 0.5f, (float)py + 0.5f, u, v, w);   // the winner's own values
                depth = (u * r.z0 + v * r.z1) + w * r.z2;
                if (shade) {
                    const int wd = dbase + r.draw;   // the frame's draw (ShadeRec::draw is frame 0's when shared)
                    if (wd < LDS_DRAWS) load_du(&sh.du[wd * 4], du);
                    else load_du(reinterpret_cast<const float4 *>(draws[wd].light), du);
                    shading = sr.shading;
                    interp_varyings(sr, u, v, w, A, N);
                }
            }
            if (shade) {
                float pre[3];
                shade_interp(du, shading, A, N, pre);
                const uint32_t cr = (uint32_t)(uint8_t)pre[0], cg = (uint32_t)(uint8_t)pre[1], cb = (uint32_t)(uint8_t)pre[2];
                rgba = cr | (cg << 8) | (cb << 16) | (255u << 24);
                pq = make_float4(pre[0], pre[1], pre[2], 1.0f);
            }
        }
        }
    tl_mark(tl, tls, 4);
    if (tl && tid == 0) { tl[TL_STRIDE * tls + 8] = seq; tl[TL_STRIDE * tls + 9] = (uint64_t)pairs; }
    const uint64_t cm = __ballot(covered);
    if (lane == 0 && cm) atomicAdd(&sh.cov, (uint32_t)__popcll(cm));
    // (DBG_SKIP_TILE_STORES, timing experiments: the busy tile's stores dropped, its values kept live)
    const bool dbg_nost = SHS_DBG(fp, DBG_SKIP_TILE_STORES) && !(rgba == 0x12345678u && depth == -1.0f);
    if (px < fp.W && py < fp.H && !dbg_nost) {
        LEGACY_STORE(rgba, &reinterpret_cast<uint32_t *>(fb.color)[(size_t)(fp.H - 1 - py) * fp.W + px]);
        LEGACY_STORE(depth, &fb.depth[(size_t)py * fp.W + px]);
        if (fb.prequant) fb.prequant[(size_t)(fp.H - 1 - py) * fp.W + px] = pq;
        // copy_to_SDLSurface: surface row h-1-y takes canvas row y, i.e. the screen row
        if (fb.present) LEGACY_STORE(rgba, &fb.present[(size_t)py * fp.W + px]);
    }
    tl_mark(tl, tls, 5);
}

// A tile with no candidates: the clear, one pixel per thread (rows of 32 px: 128-B segments).
__device__ __forceinline__ void clear_tile(const FrameParams &fp, const FrameBuffers &fb, int rt) {
    const int tid = threadIdx.x;
    const int col = rt % fp.tiles_x, row = rt / fp.tiles_x;
    const int px = col * RTW + (tid & 31), py = row * RTH + (tid >> 5);
    if (px < fp.W && py < fp.H) {
        const size_t c = (size_t)(fp.H - 1 - py) * fp.W + px;
        LEGACY_STORE(fp.clear_rgba, &reinterpret_cast<uint32_t *>(fb.color)[c]);
        LEGACY_STORE(FLT_MAX, &fb.depth[(size_t)py * fp.W + px]);
        if (fb.prequant) fb.prequant[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (fb.present) LEGACY_STORE(fp.clear_rgba, &fb.present[(size_t)py * fp.W + px]);
    }
}

// One clear strip: raster-tile row ry of frame f, full width -- every pixel of the row's tiles that
// are owned and not busy gets the clear colour (canvas rows) and FLT_MAX (screen rows), as 16-B
// stores (4 pixels per lane) along whole rows when W % 4 == 0.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void clear_strip(const FrameParams &fp, const FrameBuffers &fb, int f, int ry) {
    // No barrier and no LDS: each thread looks up the busy flag / ownership of the 32-px tile its
    // 4-px column group lies in and writes that group down the strip's rows.
    const int tid = threadIdx.x;
    const FrameBuffers fv = frame_view(fp, fb, f);
    const int y0 = ry * RTH, y1 = min(y0 + RTH, fp.H);
    const int by = ry / (TILE / RTH);
    uint32_t *color = reinterpret_cast<uint32_t *>(fv.color);
    if ((fp.W & 3) == 0) {
        const int ng = fp.W >> 2;
        const u32x4 c4 = {fp.clear_rgba, fp.clear_rgba, fp.clear_rgba, fp.clear_rgba};
        const f32x4 d4 = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
        for (int g = tid; g < ng; g += 256) {
            const int t = g >> 3;   // 8 groups of 4 px per 32-px tile
            if (fv.busy[ry * fp.tiles_x + t] == fp.epoch || (fp.count > 1 && !owned_bin_tile(fp, t, by))) continue;
            for (int y = y0; y < y1; ++y) {
                LEGACY_STORE(c4, &reinterpret_cast<u32x4 *>(color + (size_t)(fp.H - 1 - y) * fp.W)[g]);
                LEGACY_STORE(d4, &reinterpret_cast<f32x4 *>(fv.depth + (size_t)y * fp.W)[g]);
                if (fv.present) LEGACY_STORE(c4, &reinterpret_cast<u32x4 *>(fv.present + (size_t)y * fp.W)[g]);
                if (fv.prequant) {
                    float4 *pq = fv.prequant + (size_t)(fp.H - 1 - y) * fp.W + 4 * g;
                    pq[0] = pq[1] = pq[2] = pq[3] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
    } else {
        for (int x = tid; x < fp.W; x += 256) {
            const int t = x >> 5;
            if (fv.busy[ry * fp.tiles_x + t] == fp.epoch || (fp.count > 1 && !owned_bin_tile(fp, t, by))) continue;
            for (int y = y0; y < y1; ++y) {
                const size_t c = (size_t)(fp.H - 1 - y) * fp.W + x;
                LEGACY_STORE(fp.clear_rgba, &color[c]);
                LEGACY_STORE(FLT_MAX, &fv.depth[(size_t)y * fp.W + x]);
                if (fv.prequant) fv.prequant[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (fv.present) LEGACY_STORE(fp.clear_rgba, &fv.present[(size_t)y * fp.W + x]);
            }
        }
    }
}

// Raster-tile rows per clear item.  Eight (a 64-row strip of one frame) against two: C2 0.275 ->
// 0.272 ms per step in five A/B pairs, C3 unchanged.  The k_raster event grows (C2 0.242 -> 0.248 ms),
// but fewer, longer strip items let the next batch's setup take CUs sooner; 16 rows was slower
// (0.287 ms), 6 or 12 no better.  -DSHS_STRIP_RT=...: timing experiments.
#ifndef SHS_STRIP_RT
#define SHS_STRIP_RT 8
#endif
constexpr int STRIP_RT = SHS_STRIP_RT;

// Persistent raster over the whole batch.  Work items are the busy tiles (the busy list k_setup /
// k_ghost built: latency-bound raster) and the clear strips (one raster-tile row of one frame:
// streaming stores), interleaved in proportion so that every CU mixes both kinds at all times.
// Workgroup b's first item is b (no atomic: a single frame needs none); the rest come from N_WORKQ
// ticket queues -- queue q deals items G + q + N_WORKQ * j to the workgroups b = q (mod N_WORKQ) --
// fetched one item ahead.  Every owned pixel of every frame is written exactly once: by its busy
// tile or by its strip.
#ifndef SHS_LEGACY_RASTER_WAVES
#define SHS_LEGACY_RASTER_WAVES 4   // minimum waves per SIMD (-D...: timing experiments)
#endif
template <bool KARG, bool NO_RECS, bool SPANS, bool PIX, int SCAN>
__global__ __launch_bounds__(256, SHS_LEGACY_RASTER_WAVES) void k_raster(FrameParams fp, FrameBuffers fb, KArgDraws ka) {
    __shared__ RasterShared sh;
    const int tid = threadIdx.x;
    uint32_t *cnt = fb.counters + fp.parity * CSET;
    const DrawGPU *draws = draw_table<KARG>(fb, ka);
    const int n_rt = fp.tiles_x * fp.rtiles_y;            // raster tiles per frame
    const uint64_t t_start = fb.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint64_t c_start = fb.timeline ? __builtin_amdgcn_s_memtime() : 0ull;
    if (tid == 0) { sh.cov = 0; sh.maxbin = 0; }
    sh.key[tid] = KEY_EMPTY;
    // Every independent first-touch load is issued up front so their round trips overlap: the
    // busy-list length, the ghost-fragment count and the draws' shading uniforms.  (A single-frame
    // scan-mode scene's bin boxes held in registers from the start -- rounds 1-4 -- cost the batch
    // kernel two spilled registers and bought the single frame nothing measurable: C2 0.0361 ->
    // 0.0356 ms per single frame without them.)
    const uint32_t n_busy = min(cnt[C_BUSY], (uint32_t)(fp.tiles_x * fp.tiles_y * (TILE / RTH) * fp.n_frames));
    const uint32_t n_frag = min(cnt[C_FRAG], fp.frag_cap);
    static_assert(LDS_DRAWS * 4 == 256, "one per-draw uniform float4 per thread");
    const int n_draws_all = fp.n_draws * fp.n_frames;
    const float4 du_first = tid < min(n_draws_all, LDS_DRAWS) * 4 ? reinterpret_cast<const float4 *>(draws[tid >> 2].light)[tid & 3]
                                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < min(n_draws_all, LDS_DRAWS) * 4) sh.du[tid] = du_first;
    // a strip item clears STRIP_RT raster-tile rows of one frame (fewer items: fewer tickets and
    // barriers per cleared byte)
    const int strips_y = (fp.rtiles_y + STRIP_RT - 1) / STRIP_RT;
    const uint32_t n_strips = (uint32_t)(strips_y * fp.n_frames);
    const uint64_t n_items = (uint64_t)n_strips + n_busy;
    const uint32_t G = gridDim.x, q = blockIdx.x % (uint32_t)N_WORKQ;
    uint32_t *queue = &cnt[C_WORK + WORKQ_STRIDE * q];
    const bool queued = (uint64_t)G + q < n_items;        // this queue deals any item at all
    uint32_t item = blockIdx.x, ticket = 0u;
    bool first = true;
    while ((uint64_t)item < n_items) {
        if (tid == 0 && queued) ticket = atomicAdd(queue, 1u);   // the next item, in flight meanwhile
        // interleave: item i is a strip when the count of strips among items < i + 1 grows
        const uint32_t s_lo = (uint32_t)(((uint64_t)item * n_strips) / n_items);
        const uint32_t s_hi = (uint32_t)(((uint64_t)(item + 1) * n_strips) / n_items);
        if (s_hi > s_lo) {
            const int f = (int)(s_lo / (uint32_t)strips_y);
            const int sy = (int)s_lo - f * strips_y;
            if (!SHS_DBG(fp, DBG_SKIP_CLEAR))   // (timing experiments: the busy tiles alone)
                for (int ry = sy * STRIP_RT; ry < min((sy + 1) * STRIP_RT, fp.rtiles_y); ++ry) clear_strip(fp, fb, f, ry);
        } else {
            uint32_t k = item - s_lo;
            if ((fp.flags & RF_XCD_ROWS) && k < (n_busy & ~31u))   // busy item 32B + 8r + x <- entry 32B + 4x + r:
                k = (k & ~31u) | ((k & 7u) << 2) | ((k >> 3) & 3u);  // a row group's items 8 apart (one queue)
            const uint32_t g = fb.busy_list[k];
            const int f = (int)(g / (uint32_t)n_rt), rt = (int)g - f * n_rt;
            const FrameBuffers fv = frame_view(fp, fb, f);
            if (g == BUSY_SKIP) {
                // padding of a row group (a bin tile's row below the screen): nothing to draw
            } else if (SHS_DBG(fp, DBG_CLEAR_ONLY)) {
                __syncthreads();
                clear_tile(fp, fv, rt);
            } else {
                if (SHS_DBG(fp, DBG_TWICE)) raster_tile<NO_RECS, SPANS, PIX, SCAN>(fp, fv, draws, cnt, n_frag, f, rt, sh, nullptr);   // warm run
                tl_mark(first ? fb.timeline : nullptr, fp.setup_grid + (int)blockIdx.x, 0);
                raster_tile<NO_RECS, SPANS, PIX, SCAN>(fp, fv, draws, cnt, n_frag, f, rt, sh, first ? fb.timeline : nullptr);
                first = false;
            }
        }
        if (!queued) break;
        __syncthreads();   // every thread is done with sh.item of the previous round
        if (tid == 0) sh.item = G + q + (uint32_t)N_WORKQ * ticket;
        __syncthreads();
        item = sh.item;
    }
    __syncthreads();
    if (tid == 0) {
        fb.rstat[blockIdx.x] = make_uint2(sh.cov, sh.maxbin);
        if (fb.timeline) {
            fb.timeline[TL_STRIDE * (fp.setup_grid + blockIdx.x)] = t_start;
            fb.timeline[TL_STRIDE * (fp.setup_grid + blockIdx.x) + 1] = __builtin_amdgcn_s_memrealtime();
            fb.timeline[TL_STRIDE * (fp.setup_grid + blockIdx.x) + 10] = c_start;
            fb.timeline[TL_STRIDE * (fp.setup_grid + blockIdx.x) + 11] = __builtin_amdgcn_s_memtime();
        }
    }
}

// Pipelined batches (SHS_OPT_LEGACY_PIPELINE, shs_abi.cpp): ONE persistent launch renders batch k - 1's
// raster (fpR / fbR: its busy tiles and clear strips, exactly k_raster's items) and runs batch k's setup
// (fpS / fbS: exactly k_setup's blocks).  Nothing in the launch waits on anything else in it: batch
// k - 1's setup finished in the previous launch, and batch k's raster runs in the next.  The setup
// blocks are dealt among the raster items in proportion (item i is a setup block when the count of
// setup blocks among items < i + 1 grows), so they fill the raster's latency gaps and its tail instead
// of running as a kernel of their own between two rasters (the cross-queue hop and the wait for CUs
// of the two-stream pipeline).  Scan-mode batches with a device draw table only
// (no k_ghost, no kernel-argument draws).
__global__ __launch_bounds__(256, SHS_LEGACY_RASTER_WAVES) void k_pipe(FrameParams fp, FrameBuffers fb, FrameParams fpS,
                                                                       FrameBuffers fbS) {
    __shared__ RasterShared sh;
    __shared__ SliverRecs s_sliv[4];
    __shared__ GhostScratch s_ghost[4];
    __shared__ uint32_t s_stat[4];
    __shared__ NewBusy s_new;
    const int tid = threadIdx.x;
    uint32_t *cnt = fb.counters + fp.parity * CSET;
    const DrawGPU *draws = fb.draws;
    const int n_rt = fp.tiles_x * fp.rtiles_y;            // raster tiles per frame
    if (tid == 0) { sh.cov = 0; sh.maxbin = 0; }
    sh.key[tid] = KEY_EMPTY;
    const uint32_t n_busy = min(cnt[C_BUSY], (uint32_t)(n_rt * fp.n_frames));
    const uint32_t n_frag = min(cnt[C_FRAG], fp.frag_cap);
    const int n_draws_all = fp.n_draws * fp.n_frames;
    const float4 du_first = tid < min(n_draws_all, LDS_DRAWS) * 4 ? reinterpret_cast<const float4 *>(draws[tid >> 2].light)[tid & 3]
                                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < min(n_draws_all, LDS_DRAWS) * 4) sh.du[tid] = du_first;
    const int strips_y = (fp.rtiles_y + STRIP_RT - 1) / STRIP_RT;
    const uint32_t n_strips = (uint32_t)(strips_y * fp.n_frames);
    const uint64_t n_raster = (uint64_t)n_strips + n_busy;
    const uint32_t n_setup = (uint32_t)fpS.setup_grid;
    const uint64_t n_items = n_raster + n_setup;
    const uint32_t G = gridDim.x, q = blockIdx.x % (uint32_t)N_WORKQ;
    uint32_t *queue = &cnt[C_WORK + WORKQ_STRIDE * q];
    const bool queued = (uint64_t)G + q < n_items;
    uint32_t item = blockIdx.x, ticket = 0u;
    while ((uint64_t)item < n_items) {
        if (tid == 0 && queued) ticket = atomicAdd(queue, 1u);   // the next item, in flight meanwhile
        const uint32_t k_lo = (uint32_t)(((uint64_t)item * n_setup) / n_items);
        const uint32_t k_hi = (uint32_t)(((uint64_t)(item + 1) * n_setup) / n_items);
        if (k_hi > k_lo) {
            setup_item<false>(fpS, fbS, fbS.draws, (int)k_lo, s_ghost, s_stat, s_new, s_sliv);
        } else {
            const uint32_t j = item - k_lo;                   // raster item j of n_raster (k_raster's order)
            const uint32_t s_lo = (uint32_t)(((uint64_t)j * n_strips) / n_raster);
            const uint32_t s_hi = (uint32_t)(((uint64_t)(j + 1) * n_strips) / n_raster);
            if (s_hi > s_lo) {
                const int f = (int)(s_lo / (uint32_t)strips_y);
                const int sy = (int)s_lo - f * strips_y;
                for (int ry = sy * STRIP_RT; ry < min((sy + 1) * STRIP_RT, fp.rtiles_y); ++ry) clear_strip(fp, fb, f, ry);
            } else {
                const uint32_t g = fb.busy_list[j - s_lo];
                const int f = (int)(g / (uint32_t)n_rt), rt = (int)g - f * n_rt;
                const FrameBuffers fv = frame_view(fp, fb, f);
                raster_tile<false, false, true, SCAN_RUNTIME>(fp, fv, draws, cnt, n_frag, f, rt, sh, nullptr);
            }
        }
        if (!queued) break;
        __syncthreads();   // every thread is done with sh.item of the previous round
        if (tid == 0) sh.item = G + q + (uint32_t)N_WORKQ * ticket;
        __syncthreads();
        item = sh.item;
    }
    __syncthreads();
    if (tid == 0) fb.rstat[blockIdx.x] = make_uint2(sh.cov, sh.maxbin);
}

}  // namespace shs_dev

// ---- launch wrappers (called by shs_abi.cpp) -----------------------------------------------
namespace shs_internal {
using namespace shs_dev;

hipError_t launch_setup(const FrameParams &fp, const FrameBuffers &fb, const KArgDraws &ka, hipStream_t s) {
    const int grid = fp.setup_grid;   // n_frames * frame_blocks
    const bool karg = fp.n_draws * fp.n_frames <= KARG_DRAWS;   // the whole batch's draws as kernel arguments
    const dim3 g(grid > 0 ? grid : 1);
    if (fp.scan_mode) {
        if (karg) hipLaunchKernelGGL((k_setup<true, false>), g, dim3(256), 0, s, fp, fb, ka);
        else hipLaunchKernelGGL((k_setup<false, false>), g, dim3(256), 0, s, fp, fb, ka);
    } else {
        if (karg) hipLaunchKernelGGL((k_setup<true, true>), g, dim3(256), 0, s, fp, fb, ka);
        else hipLaunchKernelGGL((k_setup<false, true>), g, dim3(256), 0, s, fp, fb, ka);
    }
    return hipGetLastError();
}

hipError_t launch_ghost(const FrameParams &fp, const FrameBuffers &fb, hipStream_t s) {
    hipLaunchKernelGGL(k_ghost, dim3(GHOST_LIST_BLOCKS), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}

hipError_t launch_pipe(const FrameParams &fpR, const FrameBuffers &fbR, int grid, const FrameParams &fpS, const FrameBuffers &fbS,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_pipe, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, fpR, fbR, fpS, fbS);
    return hipGetLastError();
}

hipError_t launch_raster(const FrameParams &fp, const FrameBuffers &fb, const KArgDraws &ka, int grid, hipStream_t s) {
    const dim3 g(grid > 0 ? grid : 1);
    const bool karg = fp.n_draws * fp.n_frames <= KARG_DRAWS;   // the whole batch's draws as kernel arguments
    // binned frames test conservative row spans, scan-mode frames whole boxes (raster_tile); the
    // per-pixel loop (SHS_OPT_RASTER_LOOP 0) has kernels of its own, so the pair kernels carry none of
    // its registers
#define SHS_RASTER(NR, SP, PX, SC)                                                                          \
    do {                                                                                                   \
        if (karg) hipLaunchKernelGGL((k_raster<true, NR, SP, PX, SC>), g, dim3(256), 0, s, fp, fb, ka);      \
        else hipLaunchKernelGGL((k_raster<false, NR, SP, PX, SC>), g, dim3(256), 0, s, fp, fb, ka);          \
    } while (0)
    const bool pix = (fp.flags & RF_PER_PIXEL) != 0u;
    if (DBG_BUILD && (fp.flags & RF_NO_RECS)) {   // binned frames, records recomputed (either loop; experiments build)
#ifdef SHS_TIMING_EXPERIMENTS
        SHS_RASTER(true, true, false, SCAN_BINNED);
#endif
    } else if (pix) SHS_RASTER(false, false, true, SCAN_RUNTIME);              // (binned frames: boxes)
    else if (!fp.scan_mode) SHS_RASTER(false, true, false, SCAN_BINNED);
#ifdef SHS_SCAN_SPANS   // (timing experiments: scan-mode frames on row spans)
    else SHS_RASTER(false, true, false, SCAN_ALL);
#else
    else SHS_RASTER(false, false, false, SCAN_ALL);
#endif
#undef SHS_RASTER
    return hipGetLastError();
}

}  // namespace shs_internal
