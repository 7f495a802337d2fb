// shs_legacy.hip -- gfx950 kernels for the shs_renderer legacy triangle scan-conversion path.
//
// Replaces RendererSystem::process + draw_triangle_tile + the four legacy shader pairs
// (cpp-folders/src/hello-3d-primitives/hello_pipeline_{blinn_phong,phong,gouraud,flat}_shading.cpp).
//
// Pipeline per frame (all on one HIP stream):
//   k_setup   one thread per triangle: VS x3 (mvp), clip_to_screen, area/denominator culls, the
//             per-triangle half of barycentric_coordinate, 96-B raster record, bin counts.
//   k_scan    one workgroup: exclusive scan of per-tile counts -> list offsets.
//   k_scatter one thread per triangle: triangle ids into per-tile lists (unordered).
//   k_raster  one workgroup per 32x32 tile: stage the tile's records in LDS, each lane resolves
//             4 pixels to the lexicographic minimum (z, submission index) -- identical to the
//             reference's in-order strict-less z test (first triangle with the minimal z wins) --
//             then shades only the winners and writes colour (canvas rows) and depth (screen
//             rows) once, coalesced, with the clear fused.
// The z-buffer therefore never round-trips through HBM: HBM sees each input once and each
// output pixel once.
#include <float.h>

#include "shs_device.hpp"
#include "shs_internal.hpp"

namespace shs_dev {

// ---- k_setup --------------------------------------------------------------------------------

// Sound filter for the reference's tile-clamp "ghost" pixels.  draw_triangle_tile clamps each
// triangle's bbox to the tile that runs it (blinn_phong_shading.cpp:208-215), so every triangle is
// tested against pixels of every tile -- also pixels outside its own bbox.  Those pixels are at
// least 0.5 px outside the bbox, so some exact barycentric is <= -0.49/(2*extent); this returns
// false only when a forward error bound of barycentric_coordinate's float arithmetic proves the
// computed (u,v,w) keep a negative component there.  Triangles it cannot clear (slivers) are
// rasterised over the reference's exact visited-pixel set by every tile (ghost list).  DESIGN.md
// "Tile-clamp semantics" has the derivation.
__device__ bool ghost_risk(const TriRec &r) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double a = fabs((double)r.v0x), b = fabs((double)r.v0y);
    const double c = fabs((double)r.v1x), d = fabs((double)r.v1y);
    const double Wx = (double)r.fmaxx - (double)r.fminx, Wy = (double)r.fmaxy - (double)r.fminy;
    if (!(Wx > 0.0) || !(Wy > 0.0)) return true;
    const double A00 = a * a + b * b, A11 = c * c + d * d, A01 = a * c + b * d;
    const double Dabs = fabs((double)r.denom);
    const double ED = 6.1 * u * (A00 * A11 + A01 * A01);
    const double Dlow = Dabs - ED;
    if (!(Dlow > 0.0) || !(Dabs < 1e300)) return true;
    const double K1 = 7.2 * u + ED / Dlow;
    const double p0 = Wx + 0.01, q0 = Wy + 0.01;
    const double A20 = p0 * a + q0 * b, A21 = p0 * c + q0 * d;
    const double Nv0 = A11 * A20 + A01 * A21, Nvx = A11 * a + A01 * c, Nvy = A11 * b + A01 * d;
    const double Nw0 = A00 * A21 + A01 * A20, Nwx = A00 * c + A01 * a, Nwy = A00 * d + A01 * b;
    const double s = K1 / Dabs * (2.0 + 2.0 * u);
    double e0 = (Nv0 + Nw0) * s + u * (2.0 + (2.0 * Nv0 + Nw0) / Dlow);
    double ex = (Nvx + Nwx) * s + u * (2.0 * Nvx + Nwx) / Dlow;
    double ey = (Nvy + Nwy) * s + u * (2.0 * Nvy + Nwy) / Dlow;
    e0 *= 1.25; ex *= 1.25; ey *= 1.25;
    const double Wm = Wx > Wy ? Wx : Wy;
    const bool safe = (ex <= 1.0 / (8.0 * Wx)) && (ey <= 1.0 / (8.0 * Wy)) && (e0 <= 0.49 / (8.0 * Wm));
    return !safe;
}

__device__ __forceinline__ bool finitef(float x) { return fabsf(x) <= FLT_MAX; }

__global__ __launch_bounds__(256) void k_setup(FrameParams fp, FrameBuffers fb) {
    const int gid = blockIdx.x * 256 + threadIdx.x;
    if (gid >= fp.n_tris) return;
    int lo = 0, hi = fp.n_draws - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fb.draw_base[mid] <= gid) lo = mid; else hi = mid - 1;
    }
    const DrawGPU &dr = fb.draws[lo];
    const int local = gid - dr.tri_base;
    const float *p = dr.pos + 9 * (size_t)local;

    // VS position (mvp * vec4(p,1)) + Canvas::clip_to_screen (shs_renderer.hpp:823-831)
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
    r.draw = lo;
    r.local = local;
    r.fminx = g_min(g_min(sx[0], sx[1]), sx[2]);
    r.fmaxx = g_max(g_max(sx[0], sx[1]), sx[2]);
    r.fminy = g_min(g_min(sy[0], sy[1]), sy[2]);
    r.fmaxy = g_max(g_max(sy[0], sy[1]), sy[2]);

    uint32_t flags = 0;
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) finite = finite && finitef(sx[k]) && finitef(sy[k]);
    // area test of draw_triangle_tile (blinn_phong_shading.cpp:219-220)
    const float area = (sx[1] - sx[0]) * (sy[2] - sy[0]) - (sy[1] - sy[0]) * (sx[2] - sx[0]);
    // A non-finite corner makes denom NaN for every pixel (no write); |denom| < 1e-5 (a double
    // compare, shs_renderer.hpp:816) returns bc = -1 everywhere.
    if (!finite || area <= 0.0f || !((double)fabsf(r.denom) >= 1e-5)) flags |= TRI_CULLED;

    int ix0 = 0, ix1 = -1, iy0 = 0, iy1 = -1;
    if (!(flags & TRI_CULLED)) {
        const bool dfin = finitef(r.d00) && finitef(r.d01) && finitef(r.d11) && finitef(r.denom);
        if (!dfin || ghost_risk(r)) flags |= TRI_GHOST;
        ix0 = (int)fminf(fmaxf(floorf(r.fminx), 0.0f), (float)fp.W);
        ix1 = (int)fminf(fmaxf(floorf(r.fmaxx), -1.0f), (float)(fp.W - 1));
        iy0 = (int)fminf(fmaxf(floorf(r.fminy), 0.0f), (float)fp.H);
        iy1 = (int)fminf(fmaxf(floorf(r.fmaxy), -1.0f), (float)(fp.H - 1));
    }
    r.flags = flags;
    r.ix0 = ix0; r.ix1 = ix1; r.iy0 = iy0; r.iy1 = iy1;
    {
        const float4 *src = reinterpret_cast<const float4 *>(&r);
        float4 *dst = reinterpret_cast<float4 *>(&fb.recs[gid]);
#pragma unroll
        for (int j = 0; j < 6; ++j) dst[j] = src[j];
    }
    if (flags & TRI_CULLED) return;
    atomicAdd(&fb.counters[C_SETUP], 1u);
    if (flags & TRI_GHOST) {
        const uint32_t slot = atomicAdd(&fb.counters[C_GHOST], 1u);
        if (slot < fp.ghost_capacity) fb.ghost_list[slot] = (uint32_t)gid;
        else atomicOr(&fb.counters[C_OVERFLOW], 2u);
        return;
    }
    if (ix0 > ix1 || iy0 > iy1) return;
    const int tx0 = ix0 / TILE, tx1 = ix1 / TILE, ty0 = iy0 / TILE, ty1 = iy1 / TILE;
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            const int t = ty * fp.tiles_x + tx;
            if (t % fp.count == fp.rank) atomicAdd(&fb.tile_count[t], 1u);
        }
}

// ---- k_scan ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan(FrameParams fp, FrameBuffers fb, int n_tiles) {
    __shared__ uint32_t s[1024];
    const int tid = threadIdx.x;
    const int per = (n_tiles + 1023) / 1024;
    const int b = tid * per, e = min(b + per, n_tiles);
    uint32_t sum = 0;
    for (int i = b; i < e; ++i) sum += fb.tile_count[i];
    s[tid] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t v = tid >= off ? s[tid - off] : 0u;
        __syncthreads();
        s[tid] += v;
        __syncthreads();
    }
    uint32_t run = s[tid] - sum;  // exclusive prefix
    for (int i = b; i < e; ++i) {
        fb.tile_offset[i] = run;
        fb.tile_cursor[i] = run;
        run += fb.tile_count[i];
    }
    if (tid == 1023) {
        fb.counters[C_BINS] = s[1023];
        if (s[1023] > fp.list_capacity) atomicOr(&fb.counters[C_OVERFLOW], 1u);
    }
}

// ---- k_scatter ------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scatter(FrameParams fp, FrameBuffers fb) {
    const int gid = blockIdx.x * 256 + threadIdx.x;
    if (gid >= fp.n_tris) return;
    const int4 q = reinterpret_cast<const int4 *>(&fb.recs[gid])[3];   // z2, flags, draw, local
    const uint32_t flags = (uint32_t)q.y;
    if (flags & (TRI_CULLED | TRI_GHOST)) return;
    const int4 bb = reinterpret_cast<const int4 *>(&fb.recs[gid])[4];  // ix0, ix1, iy0, iy1
    if (bb.x > bb.y || bb.z > bb.w) return;
    const int tx0 = bb.x / TILE, tx1 = bb.y / TILE, ty0 = bb.z / TILE, ty1 = bb.w / TILE;
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            const int t = ty * fp.tiles_x + tx;
            if (t % fp.count != fp.rank) continue;
            const uint32_t pos = atomicAdd(&fb.tile_cursor[t], 1u);
            if (pos < fp.list_capacity) fb.tile_list[pos] = (uint32_t)gid;
        }
}

// ---- k_raster -------------------------------------------------------------------------------

__device__ __forceinline__ TriRec rec_from_lds(const float4 *s) {
    TriRec r;
    float4 *d = reinterpret_cast<float4 *>(&r);
#pragma unroll
    for (int j = 0; j < 6; ++j) d[j] = s[j];
    return r;
}

// Fragment shaders of the four legacy pipelines, evaluated for the winning triangle only.
// Returns the pre-truncation floats; the caller truncates to uint8 exactly like the reference.
__device__ void shade_winner(const FrameBuffers &fb, const TriRec &r, float u, float v, float w, float pre[3]) {
    const DrawGPU &dr = fb.draws[r.draw];
    const float *P = dr.pos + 9 * (size_t)r.local;
    const float *N = dr.nrm + 9 * (size_t)r.local;
    const int sh = dr.shading;
    if (sh == 0) {
        // Flat (flat_shading.cpp:46-98): VS normal = mat3(mv) * n; interpolated normal normalised;
        // FS: n = normalize(n), l = normalize(light_dir_view), intensity = min(0.2 + max(n.l,0), 1)
        f3 n[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) n[k] = m3v(dr.nmat, f3{N[3 * k], N[3 * k + 1], N[3 * k + 2]});
        const f3 in_n = normalize3(add3(add3(sc3(n[0], u), sc3(n[1], v)), sc3(n[2], w)));
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
    f3 wp[3], nr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x, y, z, ww;
        m4p(dr.model, P[3 * k], P[3 * k + 1], P[3 * k + 2], x, y, z, ww);
        wp[k] = f3{x, y, z};
        nr[k] = normalize3(m3v(dr.nmat, f3{N[3 * k], N[3 * k + 1], N[3 * k + 2]}));
    }
    const f3 L = {dr.light[0], dr.light[1], dr.light[2]};
    const f3 cam = {dr.cam[0], dr.cam[1], dr.cam[2]};
    const f3 oc = {dr.ocol[0], dr.ocol[1], dr.ocol[2]};
    if (sh == 1) {
        // Gouraud (gouraud_shading.cpp:46-89): Blinn-Phong (shininess 32, powf) per vertex, the
        // clamped colour interpolated through world_pos, FS truncates colour*255.
        f3 col[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const f3 viewDir = normalize3(sub3(cam, wp[k]));
            const float diff = g_max(dot3(nr[k], L), 0.0f);
            const f3 half = normalize3(add3(L, viewDir));
            const float spec = (float)pow((double)g_max(dot3(nr[k], half), 0.0f), 32.0);
            const float s = (0.15f + diff * 1.0f) + (0.5f * spec) * 1.0f;
            col[k] = f3{g_clamp01(s * oc.x), g_clamp01(s * oc.y), g_clamp01(s * oc.z)};
        }
        const f3 c = add3(add3(sc3(col[0], u), sc3(col[1], v)), sc3(col[2], w));
        pre[0] = c.x * 255.0f;
        pre[1] = c.y * 255.0f;
        pre[2] = c.z * 255.0f;
        return;
    }
    // Phong / Blinn-Phong: normal and world position interpolated (blinn_phong_shading.cpp:235-236)
    const f3 in_n = normalize3(add3(add3(sc3(nr[0], u), sc3(nr[1], v)), sc3(nr[2], w)));
    const f3 in_w = add3(add3(sc3(wp[0], u), sc3(wp[1], v)), sc3(wp[2], w));
    const f3 norm = normalize3(in_n);
    const f3 viewDir = normalize3(sub3(cam, in_w));
    const float diff = g_max(dot3(norm, L), 0.0f);
    float specular;
    if (sh == 2) {
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
    const float s = (0.15f + diff * 1.0f) + specular;
    pre[0] = g_clamp01(s * oc.x) * 255.0f;
    pre[1] = g_clamp01(s * oc.y) * 255.0f;
    pre[2] = g_clamp01(s * oc.z) * 255.0f;
}

__device__ __forceinline__ void resolve(float z, uint32_t id, float &bz, uint32_t &bid) {
    // In-order strict-less z test == lexicographic min of (z, submission index); NaN never wins,
    // z == FLT_MAX never beats the FLT_MAX clear (bid sentinel 0 makes id < bid false).
    if (z < bz || (z == bz && id < bid)) { bz = z; bid = id; }
}

__global__ __launch_bounds__(256) void k_raster(FrameParams fp, FrameBuffers fb) {
    __shared__ float4 s_rec[CHUNK * 6];
    __shared__ uint32_t s_id[CHUNK];
    __shared__ float s_bz[TILE * TILE];
    __shared__ uint32_t s_bid[TILE * TILE];
    __shared__ uint32_t s_cov;

    const int tile = fp.rank + (int)blockIdx.x * fp.count;
    const int tx = tile % fp.tiles_x, ty = tile / fp.tiles_x;
    const int X0 = tx * TILE, Y0 = ty * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_cov = 0;

    // raster lane mapping: wave owns rows [8w, 8w+8) of the tile, lane owns column lane&31 and
    // rows (lane>>5) + {0,2,4,6}
    const int px = X0 + (lane & 31);
    const int pyb = Y0 + wave * 8 + (lane >> 5);
    const float Px = (float)px + 0.5f;
    const int wy0 = Y0 + wave * 8, wy1 = wy0 + 7, wx0 = X0, wx1 = X0 + TILE - 1;
    float bz[4];
    uint32_t bid[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { bz[k] = FLT_MAX; bid[k] = 0u; }

    // reference tile-job bounds of this lane's pixels (ghost path only)
    const float rtminx = (float)((px / fp.rtw) * fp.rtw);
    const float rtmaxx = (float)(min((px / fp.rtw) * fp.rtw + fp.rtw, fp.W) - 1);

    const uint32_t cap = fp.list_capacity;
    const uint32_t off = fb.tile_offset[tile];
    uint32_t n_list = fb.tile_count[tile];
    if (off >= cap) n_list = 0; else if (n_list > cap - off) n_list = cap - off;
    uint32_t n_ghost = fb.counters[C_GHOST];
    if (n_ghost > fp.ghost_capacity) n_ghost = fp.ghost_capacity;

    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t n = pass == 0 ? n_list : n_ghost;
        const uint32_t *list = pass == 0 ? fb.tile_list + off : fb.ghost_list;
        for (uint32_t base = 0; base < n; base += CHUNK) {
            const int cnt = (int)min((uint32_t)CHUNK, n - base);
            __syncthreads();
            if (tid < cnt) {
                const uint32_t id = list[base + tid];
                s_id[tid] = id;
                const float4 *src = reinterpret_cast<const float4 *>(&fb.recs[id]);
#pragma unroll
                for (int j = 0; j < 6; ++j) s_rec[tid * 6 + j] = src[j];
            }
            __syncthreads();
            for (int j = 0; j < cnt; ++j) {
                const uint32_t id = s_id[j];
                if (pass == 0) {
                    const int4 bb = reinterpret_cast<const int4 *>(&s_rec[j * 6])[4];
                    if (bb.y < wx0 || bb.x > wx1 || bb.w < wy0 || bb.z > wy1) continue;  // wave-uniform
                    const TriRec r = rec_from_lds(&s_rec[j * 6]);
                    const bool inx = px >= r.ix0 && px <= r.ix1;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int py = pyb + 2 * k;
                        if (inx && py >= r.iy0 && py <= r.iy1) {
                            float u, v, w;
                            bary(r, Px, (float)py + 0.5f, u, v, w);
                            if (!(u < 0 || v < 0 || w < 0)) {
                                const float z = (u * r.z0 + v * r.z1) + w * r.z2;
                                resolve(z, id, bz[k], bid[k]);
                            }
                        }
                    }
                } else {
                    // ghost triangle: the exact visited set of the reference tile-job loop
                    // (blinn_phong_shading.cpp:208-224) for each pixel's 80x80 reference tile
                    const TriRec r = rec_from_lds(&s_rec[j * 6]);
                    const float bminx = g_max(rtminx, g_min(rtmaxx, r.fminx));
                    const float bmaxx = g_min(rtmaxx, g_max(rtminx, r.fmaxx));
                    const bool inx = !(bminx > bmaxx) && px >= (int)bminx && px <= (int)bmaxx;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int py = pyb + 2 * k;
                        const int rty = (py / fp.rth) * fp.rth;
                        const float rtminy = (float)rty;
                        const float rtmaxy = (float)(min(rty + fp.rth, fp.H) - 1);
                        const float bminy = g_max(rtminy, g_min(rtmaxy, r.fminy));
                        const float bmaxy = g_min(rtmaxy, g_max(rtminy, r.fmaxy));
                        if (inx && py < fp.H && !(bminy > bmaxy) && py >= (int)bminy && py <= (int)bmaxy) {
                            float u, v, w;
                            bary(r, Px, (float)py + 0.5f, u, v, w);
                            if (!(u < 0 || v < 0 || w < 0)) {
                                const float z = (u * r.z0 + v * r.z1) + w * r.z2;
                                resolve(z, id, bz[k], bid[k]);
                            }
                        }
                    }
                }
            }
        }
    }

    // hand the per-pixel winners to the output mapping through LDS
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ly = wave * 8 + (lane >> 5) + 2 * k;
        s_bz[ly * TILE + (lane & 31)] = bz[k];
        s_bid[ly * TILE + (lane & 31)] = bid[k];
    }
    __syncthreads();

    // output mapping: thread -> row tid>>3, 4 consecutive pixels: 8 threads cover one 32-px row
    // (128 B of colour + 128 B of depth, full lines)
    const int ly = tid >> 3, lx0 = (tid & 7) * 4;
    const int y = Y0 + ly;
    uint32_t covered = 0;
    if (y < fp.H) {
        uint32_t rgba[4];
        float dep[4];
        float4 pq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float z = s_bz[ly * TILE + lx0 + j];
            const uint32_t id = s_bid[ly * TILE + lx0 + j];
            dep[j] = z;
            rgba[j] = fp.clear_rgba;
            pq[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            const int x = X0 + lx0 + j;
            if (z < FLT_MAX && x < fp.W) {
                ++covered;
                const float4 *src = reinterpret_cast<const float4 *>(&fb.recs[id]);
                TriRec r;
                float4 *d = reinterpret_cast<float4 *>(&r);
#pragma unroll
                for (int q = 0; q < 6; ++q) d[q] = src[q];
                float u, v, w;
                bary(r, (float)x + 0.5f, (float)y + 0.5f, u, v, w);
                float pre[3];
                shade_winner(fb, r, u, v, w, pre);
                const uint32_t cr = (uint32_t)(uint8_t)pre[0], cg = (uint32_t)(uint8_t)pre[1], cb = (uint32_t)(uint8_t)pre[2];
                rgba[j] = cr | (cg << 8) | (cb << 16) | (255u << 24);
                pq[j] = make_float4(pre[0], pre[1], pre[2], 1.0f);
            }
        }
        const int x0 = X0 + lx0;
        const size_t crow = (size_t)(fp.H - 1 - y) * fp.W;
        const size_t drow = (size_t)y * fp.W;
        if (x0 + 3 < fp.W && (fp.W & 3) == 0) {
            *reinterpret_cast<uint4 *>(fb.color + (crow + x0) * 4) = make_uint4(rgba[0], rgba[1], rgba[2], rgba[3]);
            *reinterpret_cast<float4 *>(fb.depth + drow + x0) = make_float4(dep[0], dep[1], dep[2], dep[3]);
        } else {
            for (int j = 0; j < 4; ++j)
                if (x0 + j < fp.W) {
                    *reinterpret_cast<uint32_t *>(fb.color + (crow + x0 + j) * 4) = rgba[j];
                    fb.depth[drow + x0 + j] = dep[j];
                }
        }
        if (fb.prequant) {
            for (int j = 0; j < 4; ++j)
                if (x0 + j < fp.W) fb.prequant[crow + x0 + j] = pq[j];
        }
    }
    // covered-pixel count: wave reduction, one LDS atomic per wave, one global atomic per tile
    for (int o = 32; o > 0; o >>= 1) covered += __shfl_down(covered, o);
    if (lane == 0) atomicAdd(&s_cov, covered);
    __syncthreads();
    if (tid == 0) atomicAdd(&fb.counters[C_COVERED], s_cov);
}

}  // namespace shs_dev

// ---- launch wrappers (called by shs_abi.cpp) -----------------------------------------------
namespace shs_internal {
using namespace shs_dev;

hipError_t launch_setup(const FrameParams &fp, const FrameBuffers &fb, hipStream_t s) {
    if (fp.n_tris <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_setup, dim3((fp.n_tris + 255) / 256), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}
hipError_t launch_scan(const FrameParams &fp, const FrameBuffers &fb, int n_tiles, hipStream_t s) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, fp, fb, n_tiles);
    return hipGetLastError();
}
hipError_t launch_scatter(const FrameParams &fp, const FrameBuffers &fb, hipStream_t s) {
    if (fp.n_tris <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter, dim3((fp.n_tris + 255) / 256), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}
hipError_t launch_raster(const FrameParams &fp, const FrameBuffers &fb, int n_owned_tiles, hipStream_t s) {
    if (n_owned_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_raster, dim3(n_owned_tiles), dim3(256), 0, s, fp, fb);
    return hipGetLastError();
}
}  // namespace shs_internal
