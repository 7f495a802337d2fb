// Store-pattern probe (timing tool, not product code): the legacy raster's clear-strip write pattern
// in isolation, against a linear fill, to find what holds the clear-only k_raster at ~5 TB/s
// (DESIGN.md section 4).  Built by tools/store_probe.sh into tools/libstore_probe.so, driven by
// tools/store_rate.py through ctypes (device pointers from torch).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one buffer, grid-stride 16-B stores
template <bool NT>
__global__ __launch_bounds__(256) void k_fill(u32x4 *p, size_t n16) {
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) st16<NT>(p + i, v);
}

// one buffer in contiguous chunks of C16 16-B elements: PERSIST 0 -- one workgroup per chunk
// (non-persistent grid); 1 -- a persistent grid taking chunks by a ticket counter
template <bool NT, bool PERSIST>
__global__ __launch_bounds__(256) void k_fill_chunks(u32x4 *p, size_t n16, int c16, uint32_t *ticket) {
    __shared__ uint32_t s_item;
    const u32x4 v = {1u, 2u, 3u, 4u};
    const uint32_t n_items = (uint32_t)((n16 + c16 - 1) / c16);
    uint32_t item = blockIdx.x;
    while (item < n_items) {
        uint32_t next = 0;
        if (PERSIST && threadIdx.x == 0) next = gridDim.x + atomicAdd(ticket, 1u);
        const size_t e = min(n16, (size_t)(item + 1) * c16);
        for (size_t i = (size_t)item * c16 + threadIdx.x; i < e; i += 256) st16<NT>(p + i, v);
        if (!PERSIST) break;
        __syncthreads();
        if (threadIdx.x == 0) s_item = next;
        __syncthreads();
        item = s_item;
    }
}

// grid-stride, four independent stores per iteration (issue-rate check)
template <bool NT>
__global__ __launch_bounds__(256) void k_fill_unroll(u32x4 *p, size_t n16) {
    const u32x4 v = {1u, 2u, 3u, 4u};
    const size_t st = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * st < n16; i += 4 * st) { st16<NT>(p + i, v); st16<NT>(p + i + st, v); st16<NT>(p + i + 2 * st, v); st16<NT>(p + i + 3 * st, v); }
    for (; i < n16; i += st) st16<NT>(p + i, v);
}

// non-persistent, each workgroup writes four 4-KB chunks a quarter of the buffer apart
template <bool NT>
__global__ __launch_bounds__(256) void k_fill_spread(u32x4 *p, size_t n16) {
    const u32x4 v = {1u, 2u, 3u, 4u};
    const size_t q = n16 / 4;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < q) { st16<NT>(p + i, v); st16<NT>(p + i + q, v); st16<NT>(p + i + 2 * q, v); st16<NT>(p + i + 3 * q, v); }
}

// persistent, chunks of C16 dealt by Q ticket queues (k_raster's dealing: queue b % Q deals items
// G + q + Q * ticket)
template <bool NT>
__global__ __launch_bounds__(256) void k_fill_q(u32x4 *p, size_t n16, int c16, uint32_t *queues) {
    __shared__ uint32_t s_item;
    const int Q = 16;
    const u32x4 v = {1u, 2u, 3u, 4u};
    const uint32_t n_items = (uint32_t)((n16 + c16 - 1) / c16), q = blockIdx.x % Q;
    uint32_t item = blockIdx.x;
    while (item < n_items) {
        uint32_t next = 0;
        if (threadIdx.x == 0) next = gridDim.x + q + Q * atomicAdd(&queues[q * 64], 1u);
        const size_t e = min(n16, (size_t)(item + 1) * c16);
        for (size_t i = (size_t)item * c16 + threadIdx.x; i < e; i += 256) st16<NT>(p + i, v);
        __syncthreads();
        if (threadIdx.x == 0) s_item = next;
        __syncthreads();
        item = s_item;
    }
}

// Strips of SR pixel rows of one frame (F frames of W x H, colour rows bottom-up, depth rows
// top-down).  MODE 0: the current clear_strip order (per 8-row raster row: per 4-px group column of
// the thread, 8 rows of colour + depth); 1: each plane's strip block linearly, colour and depth
// interleaved per step; 2: colour block then depth block.  Persistent grid, items dealt statically
// (DYN 0) or by one ticket counter per workgroup item (DYN 1).
template <bool NT, int MODE, bool DYN>
__global__ __launch_bounds__(256) void k_strips(uint32_t *color, uint32_t *depth, int F, int W, int H, int SR,
                                                uint32_t *ticket) {
    __shared__ uint32_t s_item;
    const int tid = threadIdx.x;
    const int strips_y = (H + SR - 1) / SR;
    const uint32_t n_items = (uint32_t)(F * strips_y);
    const u32x4 c4 = {0x11223344u, 0x11223344u, 0x11223344u, 0x11223344u};
    const u32x4 d4 = {0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu, 0x7f7fffffu};
    const int ng = W >> 2;
    uint32_t item = blockIdx.x;
    while (item < n_items) {
        uint32_t next = 0;
        if (DYN && tid == 0) next = gridDim.x + atomicAdd(ticket, 1u);
        const int f = item / strips_y, sy = item - f * strips_y;
        const int y0 = sy * SR, y1 = min(y0 + SR, H);
        uint32_t *cf = color + (size_t)f * W * H, *df = depth + (size_t)f * W * H;
        if (MODE == 0) {
            for (int ry = y0; ry < y1; ry += 8) {
                for (int g = tid; g < ng; g += 256) {
                    for (int y = ry; y < min(ry + 8, y1); ++y) {
                        st16<NT>(reinterpret_cast<u32x4 *>(cf + (size_t)(H - 1 - y) * W) + g, c4);
                        st16<NT>(reinterpret_cast<u32x4 *>(df + (size_t)y * W) + g, d4);
                    }
                }
            }
        } else {
            const size_t n16 = (size_t)(y1 - y0) * ng;
            u32x4 *cb = reinterpret_cast<u32x4 *>(cf + (size_t)(H - y1) * W);
            u32x4 *db = reinterpret_cast<u32x4 *>(df + (size_t)y0 * W);
            if (MODE == 1) {
                for (size_t i = tid; i < n16; i += 256) { st16<NT>(cb + i, c4); st16<NT>(db + i, d4); }
            } else {
                for (size_t i = tid; i < n16; i += 256) st16<NT>(cb + i, c4);
                for (size_t i = tid; i < n16; i += 256) st16<NT>(db + i, d4);
            }
        }
        if (DYN) {
            __syncthreads();
            if (tid == 0) s_item = next;
            __syncthreads();
            item = s_item;
        } else {
            item += gridDim.x;
        }
    }
}

extern "C" int probe_fill(void *p, size_t bytes, int grid, int nt, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (nt) hipLaunchKernelGGL((k_fill<true>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, bytes / 16);
    else hipLaunchKernelGGL((k_fill<false>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, bytes / 16);
    return (int)hipGetLastError();
}

extern "C" int probe_fill_chunks(void *p, size_t bytes, int c16, int grid, int nt, void *ticket, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t n16 = bytes / 16;
    if (grid <= 0) grid = (int)((n16 + c16 - 1) / c16);
    const bool per = grid < (int)((n16 + c16 - 1) / c16);
    if (nt) { if (per) hipLaunchKernelGGL((k_fill_chunks<true, true>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)ticket);
              else hipLaunchKernelGGL((k_fill_chunks<true, false>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)ticket); }
    else { if (per) hipLaunchKernelGGL((k_fill_chunks<false, true>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)ticket);
           else hipLaunchKernelGGL((k_fill_chunks<false, false>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)ticket); }
    return (int)hipGetLastError();
}

extern "C" int probe_fill_var(void *p, size_t bytes, int kind, int grid, int c16, int nt, void *queues, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t n16 = bytes / 16;
    if (kind == 0) {
        if (nt) hipLaunchKernelGGL((k_fill_unroll<true>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16);
        else hipLaunchKernelGGL((k_fill_unroll<false>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16);
    } else if (kind == 1) {
        const int g = (int)((n16 / 4 + 255) / 256);
        if (nt) hipLaunchKernelGGL((k_fill_spread<true>), dim3(g), dim3(256), 0, s, (u32x4 *)p, n16);
        else hipLaunchKernelGGL((k_fill_spread<false>), dim3(g), dim3(256), 0, s, (u32x4 *)p, n16);
    } else {
        if (nt) hipLaunchKernelGGL((k_fill_q<true>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)queues);
        else hipLaunchKernelGGL((k_fill_q<false>), dim3(grid), dim3(256), 0, s, (u32x4 *)p, n16, c16, (uint32_t *)queues);
    }
    return (int)hipGetLastError();
}

extern "C" int probe_strips(void *color, void *depth, int F, int W, int H, int SR, int grid, int nt, int mode, int dyn,
                            void *ticket, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (W % 4 || SR % 8) return -1;
#define L(NTV, M, D) hipLaunchKernelGGL((k_strips<NTV, M, D>), dim3(grid), dim3(256), 0, s, (uint32_t *)color, (uint32_t *)depth, F, W, H, SR, (uint32_t *)ticket)
#define LM(NTV, D) do { if (mode == 0) L(NTV, 0, D); else if (mode == 1) L(NTV, 1, D); else L(NTV, 2, D); } while (0)
    if (nt) { if (dyn) LM(true, true); else LM(true, false); }
    else { if (dyn) LM(false, true); else LM(false, false); }
#undef LM
#undef L
    return (int)hipGetLastError();
}
