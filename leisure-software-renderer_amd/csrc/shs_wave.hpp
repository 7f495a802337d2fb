// shs_wave.hpp -- wavefront (64-lane) helpers shared by the legacy and library raster kernels:
// in-wave LDS hand-off, ballot-based appends and the order-preserving 64-bit depth key.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shs_dev {

// LDS hand-off between lanes of ONE wave: the wave's LDS operations execute in order, so only the
// compiler must be kept from reordering (no s_barrier: waves of a block may diverge).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
}

// Wave-aggregated appends to NK per-key counters (call with the whole wave converged).  Lanes with
// key[k] >= 0 get a unique slot of counter[key[k]]; each distinct key costs ONE returning atomic, and
// all of them are issued before any return value is consumed (one memory round trip in total).
template <int NK>
__device__ __forceinline__ void wave_append(uint32_t *counter, const int (&key)[NK], uint32_t (&slot)[NK]) {
    const int lane = __lane_id();
    uint32_t add[NK], rank[NK], leader[NK], ret[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        add[k] = 0u; rank[k] = 0u; leader[k] = 0u;
        uint64_t pending = __ballot(key[k] >= 0);
        while (pending) {
            const int first = __ffsll((unsigned long long)pending) - 1;
            const int lk = __shfl(key[k], first);
            const uint64_t peers = __ballot(key[k] == lk) & pending;
            if (lane == first) add[k] = (uint32_t)__popcll(peers);
            if ((peers >> lane) & 1ull) { leader[k] = (uint32_t)first; rank[k] = lanes_below(peers); }
            pending &= ~peers;
        }
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) ret[k] = add[k] ? atomicAdd(&counter[key[k]], add[k]) : 0u;
#pragma unroll
    for (int k = 0; k < NK; ++k) slot[k] = __shfl(ret[k], (int)leader[k]) + rank[k];
}

// Single-counter wave append (converged wave): slot for lanes with want.
__device__ __forceinline__ uint32_t wave_append1(uint32_t *counter, bool want) {
    const uint64_t m = __ballot(want);
    if (!m) return 0u;
    const int first = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0u;
    if (__lane_id() == first) base = atomicAdd(counter, (uint32_t)__popcll(m));
    return __shfl(base, first) + lanes_below(m);
}

// Order-preserving key of a strict-less z test run in submission order: the test keeps, per pixel,
// the lexicographic minimum of (z, submission index) (the first fragment with the minimal z wins), so
// a 64-bit key (orderable z bits << 32 | index) resolved by atomic min is exact and independent of
// the order candidates are processed in.  -0 and +0 compare equal in the reference, so -0 maps to
// +0's key.
constexpr unsigned long long KEY_EMPTY = ~0ull;

__device__ __forceinline__ unsigned long long z_key(float z, uint32_t id) {
    uint32_t b = __float_as_uint(z);
    b = (b << 1) == 0u ? 0u : b;                                 // -0 -> +0
    const uint32_t ord = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((unsigned long long)ord << 32) | id;
}

}  // namespace shs_dev
