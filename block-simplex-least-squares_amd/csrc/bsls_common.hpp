// bsls_common.hpp -- shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions
//   * wave = 64 lanes; every block size here is a multiple of 64;
//   * all arithmetic that must match the reference bit-for-bit is compiled with
//     -ffp-contract=off (Makefile) so a*b+c stays two roundings, like the
//     reference's x86-64 g++ build;
//   * reductions are deterministic: fixed lane/thread trees, fixed partial order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bsls_hip.h"

#define BSLS_CHECK(expr)                                   \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return (int)e_;              \
    } while (0)

#define BSLS_LAUNCH_CHECK() BSLS_CHECK(hipGetLastError())

namespace bsls {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (WAVE - 1)); }

// end of block b (the last block ends at n), reference proj_simplex.h:43-46
__device__ __forceinline__ int64_t block_end(const int64_t *starts, int64_t nb, int64_t b,
                                             int64_t n) {
    return (b + 1 < nb) ? starts[b + 1] : n;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T u = __shfl_xor(v, o, WAVE);
        v = (u > v) ? u : v;
    }
    return v;
}

// Sum over G consecutive lanes (G power of two <= 64); result valid in all G lanes.
template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

// Deterministic block-wide sum of NV values per thread (fixed tree); the result
// is valid in thread 0.  `red` must hold NV * (blockDim.x / 64) doubles.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *red) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = group_sum<WAVE>(v[k]);
    const int w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k * nw + w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double s = red[k * nw];
            for (int i = 1; i < nw; ++i) s += red[k * nw + i];
            v[k] = s;
        }
    }
    __syncthreads();
}

// "Last workgroup reduces": every workgroup publishes NV partials; the
// workgroup whose ticket add comes last sums all partials in index order
// (deterministic) and returns true with the totals in thread 0's `tot`.
//
// Hand-off without fences (MI355X_MICROARCH.md "Valid forms", table row 1):
// one lane stores the partials with agent-scope relaxed atomic stores (sc1),
// drains them (vmcnt(0)), then adds to a ticket (agent-scope atomic); the last
// arriver -- told by the value its add returned -- reads every partial with
// sc1 loads after a workgroup barrier.  (An agent release fence per workgroup,
// buffer_wbl2, measured ~1 ms extra on a 25k-workgroup SpMV.)
//
// Tickets are sharded 8 ways by blockIdx % 8 (the XCD group label; speed only,
// correctness never depends on placement) plus one top-level ticket, each on
// its own 64-B line: one device-scope word saturates near 88 adds/us (price
// list "dequeue"), which 7.8k arrivals turned into ~90 us.  `tickets` points
// at TICKET_BYTES of zeroed memory; the last arriver re-zeroes it.
constexpr int TICKET_STRIDE = 16;               // unsigned words = 64 B
constexpr int TICKET_BYTES = 9 * TICKET_STRIDE * 4;

template <int NV>
__device__ bool last_block_sum(const double (&mine)[NV], double *partials, unsigned *tickets,
                               double (&tot)[NV], double *red) {
    __shared__ int am_last;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            __hip_atomic_store(&partials[(size_t)blockIdx.x * NV + k], mine[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned shard = blockIdx.x & 7u;
        const unsigned members = (gridDim.x - shard + 7u) / 8u;
        const unsigned shards = gridDim.x < 8u ? gridDim.x : 8u;
        unsigned prev = __hip_atomic_fetch_add(&tickets[shard * TICKET_STRIDE], 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (prev == members - 1) {
            prev = __hip_atomic_fetch_add(&tickets[8 * TICKET_STRIDE], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            last = (prev == shards - 1);
        }
        am_last = last;
    }
    __syncthreads();
    if (!am_last) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep loads below the ticket
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += blockDim.x) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            acc[k] += __hip_atomic_load(&partials[(size_t)i * NV + k], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    }
    block_sum<NV>(acc, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] = acc[k];
        for (int k = 0; k < 9; ++k) tickets[k * TICKET_STRIDE] = 0u;
    }
    return true;
}

// Same hand-off for a subset of the workgroups: `count` participants, this
// one publishing slot `idx`; one ticket word (few arrivals).  The last arriver
// sums slots 0 .. count-1 in order and re-zeroes the ticket.
template <int NV>
__device__ bool last_of_sum(const double (&mine)[NV], double *partials, unsigned idx,
                            unsigned count, unsigned *ticket, double (&tot)[NV], double *red) {
    __shared__ int am_last_n;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            __hip_atomic_store(&partials[(size_t)idx * NV + k], mine[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev =
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        am_last_n = (prev == count - 1);
    }
    __syncthreads();
    if (!am_last_n) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (unsigned i = threadIdx.x; i < count; i += blockDim.x) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            acc[k] += __hip_atomic_load(&partials[(size_t)i * NV + k], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    }
    block_sum<NV>(acc, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] = acc[k];
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// last_block_sum with some slots reduced by max instead of sum (bit k of
// MAXMASK): NaN-propagating max, fixed order like the sums.  `red` must hold
// NV * (blockDim.x / 64) doubles.
__device__ __forceinline__ double nan_max(double a, double b) {
    return (b > a || b != b) ? b : a;
}

template <int NV, unsigned MAXMASK>
__device__ __forceinline__ void block_reduce(double (&v)[NV], double *red) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        if ((MAXMASK >> k) & 1u) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v[k] = nan_max(v[k], __shfl_xor(v[k], o, WAVE));
        } else {
            v[k] = group_sum<WAVE>(v[k]);
        }
    }
    const int w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k * nw + w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double s = red[k * nw];
            for (int i = 1; i < nw; ++i)
                s = ((MAXMASK >> k) & 1u) ? nan_max(s, red[k * nw + i]) : s + red[k * nw + i];
            v[k] = s;
        }
    }
    __syncthreads();
}

template <int NV, unsigned MAXMASK>
__device__ bool last_block_reduce(const double (&mine)[NV], double *partials, unsigned *tickets,
                                  double (&tot)[NV], double *red) {
    __shared__ int am_last_r;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            __hip_atomic_store(&partials[(size_t)blockIdx.x * NV + k], mine[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // sharded tickets, as last_block_sum (one word: ~11 ns per arrival)
        const unsigned shard = blockIdx.x & 7u;
        const unsigned members = (gridDim.x - shard + 7u) / 8u;
        const unsigned shards = gridDim.x < 8u ? gridDim.x : 8u;
        unsigned prev = __hip_atomic_fetch_add(&tickets[shard * TICKET_STRIDE], 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (prev == members - 1) {
            prev = __hip_atomic_fetch_add(&tickets[8 * TICKET_STRIDE], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            last = (prev == shards - 1);
        }
        am_last_r = last;
    }
    __syncthreads();
    if (!am_last_r) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += blockDim.x) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const double v = __hip_atomic_load(&partials[(size_t)i * NV + k], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
            acc[k] = ((MAXMASK >> k) & 1u) ? nan_max(acc[k], v) : acc[k] + v;
        }
    }
    block_reduce<NV, MAXMASK>(acc, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] = acc[k];
        for (int k = 0; k < 9; ++k)
            __hip_atomic_store(&tickets[k * TICKET_STRIDE], 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// numpy.minimum(v, 1.) then numpy.maximum(., 0.) (python/main.py:65) as
// numpy 2.x computes them: NaN propagates, and on a tie maximum returns its
// second operand, so maximum(-0.0, 0.) is +0.0 (a -0.0 input leaves as +0.0).
__device__ __forceinline__ double clip01(double v) {
    double a = (v > 1.0) ? 1.0 : v;
    return (a > 0.0 || a != a) ? a : 0.0;
}

// std::max(v, 0.) as in proj_simplex.h:33.
__device__ __forceinline__ double relu_ref(double v) { return (v < 0.) ? 0. : v; }

inline int grid_for(int64_t work, int per_block) {
    int64_t g = (work + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace bsls
