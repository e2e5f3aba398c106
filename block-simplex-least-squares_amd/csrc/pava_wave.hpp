// pava_wave.hpp -- wave-parallel PAVA v1, bit-identical to the serial reference
// (python/c_extensions/isotonic_regression.h:13-58).
//
// A wave holds a "pack": up to 64 consecutive elements forming whole blocks,
// one element per lane.  Run structure lives in two wave-uniform 64-bit masks:
//   H  run heads (initially every element; the run of head h is [h, next head))
//   B  block starts (forced chain starts; chains never cross blocks)
// One reference pass = split every block's run sequence into maximal
// non-increasing chains (the reference's `while (y[k] <= y[j])` walk: a chain
// breaks at the first head r with !(y[r] <= y[previous head])), then pool each
// chain whose first and last values differ: num = sum over its runs, in order,
// of y*w, den = sum of w, y = num / den -- the same sequence of roundings as the
// reference, computed by the chain's head lane from lane shuffles.  Passes
// repeat until no chain pools; a block that did not pool is unchanged by later
// passes, so running the wave to the slowest block's convergence is exact.
// Every shuffle runs with all lanes active (ds_bpermute reads only active lanes).
#pragma once
#include "bsls_common.hpp"

namespace bsls {

// bits [0, l); l may be 64 (a 64-bit shift by 64 is undefined, and wraps on the GPU)
__device__ __forceinline__ uint64_t mask_lt(int l) {
    return (l >= 64) ? ~0ull : ((1ull << l) - 1ull);
}
__device__ __forceinline__ uint64_t mask_le(int l) {
    return (l >= 63) ? ~0ull : ((2ull << l) - 1ull);
}
__device__ __forceinline__ int hi_bit(uint64_t m) { return 63 - __clzll((long long)m); }
__device__ __forceinline__ int lo_bit(uint64_t m) { return __ffsll((long long)m) - 1; }

__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, WAVE); }
__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, WAVE); }

// y / w: this lane's element value and run length (meaningful at run heads);
// L: active lanes (elements) in the pack; B: block-start mask.
// On return y holds the expanded isotonic fit of this lane's element
// (update = 1 semantics); w the run length if this lane heads a run, and
// `heads` the final run-head mask.
__device__ __forceinline__ void pava_v1_wave(double &y, int &w, int L, uint64_t B,
                                             uint64_t &heads) {
    const int l = lane_id();
    const bool act = l < L;
    uint64_t H = (L >= 64) ? ~0ull : mask_lt(L);
    for (int pass = 0; pass <= L; ++pass) {
        // previous head of every head lane, and the chain starts
        const uint64_t below = H & mask_lt(l);
        const int p = below ? hi_bit(below) : l;
        const double yp = shfl_d(y, p);
        const bool head = act && ((H >> l) & 1ull);
        const bool cs = head && (((B >> l) & 1ull) || !(y <= yp));
        const uint64_t CS = __ballot(cs);
        // chain of a chain start: heads in [l, next chain start)
        const uint64_t above = CS & ~mask_le(l);
        const int nxt = above ? lo_bit(above) : L;
        const uint64_t chain = H & mask_lt(nxt) & ~mask_lt(l);
        const int last = chain ? hi_bit(chain) : l;
        const double ylast = shfl_d(y, last);
        const bool pool = cs && (y != ylast);
        uint64_t cur = pool ? chain : 0ull;
        double num = 0.0;
        int den = 0;
        while (__ballot(cur != 0ull)) {
            const int src = cur ? lo_bit(cur) : l;
            const double ys = shfl_d(y, src);
            const int ws = shfl_i(w, src);
            if (cur) {
                num += ys * (double)ws;
                den += ws;
                cur &= cur - 1ull;
            }
        }
        const uint64_t POOL = __ballot(pool);
        if (!POOL) break;
        // heads absorbed into a pooled chain (every head of it but the first)
        const uint64_t cs_le = CS & mask_le(l);
        const int mycs = cs_le ? hi_bit(cs_le) : l;
        const bool absorbed = head && !cs && ((POOL >> mycs) & 1ull);
        const uint64_t ABS = __ballot(absorbed);
        if (pool) {
            y = num / (double)den;
            w = den;
        }
        H &= ~ABS;
    }
    heads = H;
    // expand: every element takes its run head's value (update = 1)
    const uint64_t hl = H & mask_le(l);
    const int myhead = hl ? hi_bit(hl) : l;
    const double yh = shfl_d(y, myhead);
    if (act) y = yh;
}

}  // namespace bsls
