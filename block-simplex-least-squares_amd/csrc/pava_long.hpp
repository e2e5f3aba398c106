// pava_long.hpp -- PAVA v1 on one long block with a whole workgroup,
// bit-identical to the serial reference (python/c_extensions/
// isotonic_regression.h:13-58, unit initial run lengths, update = 1).
//
// The wave-parallel form (pava_wave.hpp) covers blocks of <= 64 elements; a
// longer block used to run serially in one lane (a 1e6-element log-trend block:
// 880 ms against 9 ms for the CPU reference).  Here the runs live in global
// buffers and one 1024-thread workgroup runs each reference pass in parallel:
//   A  chain starts (a run starts a chain at the block start or where
//      !(y[r] <= y[r-1]), the reference's `while (y[k] <= y[j])` walk) --
//      counted per thread over a contiguous run segment, placed by a
//      workgroup scan;
//   B  per chain: pooled iff its first and last runs differ (the reference's
//      y[i] != y[j]); survivors = 1 for a pooled chain, its runs otherwise --
//      placed by a second scan;
//   C  a pooled chain's sum in run order, num += y * w, den += w, then
//      y = num / den (the reference's roundings), by the thread owning the
//      chain; unpooled runs copied.
// Passes repeat until no chain pools; a pass decides from the values at its
// start, as the reference's left-to-right walk does (a pooled chain never
// changes the runs of the next chain).  Then every element takes its run's
// value (expand).  Threads own contiguous segments of runs / chains / elements.
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int LONG_T = 1024;

// exclusive scan of v over the LONG_T-thread workgroup; `tot` = the sum
__device__ __forceinline__ int64_t wg_exscan(int64_t v, int64_t *sh, int64_t &tot) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t u = __shfl_up(x, d, 64);
        if (lane >= d) x += u;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    if (t == 0) {
        int64_t a = 0;
        for (int i = 0; i < LONG_T / 64; ++i) {
            const int64_t q = sh[i];
            sh[i] = a;
            a += q;
        }
        sh[LONG_T / 64] = a;
    }
    __syncthreads();
    const int64_t r = sh[w] + x - v;
    tot = sh[LONG_T / 64];
    __syncthreads();
    return r;
}

__device__ __forceinline__ int64_t seg_lo(int64_t n, int64_t t) {
    const int64_t s = (n + LONG_T - 1) / LONG_T;
    return (t * s < n) ? t * s : n;
}

// y[0, k): in place.  Y0/Y1 (k doubles each), W0/W1 (k int32 each) and CH
// (k + 1 int32) are this block's scratch.  sh: LDS, LONG_T / 64 + 1 int64;
// flag: LDS int.
__device__ __forceinline__ void pava_v1_long(double *__restrict__ y, int64_t k,
                                             double *__restrict__ Y0, double *__restrict__ Y1,
                                             int32_t *__restrict__ W0, int32_t *__restrict__ W1,
                                             int32_t *__restrict__ CH, int64_t *sh, int *flag) {
    const int t = threadIdx.x;
    for (int64_t i = t; i < k; i += LONG_T) {
        Y0[i] = y[i];
        W0[i] = 1;
    }
    __syncthreads();
    double *Yc = Y0, *Yn = Y1;
    int32_t *Wc = W0, *Wn = W1;
    int64_t nh = k;
    for (int64_t pass = 0; pass <= k; ++pass) {
        // A: chain starts
        const int64_t a = seg_lo(nh, t), b = seg_lo(nh, t + 1);
        int64_t c = 0;
        double prev = (a > 0 && a < b) ? Yc[a - 1] : 0.0;
        for (int64_t r = a; r < b; ++r) {
            const double v = Yc[r];
            c += (r == 0 || !(v <= prev)) ? 1 : 0;
            prev = v;
        }
        int64_t C;
        int64_t q = wg_exscan(c, sh, C);
        prev = (a > 0 && a < b) ? Yc[a - 1] : 0.0;
        for (int64_t r = a; r < b; ++r) {
            const double v = Yc[r];
            if (r == 0 || !(v <= prev)) CH[q++] = (int32_t)r;
            prev = v;
        }
        if (t == 0) CH[C] = (int32_t)nh;
        __syncthreads();
        // B: survivors per chain
        const int64_t ca = seg_lo(C, t), cb = seg_lo(C, t + 1);
        int64_t sv = 0;
        int any = 0;
        for (int64_t h = ca; h < cb; ++h) {
            const int64_t r0 = CH[h], r1 = CH[h + 1];
            const bool pooled = Yc[r0] != Yc[r1 - 1];
            sv += pooled ? 1 : (r1 - r0);
            any |= pooled ? 1 : 0;
        }
        if (t == 0) *flag = 0;
        int64_t NS;
        int64_t o = wg_exscan(sv, sh, NS);   // (its barriers order the flag reset)
        if (any) *flag = 1;
        __syncthreads();
        if (*flag == 0) break;
        // C: pooled sums in run order, unpooled runs copied
        for (int64_t h = ca; h < cb; ++h) {
            const int64_t r0 = CH[h], r1 = CH[h + 1];
            if (Yc[r0] != Yc[r1 - 1]) {
                double num = 0.0;
                int den = 0;
                for (int64_t r = r0; r < r1; ++r) {
                    const int wr = Wc[r];
                    num += Yc[r] * (double)wr;
                    den += wr;
                }
                Yn[o] = num / (double)den;
                Wn[o] = den;
                ++o;
            } else {
                for (int64_t r = r0; r < r1; ++r, ++o) {
                    Yn[o] = Yc[r];
                    Wn[o] = Wc[r];
                }
            }
        }
        __syncthreads();
        double *ty = Yc;
        Yc = Yn;
        Yn = ty;
        int32_t *tw = Wc;
        Wc = Wn;
        Wn = tw;
        nh = NS;
    }
    // expand: run offsets (exclusive prefix of the run lengths) into CH
    {
        const int64_t a = seg_lo(nh, t), b = seg_lo(nh, t + 1);
        int64_t s = 0;
        for (int64_t r = a; r < b; ++r) s += Wc[r];
        int64_t tot;
        int64_t off = wg_exscan(s, sh, tot);
        for (int64_t r = a; r < b; ++r) {
            CH[r] = (int32_t)off;
            off += Wc[r];
        }
        if (t == 0) CH[nh] = (int32_t)k;
        __syncthreads();
    }
    const int64_t ea = seg_lo(k, t), eb = seg_lo(k, t + 1);
    if (ea < eb) {
        int64_t lo = 0, hi = nh - 1;              // last run with CH[r] <= ea
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (CH[mid] <= ea) lo = mid;
            else hi = mid - 1;
        }
        int64_t r = lo;
        for (int64_t e = ea; e < eb; ++e) {
            while (CH[r + 1] <= e) ++r;
            y[e] = Yc[r];
        }
    }
    __syncthreads();
}

}  // namespace bsls
