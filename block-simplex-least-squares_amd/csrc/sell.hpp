// sell.hpp -- sliced ELLPACK (SELL-C-64) row dot products for the fused BB SpMVs.
//
// Layout (built on the host once per matrix, device.build_sell): rows are cut
// into slices of 64 (optionally permuted, `perm`); slice s holds W_s = its
// longest row's length columns, stored column-major: entry k of the row at
// slice position p sits at sptr[s] + 64 k + p.  Padding entries carry column
// -1.  One wave = one slice: every index / value load is a fully coalesced
// 256-B / 512-B wave access, all independent (no row-pointer chain), and each
// lane sums its own row sequentially in CSR order -- the summation order of
// SciPy's csr_matvec (bit-identical partial sums).
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int SELL_C = 64;
constexpr int SELL_U = 8;   // entries in flight per lane

// Sequential row sum (in storage order) of entries [0, W) of the row at
// `base` (= sptr[s] + p), gathering x; `v` is the running sum to continue.
__device__ __forceinline__ double sell_row(const int32_t *__restrict__ sidx,
                                           const double *__restrict__ sval,
                                           const double *__restrict__ x, int64_t base, int W,
                                           double v) {
    for (int k0 = 0; k0 < W; k0 += SELL_U) {
        int32_t col[SELL_U];
        double val[SELL_U];
#pragma unroll
        for (int u = 0; u < SELL_U; ++u) {
            const int k = k0 + u;
            if (k < W) {
                const int64_t e = base + (int64_t)k * SELL_C;
                col[u] = __builtin_nontemporal_load(&sidx[e]);
                val[u] = __builtin_nontemporal_load(&sval[e]);
            } else {
                col[u] = -1;
                val[u] = 0.0;
            }
        }
        double xv[SELL_U];
#pragma unroll
        for (int u = 0; u < SELL_U; ++u) xv[u] = (col[u] >= 0) ? x[col[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < SELL_U; ++u)
            if (col[u] >= 0) v += val[u] * xv[u];
    }
    return v;
}

}  // namespace bsls
