// spmv.hpp -- CSR-stream tile SpMV shared by the generic SpMV and the fused BB
// kernels (csrc/bb.hip).
//
// A host-planned tile = a run of whole rows [r0, r1) (bsls_csr_plan_tiles).  One
// 256-thread workgroup per tile walks the tile's nonzeros in chunks of NZT:
// every thread loads NZT/256 (index, value) pairs -- coalesced, all in flight
// at once -- gathers x and stores the products in LDS; then G lanes per row sum
// the row's products (fixed strided order + xor tree) into wl[row - r0].  Long
// rows simply span several chunks (partials added in chunk order).  The order
// of every sum is fixed by (tile, G), so results are bit-reproducible.
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int TB = 256;        // threads per tile workgroup
constexpr int NZT = 2048;      // nonzeros staged per chunk (16 KiB of products)
constexpr int RMAX = 1024;     // rows per tile (capacity of wl)
constexpr int MAX_TILE_WG = 1024;  // persistent grid: workgroups walk tiles round-robin

template <int G>
__device__ __forceinline__ void tile_rows(const int64_t *__restrict__ indptr,
                                          const int32_t *__restrict__ indices,
                                          const double *__restrict__ data,
                                          const double *__restrict__ x, int64_t r0, int64_t r1,
                                          double *__restrict__ prod, double *__restrict__ wl) {
    const int nrows = (int)(r1 - r0);
    __syncthreads();   // the previous tile's epilogue may still be reading wl
    for (int t = threadIdx.x; t < nrows; t += TB) wl[t] = 0.0;
    const int64_t e0 = indptr[r0], e1 = indptr[r1];
    const int gl = (int)(threadIdx.x % G);
    for (int64_t cs = e0; cs < e1; cs += NZT) {
        const int64_t ce = (cs + NZT < e1) ? cs + NZT : e1;
        __syncthreads();
        int32_t col[NZT / TB];
        double val[NZT / TB];
#pragma unroll
        for (int k = 0; k < NZT / TB; ++k) {
            const int64_t e = cs + threadIdx.x + k * TB;
            col[k] = (e < ce) ? indices[e] : 0;
            val[k] = (e < ce) ? data[e] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < NZT / TB; ++k) {
            const int64_t e = cs + threadIdx.x + k * TB;
            if (e < ce) prod[e - cs] = val[k] * x[col[k]];
        }
        __syncthreads();
        for (int rr = (int)(threadIdx.x / G); rr < nrows; rr += TB / G) {
            int64_t a = indptr[r0 + rr], b = indptr[r0 + rr + 1];
            a = a > cs ? a : cs;
            b = b < ce ? b : ce;
            double v = 0.0;
            for (int64_t q = a + gl; q < b; q += G) v += prod[q - cs];
            v = group_sum<G>(v);
            if (gl == 0 && a < b) wl[rr] += v;
        }
    }
    __syncthreads();
}

}  // namespace bsls
