// spmv.hpp -- CSR row dot product shared by the generic SpMV and the fused BB
// kernels.
#pragma once
#include "bsls_common.hpp"

namespace bsls {

// Sum over row `row` of data[e] * x[indices[e]] by G consecutive lanes; the
// result is valid in every lane of the group (0 for row >= m).
template <int G>
__device__ __forceinline__ double csr_row_dot(int64_t row, int64_t m,
                                              const int64_t *__restrict__ indptr,
                                              const int32_t *__restrict__ indices,
                                              const double *__restrict__ data,
                                              const double *__restrict__ x) {
    double v = 0.0;
    if (row < m) {
        const int gl = (int)(threadIdx.x % G);
        const int64_t e0 = indptr[row], e1 = indptr[row + 1];
        for (int64_t e = e0 + gl; e < e1; e += G) v += data[e] * x[indices[e]];
    }
    return group_sum<G>(v);
}

}  // namespace bsls
