// spmv.hip -- CSR sparse matrix-vector product (replaces SciPy csr_matvec behind
// A.dot(x), python/main.py:53-54; python/mirror_descent.py:32-34).
//
// G lanes per row (G = power of two <= 64, ~ the mean row length): the row's
// values and column indices stream coalesced across the group, x is gathered,
// the group sums by xor-shuffles (fixed tree).  HBM-bound: 12 B per nonzero +
// 8 B per row of output; the x gather is served mostly by L2 / Infinity Cache.
#include "spmv.hpp"

namespace bsls {

template <int G>
__global__ __launch_bounds__(256) void csr_spmv_kernel(
    int64_t m, const int64_t *__restrict__ indptr, const int32_t *__restrict__ indices,
    const double *__restrict__ data, const double *__restrict__ x,
    const double *__restrict__ add, double alpha, double *__restrict__ out,
    double *__restrict__ part, unsigned *__restrict__ ticket, double *__restrict__ sq_out) {
    constexpr int RPB = 256 / G;
    __shared__ double red[4];
    const int64_t row = (int64_t)blockIdx.x * RPB + threadIdx.x / G;
    const double v = csr_row_dot<G>(row, m, indptr, indices, data, x);
    double sq[1] = {0.0};
    if (row < m && (threadIdx.x % G) == 0) {
        double o = (alpha == 1.0) ? v : alpha * v;
        if (add) o += add[row];
        out[row] = o;
        sq[0] = o * o;
    }
    if (!sq_out) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0) *sq_out = tot[0];
}

template <int G>
static void launch_spmv(int64_t m, const int64_t *ip, const int32_t *ix, const double *d,
                        const double *x, const double *add, double alpha, double *out,
                        double *part, unsigned *ticket, double *sq, hipStream_t st) {
    constexpr int RPB = 256 / G;
    csr_spmv_kernel<G><<<grid_for(m, RPB), 256, 0, st>>>(m, ip, ix, d, x, add, alpha, out, part,
                                                         ticket, sq);
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_spmv_workspace_size(int64_t m) {
    return 16 + (size_t)(((m + 3) / 4 + 1) * 8);
}

extern "C" int bsls_csr_spmv(int64_t m, const int64_t *d_indptr, const int32_t *d_indices,
                             const double *d_data, const double *d_x, const double *d_add,
                             double alpha, double *d_out, double *d_sq_out, int group,
                             void *d_work, size_t work_bytes, void *stream) {
    if (m <= 0 || !d_indptr || !d_x || !d_out) return BSLS_E_ARG;
    if (d_sq_out && (!d_work || work_bytes < bsls_spmv_workspace_size(m))) return BSLS_E_WORKSPACE;
    unsigned *ticket = d_work ? (unsigned *)d_work : nullptr;
    double *part = d_work ? (double *)((char *)d_work + 16) : nullptr;
    hipStream_t st = (hipStream_t)stream;
    switch (group) {
        case 1: launch_spmv<1>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 2: launch_spmv<2>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 4: launch_spmv<4>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 8: launch_spmv<8>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 16: launch_spmv<16>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 32: launch_spmv<32>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        case 64: launch_spmv<64>(m, d_indptr, d_indices, d_data, d_x, d_add, alpha, d_out, part, ticket, d_sq_out, st); break;
        default: return BSLS_E_ARG;
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
