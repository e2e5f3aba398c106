// spmv.hip -- CSR sparse matrix-vector product (replaces SciPy csr_matvec behind
// A.dot(x), python/main.py:53-54; python/mirror_descent.py:32-34) and the host
// tile planner shared with the fused BB kernels.
//
// HBM-bound: 12 B per nonzero (fp64 value + int32 index) + 8 B per row of
// output + the x gather.  One workgroup per host-planned tile (spmv.hpp).
#include <algorithm>
#include <vector>

#include "spmv.hpp"

namespace bsls {

template <int G>
__global__ __launch_bounds__(TB) void csr_spmv_tiles(
    const int64_t *__restrict__ tiles, int64_t ntiles, const int64_t *__restrict__ indptr,
    const int32_t *__restrict__ indices, const double *__restrict__ data,
    const double *__restrict__ x, const double *__restrict__ add, double alpha,
    double *__restrict__ out, double *__restrict__ part, unsigned *__restrict__ ticket,
    double *__restrict__ sq_out) {
    __shared__ double prod[NZT];
    __shared__ double wl[RMAX];
    __shared__ double red[4];
    double sq[1] = {0.0};
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tiles[tile], r1 = tiles[tile + 1];
        tile_rows<G>(indptr, indices, data, x, r0, r1, prod, wl);
        for (int t = threadIdx.x; t < (int)(r1 - r0); t += TB) {
            double o = (alpha == 1.0) ? wl[t] : alpha * wl[t];
            if (add) o += add[r0 + t];
            out[r0 + t] = o;
            sq[0] += o * o;
        }
    }
    if (!sq_out) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0) *sq_out = tot[0];
}

// Greedy tiles of whole rows: <= nzt nonzeros (unless one row alone is longer)
// and <= rmax rows; when `ends` is given a tile may only end at one of those
// row indices (used to keep z-blocks inside one tile for the fused N').
static int64_t plan_tiles(const int64_t *indptr, int64_t m, int64_t nzt, int64_t rmax,
                          const int64_t *ends, int64_t nends, int64_t *out, int64_t cap) {
    std::vector<int64_t> allowed;
    if (ends) {
        allowed.assign(ends, ends + nends);
        std::sort(allowed.begin(), allowed.end());
        if (allowed.empty() || allowed.back() != m) allowed.push_back(m);
    }
    int64_t cnt = 0;
    if (cap > 0) out[0] = 0;
    int64_t r0 = 0;
    while (r0 < m) {
        // largest r with indptr[r] - indptr[r0] <= nzt
        const int64_t lim = indptr[r0] + nzt;
        int64_t r = std::upper_bound(indptr + r0, indptr + m + 1, lim) - indptr - 1;
        if (r > r0 + rmax) r = r0 + rmax;
        if (r > m) r = m;
        int64_t r1;
        if (ends) {
            auto it = std::upper_bound(allowed.begin(), allowed.end(), r);
            // last allowed end <= r that is > r0, else the first allowed end > r0
            if (it != allowed.begin() && *(it - 1) > r0) r1 = *(it - 1);
            else r1 = *std::upper_bound(allowed.begin(), allowed.end(), r0);
        } else {
            r1 = (r > r0) ? r : r0 + 1;
        }
        if (r1 - r0 > rmax) return -2;   // a block longer than rmax rows (fused N' limit)
        ++cnt;
        if (cnt < cap) out[cnt] = r1;
        r0 = r1;
    }
    return cnt;
}

}  // namespace bsls

using namespace bsls;

extern "C" int64_t bsls_csr_plan_tiles(const int64_t *indptr, int64_t m, int64_t nzt,
                                       int64_t rmax, const int64_t *ends, int64_t nends,
                                       int64_t *tiles_out, int64_t cap) {
    if (!indptr || m <= 0) return -1;
    if (nzt <= 0) nzt = NZT;
    if (rmax <= 0 || rmax > RMAX) rmax = RMAX;
    return plan_tiles(indptr, m, nzt, rmax, ends, nends, tiles_out, cap);
}

extern "C" size_t bsls_spmv_workspace_size(int64_t ntiles) {
    return TICKET_BYTES + (size_t)((ntiles + 1) * 8);
}

extern "C" int bsls_csr_spmv(int64_t m, const int64_t *d_indptr, const int32_t *d_indices,
                             const double *d_data, const int64_t *d_tiles, int64_t ntiles,
                             const double *d_x, const double *d_add, double alpha,
                             double *d_out, double *d_sq_out, int group, void *d_work,
                             size_t work_bytes, void *stream) {
    if (m <= 0 || !d_indptr || !d_tiles || ntiles <= 0 || !d_x || !d_out) return BSLS_E_ARG;
    if (d_sq_out && (!d_work || work_bytes < bsls_spmv_workspace_size(ntiles)))
        return BSLS_E_WORKSPACE;
    unsigned *ticket = d_work ? (unsigned *)d_work : nullptr;
    double *part = d_work ? (double *)((char *)d_work + TICKET_BYTES) : nullptr;
    hipStream_t st = (hipStream_t)stream;
    const int grid = (int)(ntiles < MAX_TILE_WG ? ntiles : MAX_TILE_WG);
    switch (group) {
#define SPMV_CASE(G)                                                                       \
    case G:                                                                                \
        csr_spmv_tiles<G><<<grid, TB, 0, st>>>(d_tiles, ntiles, d_indptr, d_indices, d_data, d_x,   \
                                               d_add, alpha, d_out, part, ticket, d_sq_out); \
        break;
        SPMV_CASE(1) SPMV_CASE(2) SPMV_CASE(4) SPMV_CASE(8) SPMV_CASE(16) SPMV_CASE(32)
        SPMV_CASE(64)
#undef SPMV_CASE
        default:
            return BSLS_E_ARG;
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
