// pava.hip -- multi-block isotonic regression entry point
// (replaces isotonic_regression_multi{,_2,_3}, isotonic_regression.h:85-102,157-164).
//
// Layout: one 64-lane workgroup per 64 consecutive blocks, one lane per block.
// The wave's contiguous element range is staged into LDS with coalesced loads
// (y as fp64, run lengths as int32), every lane runs the serial PAVA of its own
// block in LDS, and the range is written back coalesced.  A wave whose range
// exceeds ISO_CAP elements runs the same code on global memory instead (run
// lengths then live in the caller's weight array or in the workspace).
#include "pava.hpp"

namespace bsls {

constexpr int ISO_CAP = 2048;

template <int VARIANT>
__global__ __launch_bounds__(WAVE) void iso_kernel(double *__restrict__ y,
                                                   const int64_t *__restrict__ starts,
                                                   int64_t nb, int64_t n,
                                                   int32_t *__restrict__ wio, int expand,
                                                   int32_t *__restrict__ wscratch,
                                                   int32_t *__restrict__ status) {
    __shared__ double ly[ISO_CAP];
    __shared__ int32_t lw[ISO_CAP];
    const int lane = lane_id();
    const int64_t b0 = (int64_t)blockIdx.x * WAVE;
    const int64_t b = b0 + lane;
    const bool valid = b < nb;
    const int64_t s = valid ? starts[b] : 0;
    const int64_t e = valid ? block_end(starts, nb, b, n) : 0;
    const int64_t blast = (b0 + WAVE - 1 < nb) ? b0 + WAVE - 1 : nb - 1;
    const int64_t R0 = starts[b0];
    const int64_t R = block_end(starts, nb, blast, n) - R0;
    bool ok = true;
    if (R <= ISO_CAP) {
        const int r = (int)R;
        for (int j = lane; j < r; j += WAVE) {
            ly[j] = y[R0 + j];
            if (VARIANT != 2) lw[j] = wio ? wio[R0 + j] : 1;
        }
        __syncthreads();
        if (valid) {
            const int lo = (int)(s - R0), hi = (int)(e - R0);
            if (VARIANT == 1) ok = pava_v1(ly, lw, lo, hi, expand);
            else if (VARIANT == 2) pava_v2(ly, lo, hi);
            else ok = pava_v3(ly, lw, lo, hi, expand);
        }
        __syncthreads();
        for (int j = lane; j < r; j += WAVE) {
            y[R0 + j] = ly[j];
            if (VARIANT != 2 && wio) wio[R0 + j] = lw[j];
        }
    } else if (valid) {
        if (VARIANT == 2) {
            pava_v2(y, s, e);
        } else {
            int32_t *W = wio ? wio : wscratch;
            if (!wio)
                for (int64_t j = s; j < e; ++j) W[j] = 1;
            ok = (VARIANT == 1) ? pava_v1(y, W, s, e, expand) : pava_v3(y, W, s, e, expand);
        }
    }
    if (!ok && status) atomicOr(status, 1);
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_isotonic_workspace_size(int64_t n) {
    return (size_t)((n * 4 + 15) & ~(int64_t)15);
}

extern "C" int bsls_isotonic_multi(int variant, double *d_y, const int64_t *d_starts,
                                   int64_t nblocks, int64_t n, int32_t *d_weight, int expand,
                                   int64_t max_block, void *d_work, size_t work_bytes,
                                   int32_t *d_status, void *stream) {
    (void)max_block;
    if (nblocks <= 0 || n <= 0 || !d_y || !d_starts) return BSLS_E_ARG;
    if (variant < 1 || variant > 3) return BSLS_E_ARG;
    if (variant != 2 && !d_weight && (!d_work || work_bytes < bsls_isotonic_workspace_size(n)))
        return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const int grid = grid_for(nblocks, WAVE);
    int32_t *ws = (int32_t *)d_work;
    if (variant == 1)
        iso_kernel<1><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, d_weight, expand, ws, d_status);
    else if (variant == 2)
        iso_kernel<2><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, nullptr, 0, nullptr, d_status);
    else
        iso_kernel<3><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, d_weight, expand, ws, d_status);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
