// misc.hip -- z<->x change of variables, the dense-QP helpers kept for ABI
// parity, and the mirror-descent block update.
#include "bsls_common.hpp"

#include <string.h>

namespace bsls {

// x2z_c (c_extensions.pyx:195-220): z = running sum of each block's first k-1
// entries (sequential, as the reference).  One lane per block.
__global__ __launch_bounds__(256) void x2z_kernel(const double *__restrict__ x,
                                                  double *__restrict__ z,
                                                  const int64_t *__restrict__ starts,
                                                  int64_t nb, int64_t n) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t s = starts[b], e = block_end(starts, nb, b, n);
    int64_t j = s - b;  // z offset: every earlier block contributed k-1 entries
    double acc = 0.0;
    for (int64_t i = s; i < e - 1; ++i) {
        acc += x[i];
        z[j++] = acc;
    }
}

// z2x_c (c_extensions.pyx:223-248): x_i = z_j - z_{j-1}, last = 1 - z_last.
// Element-parallel: each x entry needs only its two z neighbours.
__global__ __launch_bounds__(256) void z2x_kernel(double *__restrict__ x,
                                                  const double *__restrict__ z,
                                                  const int64_t *__restrict__ starts,
                                                  int64_t nb, int64_t n) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t s = starts[b], e = block_end(starts, nb, b, n);
    const int64_t zs = s - b;
    double prev = 0.0;
    for (int64_t i = s; i < e - 1; ++i) {
        const double zj = z[zs + (i - s)];
        x[i] = zj - prev;
        prev = zj;
    }
    x[e - 1] = 1.0 - prev;
}

// N z / x0 + N z, element-parallel with a per-block lane (one lane per block).
__global__ __launch_bounds__(256) void n_apply_kernel(double *__restrict__ x,
                                                      const double *__restrict__ z,
                                                      const int64_t *__restrict__ starts,
                                                      int64_t nb, int64_t n, double last) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t s = starts[b], e = block_end(starts, nb, b, n);
    const int64_t zs = s - b;
    double prev = 0.0;
    for (int64_t i = s; i < e - 1; ++i) {
        const double zj = z[zs + (i - s)];
        x[i] = zj - prev;
        prev = zj;
    }
    x[e - 1] = last - prev;
}

// g = N' w: g_j = w_i - w_{i+1} for every x entry i that is not a block's last.
__global__ __launch_bounds__(256) void nt_apply_kernel(const double *__restrict__ w,
                                                       double *__restrict__ g,
                                                       const int64_t *__restrict__ starts,
                                                       int64_t nb, int64_t n) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t s = starts[b], e = block_end(starts, nb, b, n);
    const int64_t zs = s - b;
    for (int64_t i = s; i < e - 1; ++i) g[zs + (i - s)] = w[i] - w[i + 1];
}

// quad_obj (quadratic_objective.h:15-26): g = Q x + c row by row (sequential in
// j), f = sum_i 0.5 (g_i + c_i) x_i (sequential in i).  One workgroup.
__device__ void quad_obj_block(const double *x, const double *Q, const double *c, double *g,
                               int64_t n, double *f_out) {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        double gi = c[i];
        const double *row = Q + i * n;
        for (int64_t j = 0; j < n; ++j) gi += row[j] * x[j];
        g[i] = gi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double f = 0;
        for (int64_t i = 0; i < n; ++i) f += 0.5 * (g[i] + c[i]) * x[i];
        *f_out = f;
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void quad_obj_kernel(const double *x, const double *Q,
                                                       const double *c, double *g, int64_t n,
                                                       double *f_out) {
    quad_obj_block(x, Q, c, g, n, f_out);
}

// line_search (quadratic_objective.h:29-61), halving backtracking.  The
// reference's "step too small" branch stores g_new[n] out of bounds instead of
// copying g into g_new (an unbraced for); on valid memory g_new therefore keeps
// its last value -- reproduced here without the stray store.
__global__ __launch_bounds__(256) void line_search_kernel(const double *x, double f,
                                                          const double *g, double *x_new,
                                                          double f_new, double *g_new,
                                                          const double *Q, const double *c,
                                                          int64_t n, double *f_out) {
    __shared__ double sh[4];  // upper, t, f_new, flag
    const double suff = 1e-4, prog = 1e-8;
    if (threadIdx.x == 0) {
        double upper = f;
        for (int64_t i = 0; i < n; ++i) upper += suff * g[i] * (x_new[i] - x[i]);
        sh[0] = upper;
        sh[1] = 1.0;
        sh[2] = f_new;
    }
    __syncthreads();
    for (;;) {
        if (threadIdx.x == 0) {
            double stop = 0.0;
            if (!(sh[2] > sh[0])) {
                stop = 1.0;
            } else {
                sh[1] *= .5;
                double span = 0.0;
                for (int64_t i = 0; i < n; ++i) {
                    if (x_new[i] - x[i] > span) span = x_new[i] - x[i];
                    if (x[i] - x_new[i] > span) span = x[i] - x_new[i];
                }
                if (sh[1] * span < prog) stop = 2.0;
            }
            sh[3] = stop;
        }
        __syncthreads();
        const double stop = sh[3];
        if (stop == 1.0) break;
        if (stop == 2.0) {
            for (int64_t i = threadIdx.x; i < n; i += blockDim.x) x_new[i] = x[i];
            if (threadIdx.x == 0) sh[2] = f;
            __syncthreads();
            break;
        }
        const double t = sh[1];
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) x_new[i] = x[i] + t * (x_new[i] - x[i]);
        __syncthreads();
        quad_obj_block(x_new, Q, c, g_new, n, &sh[2]);
        if (threadIdx.x == 0) {
            double upper = sh[0];
            for (int64_t i = 0; i < n; ++i) upper += suff * g[i] * (x_new[i] - x[i]);
            sh[0] = upper;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *f_out = sh[2];
}

// Mirror-descent step (mirror_descent.py:37-47): per coordinate
// up = g * t, t = sqrt(2 ln k_b) / scale (scale = sqrt(k) Lf from the host),
// x <- x * exp(-up), then each block divided by its sum; per-block
// max|x_new - x_old| into part[], reduced by the last workgroup into *dxinf.
// With `state` (gated form): nothing happens once state[0] != 0; the launch
// that sees ||x_new - x_old||_inf < tol sets state[0] = 1 and state[2] = iter
// (the reference's break), state[1] = the norm every launch.
__global__ __launch_bounds__(256) void md_kernel(double *__restrict__ x,
                                                 const double *__restrict__ g,
                                                 const int64_t *__restrict__ starts,
                                                 int64_t nb, int64_t n, double scale,
                                                 double *__restrict__ dxinf,
                                                 double *__restrict__ part,
                                                 unsigned *__restrict__ ticket,
                                                 double *__restrict__ state, double tol,
                                                 int64_t iter) {
    __shared__ double red[4];
    if (state && state[0] != 0.0) return;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double dmax = 0.0;
    if (b < nb) {
        const int64_t s = starts[b], e = block_end(starts, nb, b, n);
        const double t = sqrt(2.0 * log((double)(e - s))) / scale;
        double acc = 0.0;
        for (int64_t i = s; i < e; ++i) {
            const double up = g[i] * t;
            acc += x[i] * exp(-up);
        }
        for (int64_t i = s; i < e; ++i) {
            const double up = g[i] * t;
            const double xo = x[i];
            const double xn = (xo * exp(-up)) / acc;
            const double d = fabs(xn - xo);
            dmax = (d > dmax || d != d) ? d : dmax;
            x[i] = xn;
        }
    }
    // block max (order-independent), then last-workgroup max over partials
    dmax = wave_max(dmax);
    if (lane_id() == 0) red[threadIdx.x / WAVE] = dmax;
    __syncthreads();
    double mine[1] = {0.0};
    if (threadIdx.x == 0) {
        double m = red[0];
        for (int w = 1; w < (int)(blockDim.x / WAVE); ++w) m = red[w] > m ? red[w] : m;
        mine[0] = m;
    }
    __shared__ int am_last;
    if (threadIdx.x == 0) {   // sc1 hand-off, as bsls_common.hpp last_block_sum
        __hip_atomic_store(&part[blockIdx.x], mine[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        am_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!am_last) return;
    if (threadIdx.x == 0) {
        double m = 0.0;
        for (unsigned i = 0; i < gridDim.x; ++i) {
            const double v = __hip_atomic_load(&part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            m = v > m ? v : m;
        }
        if (dxinf) *dxinf = m;
        if (state) {
            state[1] = m;
            if (m < tol) {                       // mirror_descent.py:50-51
                state[0] = 1.0;
                state[2] = (double)iter;
            }
        }
        *ticket = 0u;
    }
}

// The same update with one wave per PACK of whole blocks (<= 64 entries, one
// lane per entry; host-planned, like K3's packs): coalesced loads and stores,
// one exp per entry, the block sums by a segmented shuffle scan (a fixed tree
// order instead of left to right -- mirror descent is not bit-pinned: np.exp
// and np.sum differ from any device order anyway).  A block longer than 64
// entries is a pack of its own, summed by the whole wave.  Gated form only.
__device__ __forceinline__ double md_shfl(double v, int src) { return __shfl(v, src, WAVE); }
constexpr int MD_PACK_WAVES = 16;   // packs per 1024-thread workgroup
// max over the wave, NaN-propagating (the reference's inf-norm is NaN then)
__device__ __forceinline__ double wave_nan_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = nan_max(v, __shfl_xor(v, o, WAVE));
    return v;
}

__global__ __launch_bounds__(1024) void md_pack_kernel(double *__restrict__ x,
                                                      const double *__restrict__ g,
                                                      const int64_t *__restrict__ pk_x0,
                                                      const int64_t *__restrict__ pk_mask,
                                                      const int32_t *__restrict__ pk_len,
                                                      int64_t npacks, double scale,
                                                      double *__restrict__ part,
                                                      unsigned *__restrict__ ticket,
                                                      double *__restrict__ state, double tol,
                                                      int64_t iter) {
    __shared__ double red[MD_PACK_WAVES];
    __shared__ double c2lk[WAVE + 1];   // sqrt(2 log k), k = 1 .. 64: blocks of a packed wave
    if (state[0] != 0.0) return;
    const int l = threadIdx.x % WAVE, wv = threadIdx.x / WAVE;
    const int64_t pk = (int64_t)blockIdx.x * MD_PACK_WAVES + wv;
    // one log and one sqrt per size class and workgroup instead of per entry
    // (they were ~60 of the ~150 VALU instructions an entry cost)
    if (threadIdx.x < WAVE) c2lk[threadIdx.x + 1] = sqrt(2.0 * log((double)(threadIdx.x + 1)));
    __syncthreads();
    double dmax = 0.0;
    if (pk < npacks) {
        const int64_t x0 = pk_x0[pk];
        const int L = pk_len[pk];
        if (L <= WAVE) {
            const uint64_t B = (uint64_t)pk_mask[pk];
            const bool act = l < L;
            const uint64_t le = (l >= 63) ? ~0ull : ((2ull << l) - 1ull);
            const uint64_t below = B & le;                        // block starts at or before l
            const int st = 63 - __clzll((long long)below);        // this entry's block start
            const uint64_t above = B & ~le;
            const int en = (above ? (__ffsll((long long)above) - 1) : L) - 1;   // its last entry
            const double xo = act ? x[x0 + l] : 0.0;
            const double gv = act ? g[x0 + l] : 0.0;
            const double t = c2lk[en - st + 1] / scale;
            const double v = act ? xo * exp(-(gv * t)) : 0.0;
            // segmented inclusive scan (segments = blocks)
            double acc = v;
#pragma unroll
            for (int off = 1; off < WAVE; off <<= 1) {
                const double y = md_shfl(acc, l >= off ? l - off : l);
                if (l - off >= st) acc += y;
            }
            const double tot = md_shfl(acc, en < 0 ? 0 : en);
            if (act) {
                const double xn = v / tot;
                const double d = fabs(xn - xo);
                dmax = d;
                x[x0 + l] = xn;
            }
        } else {
            // one block of L > 64 entries: strided partial sums, then the wave's
            const double t = sqrt(2.0 * log((double)L)) / scale;
            double acc = 0.0;
            for (int i = l; i < L; i += WAVE) acc += x[x0 + i] * exp(-(g[x0 + i] * t));
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, WAVE);
            for (int i = l; i < L; i += WAVE) {
                const double xo = x[x0 + i];
                const double xn = (xo * exp(-(g[x0 + i] * t))) / acc;
                const double d = fabs(xn - xo);
                dmax = (d > dmax || d != d) ? d : dmax;
                x[x0 + i] = xn;
            }
        }
    }
    double v1[1] = {dmax}, tot[1];
    block_reduce<1, 1u>(v1, red);
    if (last_block_reduce<1, 1u>(v1, part, ticket, tot, red) && threadIdx.x == 0) {
        state[1] = tot[0];
        if (tot[0] < tol) {                      // mirror_descent.py:50-51
            state[0] = 1.0;
            state[2] = (double)iter;
        }
    }
}

// BATCH.solve_MD's update (python/BATCH.py:238-240) and
// algorithm_utils.normalization (python/algorithm_utils.py:175-179):
// y = x * exp((-t) * g) elementwise (y = x when g == NULL), then every block
// [starts[b], end_b) divided by its sum (x[s:e] / np.sum(x[s:e])).  Entries
// before starts[0] get the elementwise update only.  One lane per block; the
// block sum is sequential (NumPy's pairwise sum differs from it only in the
// last bits for blocks >= 8, and np.exp is not correctly rounded either).
__global__ __launch_bounds__(256) void md_step_kernel(const double *x,
                                                      const double *__restrict__ g,
                                                      double *y,
                                                      const int64_t *__restrict__ starts,
                                                      int64_t nb, int64_t n, double t) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const double mt = -t;
    if (b == 0) {
        for (int64_t i = 0; i < starts[0]; ++i) y[i] = g ? x[i] * exp(mt * g[i]) : x[i];
    }
    const int64_t s = starts[b], e = block_end(starts, nb, b, n);
    double acc = 0.0;
    for (int64_t i = s; i < e; ++i) {
        const double v = g ? x[i] * exp(mt * g[i]) : x[i];
        y[i] = v;
        acc += v;
    }
    for (int64_t i = s; i < e; ++i) y[i] = y[i] / acc;
}

}  // namespace bsls

using namespace bsls;

extern "C" int bsls_x2z(const double *d_x, double *d_z, const int64_t *d_starts, int64_t nblocks,
                        int64_t n, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_starts) return BSLS_E_ARG;
    x2z_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(d_x, d_z, d_starts, nblocks, n);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_z2x(double *d_x, const double *d_z, const int64_t *d_starts, int64_t nblocks,
                        int64_t n, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_starts) return BSLS_E_ARG;
    z2x_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(d_x, d_z, d_starts, nblocks, n);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_n_apply(double *d_x, const double *d_z, const int64_t *d_starts,
                            int64_t nblocks, int64_t n, int with_x0, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_starts) return BSLS_E_ARG;
    n_apply_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(
        d_x, d_z, d_starts, nblocks, n, with_x0 ? 1.0 : 0.0);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_nt_apply(const double *d_w, double *d_g, const int64_t *d_starts,
                             int64_t nblocks, int64_t n, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_w || !d_starts) return BSLS_E_ARG;
    nt_apply_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(d_w, d_g, d_starts,
                                                                             nblocks, n);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_quad_obj(const double *d_x, const double *d_Q, const double *d_c, double *d_g,
                             int64_t n, double *d_f, void *stream) {
    if (n <= 0 || !d_x || !d_Q || !d_c || !d_g || !d_f) return BSLS_E_ARG;
    quad_obj_kernel<<<1, 256, 0, (hipStream_t)stream>>>(d_x, d_Q, d_c, d_g, n, d_f);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_line_search(const double *d_x, double f, const double *d_g, double *d_x_new,
                                double f_new, double *d_g_new, const double *d_Q,
                                const double *d_c, int64_t n, double *d_f_out, void *stream) {
    if (n <= 0 || !d_x || !d_g || !d_x_new || !d_g_new || !d_Q || !d_c || !d_f_out) return BSLS_E_ARG;
    line_search_kernel<<<1, 256, 0, (hipStream_t)stream>>>(d_x, f, d_g, d_x_new, f_new, d_g_new, d_Q,
                                                           d_c, n, d_f_out);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" size_t bsls_md_workspace_size(int64_t nblocks) {
    const int64_t grid = (nblocks + 255) / 256;
    return (size_t)(TICKET_BYTES + ((grid * 8 + 15) & ~(int64_t)15));
}

extern "C" int bsls_md_update(double *d_x, const double *d_g, const int64_t *d_starts,
                              int64_t nblocks, int64_t n, double step_scale, double *d_dxinf,
                              void *d_work, size_t work_bytes, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_g || !d_starts || !d_dxinf) return BSLS_E_ARG;
    if (!d_work || work_bytes < bsls_md_workspace_size(nblocks)) return BSLS_E_WORKSPACE;
    unsigned *ticket = (unsigned *)d_work;
    double *part = (double *)((char *)d_work + TICKET_BYTES);
    md_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(
        d_x, d_g, d_starts, nblocks, n, step_scale, d_dxinf, part, ticket, nullptr, 0.0, 0);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_md_update_gated(double *d_x, const double *d_g, const int64_t *d_starts,
                                    int64_t nblocks, int64_t n, double step_scale, double tol,
                                    int64_t iter, double *d_state, void *d_work,
                                    size_t work_bytes, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_g || !d_starts || !d_state) return BSLS_E_ARG;
    if (!d_work || work_bytes < bsls_md_workspace_size(nblocks)) return BSLS_E_WORKSPACE;
    unsigned *ticket = (unsigned *)d_work;
    double *part = (double *)((char *)d_work + TICKET_BYTES);
    md_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(
        d_x, d_g, d_starts, nblocks, n, step_scale, nullptr, part, ticket, d_state, tol, iter);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" size_t bsls_md_pack_workspace_size(int64_t npacks) {
    const int64_t grid = (npacks + MD_PACK_WAVES - 1) / MD_PACK_WAVES;
    return (size_t)(TICKET_BYTES + ((grid * 8 + 15) & ~(int64_t)15));
}

extern "C" int bsls_md_update_packs(double *d_x, const double *d_g, const int64_t *d_pk_x0,
                                    const int64_t *d_pk_mask, const int32_t *d_pk_len,
                                    int64_t npacks, double step_scale, double tol, int64_t iter,
                                    double *d_state, void *d_work, size_t work_bytes,
                                    void *stream) {
    if (npacks <= 0 || !d_x || !d_g || !d_pk_x0 || !d_pk_mask || !d_pk_len || !d_state)
        return BSLS_E_ARG;
    if (!d_work || work_bytes < bsls_md_pack_workspace_size(npacks)) return BSLS_E_WORKSPACE;
    unsigned *ticket = (unsigned *)d_work;
    double *part = (double *)((char *)d_work + TICKET_BYTES);
    md_pack_kernel<<<(int)((npacks + MD_PACK_WAVES - 1) / MD_PACK_WAVES), 64 * MD_PACK_WAVES, 0,
                     (hipStream_t)stream>>>(
        d_x, d_g, d_pk_x0, d_pk_mask, d_pk_len, npacks, step_scale, part, ticket, d_state, tol,
        iter);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_md_step(const double *d_x, const double *d_g, double *d_y,
                            const int64_t *d_starts, int64_t nblocks, int64_t n, double t,
                            void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_x || !d_y || !d_starts) return BSLS_E_ARG;
    md_step_kernel<<<grid_for(nblocks, 256), 256, 0, (hipStream_t)stream>>>(d_x, d_g, d_y, d_starts,
                                                                            nblocks, n, t);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" const char *bsls_version(void) { return "bsls-hip 0.1 (gfx950)"; }

extern "C" int bsls_device_arch(char *buf, int buflen) {
    hipDeviceProp_t prop;
    int dev = 0;
    BSLS_CHECK(hipGetDevice(&dev));
    BSLS_CHECK(hipGetDeviceProperties(&prop, dev));
    if (buf && buflen > 0) {
        strncpy(buf, prop.gcnArchName, (size_t)buflen - 1);
        buf[buflen - 1] = 0;
    }
    return BSLS_OK;
}
