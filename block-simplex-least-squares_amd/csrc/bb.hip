// bb.hip -- fused z-space projected Barzilai-Borwein iteration on one GCD.
//
// Reference loop (python/BB.py:17-41) over main.solve_in_z's closures
// (python/main.py:53-65), stopping rule solvers.stopping (python/solvers.py:40-63):
//     g = N'A'(A N z + target);  dg = g - g_prev;  if sum(dg) == 0: break
//     t = (z - z_prev).dg / dg.dg;  z <- clip01(PAVA(z - t g));  fx = f(z); stop?
// One iteration here = three kernels, all HBM-bound, no host round trip:
//   K2  g = N'(A' r) with an explicit A' CSR (deterministic, no atomics): CSR-
//       stream tiles of A' that end at x-block ends, so the adjacent difference
//       N'w = w_i - w_{i+1} never leaves LDS; fused: dg, the four BB sums, the
//       store of g.
//   K3  t from the sums; per z-block PAVA (v1 pooling order, bit-identical to
//       isotonic_regression.h:13-58) + clip to [0,1] + the vector N z (per-block
//       differences, last entry -z_last), one lane per block over an LDS-staged
//       range.  N is never materialised.
//   K1  r = A (N z) + target, target = A x0 - b, exactly the reference's
//       A.dot(N.dot(z)) + target; ||r||^2 (next gradient's residual AND f(z)),
//       and the stopping test of the iteration, in the last workgroup.
// Every cross-workgroup sum is reduced in a fixed order by the last-arriving
// workgroup (bsls_common.hpp last_block_sum), so runs are bit-reproducible.
// Scalars live in device memory (scal[]); the host only polls them.
#include "pava.hpp"
#include "spmv.hpp"

namespace bsls {

constexpr int K3_CAP = 1024;   // z entries staged per K3 wave
constexpr int BPW = 16;        // z-blocks per K3 wave (one lane each)

struct BBWork {
    unsigned *tk1, *tk2, *tkf;
    double *p1, *p2, *pf;
    int32_t *wsc;
    size_t bytes;
};

static size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

static BBWork bb_layout(void *base, int64_t m, int64_t nz, int64_t max_tiles) {
    BBWork w{};
    char *p = (char *)base;
    size_t off = 0;
    w.tk1 = (unsigned *)(p + off);
    w.tk2 = (unsigned *)(p + off + TICKET_BYTES);
    w.tkf = (unsigned *)(p + off + 2 * TICKET_BYTES);
    off += al16(3 * TICKET_BYTES);
    w.p1 = (double *)(p + off);
    off += al16((size_t)(max_tiles + 1) * 8);
    w.p2 = (double *)(p + off);
    off += al16((size_t)(max_tiles + 1) * 4 * 8);
    w.pf = (double *)(p + off);
    off += al16((size_t)((m + 255) / 256 + 1) * 8);
    w.wsc = (int32_t *)(p + off);
    off += al16((size_t)(nz > 0 ? nz : 1) * 4);
    w.bytes = off;
    return w;
}

static BBWork bb_layout(const bsls_bb_problem &P) {
    const int64_t mt = P.A_ntiles > P.AT_ntiles ? P.A_ntiles : P.AT_ntiles;
    return bb_layout(P.work, P.m, P.nz, mt);
}

__device__ __forceinline__ void bb_stop_check(const bsls_bb_problem &P, int64_t iter, double fx) {
    double *s = P.scal;
    int reason = 0;
    if (iter >= P.max_iter) {
        reason = BSLS_STOP_MAXITER;
    } else if (P.early_exit) {
        const double gn = sqrt(s[BSLS_S_GG]);
        if (gn * gn <= P.opt_tol * (1 + fabs(fx))) reason = BSLS_STOP_GRAD;
        else if (sqrt(s[BSLS_S_DGDG]) == 0) reason = BSLS_STOP_DG;
    }
    if (reason) s[BSLS_S_STOP] = (double)reason;
}

__device__ __forceinline__ void bb_record_f(const bsls_bb_problem &P, int64_t iter, double rr,
                                            bool iterating) {
    double *s = P.scal;
    const double nr = sqrt(rr);
    const double fx = 0.5 * (nr * nr);  // 0.5 * la.norm(r)**2, main.py:53
    s[BSLS_S_RR] = rr;
    s[BSLS_S_FX] = fx;
    if (iterating) {
        s[BSLS_S_ITER] = (double)iter;
        s[BSLS_S_ZBUF] = (double)(iter & 1);
        bb_stop_check(P, iter, fx);
    }
}

// K1: r = A x (+ target); optional ||r||^2 and stopping test.  One workgroup
// per A tile (spmv.hpp); the tiles' partial ||r||^2 are reduced in tile order
// by the last workgroup.
template <int G, bool ADD, bool REDUCE, bool ITER>
__global__ __launch_bounds__(TB) void bb_k1(bsls_bb_problem P, int64_t iter, double *part,
                                            unsigned *ticket) {
    __shared__ double prod[NZT];
    __shared__ double wl[RMAX];
    __shared__ double red[4];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) return;
    double sq[1] = {0.0};
    for (int64_t tile = blockIdx.x; tile < P.A_ntiles; tile += gridDim.x) {
        const int64_t r0 = P.A_tiles[tile], r1 = P.A_tiles[tile + 1];
        tile_rows<G>(P.A_indptr, P.A_indices, P.A_data, P.x, r0, r1, prod, wl);
        for (int t = threadIdx.x; t < (int)(r1 - r0); t += TB) {
            double o = wl[t];
            if (ADD) o += P.target[r0 + t];
            P.r[r0 + t] = o;
            sq[0] += o * o;
        }
    }
    if (!REDUCE) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0)
        bb_record_f(P, iter, tot[0], ITER);
}

// Multi-GPU stage 2: r (already all-reduced) += target, ||r||^2, stop test.
__global__ __launch_bounds__(256) void bb_r_finish(bsls_bb_problem P, int64_t iter, double *part,
                                                   unsigned *ticket) {
    __shared__ double red[4];
    if (iter > 0 && P.scal[BSLS_S_STOP] != 0.0) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sq[1] = {0.0};
    if (i < P.m) {
        const double o = P.r[i] + P.target[i];
        P.r[i] = o;
        sq[0] = o * o;
    }
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0)
        bb_record_f(P, iter, tot[0], iter > 0);
}

// K2: g = N'(A' r); with ITER also dg = g - g_prev and the BB sums.  A' tiles
// end at x-block ends, so both rows of every N' difference sit in this
// workgroup's LDS.
template <int G, bool ITER>
__global__ __launch_bounds__(TB) void bb_k2(bsls_bb_problem P, const double *__restrict__ zc,
                                            const double *__restrict__ zp,
                                            const double *__restrict__ gp,
                                            double *__restrict__ gout, double *part,
                                            unsigned *ticket) {
    __shared__ double prod[NZT];
    __shared__ double wl[RMAX];
    __shared__ double red[16];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) return;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t tile = blockIdx.x; tile < P.AT_ntiles; tile += gridDim.x) {
        const int64_t r0 = P.AT_tiles[tile], r1 = P.AT_tiles[tile + 1];
        tile_rows<G>(P.AT_indptr, P.AT_indices, P.AT_data, P.r, r0, r1, prod, wl);
        for (int t = threadIdx.x; t < (int)(r1 - r0); t += TB) {
            const int32_t j = P.xz[r0 + t];
            if (j >= 0) {
                const double g = wl[t] - wl[t + 1];
                gout[j] = g;
                if (ITER) {
                    const double dg = g - gp[j];
                    const double dz = zc[j] - zp[j];
                    acc[0] += dg;
                    acc[1] += dz * dg;
                    acc[2] += dg * dg;
                    acc[3] += g * g;
                }
            }
        }
    }
    if (!ITER) return;
    block_sum<4>(acc, red);
    double tot[4];
    if (last_block_sum<4>(acc, part, ticket, tot, red) && threadIdx.x == 0) {
        P.scal[BSLS_S_SUMDG] = tot[0];
        P.scal[BSLS_S_DZDG] = tot[1];
        P.scal[BSLS_S_DGDG] = tot[2];
        P.scal[BSLS_S_GG] = tot[3];
    }
}

__device__ __forceinline__ int64_t zend(const bsls_bb_problem &P, int64_t b) {
    return (b + 1 < P.nblocks) ? P.zstarts[b + 1] : P.nz;
}
__device__ __forceinline__ int64_t xend(const bsls_bb_problem &P, int64_t b) {
    return (b + 1 < P.nblocks) ? P.xstarts[b + 1] : P.n;
}

// K3: t, z_new = clip01(PAVA(z - t g)) per block, x = N z_new.  One wave per
// BPW consecutive blocks: all 64 lanes stage the blocks' contiguous z range
// into LDS (loads kept in flight), lanes 0..BPW-1 run the serial PAVA of one
// block each, then the z and x ranges are written back coalesced.
__global__ __launch_bounds__(WAVE) void bb_k3(bsls_bb_problem P, int64_t iter,
                                              const double *__restrict__ zc,
                                              const double *__restrict__ g,
                                              double *__restrict__ zn,
                                              int32_t *__restrict__ wsc) {
    __shared__ double ly[K3_CAP];
    __shared__ double lx[K3_CAP + BPW];
    __shared__ int32_t lw[K3_CAP];
    double *s = P.scal;
    if (s[BSLS_S_STOP] != 0.0) return;
    if (P.early_exit && s[BSLS_S_SUMDG] == 0.0) {  // BB.py:22
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            s[BSLS_S_STOP] = (double)BSLS_STOP_NOCHANGE;
            s[BSLS_S_ITER] = (double)iter;
            s[BSLS_S_ZBUF] = (double)((iter - 1) & 1);
        }
        return;
    }
    const double t = s[BSLS_S_DZDG] / s[BSLS_S_DGDG];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s[BSLS_S_T] = t;
        if (fabs(t) <= 1e-10 || fabs(t) > 1e10) s[BSLS_S_WARN] += 1.0;
    }
    const int lane = lane_id();
    const int64_t b0 = (int64_t)blockIdx.x * BPW;
    const int64_t b = b0 + lane;
    const bool valid = lane < BPW && b < P.nblocks;
    const int64_t blast = (b0 + BPW - 1 < P.nblocks) ? b0 + BPW - 1 : P.nblocks - 1;
    const int64_t Z0 = P.zstarts[b0], Z1 = zend(P, blast);
    const int64_t X0 = P.xstarts[b0], X1 = xend(P, blast);
    const int64_t zs = valid ? P.zstarts[b] : 0, ze = valid ? zend(P, b) : 0;
    const int64_t xs = valid ? P.xstarts[b] : 0, xe = valid ? xend(P, b) : 0;
    if (Z1 - Z0 <= K3_CAP) {
        const int nzr = (int)(Z1 - Z0), nxr = (int)(X1 - X0);
        constexpr int U = 4;
        for (int j0 = 0; j0 < nzr; j0 += U * WAVE) {
            double a[U], c[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int j = j0 + lane + k * WAVE;
                a[k] = (j < nzr) ? zc[Z0 + j] : 0.0;
                c[k] = (j < nzr) ? g[Z0 + j] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int j = j0 + lane + k * WAVE;
                if (j < nzr) {
                    ly[j] = a[k] - t * c[k];  // x_next = x - t * g (BB.py:29)
                    lw[j] = 1;
                }
            }
        }
        __syncthreads();
        if (valid) {
            const int lo = (int)(zs - Z0), hi = (int)(ze - Z0);
            pava_v1(ly, lw, lo, hi, 1);
            double prev = 0.0;
            int xo = (int)(xs - X0);
            for (int j = lo; j < hi; ++j) {
                const double v = clip01(ly[j]);
                ly[j] = v;
                lx[xo++] = v - prev;
                prev = v;
            }
            lx[xe - 1 - X0] = 0.0 - prev;   // (N z)_last = -z_last
        }
        __syncthreads();
        for (int j = lane; j < nzr; j += WAVE) zn[Z0 + j] = ly[j];
        for (int j = lane; j < nxr; j += WAVE) P.x[X0 + j] = lx[j];
    } else if (valid) {
        for (int64_t j = zs; j < ze; ++j) {
            zn[j] = zc[j] - t * g[j];
            wsc[j] = 1;
        }
        pava_v1(zn, wsc, zs, ze, 1);
        double prev = 0.0;
        int64_t xo = xs;
        for (int64_t j = zs; j < ze; ++j) {
            const double v = clip01(zn[j]);
            zn[j] = v;
            P.x[xo++] = v - prev;
            prev = v;
        }
        P.x[xe - 1] = 0.0 - prev;
    }
}

// Prologue helpers (BB.py:14-15: x_prev = x + 1); bb_z2x writes N z.
__global__ __launch_bounds__(256) void bb_plus_one(const double *__restrict__ a,
                                                   double *__restrict__ o, int64_t nz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nz) o[i] = a[i] + 1;
}

__global__ __launch_bounds__(256) void bb_z2x(bsls_bb_problem P, const double *__restrict__ z) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P.nblocks) return;
    const int64_t zs = P.zstarts[b], ze = zend(P, b), xs = P.xstarts[b];
    double prev = 0.0;
    int64_t xo = xs;
    for (int64_t j = zs; j < ze; ++j) {
        const double v = z[j];
        P.x[xo++] = v - prev;
        prev = v;
    }
    P.x[xo] = 0.0 - prev;
}

template <bool ADD, bool REDUCE, bool ITER>
static void launch_k1(const bsls_bb_problem &P, int64_t iter, const BBWork &w, hipStream_t st) {
    const int grid = (int)(P.A_ntiles < MAX_TILE_WG ? P.A_ntiles : MAX_TILE_WG);
    switch (P.a_group) {
#define K1CASE(G)                                                               \
    case G:                                                                     \
        bb_k1<G, ADD, REDUCE, ITER><<<grid, TB, 0, st>>>(P, iter, w.p1, w.tk1); \
        break;
        K1CASE(1) K1CASE(2) K1CASE(4) K1CASE(8) K1CASE(16) K1CASE(32) K1CASE(64)
#undef K1CASE
    }
}

template <bool ITER>
static void launch_k2(const bsls_bb_problem &P, const double *zc, const double *zp,
                      const double *gp, double *gout, const BBWork &w, hipStream_t st) {
    const int grid = (int)(P.AT_ntiles < MAX_TILE_WG ? P.AT_ntiles : MAX_TILE_WG);
    switch (P.at_group) {
#define K2CASE(G)                                                               \
    case G:                                                                     \
        bb_k2<G, ITER><<<grid, TB, 0, st>>>(P, zc, zp, gp, gout, w.p2, w.tk2);  \
        break;
        K2CASE(1) K2CASE(2) K2CASE(4) K2CASE(8) K2CASE(16) K2CASE(32) K2CASE(64)
#undef K2CASE
    }
}

static void launch_k3(const bsls_bb_problem &P, int64_t iter, const double *zc, const double *g,
                      double *zn, const BBWork &w, hipStream_t st) {
    bb_k3<<<grid_for(P.nblocks, BPW), WAVE, 0, st>>>(P, iter, zc, g, zn, w.wsc);
}

static int check_problem(const bsls_bb_problem *p) {
    if (!p || p->m <= 0 || p->n <= 0 || p->nblocks <= 0 || p->nz != p->n - p->nblocks) return BSLS_E_ARG;
    if (!p->A_indptr || !p->AT_indptr || !p->target || !p->xstarts || !p->zstarts || !p->xz)
        return BSLS_E_ARG;
    if (!p->A_tiles || !p->AT_tiles || p->A_ntiles <= 0 || p->AT_ntiles <= 0) return BSLS_E_ARG;
    if (!p->z[0] || !p->z[1] || !p->g[0] || !p->g[1] || !p->x || !p->r || !p->scal || !p->work)
        return BSLS_E_ARG;
    const int ag = p->a_group, tg = p->at_group;
    if (ag < 1 || ag > 64 || (ag & (ag - 1)) || tg < 1 || tg > 64 || (tg & (tg - 1)))
        return BSLS_E_ARG;
    return BSLS_OK;
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_bb_workspace_size(int64_t m, int64_t n, int64_t nz, int64_t max_tiles) {
    (void)n;
    return bb_layout(nullptr, m, nz, max_tiles).bytes;
}

extern "C" int bsls_bb_stage(const bsls_bb_problem *p, int stage, int64_t iter, void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    const bsls_bb_problem &P = *p;
    hipStream_t st = (hipStream_t)stream;
    const BBWork w = bb_layout(P);
    const int zc = (int)((iter - 1) & 1), zn = (int)(iter & 1);
    switch (stage) {
        case 0:  // reset scalars and tickets
            BSLS_CHECK(hipMemsetAsync(P.scal, 0, BSLS_S_COUNT * sizeof(double), st));
            BSLS_CHECK(hipMemsetAsync(P.work, 0, al16(3 * TICKET_BYTES), st));
            return BSLS_OK;
        case 1:  // r_partial = A_g x_g
            if (iter > 0) launch_k1<false, false, true>(P, iter, w, st);
            else launch_k1<false, false, false>(P, iter, w, st);
            break;
        case 2:  // r += target, ||r||^2, stop test
            bb_r_finish<<<grid_for(P.m, 256), 256, 0, st>>>(P, iter, w.pf, w.tkf);
            break;
        case 3:  // g = N'A'r (+ sums)
            if (iter > 0) launch_k2<true>(P, P.z[zc], P.z[zn], P.g[zc], P.g[zn], w, st);
            else launch_k2<false>(P, nullptr, nullptr, nullptr, P.g[0], w, st);
            break;
        case 4:  // t, projection, x
            if (iter <= 0) return BSLS_E_ARG;
            launch_k3(P, iter, P.z[zc], P.g[zn], P.z[zn], w, st);
            break;
        case 5:  // z[1] = z[0] + 1; x = N z[1]
            bb_plus_one<<<grid_for(P.nz > 0 ? P.nz : 1, 256), 256, 0, st>>>(P.z[0], P.z[1], P.nz);
            BSLS_LAUNCH_CHECK();
            bb_z2x<<<grid_for(P.nblocks, 256), 256, 0, st>>>(P, P.z[1]);
            break;
        case 6:  // x = N z[0]
            bb_z2x<<<grid_for(P.nblocks, 256), 256, 0, st>>>(P, P.z[0]);
            break;
        case 7:  // single GCD K1: r = A x + target, ||r||^2, stop test (iter > 0)
            if (iter > 0) launch_k1<true, true, true>(P, iter, w, st);
            else launch_k1<true, true, false>(P, iter, w, st);
            break;
        default:
            return BSLS_E_ARG;
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_bb_prologue(const bsls_bb_problem *p, void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    const bsls_bb_problem &P = *p;
    hipStream_t st = (hipStream_t)stream;
    const BBWork w = bb_layout(P);
    int e;
    if ((e = bsls_bb_stage(p, 0, 0, stream)) != BSLS_OK) return e;
    if ((e = bsls_bb_stage(p, 5, 0, stream)) != BSLS_OK) return e;
    launch_k1<true, false, false>(P, 0, w, st);  // r(z0 + 1)
    BSLS_LAUNCH_CHECK();
    if ((e = bsls_bb_stage(p, 3, 0, stream)) != BSLS_OK) return e;  // g_prev -> g[0]
    if ((e = bsls_bb_stage(p, 6, 0, stream)) != BSLS_OK) return e;
    launch_k1<true, true, false>(P, 0, w, st);  // r(z0), f(z0)
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_bb_iterate(const bsls_bb_problem *p, int64_t first_iter, int64_t count,
                               void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    if (first_iter < 1 || count < 0) return BSLS_E_ARG;
    const bsls_bb_problem &P = *p;
    hipStream_t st = (hipStream_t)stream;
    const BBWork w = bb_layout(P);
    for (int64_t i = first_iter; i < first_iter + count; ++i) {
        const int zc = (int)((i - 1) & 1), zn = (int)(i & 1);
        launch_k2<true>(P, P.z[zc], P.z[zn], P.g[zc], P.g[zn], w, st);
        launch_k3(P, i, P.z[zc], P.g[zn], P.z[zn], w, st);
        launch_k1<true, true, true>(P, i, w, st);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}
