// bb.hip -- fused z-space projected Barzilai-Borwein iteration on one GCD.
//
// Reference loop (python/BB.py:17-41) over main.solve_in_z's closures
// (python/main.py:53-65), stopping rule solvers.stopping (python/solvers.py:40-63):
//     g = N'A'(A N z + target);  dg = g - g_prev;  if sum(dg) == 0: break
//     t = (z - z_prev).dg / dg.dg;  z <- clip01(PAVA(z - t g));  fx = f(z); stop?
// One iteration here = three kernels, all HBM-bound, no host round trip:
//   K2  g = N'(A' r) with an explicit A' in SELL-C-64 (deterministic, no atomics):
//       one lane per x-row, each wave owning 63 rows plus one halo row, so the
//       adjacent difference N'w = w_i - w_{i+1} is a lane shuffle; fused: dg,
//       the four BB sums, the store of g.
//   K3  t from the sums; per z-block PAVA (v1 pooling order, bit-identical to
//       isotonic_regression.h:13-58) + clip to [0,1] + the vector N z (per-block
//       differences, last entry -z_last), one lane per block over an LDS-staged
//       range.  N is never materialised.
//   K1  r = A (N z) + target, target = A x0 - b, exactly the reference's
//       A.dot(N.dot(z)) + target.  A in SELL-C-64 cut into column chunks, one
//       per XCD group, so each XCD's L2 serves the x gather of one chunk
//       (K1a: partial per chunk); K1b sums the chunk partials in chunk order,
//       adds target, ||r||^2 (next gradient's residual AND f(z)) and runs the
//       stopping test of the iteration in the last workgroup.
// Every cross-workgroup sum is reduced in a fixed order by the last-arriving
// workgroup (bsls_common.hpp last_block_sum), so runs are bit-reproducible.
// Scalars live in device memory (scal[]); the host only polls them.
#include "pava.hpp"
#include "pava_wave.hpp"
#include "sell.hpp"

namespace bsls {


struct BBWork {
    unsigned *tk1, *tk2, *tkf;
    double *p1, *p2, *pf;
    int32_t *wsc;
    size_t bytes;
};

static size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

constexpr int K2_ROWS = 4 * (SELL_C - 1);   // own x-rows per K2 workgroup (4 waves)

static BBWork bb_layout(void *base, int64_t m, int64_t n, int64_t nz) {
    BBWork w{};
    char *p = (char *)base;
    size_t off = 0;
    w.tk1 = (unsigned *)(p + off);
    w.tk2 = (unsigned *)(p + off + TICKET_BYTES);
    w.tkf = (unsigned *)(p + off + 2 * TICKET_BYTES);
    off += al16(3 * TICKET_BYTES);
    w.p1 = (double *)(p + off);
    off += al16((size_t)((m + 255) / 256 + 1) * 8);
    w.p2 = (double *)(p + off);
    off += al16((size_t)((n + K2_ROWS - 1) / K2_ROWS + 1) * 4 * 8);
    w.pf = (double *)(p + off);
    off += al16((size_t)((m + 255) / 256 + 1) * 8);
    w.wsc = (int32_t *)(p + off);
    off += al16((size_t)(nz > 0 ? nz : 1) * 4);
    w.bytes = off;
    return w;
}

static BBWork bb_layout(const bsls_bb_problem &P) { return bb_layout(P.work, P.m, P.n, P.nz); }

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

// K1a: per column chunk c, rpart[c][row] = sum over the row's entries in that
// chunk (SELL, one wave per slice).  Workgroup b takes chunk b % nchunk.
template <bool ITER>
__global__ __launch_bounds__(256) void bb_k1a(bsls_bb_problem P) {
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) return;
    const int64_t nc = P.A_nchunk;
    const int64_t c = blockIdx.x % nc;
    const int64_t sl = P.A_coff[c] + (int64_t)(blockIdx.x / nc) * 4 + threadIdx.x / WAVE;
    if (sl >= P.A_coff[c + 1]) return;
    const int lane = lane_id();
    const int32_t row = P.A_perm[sl * SELL_C + lane];
    const int64_t s0 = P.A_sptr[sl];
    const int W = (int)((P.A_sptr[sl + 1] - s0) / SELL_C);
    const double v = sell_row(P.A_sidx, P.A_sval, P.x, s0 + lane, W, 0.0);
    if (row >= 0) P.rpart[c * P.m + row] = v;
}

// K1b: r = sum_c rpart[c] (+ target); optional ||r||^2 and the stopping test.
template <bool ADD, bool REDUCE, bool ITER>
__global__ __launch_bounds__(256) void bb_k1b(bsls_bb_problem P, int64_t iter, double *part,
                                              unsigned *ticket) {
    __shared__ double red[4];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sq[1] = {0.0};
    if (i < P.m) {
        double o = P.rpart[i];
        for (int64_t c = 1; c < P.A_nchunk; ++c) o += P.rpart[c * P.m + i];
        if (ADD) o += P.target[i];
        P.r[i] = o;
        sq[0] = o * o;
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

// K2: g = N'(A' r); with ITER also dg = g - g_prev and the BB sums.  Lane l of
// wave w takes x-row i = 63 w + l; lane 63 is the halo (the next wave's first
// row), so N' w = w_i - w_{i+1} is one shuffle.  The epilogue operands are
// loaded before the row sum so their latency overlaps it.
template <bool ITER>
__global__ __launch_bounds__(256) void bb_k2(bsls_bb_problem P, const double *__restrict__ zc,
                                             const double *__restrict__ zp,
                                             const double *__restrict__ gp,
                                             double *__restrict__ gout, double *part,
                                             unsigned *ticket) {
    __shared__ double red[16];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) return;
    const int lane = lane_id();
    const int64_t wv = (int64_t)blockIdx.x * 4 + threadIdx.x / WAVE;
    const int64_t i = wv * (SELL_C - 1) + lane;
    int32_t j = -1;
    double gpj = 0.0, zcj = 0.0, zpj = 0.0;
    if (lane < SELL_C - 1 && i < P.n) {
        j = P.xz[i];
        if (ITER && j >= 0) {
            gpj = gp[j];
            zcj = zc[j];
            zpj = zp[j];
        }
    }
    double v = 0.0;
    if (i < P.n) {
        const int64_t sl = i / SELL_C;
        const int64_t s0 = P.AT_sptr[sl];
        const int W = (int)((P.AT_sptr[sl + 1] - s0) / SELL_C);
        v = sell_row(P.AT_sidx, P.AT_sval, P.r, s0 + (i % SELL_C), W, 0.0);
    }
    const double vn = __shfl_down(v, 1, WAVE);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (j >= 0) {
        const double g = v - vn;
        gout[j] = g;
        if (ITER) {
            const double dg = g - gpj;
            const double dz = zcj - zpj;
            acc[0] = dg;
            acc[1] = dz * dg;
            acc[2] = dg * dg;
            acc[3] = g * g;
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
// pack of whole z-blocks (<= 64 entries, one lane each): the PAVA passes run
// wave-parallel (pava_wave.hpp, bit-identical to the serial reference); a
// block longer than 64 entries gets a pack of its own and the serial PAVA.
__device__ __forceinline__ bool bb_step_t(const bsls_bb_problem &P, int64_t iter, double &t) {
    double *s = P.scal;
    if (s[BSLS_S_STOP] != 0.0) return false;
    if (P.early_exit && s[BSLS_S_SUMDG] == 0.0) {  // BB.py:22
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            s[BSLS_S_STOP] = (double)BSLS_STOP_NOCHANGE;
            s[BSLS_S_ITER] = (double)iter;
            s[BSLS_S_ZBUF] = (double)((iter - 1) & 1);
        }
        return false;
    }
    t = s[BSLS_S_DZDG] / s[BSLS_S_DGDG];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s[BSLS_S_T] = t;
        if (fabs(t) <= 1e-10 || fabs(t) > 1e10) s[BSLS_S_WARN] += 1.0;
    }
    return true;
}

__global__ __launch_bounds__(256) void bb_k3(bsls_bb_problem P, int64_t iter,
                                             const double *__restrict__ zc,
                                             const double *__restrict__ g,
                                             double *__restrict__ zn,
                                             int32_t *__restrict__ wsc) {
    double t;
    if (!bb_step_t(P, iter, t)) return;
    const int64_t pk = (int64_t)blockIdx.x * 4 + threadIdx.x / WAVE;
    if (pk >= P.npacks) return;
    const int l = lane_id();
    const int64_t z0 = P.pk_z0[pk], b0 = P.pk_b0[pk];
    const int L = P.pk_len[pk];
    if (L <= WAVE) {
        const uint64_t B = (uint64_t)P.pk_mask[pk];
        const bool act = l < L;
        double y = act ? zc[z0 + l] - t * g[z0 + l] : 0.0;  // x_next = x - t g (BB.py:29)
        int w = 1;
        uint64_t heads;
        pava_v1_wave(y, w, L, B, heads);
        const double v = clip01(y);
        const double vprev = shfl_d(v, l > 0 ? l - 1 : 0);
        if (act) {
            zn[z0 + l] = v;
            const bool bstart = (B >> l) & 1ull;
            const int64_t blk = b0 + __popcll(B & mask_le(l)) - 1;
            const int64_t xi = z0 + l + blk;            // x index of this z entry
            P.x[xi] = v - (bstart ? 0.0 : vprev);
            const bool bend = (l == L - 1) || (l < 63 && ((B >> (l + 1)) & 1ull));
            if (bend) P.x[xi + 1] = 0.0 - v;            // (N z)_last = -z_last
        }
    } else if (l == 0) {
        // one block longer than a wave: serial PAVA in global memory
        const int64_t xs = P.xstarts[b0];
        for (int64_t j = z0; j < z0 + L; ++j) {
            zn[j] = zc[j] - t * g[j];
            wsc[j] = 1;
        }
        pava_v1(zn, wsc, z0, z0 + L, 1);
        double prev = 0.0;
        int64_t xo = xs;
        for (int64_t j = z0; j < z0 + L; ++j) {
            const double v = clip01(zn[j]);
            zn[j] = v;
            P.x[xo++] = v - prev;
            prev = v;
        }
        P.x[xo] = 0.0 - prev;
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
    const int ga = (int)(P.A_nchunk * ((P.A_maxsl + 3) / 4));
    bb_k1a<ITER><<<ga, 256, 0, st>>>(P);
    bb_k1b<ADD, REDUCE, ITER><<<grid_for(P.m, 256), 256, 0, st>>>(P, iter, w.p1, w.tk1);
}

template <bool ITER>
static void launch_k2(const bsls_bb_problem &P, const double *zc, const double *zp,
                      const double *gp, double *gout, const BBWork &w, hipStream_t st) {
    bb_k2<ITER><<<grid_for(P.n, K2_ROWS), 256, 0, st>>>(P, zc, zp, gp, gout, w.p2, w.tk2);
}

static void launch_k3(const bsls_bb_problem &P, int64_t iter, const double *zc, const double *g,
                      double *zn, const BBWork &w, hipStream_t st) {
    bb_k3<<<grid_for(P.npacks, 4), 256, 0, st>>>(P, iter, zc, g, zn, w.wsc);
}

static int check_problem(const bsls_bb_problem *p) {
    if (!p || p->m <= 0 || p->n <= 0 || p->nblocks <= 0 || p->nz != p->n - p->nblocks) return BSLS_E_ARG;
    if (!p->A_sidx || !p->A_sval || !p->A_sptr || !p->A_perm || !p->A_coff || !p->rpart)
        return BSLS_E_ARG;
    if (p->A_nchunk < 1 || p->A_maxsl < 1) return BSLS_E_ARG;
    if (!p->AT_sidx || !p->AT_sval || !p->AT_sptr) return BSLS_E_ARG;
    if (!p->target || !p->xstarts || !p->zstarts || !p->xz) return BSLS_E_ARG;
    if (!p->pk_z0 || !p->pk_b0 || !p->pk_mask || !p->pk_len || p->npacks < 1) return BSLS_E_ARG;
    if (!p->z[0] || !p->z[1] || !p->g[0] || !p->g[1] || !p->x || !p->r || !p->scal || !p->work)
        return BSLS_E_ARG;
    return BSLS_OK;
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_bb_workspace_size(int64_t m, int64_t n, int64_t nz) {
    return bb_layout(nullptr, m, n, nz).bytes;
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
