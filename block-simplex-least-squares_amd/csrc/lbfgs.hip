// lbfgs.hip -- LBFGS.solve's search direction (python/LBFGS.py:59-71) over a
// device ring of the m history pairs (s_k, y_k, rho_k), "vector-free":
//
// The two-loop recursion keeps q and r in the span of g and the stored s_k,
// y_k, so it runs on their dot products instead of on vectors:
//   q = g - sum_j cq_j y_j          alpha_k = rho_k (s_k . q),  cq_k += alpha_k
//   r = H q,  H = (y.s) / (y.y) of the latest pair (not yet in the ring)
//   r = H g - sum_j H cq_j y_j + sum_j cs_j s_j
//                                   beta = rho_k (y_k . r),     cs_k += alpha_k - beta
//   d = -r
// so one iteration costs ONE pass computing every dot it needs
// (bsls_multi_dot: g, y_new and s_new against every stored s_k, y_k and
// against y_new, s_new -- also the rows of the Gram matrices the push of the
// new pair needs), the m-step loops on scalars (bsls_lbfgs_coef, one wave),
// ONE combine pass (bsls_multi_axpy: d = a g + sum b_k s_k + sum c_k y_k) and
// the push (bsls_lbfgs_push: the new pair copied into the oldest slot, its
// Gram rows filled in) -- instead of 2m dependent dot products, each a
// device -> host read, and 2m AXPYs.  Summation order differs from the
// reference's vector recursion; the iterates stay within the 1e-6 contract.
//
// Ring: slot (head + k) % m holds logical pair k (0 = oldest), as the
// reference's lists Y, S, rho (initially m zero vectors and zeros).  Gram
// matrices by slot: SY[a][b] = s_a . y_b, YY[a][b] = y_a . y_b (m x m).
#include "bsls_common.hpp"

namespace bsls {

constexpr int MD_T = 256;
constexpr int MD_KC = 16;     // columns per workgroup
constexpr int MD_JMAX = 4;    // rows per call
constexpr int MD_NB = 256;    // element blocks (partials per column chunk)

// stage 1: workgroup (eb, kc) sums rows[j][i] * cols[k][i] over its element
// blocks for the kc-th chunk of MD_KC columns; partials in index order
template <int J>
__global__ __launch_bounds__(MD_T) void mdot_partial(const double *const *__restrict__ rows,
                                                     const double *const *__restrict__ cols,
                                                     int K, int64_t n,
                                                     double *__restrict__ part) {
    __shared__ double red[J * MD_KC * (MD_T / WAVE)];
    const int eb = blockIdx.x % MD_NB, kc = blockIdx.x / MD_NB;
    const int k0 = kc * MD_KC;
    const int nk = (K - k0 < MD_KC) ? K - k0 : MD_KC;
    double acc[J * MD_KC];
#pragma unroll
    for (int q = 0; q < J * MD_KC; ++q) acc[q] = 0.0;
    const double *cp[MD_KC];
#pragma unroll
    for (int c = 0; c < MD_KC; ++c) cp[c] = cols[k0 + (c < nk ? c : 0)];
    const double *rp[J];
#pragma unroll
    for (int j = 0; j < J; ++j) rp[j] = rows[j];
    // every column load unconditional (columns past nk re-read column k0 into
    // accumulators that are never written out): a branch per column kept the
    // compiler from issuing the loads of an iteration together -- one memory
    // latency per column, 302 us for C3's 3 x 102 dots against ~130 of bytes
    for (int64_t i = (int64_t)eb * MD_T + threadIdx.x; i < n; i += (int64_t)MD_NB * MD_T) {
        double r[J], v[MD_KC];
#pragma unroll
        for (int j = 0; j < J; ++j) r[j] = rp[j][i];
#pragma unroll
        for (int c = 0; c < MD_KC; ++c) v[c] = cp[c][i];
#pragma unroll
        for (int c = 0; c < MD_KC; ++c) {
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j * MD_KC + c] += r[j] * v[c];
        }
    }
    block_sum<J * MD_KC>(acc, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < J * MD_KC; ++q) part[((size_t)kc * MD_NB + eb) * (J * MD_KC) + q] = acc[q];
    }
}

// stage 2: out[j * K + k] = the sum of the element blocks' partials, one wave
// per output: lane l adds blocks l, l + 64, ... in order, then a fixed-tree
// wave sum (deterministic; one thread walking all MD_NB partials took 31 us)
template <int J>
__global__ __launch_bounds__(256) void mdot_finish(const double *__restrict__ part, int K,
                                                   double *__restrict__ out) {
    const int t = (int)((blockIdx.x * blockDim.x + threadIdx.x) / WAVE);
    if (t >= J * K) return;
    const int j = t / K, k = t % K;
    const int kc = k / MD_KC, c = k % MD_KC;
    const int l = lane_id();
    double v[MD_NB / WAVE];
#pragma unroll
    for (int q = 0; q < MD_NB / WAVE; ++q)
        v[q] = part[((size_t)kc * MD_NB + l + q * WAVE) * (J * MD_KC) + j * MD_KC + c];
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < MD_NB / WAVE; ++q) s += v[q];
    s = group_sum<WAVE>(s);
    if (l == 0) out[t] = s;
}

// out[i] = sum_k coef[k] * vecs[k][i]
constexpr int MAXPY_T = 256, MAXPY_TILE = 2 * MAXPY_T;
__global__ __launch_bounds__(MAXPY_T) void maxpy_kernel(const double *const *__restrict__ vecs, int K,
                                                    const double *__restrict__ coef, int64_t n,
                                                    double *__restrict__ out) {
    __shared__ double cs[256];
    __shared__ const double *vp[256];
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        cs[k] = coef[k];
        vp[k] = vecs[k];
    }
    __syncthreads();
    // one 512-element tile per workgroup, two elements per thread, the vectors
    // eight at a time with all 16 loads of a batch in flight (the one-element
    // loop waited once per 8 loads); the same left-to-right sum per element
    const int64_t i0 = (int64_t)blockIdx.x * MAXPY_TILE + threadIdx.x, i1 = i0 + MAXPY_T;
    const int64_t j0 = i0 < n ? i0 : n - 1, j1 = i1 < n ? i1 : n - 1;
    double a0 = 0.0, a1 = 0.0;
    int k = 0;
    for (; k + 8 <= K; k += 8) {
        double v0[8], v1[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            v0[q] = vp[k + q][j0];
            v1[q] = vp[k + q][j1];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            a0 += cs[k + q] * v0[q];
            a1 += cs[k + q] * v1[q];
        }
    }
    for (; k < K; ++k) {
        a0 += cs[k] * vp[k][j0];
        a1 += cs[k] * vp[k][j1];
    }
    if (i0 < n) out[i0] = a0;
    if (i1 < n) out[i1] = a1;
}

// wave sum, result in every lane
__device__ __forceinline__ double wsum(double v) { return group_sum<WAVE>(v); }

// The two loops on scalars (one wave; lane j works on slot j, and on slots
// j + 64, ... for m > 64).  dots: row g of bsls_multi_dot over the columns
// [S slot 0..m-1, Y slot 0..m-1, y_new, s_new] (gS, gY), then rows y_new and
// s_new (their y_new / s_new columns give y.y and y.s for H).  coef out:
// [a (g), b (S slots), c (Y slots)] of d = -r.
__global__ __launch_bounds__(64) void lbfgs_coef_kernel(int m, int head, const double *__restrict__ rho,
                                                        const double *__restrict__ SY,
                                                        const double *__restrict__ YY,
                                                        const double *__restrict__ dots,
                                                        double *__restrict__ coef,
                                                        double *__restrict__ work) {
    const int l = threadIdx.x;
    const int K = 2 * m + 2;
    const double *gS = dots, *gY = dots + m;
    const double yy = dots[K + 2 * m];        // row y_new, column y_new
    const double ys = dots[K + 2 * m + 1];    // row y_new, column s_new
    double *cq = work, *cs = work + m, *alpha = work + 2 * m;
    for (int j = l; j < m; j += WAVE) {
        cq[j] = 0.0;
        cs[j] = 0.0;
        alpha[j] = 0.0;
    }
    __syncthreads();
    // loop 1, newest first (LBFGS.py:62-64)
    for (int k = m - 1; k >= 0; --k) {
        const int sk = (head + k) % m;
        double p = 0.0;
        for (int j = l; j < m; j += WAVE) p += cq[j] * SY[(size_t)sk * m + j];
        const double sq = gS[sk] - wsum(p);
        const double a = rho[sk] * sq;
        __syncthreads();
        if (l == 0) {
            alpha[sk] = a;
            cq[sk] += a;
        }
        __syncthreads();
    }
    // r = H q (LBFGS.py:65-66): coefficients H (g), -H cq (Y), 0 (S)
    const double H = ys / yy;
    // loop 2, oldest first (LBFGS.py:67-69): y_k . r
    for (int k = 0; k < m; ++k) {
        const int sk = (head + k) % m;
        double p = 0.0;
        for (int j = l; j < m; j += WAVE)
            p += -H * cq[j] * YY[(size_t)sk * m + j] + cs[j] * SY[(size_t)j * m + sk];
        const double yr = H * gY[sk] + wsum(p);
        const double beta = rho[sk] * yr;
        __syncthreads();
        if (l == 0) cs[sk] += alpha[sk] - beta;
        __syncthreads();
    }
    // d = -r = -(H g - sum H cq_j y_j + sum cs_j s_j)
    if (l == 0) coef[0] = -H;
    for (int j = l; j < m; j += WAVE) {
        coef[1 + j] = -cs[j];
        coef[1 + m + j] = H * cq[j];
    }
}

// The same recursion with the Gram matrices staged in LDS and the
// coefficients in registers (lane j holds slot j, and slot j + 64 when m >
// 64): each of the 2m steps is an LDS read, a wave sum and a readlane instead
// of global reads, two barriers and global writes (the form above spends ~1 us
// a step on those round trips).  Same operations in the same order as
// lbfgs_coef_kernel, so the same bits.  LDS: SY, YY (m^2 each), m <= COEF_LDS_M.
constexpr int COEF_LDS_M = 90;

__device__ __forceinline__ double lane_bcast(double v, int src) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}

// stage the m x m Gram matrices into LDS, COEF_B loads per lane in flight
// (a plain strided loop waited for every load: ~40 us of round trips at m = 50)
constexpr int COEF_B = 16;
__device__ __forceinline__ void stage_gram(const double *__restrict__ SY,
                                           const double *__restrict__ YY, double *sy, double *yy,
                                           int mm, int l) {
    for (int i0 = 0; i0 < mm; i0 += COEF_B * WAVE) {
        double a[COEF_B], b[COEF_B];
#pragma unroll
        for (int q = 0; q < COEF_B; ++q) {
            const int i = i0 + q * WAVE + l;
            a[q] = (i < mm) ? SY[i] : 0.0;
            b[q] = (i < mm) ? YY[i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < COEF_B; ++q) {
            const int i = i0 + q * WAVE + l;
            if (i < mm) {
                sy[i] = a[q];
                yy[i] = b[q];
            }
        }
    }
}

__global__ __launch_bounds__(64) void lbfgs_coef_lds(int m, int head, const double *__restrict__ rho,
                                                     const double *__restrict__ SY,
                                                     const double *__restrict__ YY,
                                                     const double *__restrict__ dots,
                                                     double *__restrict__ coef) {
    extern __shared__ double gram[];
    double *sy = gram, *yy = gram + (size_t)m * m;
    const int l = threadIdx.x;
    const int K = 2 * m + 2;
    stage_gram(SY, YY, sy, yy, m * m, l);
    const bool two = m > WAVE;
    const int l2 = l + WAVE;
    // per-slot values, lane j (and j + 64)
    const double rho0 = (l < m) ? rho[l] : 0.0, rho1 = (two && l2 < m) ? rho[l2] : 0.0;
    const double gS0 = (l < m) ? dots[l] : 0.0, gS1 = (two && l2 < m) ? dots[l2] : 0.0;
    const double gY0 = (l < m) ? dots[m + l] : 0.0, gY1 = (two && l2 < m) ? dots[m + l2] : 0.0;
    const double yyn = dots[K + 2 * m];       // row y_new, column y_new
    const double ysn = dots[K + 2 * m + 1];   // row y_new, column s_new
    double cq0 = 0.0, cq1 = 0.0, cs0 = 0.0, cs1 = 0.0, al0 = 0.0, al1 = 0.0;
    __syncthreads();
    // loop 1, newest first (LBFGS.py:62-64)
    for (int k = m - 1; k >= 0; --k) {
        const int sk = (head + k) % m;
        double p = 0.0;
        if (l < m) p += cq0 * sy[(size_t)sk * m + l];
        if (two && l2 < m) p += cq1 * sy[(size_t)sk * m + l2];
        const double tot = group_sum<WAVE>(p);
        const double rs = (sk < WAVE) ? lane_bcast(rho0, sk) : lane_bcast(rho1, sk - WAVE);
        const double gs = (sk < WAVE) ? lane_bcast(gS0, sk) : lane_bcast(gS1, sk - WAVE);
        const double a = rs * (gs - tot);
        if (l == sk) {
            al0 = a;
            cq0 += a;
        }
        if (l2 == sk) {
            al1 = a;
            cq1 += a;
        }
    }
    // r = H q (LBFGS.py:65-66)
    const double H = ysn / yyn;
    // loop 2, oldest first (LBFGS.py:67-69): y_k . r
    for (int k = 0; k < m; ++k) {
        const int sk = (head + k) % m;
        double p = 0.0;
        if (l < m) p += -H * cq0 * yy[(size_t)sk * m + l] + cs0 * sy[(size_t)l * m + sk];
        if (two && l2 < m) p += -H * cq1 * yy[(size_t)sk * m + l2] + cs1 * sy[(size_t)l2 * m + sk];
        const double yr = H * ((sk < WAVE) ? lane_bcast(gY0, sk) : lane_bcast(gY1, sk - WAVE)) +
                          group_sum<WAVE>(p);
        const double beta = ((sk < WAVE) ? lane_bcast(rho0, sk) : lane_bcast(rho1, sk - WAVE)) * yr;
        if (l == sk) cs0 += al0 - beta;
        if (l2 == sk) cs1 += al1 - beta;
    }
    if (l == 0) coef[0] = -H;
    if (l < m) {
        coef[1 + l] = -cs0;
        coef[1 + m + l] = H * cq0;
    }
    if (two && l2 < m) {
        coef[1 + l2] = -cs1;
        coef[1 + m + l2] = H * cq1;
    }
}

// m <= 64 (lane i = slot i): the sums the loops need kept up to date instead
// of re-reduced every step.  Loop 1 needs P_sk = sum_j cq_j SY[sk][j]; cq
// changes in one slot per step, so every lane keeps its P_i and adds
// a SY[i][sk] when slot sk takes alpha = a.  Loop 2 needs sum_j cq_j YY[sk][j]
// (cq fixed by then: Q_i, formed once) and R_sk = sum_j cs_j SY[j][sk] (kept
// like P).  A step is then three readlanes and one multiply-add per lane, no
// wave sum (lbfgs_coef_lds: six dependent lane shuffles a step, 56 us for
// m = 50).  The sums' order differs from the vector recursion's, within the
// 1e-11 the direction test holds it to.
__global__ __launch_bounds__(64) void lbfgs_coef_inc(int m, int head, const double *__restrict__ rho,
                                                     const double *__restrict__ SY,
                                                     const double *__restrict__ YY,
                                                     const double *__restrict__ dots,
                                                     double *__restrict__ coef) {
    extern __shared__ double gram[];
    double *sy = gram, *yy = gram + (size_t)m * m;
    const int l = threadIdx.x;
    const bool act = l < m;
    const int lr = act ? l : 0;                 // (rows read by idle lanes: row 0)
    const int K = 2 * m + 2;
    stage_gram(SY, YY, sy, yy, m * m, l);
    const double rho_l = act ? rho[l] : 0.0;
    const double gS_l = act ? dots[l] : 0.0, gY_l = act ? dots[m + l] : 0.0;
    const double yyn = dots[K + 2 * m];       // row y_new, column y_new
    const double ysn = dots[K + 2 * m + 1];   // row y_new, column s_new
    __syncthreads();
    // loop 1, newest first (LBFGS.py:62-64); the next step's column of SY is
    // read while this step runs
    double P = 0.0, cq = 0.0;
    int sk = (head + m - 1) % m;
    double col = sy[(size_t)lr * m + sk];
    for (int k = m - 1; k >= 0; --k) {
        const int sn = (sk == 0) ? m - 1 : sk - 1;
        const double nxt = sy[(size_t)lr * m + sn];
        const double a = lane_bcast(rho_l, sk) * (lane_bcast(gS_l, sk) - lane_bcast(P, sk));
        if (l == sk) cq += a;                       // (cq_sk was 0: alpha_sk)
        P += a * col;
        col = nxt;
        sk = sn;
    }
    // r = H q (LBFGS.py:65-66)
    const double H = ysn / yyn;
    double Q = 0.0;
    for (int j = 0; j < m; ++j) Q += lane_bcast(cq, j) * yy[(size_t)lr * m + j];
    // loop 2, oldest first (LBFGS.py:67-69): y_k . r = H gY_k - H Q_k + R_k
    double R = 0.0, cs = 0.0;
    sk = head;
    double row = sy[(size_t)sk * m + lr];
    for (int k = 0; k < m; ++k) {
        const int sn = (sk == m - 1) ? 0 : sk + 1;
        const double nxt = sy[(size_t)sn * m + lr];
        const double yr = H * lane_bcast(gY_l, sk) + (-H * lane_bcast(Q, sk) + lane_bcast(R, sk));
        const double dlt = lane_bcast(cq, sk) - lane_bcast(rho_l, sk) * yr;   // alpha - beta
        if (l == sk) cs += dlt;
        R += dlt * row;
        row = nxt;
        sk = sn;
    }
    if (l == 0) coef[0] = -H;
    if (act) {
        coef[1 + l] = -cs;
        coef[1 + m + l] = H * cq;
    }
}

// the new pair into slot `slot` (copies) and its Gram rows from the dots of
// this iteration's bsls_multi_dot (rows g, y_new, s_new against the old slots
// and the new pair), rho[slot] = rho_new
__global__ __launch_bounds__(256) void lbfgs_push_gram(int m, int slot, double rho_new,
                                                       const double *__restrict__ dots,
                                                       double *__restrict__ SY,
                                                       double *__restrict__ YY,
                                                       double *__restrict__ rho) {
    const int K = 2 * m + 2;
    const double *yrow = dots + K, *srow = dots + 2 * K;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m && j != slot) {
        SY[(size_t)slot * m + j] = srow[m + j];     // s_new . y_j
        SY[(size_t)j * m + slot] = yrow[j];         // s_j . y_new
        YY[(size_t)slot * m + j] = yrow[m + j];     // y_new . y_j
        YY[(size_t)j * m + slot] = yrow[m + j];
    }
    if (j == 0) {
        SY[(size_t)slot * m + slot] = srow[2 * m];  // s_new . y_new
        YY[(size_t)slot * m + slot] = yrow[2 * m];  // y_new . y_new
        rho[slot] = rho_new;
    }
}

__global__ __launch_bounds__(256) void lbfgs_copy2(const double *__restrict__ a,
                                                   double *__restrict__ da,
                                                   const double *__restrict__ b,
                                                   double *__restrict__ db, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        da[i] = a[i];
        db[i] = b[i];
    }
}

static int grid_cap(int64_t n, int per, int cap) {
    const int g = grid_for(n, per);
    return g < cap ? g : cap;
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_multi_dot_workspace_size(int64_t J, int64_t K) {
    if (J < 1 || J > MD_JMAX || K < 1) return 0;
    return (size_t)((K + MD_KC - 1) / MD_KC) * MD_NB * J * MD_KC * sizeof(double);
}

extern "C" int bsls_multi_dot(const double *const *d_rows, int J, const double *const *d_cols,
                              int K, int64_t n, double *d_out, void *d_work, size_t work_bytes,
                              void *stream) {
    if (!d_rows || !d_cols || !d_out || J < 1 || J > MD_JMAX || K < 1 || n < 0) return BSLS_E_ARG;
    if (!d_work || work_bytes < bsls_multi_dot_workspace_size(J, K)) return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    double *part = (double *)d_work;
    const int grid = ((K + MD_KC - 1) / MD_KC) * MD_NB;
    switch (J) {
        case 1: mdot_partial<1><<<grid, MD_T, 0, st>>>(d_rows, d_cols, K, n, part); break;
        case 2: mdot_partial<2><<<grid, MD_T, 0, st>>>(d_rows, d_cols, K, n, part); break;
        case 3: mdot_partial<3><<<grid, MD_T, 0, st>>>(d_rows, d_cols, K, n, part); break;
        default: mdot_partial<4><<<grid, MD_T, 0, st>>>(d_rows, d_cols, K, n, part); break;
    }
    BSLS_LAUNCH_CHECK();
    const int g2 = grid_for((int64_t)J * K * WAVE, 256);
    switch (J) {
        case 1: mdot_finish<1><<<g2, 256, 0, st>>>(part, K, d_out); break;
        case 2: mdot_finish<2><<<g2, 256, 0, st>>>(part, K, d_out); break;
        case 3: mdot_finish<3><<<g2, 256, 0, st>>>(part, K, d_out); break;
        default: mdot_finish<4><<<g2, 256, 0, st>>>(part, K, d_out); break;
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_multi_axpy(const double *const *d_vecs, int K, const double *d_coef, int64_t n,
                               double *d_out, void *stream) {
    if (!d_vecs || !d_coef || !d_out || K < 1 || K > 256 || n < 0) return BSLS_E_ARG;
    if (n == 0) return BSLS_OK;
    maxpy_kernel<<<(unsigned)((n + MAXPY_TILE - 1) / MAXPY_TILE), MAXPY_T, 0, (hipStream_t)stream>>>(
        d_vecs, K, d_coef, n, d_out);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" size_t bsls_lbfgs_state_size(int64_t m) {
    // rho (m), SY (m^2), YY (m^2), coef (2m+1), scratch (3m)
    return (size_t)(m + 2 * m * m + (2 * m + 1) + 3 * m) * sizeof(double);
}

extern "C" int bsls_lbfgs_coef(int64_t m, int64_t head, double *d_state, const double *d_dots,
                               void *stream) {
    if (m < 1 || m > 127 || head < 0 || head >= m || !d_state || !d_dots) return BSLS_E_ARG;
    double *rho = d_state, *SY = rho + m, *YY = SY + m * m, *coef = YY + m * m,
           *work = coef + 2 * m + 1;
    if (m <= WAVE) {
        lbfgs_coef_inc<<<1, 64, 2 * m * m * sizeof(double), (hipStream_t)stream>>>(
            (int)m, (int)head, rho, SY, YY, d_dots, coef);
    } else if (m <= COEF_LDS_M) {
        static bool attr_set = false;
        if (!attr_set) {
            BSLS_CHECK(hipFuncSetAttribute((const void *)lbfgs_coef_lds,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(2 * COEF_LDS_M * COEF_LDS_M * sizeof(double))));
            attr_set = true;
        }
        lbfgs_coef_lds<<<1, 64, 2 * m * m * sizeof(double), (hipStream_t)stream>>>(
            (int)m, (int)head, rho, SY, YY, d_dots, coef);
    } else {
        lbfgs_coef_kernel<<<1, 64, 0, (hipStream_t)stream>>>((int)m, (int)head, rho, SY, YY, d_dots,
                                                             coef, work);
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_lbfgs_push(int64_t m, int64_t slot, double rho_new, double *d_state,
                               const double *d_dots, const double *d_y_new,
                               const double *d_s_new, double *d_y_slot, double *d_s_slot,
                               int64_t n, void *stream) {
    if (m < 1 || m > 127 || slot < 0 || slot >= m || !d_state || !d_dots || !d_y_new ||
        !d_s_new || !d_y_slot || !d_s_slot || n < 0)
        return BSLS_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    double *rho = d_state, *SY = rho + m, *YY = SY + m * m;
    lbfgs_copy2<<<grid_cap(n, 256, 2048), 256, 0, st>>>(d_y_new, d_y_slot, d_s_new, d_s_slot, n);
    BSLS_LAUNCH_CHECK();
    lbfgs_push_gram<<<grid_for(m, 256), 256, 0, st>>>((int)m, (int)slot, rho_new, d_dots, SY, YY,
                                                      rho);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
