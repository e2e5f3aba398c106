// xbb.hip -- fused x-space projected Barzilai-Borwein (BATCH.solve_BB,
// python/BATCH.py:55-106) over the sparse least-squares objective
// (algorithm_utils.sparse_least_squares_obj, python/algorithm_utils.py:88-94),
// the block simplex / l1-ball projection and the backtracking line search
// line_search_np (:113-137), with the stopping rule algorithm_utils.stopping
// (:158-172) -- every decision on the device.
//
// A round (bsls_xbb_rounds) is five launches (six for L-BFGS, BATCH.solve_LBFGS:
// xlb_step / xlb_dir in place of xbb_step, see below):
//   xbb_step    mode STEP:      x <- x_new, g <- g_new (the accepted point),
//                               x_new = x + (-t) g        (np.add(x, -t*g, x_new))
//               mode BACKTRACK: x_new = (1-tt) x + tt x_new, or x_new = x when
//                               the step became too small (the reference's
//                               revert: obj(x) then reproduces f and g exactly,
//                               every kernel here being deterministic)
//               mode INIT:      x_new = x_init
//   proj        gated on STEP:  proj_multi_simplex / proj_multi_ball on x_new
//   spmv A      r = A x_new - b, ||r||^2
//   spmv A'     g_new = A' r
//   xbb_finish  g.(x_new - x), dx.dg, dg.dg, ||dx||_inf (deterministic
//               last-workgroup reduction), then the Armijo test
//               f_new > f + 1e-4 g.(x_new - x): reject -> next round
//               BACKTRACK (tt *= .8), else accept (f_old = f, f = f_new, the
//               BB step for the next iteration, i += 1) and the stopping test.
// After the stop every launch returns at once (the SpMVs recompute the same
// values), and the final iterate is x_new / g_new.
//
// Bytes per STEP round (n routes, m rows, nnz): step 40 n, projection 16 n,
// the two SpMVs 24 nnz + 4 (m + n) + 8 (m + n) + 16 m, finish 32 n.
#include "bsls_common.hpp"

namespace bsls {

int proj_launch_gated(bool ball, double *y, const int64_t *starts, int64_t nb, int64_t n,
                      int64_t max_block, void *work, size_t work_bytes, hipStream_t st,
                      const double *gate, bool fast);

constexpr int XT = 256;
constexpr int XGRID = 1024;   // finish: partials per launch (one slot per workgroup)
constexpr int XU = 4;         // finish: 16-B pairs per thread and step

static size_t xalign(size_t v) { return (v + 255) & ~(size_t)255; }

__global__ __launch_bounds__(64) void xbb_init_kernel(double *scal, double *hist,
                                                      int64_t hist_cap) {
    const int t = threadIdx.x;
    if (t < BSLS_XS_COUNT) scal[t] = 0.0;
    if (t == 0) {
        scal[BSLS_XS_MODE] = BSLS_XM_INIT;
        scal[BSLS_XS_TT] = 1.0;
        scal[BSLS_XS_T] = 1.0;
    }
    (void)hist;
    (void)hist_cap;
}

__device__ __forceinline__ void xbb_step_body(double *__restrict__ x, double *__restrict__ g,
                                              double *__restrict__ xn,
                                              const double *__restrict__ gn, int64_t n,
                                              const double *__restrict__ scal, int mode) {
    const int64_t stride = (int64_t)gridDim.x * XT;
    int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x;
    if (mode == BSLS_XM_INIT) {
        for (; i < n; i += stride) xn[i] = x[i];
    } else if (mode == BSLS_XM_STEP) {
        const double mt = -scal[BSLS_XS_T];   // i == 1: t = 1, (-1) * g == -g exactly
        for (; i < n; i += stride) {
            const double xv = xn[i], gv = gn[i];
            x[i] = xv;
            g[i] = gv;
            const double d = mt * gv;
            xn[i] = xv + d;
        }
    } else {   // BACKTRACK (algorithm_utils.py:124-135)
        if (scal[BSLS_XS_REVERT] != 0.0) {
            for (; i < n; i += stride) xn[i] = x[i];
        } else {
            const double tt = scal[BSLS_XS_TT];
            const double om = 1.0 - tt;
            for (; i < n; i += stride) {
                const double a = om * x[i];
                const double b = tt * xn[i];
                xn[i] = a + b;
            }
        }
    }
}

__global__ __launch_bounds__(XT) void xbb_step_kernel(double *__restrict__ x,
                                                      double *__restrict__ g,
                                                      double *__restrict__ xn,
                                                      const double *__restrict__ gn, int64_t n,
                                                      const double *__restrict__ scal) {
    const int mode = (int)scal[BSLS_XS_MODE];
    if (mode == BSLS_XM_STOPPED) return;
    xbb_step_body(x, g, xn, gn, n, scal, mode);
}

// ---- L-BFGS (BATCH.solve_LBFGS, python/BATCH.py:110-214) ---------------------
// lb (doubles): [0, C) the rho ring (rho appended at iteration i' in slot
// (i' - 2) % C), [C, 2C) alpha (the slot of its rho), [2C, 2C + 4) the
// coefficients a, b, c of the last direction and its t.
static size_t lb_doubles(int64_t C) { return (size_t)(2 * C + 8); }

// STEP round of iteration i > 5: the accepted point's deltas s = x_new - x,
// y = g_new - g (np.add(x_new, -x, delta_x), BATCH.py:197-198), x <- x_new,
// g <- g_new, and g.s, g.y, s.y, y.y; the last block then runs LBFGS_helper
// (:196-214) -- every queued correction is the latest (s, y), the queues
// holding the one delta buffer -- in the coefficients of d = a g + b s + c y:
//   d = g; for j = 1..m: alpha_j = rho[-j] s.d; d -= alpha_j y
//   d *= s.y / y.y; for j = 0..m-1: beta = rho[j] y.d; d += s (alpha[-m+j] - beta)
//   d = -d
// Any other round: xbb_step (i <= 5 keeps the BB step, :179-181).
__global__ __launch_bounds__(XT) void xlb_step_kernel(
    double *__restrict__ x, double *__restrict__ g, double *__restrict__ xn,
    const double *__restrict__ gn, double *__restrict__ sv, double *__restrict__ yv, int64_t n,
    const double *__restrict__ scal, double *__restrict__ lb, int64_t C,
    double *__restrict__ part, unsigned *__restrict__ ticket) {
    __shared__ double red[4 * XT / WAVE];
    const int mode = (int)scal[BSLS_XS_MODE];
    if (mode == BSLS_XM_STOPPED) return;
    const double it = scal[BSLS_XS_ITER];
    if (mode != BSLS_XM_STEP || it <= 5.0) {
        xbb_step_body(x, g, xn, gn, n, scal, mode);
        return;
    }
    const int64_t stride = (int64_t)gridDim.x * XT;
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < n; i += stride) {
        const double xv = xn[i], gv = gn[i], xo = x[i], go = g[i];
        const double s_ = xv - xo, y_ = gv - go;
        sv[i] = s_;
        yv[i] = y_;
        x[i] = xv;
        g[i] = gv;
        v[0] += gv * s_;
        v[1] += gv * y_;
        v[2] += s_ * y_;
        v[3] += y_ * y_;
    }
    block_reduce<4, 0u>(v, red);
    double tot[4];
    if (!last_block_reduce<4, 0u>(v, part, ticket, tot, red)) return;
    if (threadIdx.x != 0) return;
    const double gs = tot[0], gy = tot[1], sy = tot[2], yy = tot[3];
    const int64_t k = (int64_t)it - 1;            // corrections appended (iterations 2..i)
    const int64_t m = k < C ? k : C;
    double *rho = lb, *alpha = lb + C, *cf = lb + 2 * C;
    double a = 1.0, b = 0.0, c = 0.0;
    for (int64_t j = 1; j <= m; ++j) {            // newest first
        const int64_t q = (k - j) % C;
        const double al = rho[q] * (a * gs + c * sy);   // s.d, d = a g + c y
        alpha[q] = al;
        c -= al;                                        // d -= alpha y
    }
    const double t = sy / yy;
    a *= t;
    c *= t;
    for (int64_t j = 0; j < m; ++j) {             // oldest first
        const int64_t q = (k - m + j) % C;
        const double beta = rho[q] * (a * gy + b * sy + c * yy);   // y.d
        b += alpha[q] - beta;                           // d += s (alpha - beta)
    }
    cf[0] = a;
    cf[1] = b;
    cf[2] = c;
    cf[3] = t;
}

// x_new = x + d, d = -(a g + b s + c y) (d *= -1.0; np.add(x, d, x_new))
__global__ __launch_bounds__(XT) void xlb_dir_kernel(const double *__restrict__ x,
                                                     const double *__restrict__ g,
                                                     const double *__restrict__ sv,
                                                     const double *__restrict__ yv,
                                                     double *__restrict__ xn, int64_t n,
                                                     const double *__restrict__ scal,
                                                     const double *__restrict__ lb, int64_t C) {
    if ((int)scal[BSLS_XS_MODE] != BSLS_XM_STEP || scal[BSLS_XS_ITER] <= 5.0) return;
    const double a = lb[2 * C], b = lb[2 * C + 1], c = lb[2 * C + 2];
    const int64_t stride = (int64_t)gridDim.x * XT;
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < n; i += stride) {
        const double d = -((a * g[i] + b * sv[i]) + c * yv[i]);
        xn[i] = x[i] + d;
    }
}

// algorithm_utils.stopping (:158-172): every test runs, the last true one names
// the reason.
__device__ __forceinline__ int xstop(double i, double max_iter, double f, double f_old,
                                     double opt_tol, double prog_tol, double f_min,
                                     int has_fmin) {
    int reason = 0;
    if (i == max_iter) reason = BSLS_XSTOP_MAXITER;
    if (has_fmin && f - f_min < opt_tol) reason = BSLS_XSTOP_OPT;
    if (fabs(f_old - f) < prog_tol) reason = BSLS_XSTOP_PROG;
    return reason;
}

__global__ __launch_bounds__(XT) void xbb_finish_kernel(
    const double *__restrict__ x, const double *__restrict__ g, const double *__restrict__ xn,
    const double *__restrict__ gn, int64_t n, double *__restrict__ scal,
    double *__restrict__ hist, int64_t hist_cap, double max_iter, double opt_tol,
    double prog_tol, double f_min, int has_fmin, double *__restrict__ part,
    unsigned *__restrict__ ticket, double *__restrict__ lb, int64_t C) {
    __shared__ double red[4 * XT / WAVE];
    const int mode = (int)scal[BSLS_XS_MODE];
    if (mode == BSLS_XM_STOPPED) return;
    // gd = g.(x_new - x), dx.dg, dg.dg, ||dx||_inf
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if (mode != BSLS_XM_INIT) {
        // XU pairs per thread and step, 16-B loads, all issued before the math
        // (the vectors are 16-B aligned device allocations); odd tail by
        // thread 0 of workgroup 0
        const int64_t n2 = n >> 1;
        const int64_t stride = (int64_t)gridDim.x * XT * XU;
        for (int64_t p0 = (int64_t)blockIdx.x * XT * XU + threadIdx.x; p0 < n2; p0 += stride) {
            double2 gv[XU], xv[XU], xnv[XU], gnv[XU];
#pragma unroll
            for (int u = 0; u < XU; ++u) {
                const int64_t p = p0 + (int64_t)u * XT;
                const int64_t q = p < n2 ? p : 0;
                gv[u] = ((const double2 *)g)[q];
                xv[u] = ((const double2 *)x)[q];
                xnv[u] = ((const double2 *)xn)[q];
                gnv[u] = ((const double2 *)gn)[q];
            }
#pragma unroll
            for (int u = 0; u < XU; ++u) {
                if (p0 + (int64_t)u * XT < n2) {
                    const double dx0 = xnv[u].x - xv[u].x, dx1 = xnv[u].y - xv[u].y;
                    const double dg0 = gnv[u].x - gv[u].x, dg1 = gnv[u].y - gv[u].y;
                    v[0] += gv[u].x * dx0;
                    v[0] += gv[u].y * dx1;
                    v[1] += dx0 * dg0;
                    v[1] += dx1 * dg1;
                    v[2] += dg0 * dg0;
                    v[2] += dg1 * dg1;
                    v[3] = nan_max(v[3], fabs(dx0));
                    v[3] = nan_max(v[3], fabs(dx1));
                }
            }
        }
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const int64_t i = n - 1;
            const double gv = g[i];
            const double dx = xn[i] - x[i];
            const double dg = gn[i] - gv;
            v[0] += gv * dx;
            v[1] += dx * dg;
            v[2] += dg * dg;
            v[3] = nan_max(v[3], fabs(dx));
        }
    }
    block_reduce<4, 8u>(v, red);
    double tot[4];
    if (!last_block_reduce<4, 8u>(v, part, ticket, tot, red)) return;
    if (threadIdx.x != 0) return;
    const double f_new = .5 * scal[BSLS_XS_SQ];          // .5 * tmp.T.dot(tmp)
    scal[BSLS_XS_ROUNDS] += 1.0;
    if (mode == BSLS_XM_INIT) {                          // f = obj(x, g); i = 1
        scal[BSLS_XS_F] = f_new;
        scal[BSLS_XS_FOLD] = INFINITY;
        scal[BSLS_XS_ITER] = 1.0;
        scal[BSLS_XS_T] = 1.0;
        scal[BSLS_XS_TT] = 1.0;
        if (hist_cap > 0) hist[0] = f_new;
        const int r = xstop(1.0, max_iter, f_new, INFINITY, opt_tol, prog_tol, f_min, has_fmin);
        scal[BSLS_XS_STOP] = r;
        scal[BSLS_XS_MODE] = r ? BSLS_XM_STOPPED : BSLS_XM_STEP;
        return;
    }
    const double f = scal[BSLS_XS_F];
    scal[BSLS_XS_GD] = tot[0];
    scal[BSLS_XS_STEPINF] = tot[3];
    const double upper = f + 1e-4 * tot[0];               // f + suffDec * g.dot(x_new - x)
    if (f_new > upper) {                                  // while f_new > upper_line
        scal[BSLS_XS_BACKTRACKS] += 1.0;
        scal[BSLS_XS_TT] = scal[BSLS_XS_TT] * .8;         // t *= .8
        scal[BSLS_XS_REVERT] = (tot[3] < 1e-12) ? 1.0 : 0.0;   // step < progTol
        scal[BSLS_XS_MODE] = BSLS_XM_BACKTRACK;
        return;
    }
    // accept: f_old = f; f = f_new; delta_x, delta_g; i += 1 (BATCH.py:99-104)
    const double it = scal[BSLS_XS_ITER] + 1.0;
    scal[BSLS_XS_FOLD] = f;
    scal[BSLS_XS_F] = f_new;
    scal[BSLS_XS_DXDG] = tot[1];
    scal[BSLS_XS_DGDG] = tot[2];
    scal[BSLS_XS_T] = tot[1] / tot[2];                    // delta_x.T.dot(delta_g) / ...
    scal[BSLS_XS_TT] = 1.0;
    scal[BSLS_XS_REVERT] = 0.0;
    scal[BSLS_XS_ITER] = it;
    // L-BFGS: q_rho.append(1 / delta_g.T.dot(delta_x)) at iteration it (BATCH.py:174)
    if (C > 0) lb[((int64_t)it - 2) % C] = 1.0 / tot[1];
    const int64_t k = (int64_t)it - 1;
    if (k < hist_cap) hist[k] = f_new;
    const int r = xstop(it, max_iter, f_new, f, opt_tol, prog_tol, f_min, has_fmin);
    scal[BSLS_XS_STOP] = r;
    scal[BSLS_XS_MODE] = r ? BSLS_XM_STOPPED : BSLS_XM_STEP;
}

struct XWork {
    void *spmv;
    size_t spmv_bytes;
    unsigned *ticket;
    double *part;
    size_t bytes;
};

static XWork xwork(void *base, int64_t A_ntiles) {
    XWork w{};
    char *p = (char *)base;
    size_t off = 0;
    w.spmv = p + off;
    w.spmv_bytes = bsls_spmv_workspace_size(A_ntiles);
    off += xalign(w.spmv_bytes);
    w.ticket = (unsigned *)(p + off);
    off += xalign(TICKET_BYTES);
    w.part = (double *)(p + off);
    off += xalign((size_t)XGRID * 4 * sizeof(double));
    w.bytes = off;
    return w;
}

static int xgrid(int64_t n) {
    const int64_t g = (n + XT - 1) / XT;
    return (int)(g < 1 ? 1 : (g > XGRID ? XGRID : g));
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_xbb_workspace_size(int64_t m, int64_t n, int64_t A_ntiles,
                                          int64_t AT_ntiles) {
    (void)m;
    (void)n;
    (void)AT_ntiles;
    return xwork(nullptr, A_ntiles).bytes;
}

extern "C" size_t bsls_xbb_lbfgs_size(int64_t corrections) {
    return (corrections > 0 ? lb_doubles(corrections) : 0) * sizeof(double);
}

extern "C" int bsls_xbb_init(const bsls_xbb_problem *p, void *stream) {
    if (!p || !p->scal) return BSLS_E_ARG;
    xbb_init_kernel<<<1, 64, 0, (hipStream_t)stream>>>(p->scal, p->hist, p->hist_cap);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_xbb_rounds(const bsls_xbb_problem *p, int64_t count, void *stream) {
    if (!p || p->n <= 0 || p->m <= 0 || p->nblocks <= 0 || !p->x || !p->g || !p->xn || !p->gn ||
        !p->r || !p->scal || !p->neg_b || !p->starts || count < 0)
        return BSLS_E_ARG;
    if (!p->lsq && (p->A.rows != p->m || p->AT.rows != p->n)) return BSLS_E_ARG;
    if (p->lbfgs < 0 || (p->lbfgs > 0 && (!p->s || !p->y || !p->lb))) return BSLS_E_ARG;
    XWork w = xwork(p->work, p->A.ntiles);
    if (!p->work || p->work_bytes < w.bytes) return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const int gs = xgrid(p->n);
    const int64_t fw = ((p->n >> 1) + XT * XU - 1) / (XT * XU);
    const int gf = (int)(fw < 1 ? 1 : (fw > XGRID ? XGRID : fw));
    for (int64_t c = 0; c < count; ++c) {
        if (p->lbfgs > 0) {
            xlb_step_kernel<<<gs, XT, 0, st>>>(p->x, p->g, p->xn, p->gn, p->s, p->y, p->n, p->scal,
                                               p->lb, p->lbfgs, w.part, w.ticket);
            BSLS_LAUNCH_CHECK();
            xlb_dir_kernel<<<gs, XT, 0, st>>>(p->x, p->g, p->s, p->y, p->xn, p->n, p->scal, p->lb,
                                              p->lbfgs);
        } else {
            xbb_step_kernel<<<gs, XT, 0, st>>>(p->x, p->g, p->xn, p->gn, p->n, p->scal);
        }
        BSLS_LAUNCH_CHECK();
        int rc = proj_launch_gated((p->ball & 1) != 0, p->xn, p->starts, p->nblocks, p->n,
                                   p->max_block, p->proj_work, p->proj_work_bytes, st,
                                   p->scal + BSLS_XS_MODE, (p->ball & 2) != 0);
        if (rc != BSLS_OK) return rc;
        if (p->lsq) {
            rc = bsls_lsq_residual(p->lsq, p->xn, p->neg_b, p->r, p->scal + BSLS_XS_SQ, stream);
            if (rc != BSLS_OK) return rc;
            rc = bsls_lsq_gradient(p->lsq, p->r, p->gn, stream);
            if (rc != BSLS_OK) return rc;
        } else {
            rc = bsls_csr_spmv(p->m, p->A.indptr, p->A.indices, p->A.data, p->A.tiles,
                               p->A.ntiles, p->xn, p->neg_b, 1.0, p->r, p->scal + BSLS_XS_SQ,
                               (int)p->A.group, w.spmv, w.spmv_bytes, stream);
            if (rc != BSLS_OK) return rc;
            rc = bsls_csr_spmv(p->n, p->AT.indptr, p->AT.indices, p->AT.data, p->AT.tiles,
                               p->AT.ntiles, p->r, nullptr, 1.0, p->gn, nullptr, (int)p->AT.group,
                               nullptr, 0, stream);
            if (rc != BSLS_OK) return rc;
        }
        xbb_finish_kernel<<<gf, XT, 0, st>>>(p->x, p->g, p->xn, p->gn, p->n, p->scal, p->hist,
                                             p->hist_cap, (double)p->max_iter, p->opt_tol,
                                             p->prog_tol, p->f_min, (int)p->has_fmin, w.part,
                                             w.ticket, p->lb, p->lbfgs);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}
