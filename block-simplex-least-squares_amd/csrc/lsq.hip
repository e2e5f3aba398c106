// lsq.hip -- the x-space least-squares operator pair on panel images:
//   residual  r = A x + add, ||r||^2      (algorithm_utils.sparse_least_squares_obj
//                                           :88-94's tmp = A.dot(x) - b, tmp.dot(tmp))
//   gradient  g = A' r                     (its np.copyto(g, A_sparse_T.dot(tmp)))
// used by the x-space BB engine (xbb.hip), the batch objective
// (algorithm_utils.SparseLSQ) and mirror descent (mirror_descent.py:31-34).
// The same LDS-chunked panel walk as the z-space engine's K1 / K2 (panels.hpp,
// bb.hip), without the N / N' algebra: the residual splits the columns into
// XCD groups with per-group partial rows summed in group order by the last
// workgroup of each row block; the gradient sums each row of A' in CSR order
// over all chunks (bit-identical to SciPy's csr_matvec).  For a scaled
// incidence (values not stored) the residual first forms colv * x (the
// products SciPy forms, one extra pass) and the gradient multiplies each
// entry by its row's colv.
#include "panels.hpp"
#include "tiles.hpp"

namespace bsls {

struct LsqWork {
    unsigned *tk;       // ||r||^2 hand-off
    unsigned *tkrb;     // one ticket per row block
    double *part;       // one partial per row block
    double *xmax;       // fixed-point residual: max |x| (of colv * x when scaled), as bits,
                        //   in XMAX_SLOTS slots (the max over them)
    size_t bytes;
};
// one 64-bit atomic max per workgroup into slot blockIdx % XMAX_SLOTS: a
// single word took every wave's atomic in turn (~11 ns each: 4096 waves made
// the C3 x-space round 105 -> 148 us)
constexpr int XMAX_SLOTS = 64;

static size_t lal(size_t v) { return (v + 255) & ~(size_t)255; }

static LsqWork lsq_layout(void *base, int64_t A_npanels) {
    LsqWork w{};
    char *p = (char *)base;
    const int64_t rbs = (A_npanels + PANEL_WAVES - 1) / PANEL_WAVES + 1;
    size_t off = 0;
    w.tk = (unsigned *)(p + off);
    off += lal(TICKET_BYTES);
    w.tkrb = (unsigned *)(p + off);
    off += lal((size_t)rbs * 4);
    w.part = (double *)(p + off);
    off += lal((size_t)rbs * 8);
    w.xmax = (double *)(p + off);
    off += lal(XMAX_SLOTS * 8);
    w.bytes = off;
    return w;
}

// max |x| over n entries (with colv: of xs = colv * x, written on the way):
// the bit patterns of non-negative doubles order as unsigned integers (a NaN's
// above inf's, as nan_max wants), so each workgroup's max goes to one of
// XMAX_SLOTS words by a 64-bit atomic max -- order-free, hence the same at
// the same x -- over a grid as wide as the scaling pass (a last-block
// reduction over 512 workgroups took 9.9 us here against 5.7 for the plain
// scaling pass).  The slots are 0 on entry: the workspace starts zeroed and
// lsq_t_sum, which runs after the walk that reads them, clears them again.
__global__ __launch_bounds__(256) void lsq_xmax_kernel(double *__restrict__ xs,
                                                       const double *__restrict__ colv,
                                                       const double *__restrict__ x, int64_t n,
                                                       double *xmax) {
    __shared__ unsigned long long wmax[4];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    double mx = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double v = x[i];
        if (colv) {
            v = colv[i] * v;
            xs[i] = v;
        }
        mx = nan_max(mx, fabs(v));
    }
    unsigned long long b = (unsigned long long)__double_as_longlong(mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(b, o);
        b = t > b ? t : b;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = wmax[w] > b ? wmax[w] : b;
        if (b != 0ull)
            atomicMax(reinterpret_cast<unsigned long long *>(xmax) + blockIdx.x % XMAX_SLOTS, b);
    }
}

// the max over the slots (every workgroup of the walk reads the 64 words)
__device__ __forceinline__ double xmax_of(const double *xmax) {
    unsigned long long b = 0ull;
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(xmax);
#pragma unroll 16
    for (int k = 0; k < XMAX_SLOTS; ++k) b = w[k] > b ? w[k] : b;
    return __longlong_as_double((long long)b);
}

__global__ __launch_bounds__(256) void lsq_scale_kernel(double *__restrict__ xs,
                                                        const double *__restrict__ colv,
                                                        const double *__restrict__ x, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        xs[i] = colv[i] * x[i];
}

// workgroup (group g = blockIdx % ngroups, row block rb): the group's chunks of
// panels 16 rb .. 16 rb + 15 -> rpart[g][row]; the row block's last arriver
// sums the partials in group order (+ add) into r; with sq_out, the last row
// block reduces ||r||^2 (fixed order).
template <int MODE>
__global__ __launch_bounds__(1024) void lsq_k1(bsls_panels M, int64_t m,
                                               const double *__restrict__ x,
                                               const double *__restrict__ add,
                                               double *__restrict__ r, double *sq_out,
                                               double *rpart, unsigned *tkrb, double *part,
                                               unsigned *ticket) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int row_last;
    const int64_t G = M.ngroups;
    const int64_t g = blockIdx.x % G, rb = blockIdx.x / G;
    const int wv = threadIdx.x / WAVE, lane = lane_id();
    const int64_t panel = rb * PANEL_WAVES + wv;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    const double sc[4] = {0.0, 0.0, 0.0, 0.0};
    panel_chunks<MODE>(M, rb, wv, M.group_chunk[g], M.group_chunk[g + 1], x, lds, s, sc);
    if (panel < M.npanels) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = 64 * q + lane;
            const int64_t row = panel * M.prow + i;
            if (i < M.prow && row < m)
                __hip_atomic_store(&rpart[g * m + row], s[q], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev =
            __hip_atomic_fetch_add(&tkrb[rb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        row_last = (prev == (unsigned)G - 1);
        if (row_last) __hip_atomic_store(&tkrb[rb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!row_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t r0 = rb * PANEL_WAVES * M.prow;
    const int64_t r1 = (r0 + PANEL_WAVES * M.prow < m) ? r0 + PANEL_WAVES * M.prow : m;
    double sq[1] = {0.0};
    for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x) {
        double o = __hip_atomic_load(&rpart[row], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int64_t c = 1; c < G; ++c)
            o += __hip_atomic_load(&rpart[c * m + row], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (add) o += add[row];
        r[row] = o;
        sq[0] += o * o;
    }
    if (!sq_out) return;
    const unsigned nrb = (unsigned)((M.npanels + PANEL_WAVES - 1) / PANEL_WAVES);
    block_sum<1>(sq, lds);
    double tot[1];
    if (last_of_sum<1>(sq, part, (unsigned)rb, nrb, ticket, tot, lds) && threadIdx.x == 0)
        *sq_out = tot[0];
}

// g = A' r: one workgroup per 16 panels of A' rows, every chunk of r.
template <int MODE>
__global__ __launch_bounds__(1024) void lsq_k2(bsls_panels M, int64_t n,
                                               const double *__restrict__ r,
                                               const double *__restrict__ colv,
                                               double *__restrict__ g) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int wv = threadIdx.x / WAVE, lane = lane_id();
    const int64_t panel = (int64_t)blockIdx.x * PANEL_WAVES + wv;
    const int64_t i0 = panel * M.prow;
    const bool live = panel < M.npanels;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    double sc[4] = {0.0, 0.0, 0.0, 0.0};
    if (MODE == 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = i0 + 64 * q + lane;
            const bool ok = live && 64 * q + lane < M.prow && i < n;
            const double v = colv[ok ? i : 0];
            sc[q] = ok ? v : 0.0;
        }
    }
    panel_chunks<MODE>(M, blockIdx.x, wv, 0, M.nchunks, r, lds, s, sc);
    if (!live) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int pos = 64 * q + lane;
        const int64_t i = i0 + pos;
        if (pos < M.prow && i < n) g[i] = s[q];
    }
}

// The residual on a tile image of A (op->At.ent set: the dealt walk of the
// z-space engine's K1, csrc/tiles.hpp): workgroup (rb, g) sums its rows over
// group g's columns of x in LDS and stores them as rpart[g][row]; lsq_t_sum
// (next in the stream) adds the groups in group order (+ add) and reduces
// ||r||^2 -- the split finish of bb_k1t / bb_k1_sum.  LDS atomic sums: the
// same sums to rounding, not run-to-run bit-identical (the panels are).
template <int MODE>
__global__ __launch_bounds__(1024) void lsq_k1t(bsls_tiles T, int64_t m,
                                                const double *__restrict__ x,
                                                double *__restrict__ rpart) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int64_t rb, g;
    tile_map(T, blockIdx.x, gridDim.x / T.ngroups, rb, g);
    const int HR = (int)tile_lds_doubles(T, false);
    for (int i = threadIdx.x; i < HR; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    tile_walk_any<MODE>(T, rb, g, x, lds, nullptr);
    __syncthreads();
    const int64_t r0 = rb * T.H, r1 = (r0 + T.H < m) ? r0 + T.H : m;
    for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
        rpart[g * m + row] = lds[row - r0];
}

// The same in 64-bit fixed point (bsls_lsq_op.fixed): the scale 2^k puts
// every term within +-2^50 (|term| <= fx_amax * max|x|, max|x| from
// lsq_xmax_kernel), the integer row sums are order-free, so r -- and f --
// repeat bit for bit at the same x (the exits of the x-space solvers need
// that), at the dealt walk's speed.  Two words (tiles.hpp fx_add): each term
// rounds by at most 2^-(51 + fx_lo_shift(n)) of fx_amax max|x| (~2^-89 at 10M
// columns), the sum converts back once; the low word cannot overflow, however
// many entries a row holds.
template <int MODE>
__global__ __launch_bounds__(1024) void lsq_k1t_fx(bsls_tiles T, int64_t m,
                                                   const double *__restrict__ x,
                                                   double *__restrict__ rpart,
                                                   const double *__restrict__ xmax, double amax,
                                                   double xb) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int64_t rb, g;
    tile_map(T, blockIdx.x, gridDim.x / T.ngroups, rb, g);
    const double B = amax * (xb > 0.0 ? xb : xmax_of(xmax));
    int ex = 0;
    if (B > 0.0 && B <= 1.7976931348623157e308) (void)frexp(B, &ex);
    const double fxs = ldexp(1.0, 50 - ex), inv = ldexp(1.0, ex - 50);
    const int HR = (int)tile_lds_doubles(T, true);   // two words per row
    for (int i = threadIdx.x; i < HR; i += blockDim.x) lds[i] = 0.0;   // integer 0 too
    __syncthreads();
    tile_walk_any<MODE, true>(T, rb, g, x, lds, nullptr, fxs);
    __syncthreads();
    const int lo_off = (int)(T.H + T.halo + 1);
    const double inv_lo = ldexp(inv, -fx_lo_shift(T.cols));
    const int64_t r0 = rb * T.H, r1 = (r0 + T.H < m) ? r0 + T.H : m;
    // a NaN / inf in x (no finite scale): the rows are NaN, as a float sum
    // would make them (the solvers' NaN checks must still see it)
    const bool bad = !(B <= 1.7976931348623157e308);
    for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
        rpart[g * m + row] = bad ? __builtin_nan("") : fx_value(lds, (int)(row - r0), lo_off, inv,
                                                                  inv_lo);
}

__global__ __launch_bounds__(256) void lsq_t_sum(int64_t m, int64_t G, const double *rpart,
                                                 const double *__restrict__ add,
                                                 double *__restrict__ r, double *sq_out,
                                                 double *part, unsigned *ticket,
                                                 double *xmax_clear = nullptr) {
    __shared__ double red[4];
    // the fixed-point walk that read the max has finished: ready for the next call
    if (xmax_clear && blockIdx.x == 0 && threadIdx.x < XMAX_SLOTS) xmax_clear[threadIdx.x] = 0.0;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double sq[1] = {0.0};
    for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < m; row += gs) {
        // the first 8 groups' partials loaded together, added in group order
        double v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = (c < G) ? rpart[c * m + row] : 0.0;
        double o = v[0];
#pragma unroll
        for (int c = 1; c < 8; ++c)
            if (c < G) o += v[c];
        for (int64_t c = 8; c < G; ++c) o += rpart[c * m + row];
        if (add) o += add[row];
        r[row] = o;
        sq[0] += o * o;
    }
    if (!sq_out) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0) *sq_out = tot[0];
}
constexpr int LSQ_SUM_GRID = 1024;

constexpr int LSQ_LDS_MAX = 163840 - 512;
template <typename K>
static void lsq_allow_lds(K kernel) {
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LSQ_LDS_MAX);
        done = true;
    }
}

// one dealt image of A' (layout 1 / 2, one group, halo 0): tile rb sums the
// entries of each of its rows in LDS (atomic adds: the sums to rounding, not
// SciPy's order) and writes g = colv_i * sum (scaled incidence, MODE 0) or
// the sum (values stored, MODE 1) -- the z-space K2's walk without its N'
// epilogue
template <int MODE>
__global__ __launch_bounds__(1024) void lsq_k2t(bsls_tiles T, int64_t n,
                                                const double *__restrict__ r,
                                                const double *__restrict__ colv,
                                                double *__restrict__ g) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int64_t rb, gg;
    tile_map(T, blockIdx.x, gridDim.x / T.ngroups, rb, gg);
    const int HR = (int)tile_lds_doubles(T, false);
    for (int i = threadIdx.x; i < HR; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    tile_walk_any<MODE>(T, rb, gg, r, lds, nullptr);
    __syncthreads();
    const int64_t r0 = rb * T.H, r1 = (r0 + T.H < n) ? r0 + T.H : n;
    for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
        g[row] = (MODE == 0) ? colv[row] * lds[row - r0] : lds[row - r0];
}

static bool lsq_ok(const bsls_lsq_op *op) {
    if (!op || op->m <= 0 || op->n <= 0) return false;
    const bsls_panels &A = op->A, &T = op->AT;
    if (op->ATt.ent) {
        const bsls_tiles &K = op->ATt;
        // the shared validator (bb.hip's) plus what lsq_k2t assumes: one group,
        // a dealt layout, values iff the matrix is not a scaled incidence
        if (!tiles_valid(K, op->n, op->m, 0, op->colv == nullptr, false, LSQ_LDS_MAX)) return false;
        if (K.ngroups != 1 || (K.layout & 3) == 0) return false;
        if ((op->colv == nullptr) != (K.val != nullptr)) return false;
    } else {
        if (T.rows != op->n || T.cols != op->m || T.halo != 0 || T.ngroups != 1) return false;
        if (T.prow < 1 || T.prow > BSLS_PANEL_ROWS) return false;
    }
    if (op->At.ent) {
        const bsls_tiles &K = op->At;
        // (the fixed-point walk keeps two words per row: twice the LDS)
        if (!tiles_valid(K, op->m, op->n, 0, op->colv == nullptr, op->fixed != 0, LSQ_LDS_MAX))
            return false;
        if ((K.layout & 3) == 0) return false;
        if ((op->colv == nullptr) != (K.val != nullptr)) return false;
    } else {
        if (A.rows != op->m || A.cols != op->n || A.halo != 0 || A.ngroups < 1) return false;
        if (A.prow < 1 || A.prow > BSLS_PANEL_ROWS) return false;
    }
    if (!op->rpart || !op->work) return false;
    if (op->fixed && (!op->At.ent || (op->At.layout & 3) == 0 || !(op->fx_amax > 0.0) ||
                      op->fx_amax > 1e300 || (op->colv && !op->xs)))
        return false;
    if (!(op->x_bound >= 0.0) || op->x_bound > 1e300) return false;
    if (op->colv && !op->xs) return false;
    if (!op->ATt.ent && (op->colv ? T.val != nullptr : !T.val)) return false;
    if (!op->At.ent && (op->colv ? A.val != nullptr : !A.val)) return false;
    return true;
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_lsq_workspace_size(int64_t m, int64_t A_npanels) {
    (void)m;
    // (the tile residual's reduction uses part's first LSQ_SUM_GRID slots)
    const int64_t np = A_npanels > LSQ_SUM_GRID * PANEL_WAVES ? A_npanels : LSQ_SUM_GRID * PANEL_WAVES;
    return lsq_layout(nullptr, np).bytes;
}

extern "C" int bsls_lsq_residual(const bsls_lsq_op *op, const double *d_x, const double *d_add,
                                 double *d_r, double *d_sq_out, void *stream) {
    if (!lsq_ok(op) || !d_x || !d_r) return BSLS_E_ARG;
    LsqWork w = lsq_layout(op->work, op->At.ent ? LSQ_SUM_GRID * PANEL_WAVES : op->A.npanels);
    if (op->work_bytes < w.bytes) return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    if (op->At.ent && op->fixed) {
        const bsls_tiles &K = op->At;
        const double xb = op->x_bound;
        if (xb > 0.0) {
            // the caller's bound (bsls_lsq_op.x_bound): only colv * x to form
            if (op->colv)
                lsq_scale_kernel<<<grid_for(op->n < 262144 ? op->n : 262144, 256), 256, 0, st>>>(
                    op->xs, op->colv, d_x, op->n);
        } else {
            lsq_xmax_kernel<<<grid_for(op->n < 262144 ? op->n : 262144, 256), 256, 0, st>>>(
                op->xs, op->colv, d_x, op->n, w.xmax);
        }
        BSLS_LAUNCH_CHECK();
        const double *xin = op->colv ? op->xs : d_x;
        const int grid = (int)(K.nrb * K.ngroups);
        const size_t lds = tile_lds_doubles(K, true) * 8;
        if (op->colv) {
            lsq_allow_lds(lsq_k1t_fx<0>);
            lsq_k1t_fx<0><<<grid, BSLS_TILE_THREADS, lds, st>>>(K, op->m, xin, op->rpart, w.xmax,
                                                               op->fx_amax, xb);
        } else {
            lsq_allow_lds(lsq_k1t_fx<1>);
            lsq_k1t_fx<1><<<grid, BSLS_TILE_THREADS, lds, st>>>(K, op->m, xin, op->rpart, w.xmax,
                                                               op->fx_amax, xb);
        }
        BSLS_LAUNCH_CHECK();
        const int gk = grid_for(op->m, 256);
        lsq_t_sum<<<gk < LSQ_SUM_GRID ? gk : LSQ_SUM_GRID, 256, 0, st>>>(
            op->m, K.ngroups, op->rpart, d_add, d_r, d_sq_out, w.part, w.tk,
            xb > 0.0 ? nullptr : w.xmax);
        BSLS_LAUNCH_CHECK();
        return BSLS_OK;
    }
    if (op->At.ent) {
        const bsls_tiles &K = op->At;
        const double *xin = d_x;
        if (op->colv) {
            lsq_scale_kernel<<<grid_for(op->n < 262144 ? op->n : 262144, 256), 256, 0, st>>>(
                op->xs, op->colv, d_x, op->n);
            BSLS_LAUNCH_CHECK();
            xin = op->xs;
        }
        const int grid = (int)(K.nrb * K.ngroups);
        const size_t lds = tile_lds_doubles(K, false) * 8;
        if (op->colv) {
            lsq_allow_lds(lsq_k1t<0>);
            lsq_k1t<0><<<grid, BSLS_TILE_THREADS, lds, st>>>(K, op->m, xin, op->rpart);
        } else {
            lsq_allow_lds(lsq_k1t<1>);
            lsq_k1t<1><<<grid, BSLS_TILE_THREADS, lds, st>>>(K, op->m, xin, op->rpart);
        }
        BSLS_LAUNCH_CHECK();
        const int gk = grid_for(op->m, 256);
        lsq_t_sum<<<gk < LSQ_SUM_GRID ? gk : LSQ_SUM_GRID, 256, 0, st>>>(
            op->m, K.ngroups, op->rpart, d_add, d_r, d_sq_out, w.part, w.tk);
        BSLS_LAUNCH_CHECK();
        return BSLS_OK;
    }
    const int64_t rbs = (op->A.npanels + PANEL_WAVES - 1) / PANEL_WAVES;
    const int grid = (int)(op->A.ngroups * rbs);
    if (op->colv) {
        lsq_scale_kernel<<<grid_for(op->n < 262144 ? op->n : 262144, 256), 256, 0, st>>>(
            op->xs, op->colv, d_x, op->n);
        BSLS_LAUNCH_CHECK();
        lsq_allow_lds(lsq_k1<0>);
        lsq_k1<0><<<grid, 1024, panel_lds_bytes(op->A), st>>>(op->A, op->m, op->xs, d_add, d_r,
                                                              d_sq_out, op->rpart, w.tkrb, w.part,
                                                              w.tk);
    } else {
        lsq_allow_lds(lsq_k1<1>);
        lsq_k1<1><<<grid, 1024, panel_lds_bytes(op->A), st>>>(op->A, op->m, d_x, d_add, d_r,
                                                              d_sq_out, op->rpart, w.tkrb, w.part,
                                                              w.tk);
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_lsq_gradient(const bsls_lsq_op *op, const double *d_r, double *d_g,
                                 void *stream) {
    if (!lsq_ok(op) || !d_r || !d_g) return BSLS_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (op->ATt.ent) {
        const bsls_tiles &K = op->ATt;
        const size_t lds = tile_lds_doubles(K, false) * 8;
        if (op->colv) {
            lsq_allow_lds(lsq_k2t<0>);
            lsq_k2t<0><<<(int)K.nrb, BSLS_TILE_THREADS, lds, st>>>(K, op->n, d_r, op->colv, d_g);
        } else {
            lsq_allow_lds(lsq_k2t<1>);
            lsq_k2t<1><<<(int)K.nrb, BSLS_TILE_THREADS, lds, st>>>(K, op->n, d_r, nullptr, d_g);
        }
        BSLS_LAUNCH_CHECK();
        return BSLS_OK;
    }
    const int grid = grid_for(op->AT.npanels, PANEL_WAVES);
    if (op->colv) {
        lsq_allow_lds(lsq_k2<2>);
        lsq_k2<2><<<grid, 1024, panel_lds_bytes(op->AT), st>>>(op->AT, op->n, d_r, op->colv, d_g);
    } else {
        lsq_allow_lds(lsq_k2<1>);
        lsq_k2<1><<<grid, 1024, panel_lds_bytes(op->AT), st>>>(op->AT, op->n, d_r, nullptr, d_g);
    }
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
