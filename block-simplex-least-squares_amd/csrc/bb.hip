// bb.hip -- fused z-space projected Barzilai-Borwein iteration on one GCD.
//
// Reference loop (python/BB.py:17-41) over main.solve_in_z's closures
// (python/main.py:53-65), stopping rule solvers.stopping (python/solvers.py:40-63):
//     g = N'A'(A N z + target);  dg = g - g_prev;  if sum(dg) == 0: break
//     t = (z - z_prev).dg / dg.dg;  z <- clip01(PAVA(z - t g));  fx = f(z); stop?
// One iteration here = three kernels, all HBM-bound, no host round trip:
//   K2  g = N'(A' r) with an explicit A' in panel format (panels.hpp): each
//       workgroup stages r chunk by chunk into LDS and sums its rows there in
//       CSR order (bit-identical to SciPy's csr_matvec); each panel carries the
//       next panel's first row, so the adjacent difference N'w = w_i - w_{i+1}
//       stays in the wave; fused: dg, the four BB sums, the store of g.
//   K3  t from the sums; per z-block PAVA (v1 pooling order, bit-identical to
//       isotonic_regression.h:13-58) + clip to [0,1] + the vector N z (per-block
//       differences, last entry -z_last), one wave per pack of whole blocks
//       (<= 64 entries, one lane per entry, pava_wave.hpp).  N is never
//       materialised.
//   K1  r = A (N z) + target, target = A x0 - b, exactly the reference's
//       A.dot(N.dot(z)) + target.  A in panel format with its column chunks
//       split into G groups (device.k1_plan: C3 10), group = blockIdx % G;
//       each workgroup stages its group's slice of x chunk by chunk into LDS
//       and publishes one partial per (row, group); the last of a row
//       block's G workgroups sums them in group order, adds target,
//       ||r||^2 (next gradient's residual AND f(z)); the last row block runs
//       the stopping test.
//   For a scaled incidence A (bsls_utils.py:494) the values are not stored:
//   K3 writes colv * (N z) (the same products SciPy forms), K2 multiplies by
//   the row's colv.
// Sparse row blocks (C5: 1M links, ~0.3 entries per row per panel chunk) take
// the streamed-tile format instead of the panels for K1 and/or K2 (tiles.hpp;
// bb_k1t / bb_k2t, chosen per matrix by the host: P.At / P.ATt).
// Every cross-workgroup sum of a reduction (the BB sums, ||r||^2) is reduced in
// a fixed order by the last-arriving workgroup (bsls_common.hpp last_block_sum).
// The SpMV row sums are fixed-order on the panels and the thread-stream tiles
// (BBEngine(deterministic=True): runs bit-reproducible); the dealt tiles, the
// default, add them with LDS atomics, so their rounding varies run to run at
// the 1e-16 level.
// Scalars live in device memory (scal[]); the host only polls them.
#include "pava.hpp"
#include "pava_long.hpp"
#include "pava_wave.hpp"
#include "panels.hpp"
#include "tiles.hpp"

namespace bsls {


struct BBWork {
    unsigned *tk1, *tk2, *tkf, *tkrb, *tk2rb;
    double *p1, *p2, *pf;
    int32_t *wsc;
    double *dz;   // z - z_prev, written by K3 (and the prologue) for the next K2
    uint64_t *hd; // K3's warm start: each pack's last run-head mask (<= n - nz packs),
                  //   two sets (slot 1: DORE's second projection, the line search's trials)
    int64_t hd_stride;
    size_t bytes;
};

static size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }


static BBWork bb_layout(void *base, int64_t m, int64_t n, int64_t nz) {
    BBWork w{};
    char *p = (char *)base;
    size_t off = 0;
    w.tk1 = (unsigned *)(p + off);
    w.tk2 = (unsigned *)(p + off + TICKET_BYTES);
    w.tkf = (unsigned *)(p + off + 2 * TICKET_BYTES);
    off += al16(3 * TICKET_BYTES);
    w.tkrb = (unsigned *)(p + off);              // K1: one ticket per row block
    off += al16((size_t)(m / 16 + 2) * 4);
    w.tk2rb = (unsigned *)(p + off);             // K2 tiles: one ticket per row block (H >= 64)
    off += al16((size_t)(n / 64 + 2) * 4);
    // K1's per-row-block partials of ||r||^2: one per row block (two slots
    // reserved), and a row block holds >= 16 rows (16 panels of >= 1 row;
    // tiles of >= 64 rows)
    w.p1 = (double *)(p + off);
    off += al16((size_t)(m / 16 + 2) * 2 * 8);
    w.p2 = (double *)(p + off);
    off += al16((size_t)((n + PANEL_WAVES - 1) / PANEL_WAVES + 1) * 5 * 8);   // (5 sums fused)
    w.pf = (double *)(p + off);
    off += al16((size_t)((m + 255) / 256 + 1) * 2 * 8);
    w.wsc = (int32_t *)(p + off);
    off += al16((size_t)(nz > 0 ? nz : 1) * 4);
    w.dz = (double *)(p + off);
    off += al16((size_t)(nz > 0 ? nz : 1) * 8);
    w.hd = (uint64_t *)(p + off);
    w.hd_stride = n - nz > 0 ? n - nz : 1;
    off += al16((size_t)w.hd_stride * 2 * 8);
    w.bytes = off;
    return w;
}

static BBWork bb_layout(const bsls_bb_problem &P) { return bb_layout(P.work, P.m, P.n, P.nz); }

// column scale i (bsls_bb_problem.colv_codec: exact narrow copies read instead
// of the doubles)
__device__ __forceinline__ double colv_at(const bsls_bb_problem &P, int64_t i) {
    if (P.colv_codec == 2) return (double)reinterpret_cast<const _Float16 *>(P.colv_n)[i];
    if (P.colv_codec == 1) return (double)reinterpret_cast<const float *>(P.colv_n)[i];
    return P.colv[i];
}

// the same with the codec known at compile time (the hot kernels are
// instantiated per codec: a runtime switch among three loads inside K2's
// batched epilogue kept its loads from being in flight together)
template <int CV>
__device__ __forceinline__ double colv_t(const bsls_bb_problem &P, int64_t i) {
    if constexpr (CV == 2) return (double)reinterpret_cast<const _Float16 *>(P.colv_n)[i];
    else if constexpr (CV == 1) return (double)reinterpret_cast<const float *>(P.colv_n)[i];
    else return P.colv[i];
}

// solvers.py:40-63 on iteration iter's g.g and dg.dg (the all-reduced sums)
__device__ __forceinline__ int bb_stop_reason(const bsls_bb_problem &P, int64_t iter, double fx,
                                              double gg, double dgdg) {
    if (iter >= P.max_iter) return BSLS_STOP_MAXITER;
    if (P.early_exit) {
        const double gn = sqrt(gg);
        if (gn * gn <= P.opt_tol * (1 + fabs(fx))) return BSLS_STOP_GRAD;
        if (sqrt(dgdg) == 0) return BSLS_STOP_DG;
    }
    return 0;
}

__device__ __forceinline__ void bb_stop_check(const bsls_bb_problem &P, int64_t iter, double fx) {
    double *s = P.scal;
    const int reason = bb_stop_reason(P, iter, fx, s[BSLS_S_GG], s[BSLS_S_DGDG]);
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

// A column shard's r in 64-bit fixed point (bsls_bb_problem.r_fx > 0): the
// stored word is the int64 llrint(r * r_fx).  r_fx_of(v): v as that word.
__device__ __forceinline__ double r_fx_of(const bsls_bb_problem &P, double v) {
    return __longlong_as_double(__double2ll_rn(v * P.r_fx));
}
__device__ __forceinline__ double r_load(const bsls_bb_problem &P, int64_t i) {
    if (P.r_fx > 0.0) return (double)__double_as_longlong(P.r[i]) * (1.0 / P.r_fx);
    return P.r[i];
}

// A column-sharded rank other than the one adding target (shard_role 2)
// writes r = 0 for its rows once the run has stopped: its K1 no longer forms a
// partial, and the all-reduce must leave the final residual (held by the
// shard_role 1 rank, whose r is not touched) as it was.
__device__ __forceinline__ void k1_stopped_rows(const bsls_bb_problem &P, int64_t r0, int64_t r1,
                                                int64_t t0, int64_t stride) {
    if (P.shard_role != 2) return;
    for (int64_t row = r0 + t0; row < r1; row += stride) P.r[row] = 0.0;
}

// K1's finish for row block rb (rows [r0, r1)), run by one workgroup: r =
// the G partials of each row summed in group order (from rpart, or from LDS
// `local` when the block had one group) + target; its share of ||r||^2 goes
// to the last row block, which records f and runs the stopping test.
template <bool ADD, bool REDUCE>
__device__ __forceinline__ void k1_finish(const bsls_bb_problem &P, int64_t iter, bool iterating,
                                          int64_t rb, unsigned nrb, int64_t r0, int64_t r1,
                                          int64_t G, const double *local, double *part,
                                          unsigned *ticket, double *red) {
    double sq[1] = {0.0};
    if (local) {
        for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x) {
            double o = local[row - r0];
            if (ADD) o += P.target[row];
            P.r[row] = o;
            sq[0] += o * o;
        }
    } else {
        // up to RPT rows per thread, every partial load of them in flight at once
        constexpr int RPT = 4;
        for (int64_t row0 = r0 + threadIdx.x; row0 < r1; row0 += RPT * blockDim.x) {
            double v[RPT][8];
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int64_t row = row0 + (int64_t)u * blockDim.x;
                const int64_t rr = row < r1 ? row : r0;
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    v[u][c] = (c < G) ? __hip_atomic_load(&P.rpart[c * P.m + rr], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : 0.0;
            }
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int64_t row = row0 + (int64_t)u * blockDim.x;
                if (row >= r1) continue;
                double o = v[u][0];
#pragma unroll
                for (int c = 1; c < 8; ++c)
                    if (c < G) o += v[u][c];
                for (int64_t c = 8; c < G; ++c)
                    o += __hip_atomic_load(&P.rpart[c * P.m + row], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                if (ADD) o += P.target[row];
                P.r[row] = o;
                sq[0] += o * o;
            }
        }
    }
    if (!REDUCE) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_of_sum<1>(sq, part, (unsigned)rb, nrb, ticket, tot, red) && threadIdx.x == 0)
        bb_record_f(P, iter, tot[0], iterating);
}

// K1: workgroup (group g = blockIdx % ngroups, panels 16 rb .. 16 rb + 15)
// stages x chunk by chunk (the group's columns) and publishes, per row, the
// sum over the group's columns in rpart[g][row] (sc1: visible across XCDs).
// The last of the row block's ngroups workgroups to arrive sums the partials
// in group order (+ target), writes r, and (REDUCE) hands its share of
// ||r||^2 to the last row block, which records f and runs the stopping test.
template <int MODE, bool ITER, bool ADD, bool REDUCE>
__global__ __launch_bounds__(1024) void bb_k1(bsls_bb_problem P, int64_t iter, unsigned *tkrb,
                                              double *part, unsigned *ticket, int64_t rb_base) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int row_last;
    const bsls_panels &M = P.A;
    const int64_t G = M.ngroups;
    const int64_t g = blockIdx.x % G, rb = rb_base + blockIdx.x / G;
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        if (g == 0) {
            const int64_t r0 = rb * PANEL_WAVES * M.prow;
            const int64_t r1 = (r0 + PANEL_WAVES * M.prow < P.m) ? r0 + PANEL_WAVES * M.prow : P.m;
            k1_stopped_rows(P, r0, r1, threadIdx.x, blockDim.x);
        }
        return;
    }
    const int wv = threadIdx.x / WAVE, lane = lane_id();
    const int64_t panel = rb * PANEL_WAVES + wv;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    const double sc[4] = {0.0, 0.0, 0.0, 0.0};
    panel_chunks<MODE>(M, rb, wv, M.group_chunk[g], M.group_chunk[g + 1], P.x, lds, s, sc);
    if (panel < M.npanels) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = 64 * q + lane;
            const int64_t row = panel * M.prow + i;
            if (i < M.prow && row < P.m)
                __hip_atomic_store(&P.rpart[g * P.m + row], s[q], __ATOMIC_RELAXED,
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
    const int64_t r1 = (r0 + PANEL_WAVES * M.prow < P.m) ? r0 + PANEL_WAVES * M.prow : P.m;
    const unsigned nrb = (unsigned)((M.npanels + PANEL_WAVES - 1) / PANEL_WAVES);
    k1_finish<ADD, REDUCE>(P, iter, ITER, rb, nrb, r0, r1, G, nullptr, part, ticket, lds);
}

// BSLS_K1_SPLIT (default 1): a K1 tile launch with several column groups ends
// once its partials are stored, and bb_k1_sum finishes the rows in a launch of
// its own -- the kernel boundary replaces the in-kernel hand-off (partials
// drained, a ticket per row block, the last arriver's loads, a second ticket
// for ||r||^2: a chain of dependent round trips that took ~half of C3's K1)
#ifndef BSLS_K1_SPLIT
#define BSLS_K1_SPLIT 1
#endif

// K1's finish as its own launch (rows [r0, r1), one thread per row): r = the G
// partials in group order (+ target, ADD), ||r||^2 and f by the last block
// (REDUCE), as k1_finish.
template <bool ITER, bool ADD, bool REDUCE>
__global__ __launch_bounds__(256) void bb_k1_sum(bsls_bb_problem P, int64_t iter, int64_t G,
                                                 int64_t r0, int64_t r1, double *part,
                                                 unsigned *ticket) {
    __shared__ double red[8];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        k1_stopped_rows(P, r0, r1, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                        (int64_t)gridDim.x * blockDim.x);
        return;
    }
    // grid-stride rows: with REDUCE the launch is capped at K1_SUM_GRID
    // workgroups (one per 256 rows made 3.9k arrivals at the ||r||^2 tickets
    // at m = 1M: 12.5 us against 4.6 without the reduction)
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double sq[1] = {0.0};
    for (int64_t row = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < r1; row += gs) {
        double v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = (c < G) ? P.rpart[c * P.m + row] : 0.0;
        double o = v[0];
#pragma unroll
        for (int c = 1; c < 8; ++c)
            if (c < G) o += v[c];
        for (int64_t c = 8; c < G; ++c) o += P.rpart[c * P.m + row];
        if (ADD) o += P.target[row];
        P.r[row] = o;
        sq[0] += o * o;
    }
    if (!REDUCE) return;
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0)
        bb_record_f(P, iter, tot[0], ITER);
}

// K1 with global atomics (BSLS_K1_ATOMIC): rows [r0, r1) of r start as
// target (ADD) or 0 for the groups to add into; once the run has stopped, the
// shard_role 1 rank keeps its r (the final residual) and the others write 0.
template <bool ITER, bool ADD>
__global__ __launch_bounds__(256) void bb_k1_init(bsls_bb_problem P, int64_t r0, int64_t r1) {
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        k1_stopped_rows(P, r0, r1, t0, gs);
        return;
    }
    for (int64_t row = r0 + t0; row < r1; row += gs) {
        const double v = ADD ? P.target[row] : 0.0;
        P.r[row] = (P.r_fx > 0.0) ? r_fx_of(P, v) : v;
    }
}

// K1 on a tile image (tiles.hpp): workgroup (rb, g) sums its rows over group
// g's columns of x in LDS; with one group it finishes the block itself,
// otherwise it publishes its partials (rpart, sc1) and the last of the block's
// G workgroups finishes (group order) -- as bb_k1.
// BSLS_K1T_WGS (variant builds): the workgroups of 1024 threads a CU must
// hold at once (2: registers capped so two tiles share a CU)
#ifndef BSLS_K1T_WGS
#define BSLS_K1T_WGS 1
#endif
template <int MODE, bool ITER, bool ADD, bool REDUCE, bool ATOM = false>
__global__ __launch_bounds__(1024, BSLS_K1T_WGS) void bb_k1t(bsls_bb_problem P, int64_t iter, unsigned *tkrb,
                                               double *part, unsigned *ticket, int64_t rb_base) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double red[32];   // (k1_finish: 2 doubles per wave)
    __shared__ int row_last;
    const bsls_tiles &T = P.At;
    int64_t rb, g;
    tile_map(T, blockIdx.x, gridDim.x / T.ngroups, rb, g);
    rb += rb_base;
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        // (several groups with the split finish: bb_k1_sum zeroes the rows;
        // ATOM: bb_k1_init did)
        if (!ATOM && g == 0 && (T.ngroups == 1 || !BSLS_K1_SPLIT))
            k1_stopped_rows(P, rb * T.H, (rb * T.H + T.H < P.m) ? rb * T.H + T.H : P.m,
                            threadIdx.x, blockDim.x);
        return;
    }
    const int HR = (int)tile_lds_doubles(T, false);
    for (int i = threadIdx.x; i < HR; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    tile_walk_any<MODE>(T, rb, g, P.x, lds, nullptr);
    __syncthreads();
    const int64_t G = T.ngroups;
    const int64_t r0 = rb * T.H, r1 = (r0 + T.H < P.m) ? r0 + T.H : P.m;
    if (G == 1) {
        k1_finish<ADD, REDUCE>(P, iter, ITER, rb, (unsigned)T.nrb, r0, r1, 1, lds, part, ticket,
                               red);
        return;
    }
    if (ATOM) {
        // r was set to target / 0 by bb_k1_init: every group adds its sums
        // (global f64 atomics; the order over groups varies run to run, as the
        // dealt walk's LDS sums do)
        // (r_fx: the sums as int64 words, added as integers -- order-free)
        if (P.r_fx > 0.0) {
            for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
                atomicAdd(reinterpret_cast<unsigned long long *>(&P.r[row]),
                          (unsigned long long)__double2ll_rn(lds[row - r0] * P.r_fx));
        } else {
            for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
                unsafeAtomicAdd(&P.r[row], lds[row - r0]);
        }
        return;
    }
    if (BSLS_K1_SPLIT) {
        // the partials only; bb_k1_sum (next in the stream) finishes the rows
        for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
            P.rpart[g * P.m + row] = lds[row - r0];
        return;
    }
    for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x)
        __hip_atomic_store(&P.rpart[g * P.m + row], lds[row - r0], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
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
    k1_finish<ADD, REDUCE>(P, iter, ITER, rb, (unsigned)T.nrb, r0, r1, G, nullptr, part, ticket,
                           red);
}

// K2's epilogue rows per thread per batch (K2E; round 6: 4 -- C3's 3.8 rows
// per thread fit one batch, C5's 19 run five at the speed of three of 8, and
// the kernel drops from 124 to 86 VGPRs: C3 13.2k -> 13.4k it/s, C5 and the
// 8-way C5 rank the same, tools/gpu_r06k.sh; A/B builds: BSLS_K2E.  Loading
// the first batch's z indices and scales before the walk instead, to land
// under it, measured no gain: 13.2k)
#ifndef BSLS_K2E
#define BSLS_K2E 4
#endif

// K2 on a tile image: w = A'r for row block rb (+ its halo row) in LDS, summed
// over r's column groups (one group: in CSR order, bit-identical to SciPy;
// several: partials in wpart, summed in group order by the block's last
// workgroup); then g = N'w, dg and the four BB sums, as bb_k2.  MODE 1: stored
// values; MODE 2: scaled incidence, each term colv[row] * r_i (SciPy's
// product; the rows' scales sit in LDS beside the sums); MODE 3: scaled
// incidence with several groups (no bit pattern to keep): w_i = colv_i *
// sum r, one product per row after the group sums, and the whole LDS for rows.
// FUSE (stage 8, column-sharded): every workgroup first sums r_i^2 over its
// slice of r (already the all-reduced residual; slice blockIdx of nrb * G, so
// the linear read also warms the caches the walk gathers r from), the
// finishing workgroup of row block rb adds its groups' slices in group order
// (through wpart's tail, see bsls_bb_problem.wpart), and the last one records
// f and runs the stopping test of iteration iter - 1 before it stores this
// iteration's sums.  (At the end of the finishing workgroups only, the slice
// sums cost 13 us of tail in the 8-way rehearsal.)
// FUSE 2 (stage 10, the sliced schedule): the same r^2, but over this rank's
// rows [P.rr_lo, P.rr_hi) of r only (1/world of m: the other ranks sum the
// rest), stored with the sums as scal[RR] for the all-reduce; the last
// workgroup keeps iteration iter - 1's sums in scal[PSUMDG..PGG] for the
// stop test that follows the all-reduce (stage 12), instead of testing.
// K2 of a stopped sharded run: the driver still all-reduces scal[SUMDG..RR]
// after every K2 it enqueues, so the shard_role 2 ranks zero their copy and
// the sum leaves role 1's -- the stop iteration's sums -- instead of world
// times them, growing with every iteration enqueued past the stop
// (fuse 2 all-reduces scal[RR] with the four sums)
template <int FUSE>
__device__ __forceinline__ void k2_stopped_sums(const bsls_bb_problem &P) {
    if (P.shard_role == 2 && blockIdx.x == 0 && threadIdx.x == 0)
        for (int q = 0; q < (FUSE == 2 ? 5 : 4); ++q) P.scal[BSLS_S_SUMDG + q] = 0.0;
}

// gsel >= 0 (bsls_bb_k2_part): only column group gsel, one workgroup per row
// block -- the link-part pipeline of the sharded schedule launches the groups
// one by one, each as soon as its rows of r are all-reduced.  The launches
// are ordered on one stream, so the roles are fixed: groups < G - 1 leave
// their partial row sums (and r^2 slices) in wpart and return; the last group
// adds them in group order and runs the epilogue -- no tickets.  Its slice of
// ||r||^2 stays inside its own link range (rows of r the earlier parts'
// exchanges have not finished may not be read).
template <int MODE, bool ITER, int FUSE = 0, int CV = 0>
__global__ __launch_bounds__(1024) void bb_k2t(bsls_bb_problem P, const double *__restrict__ dzv,
                                               const double *__restrict__ gp,
                                               double *__restrict__ gout, double *part,
                                               unsigned *ticket, unsigned *tk2rb, int64_t iter,
                                               int gsel) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double red[5 * 16];
    __shared__ int row_last;
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        if (gsel < 0 || gsel == P.ATt.ngroups - 1) k2_stopped_sums<FUSE>(P);
        return;
    }
    const bsls_tiles &T = P.ATt;
    int64_t rb, g;
    if (gsel >= 0) {
        rb = blockIdx.x;
        g = gsel;
    } else {
        tile_map(T, blockIdx.x, T.nrb, rb, g);
    }
    const int HR = (int)tile_lds_doubles(T, false);
    double *rows = lds;
    double *rc = lds + HR;
    const int64_t i0 = rb * T.H;
    const int64_t nloc = (i0 + T.H + 1 <= P.n) ? T.H + 1 : P.n - i0;   // rows incl. the halo
    const int64_t G = T.ngroups;
    double rr[1] = {0.0};
    if constexpr (FUSE) {
        if (ITER) {
            // the slice's loads RR at a time, all in flight (a load-then-add
            // loop waited out one memory latency per element, at the start of
            // every workgroup); same left-to-right order, padding adds +0
            constexpr int RR = 4;
            const int64_t ns = T.nrb * G, sl = rb * G + g;
            const bool cut = FUSE == 2 && P.rr_hi > P.rr_lo;
            int64_t lo = cut ? P.rr_lo : 0, span = (cut ? P.rr_hi : P.m) - lo;
            int64_t q0 = lo + sl * span / ns, q1 = lo + (sl + 1) * span / ns;
            if (gsel >= 0) {
                // this part's link range, cut to the rank's slice, over the row blocks
                const int64_t a = T.group_col[g] > lo ? T.group_col[g] : lo;
                const int64_t b = T.group_col[g + 1] < lo + span ? T.group_col[g + 1] : lo + span;
                const int64_t w = b > a ? b - a : 0;
                q0 = a + rb * w / T.nrb;
                q1 = a + (rb + 1) * w / T.nrb;
            }
            for (int64_t i0 = q0 + threadIdx.x; i0 < q1; i0 += RR * (int64_t)blockDim.x) {
                double v[RR];
#pragma unroll
                for (int q = 0; q < RR; ++q) {
                    const int64_t i = i0 + (int64_t)q * blockDim.x;
                    v[q] = (i < q1) ? r_load(P, i) : 0.0;
                }
#pragma unroll
                for (int q = 0; q < RR; ++q) rr[0] += v[q] * v[q];
            }
        }
    }
    for (int i = threadIdx.x; i < HR; i += blockDim.x) {
        rows[i] = 0.0;
        if (MODE == 2) rc[i] = (i < nloc) ? colv_t<CV>(P, i0 + i) : 0.0;
    }
    __syncthreads();
    if (P.r_fx > 0.0)
        tile_walk_any<(MODE == 3 ? 0 : MODE), false, true>(T, rb, g, P.r, rows, rc, 1.0,
                                                            1.0 / P.r_fx);
    else
        tile_walk_any<(MODE == 3 ? 0 : MODE)>(T, rb, g, P.r, rows, rc);
    __syncthreads();
    // wpart's tail: one slot per (group, row block) for the slices' r^2 sums
    double *rrp = P.wpart + G * T.nrb * (T.H + 1);
    if (FUSE && ITER && G > 1) {
        block_sum<1>(rr, red);
        if (threadIdx.x == 0)
            __hip_atomic_store(&rrp[g * T.nrb + rb], rr[0], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    bool fin = true;
    // dealt image, one group (MODE 3): w_i = colv_i * (sum of r over row i),
    // one product per row (the sums' order is not fixed anyway), formed in the
    // epilogue below; several groups: by the finishing workgroup
    const bool scale_epi = MODE == 3 && G == 1;
    if (G > 1 && gsel >= 0) {
        // the part pipeline: fixed roles (see above)
        if (gsel < G - 1) {
            double *wp = P.wpart + (g * T.nrb + rb) * (T.H + 1);
            for (int64_t i = threadIdx.x; i < nloc; i += blockDim.x) wp[i] = rows[i];
            return;
        }
        for (int64_t i = threadIdx.x; i < nloc; i += blockDim.x) {
            double o = 0.0;
            for (int64_t c = 0; c < G - 1; ++c)
                o += __hip_atomic_load(&P.wpart[(c * T.nrb + rb) * (T.H + 1) + i], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            o += rows[i];
            rows[i] = (MODE == 3) ? colv_t<CV>(P, i0 + i) * o : o;
        }
        __syncthreads();
    } else if (G > 1) {
        double *wp = P.wpart + (g * T.nrb + rb) * (T.H + 1);
        for (int64_t i = threadIdx.x; i < nloc; i += blockDim.x)
            __hip_atomic_store(&wp[i], rows[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned prev =
                __hip_atomic_fetch_add(&tk2rb[rb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            row_last = (prev == (unsigned)G - 1);
            if (row_last)
                __hip_atomic_store(&tk2rb[rb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        fin = row_last;
        if (fin) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int64_t i = threadIdx.x; i < nloc; i += blockDim.x) {
                double o = 0.0;
                for (int64_t c = 0; c < G; ++c)
                    o += __hip_atomic_load(&P.wpart[(c * T.nrb + rb) * (T.H + 1) + i],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rows[i] = (MODE == 3) ? colv_t<CV>(P, i0 + i) * o : o;
            }
            __syncthreads();
        }
    }
    constexpr int NS = FUSE ? 5 : 4;
    double sums[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) sums[q] = 0.0;
    if (fin && BSLS_TILE_KO != 4) {   // (KO 4: no epilogue -- timing builds only)
        // K2E rows per thread per batch: every z index, then every operand of
        // the batch in flight at once (two round trips per batch instead of
        // two per row: C5's 19 rows per thread made the epilogue ~90 us)
        const int64_t iend = (nloc < T.H) ? nloc : T.H;
        constexpr int K2E = BSLS_K2E;
        for (int64_t ib = threadIdx.x; ib < iend; ib += K2E * blockDim.x) {
            int32_t jq[K2E];
            double ca[K2E], cb[K2E], gq[K2E], dq[K2E];
#pragma unroll
            for (int q = 0; q < K2E; ++q) {
                const int64_t i = ib + (int64_t)q * blockDim.x;
                // (j < 0: a block's last x entry, also the matrix's last row)
                jq[q] = (i < iend) ? P.xz[i0 + i] : -1;
                ca[q] = cb[q] = 1.0;
                if (scale_epi && i < iend) {
                    ca[q] = colv_t<CV>(P, i0 + i);
                    cb[q] = (i + 1 < nloc) ? colv_t<CV>(P, i0 + i + 1) : 0.0;
                }
            }
#pragma unroll
            for (int q = 0; q < K2E; ++q) {
                gq[q] = dq[q] = 0.0;
                if (ITER && jq[q] >= 0) {
                    gq[q] = gp[jq[q]];
                    if (dzv) dq[q] = dzv[jq[q]];
                }
            }
#pragma unroll
            for (int q = 0; q < K2E; ++q) {
                const int64_t i = ib + (int64_t)q * blockDim.x;
                const int32_t j = jq[q];
                if (j < 0) continue;
                const double wa = scale_epi ? ca[q] * rows[i] : rows[i];
                const double wb = scale_epi ? cb[q] * rows[i + 1] : rows[i + 1];
                const double gv = wa - wb;
                gout[j] = gv;
                if (ITER) {
                    const double dg = gv - gq[q];
                    const double dz = dq[q];
                    sums[0] += dg;
                    sums[1] += dz * dg;
                    sums[2] += dg * dg;
                    sums[3] += gv * gv;
                }
            }
        }
    }
    if (!ITER || !fin) return;
    if constexpr (FUSE) {
        if (G == 1) {
            sums[4] = rr[0];
        } else if (threadIdx.x == 0) {
            // (the group partials' hand-off above orders these slots too)
            double o = 0.0;
            for (int64_t c = 0; c < G; ++c)
                o += __hip_atomic_load(&rrp[c * T.nrb + rb], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            sums[4] = o;
        }
    }
    block_sum<NS>(sums, red);
    double tot[NS];
    // one slot per row block, summed in row-block order: with several groups
    // the finishing workgroup of a block varies from run to run, so its
    // blockIdx must not decide where the block's sums enter the reduction
    const bool last = (G == 1) ? last_block_sum<NS>(sums, part, ticket, tot, red)
                               : last_of_sum<NS>(sums, part, (unsigned)rb, (unsigned)T.nrb, ticket,
                                                 tot, red);
    if (last && threadIdx.x == 0) {
        if constexpr (FUSE == 1) {
            bb_record_f(P, iter - 1, tot[4], iter - 1 > 0);
            // stopped at iter - 1: keep that iteration's sums (what the
            // unfused schedule leaves in scal); g[iter & 1], written above,
            // is the other buffer -- the stopping iterate's g is untouched
            if (P.scal[BSLS_S_STOP] != 0.0) {
                // (the sums all-reduced after this launch: as k2_stopped_sums)
                if (P.shard_role == 2)
                    for (int q = 0; q < 4; ++q) P.scal[BSLS_S_SUMDG + q] = 0.0;
                return;
            }
        }
        if constexpr (FUSE == 2) {
            double *sc = P.scal;
            for (int q = 0; q < 4; ++q) sc[BSLS_S_PSUMDG + q] = sc[BSLS_S_SUMDG + q];
            sc[BSLS_S_RR] = tot[4];
        }
        P.scal[BSLS_S_SUMDG] = tot[0];
        P.scal[BSLS_S_DZDG] = tot[1];
        P.scal[BSLS_S_DGDG] = tot[2];
        P.scal[BSLS_S_GG] = tot[3];
    }
}

// Stage 12 (the sliced schedule, after the all-reduce of scal[SUMDG..RR]):
// f(iter - 1) from the summed ||r||^2 and the stopping test of iter - 1 on
// its own g.g and dg.dg (kept by stage 10 in scal[PSUMDG..PGG]); on a stop the
// scal sums go back to that iteration's, as the unfused schedule leaves them.
__global__ void bb_shard_record(bsls_bb_problem P, int64_t iter) {
    if (threadIdx.x != 0) return;
    double *s = P.scal;
    const int64_t it = iter - 1;
    if (it > 0 && s[BSLS_S_STOP] != 0.0) return;
    const double rr = s[BSLS_S_RR];
    const double nr = sqrt(rr);
    const double fx = 0.5 * (nr * nr);      // 0.5 * la.norm(r)**2, main.py:53
    s[BSLS_S_FX] = fx;
    if (it <= 0) return;
    s[BSLS_S_ITER] = (double)it;
    s[BSLS_S_ZBUF] = (double)(it & 1);
    const int reason = bb_stop_reason(P, it, fx, s[BSLS_S_PGG], s[BSLS_S_PDGDG]);
    if (reason) {
        s[BSLS_S_STOP] = (double)reason;
        for (int q = 0; q < 4; ++q) s[BSLS_S_SUMDG + q] = s[BSLS_S_PSUMDG + q];
    }
}

// Multi-GPU stage 2: r (already all-reduced) += target, ||r||^2, stop test.
__global__ __launch_bounds__(256) void bb_r_finish(bsls_bb_problem P, int64_t iter, double *part,
                                                   unsigned *ticket, int add_target) {
    __shared__ double red[4];
    if (iter > 0 && P.scal[BSLS_S_STOP] != 0.0) return;
    // grid-stride over at most R_FINISH_GRID workgroups (the launch below):
    // one workgroup per 256 rows made 3.9k ticket arrivals at m = 1M, ~20 us
    // for 24 MB in the 8-way rehearsal
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double sq[1] = {0.0};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P.m; i += gs) {
        double o = r_load(P, i);
        if (add_target) {
            o += P.target[i];
            P.r[i] = (P.r_fx > 0.0) ? r_fx_of(P, o) : o;
        }
        sq[0] += o * o;
    }
    block_sum<1>(sq, red);
    double tot[1];
    if (last_block_sum<1>(sq, part, ticket, tot, red) && threadIdx.x == 0)
        bb_record_f(P, iter, tot[0], iter > 0);
}
constexpr int R_FINISH_GRID = 512;

// K2: g = N'(A' r); with ITER also dg = g - g_prev and the BB sums.  The
// workgroup's 16 panels (x-rows) are summed over every chunk of r; then lane
// position p of a panel has w_i in acc[p] and w_{i+1} in acc[p + 1] (the halo
// row), so N'w = w_i - w_{i+1} needs no exchange.  The column scales are
// loaded before the chunk loop; the epilogue's z indices and operands after
// it (the walk holds 122 of the 128 VGPRs; loading the indices early measured
// no faster).  The ITER epilogue reads g_prev and dz = z - z_prev (K3 wrote
// dz from the z's it holds, bit-identical to the subtraction here): 15.2 MB
// that no walk overlaps, where z and z_prev were 22.8 MB.
template <int MODE, bool ITER, int FUSE = 0>
__global__ __launch_bounds__(1024) void bb_k2(bsls_bb_problem P, const double *__restrict__ dzv,
                                              const double *__restrict__ gp,
                                              double *__restrict__ gout, double *part,
                                              unsigned *ticket, int64_t iter) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (ITER && P.scal[BSLS_S_STOP] != 0.0) {
        k2_stopped_sums<FUSE>(P);
        return;
    }
    const bsls_panels &M = P.AT;
    const int wv = threadIdx.x / WAVE, lane = lane_id();
    const int64_t panel = (int64_t)blockIdx.x * PANEL_WAVES + wv;
    const int64_t i0 = panel * M.prow;
    const bool live = panel < M.npanels;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    double sc[4] = {0.0, 0.0, 0.0, 0.0};
    if (MODE == 2) {
        // unconditional loads at clamped rows (all in flight together)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = i0 + 64 * q + lane;        // halo row included
            const bool ok = live && 64 * q + lane <= M.prow && i < P.n;
            const double v = colv_at(P, ok ? i : 0);
            sc[q] = ok ? v : 0.0;
        }
    }
    panel_chunks<MODE>(M, blockIdx.x, wv, 0, M.nchunks, P.r, lds, s, sc);
    // w_{i+1}: the next lane, or lane 0 of the next slice (the halo row is
    // row prow of the panel)
    double nx[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double dn = __shfl_down(s[q], 1, WAVE);
        const double wrap = (q < 3) ? __shfl(s[q < 3 ? q + 1 : q], 0, WAVE) : 0.0;
        nx[q] = (lane < 63) ? dn : wrap;
    }
    __syncthreads();   // the chunk table becomes the reduction scratch below
    constexpr int NS = FUSE ? 5 : 4;
    double sums[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) sums[q] = 0.0;
    // epilogue operands: unconditional loads at clamped indices, all in flight
    int32_t j[4];
    double gpj[4], dzj[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int pos = 64 * q + lane;
        const int64_t i = i0 + pos;
        const bool ok = live && pos < M.prow && i < P.n;
        const int32_t jj = P.xz[ok ? i : 0];
        j[q] = ok ? jj : -1;
    }
    if (ITER) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int32_t jc = j[q] >= 0 ? j[q] : 0;
            gpj[q] = gp[jc];
            dzj[q] = dzv ? dzv[jc] : 0.0;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (j[q] >= 0) {
            const double g = s[q] - nx[q];
            gout[j[q]] = g;
            if (ITER) {
                const double dg = g - gpj[q];
                const double dz = dzj[q];
                sums[0] += dg;
                sums[1] += dz * dg;
                sums[2] += dg * dg;
                sums[3] += g * g;
            }
        }
    }
    if (!ITER) return;
    if constexpr (FUSE) {   // stage 8 / 10: this workgroup's slice of ||r||^2 (see bb_k2t)
        const bool cut = FUSE == 2 && P.rr_hi > P.rr_lo;
        const int64_t lo = cut ? P.rr_lo : 0, span = (cut ? P.rr_hi : P.m) - lo;
        const int64_t q0 = lo + (int64_t)blockIdx.x * span / gridDim.x;
        const int64_t q1 = lo + ((int64_t)blockIdx.x + 1) * span / gridDim.x;
        for (int64_t i = q0 + threadIdx.x; i < q1; i += blockDim.x) {
            const double v = P.r[i];
            sums[4] += v * v;
        }
    }
    block_sum<NS>(sums, lds);
    double tot[NS];
    if (last_block_sum<NS>(sums, part, ticket, tot, lds) && threadIdx.x == 0) {
        if constexpr (FUSE == 1) {
            bb_record_f(P, iter - 1, tot[4], iter - 1 > 0);
            if (P.scal[BSLS_S_STOP] != 0.0) {
                // (the sums all-reduced after this launch: as k2_stopped_sums)
                if (P.shard_role == 2)
                    for (int q = 0; q < 4; ++q) P.scal[BSLS_S_SUMDG + q] = 0.0;
                return;
            }   // as bb_k2t
        }
        if constexpr (FUSE == 2) {
            double *sc = P.scal;
            for (int q = 0; q < 4; ++q) sc[BSLS_S_PSUMDG + q] = sc[BSLS_S_SUMDG + q];
            sc[BSLS_S_RR] = tot[4];
        }
        P.scal[BSLS_S_SUMDG] = tot[0];
        P.scal[BSLS_S_DZDG] = tot[1];
        P.scal[BSLS_S_DGDG] = tot[2];
        P.scal[BSLS_S_GG] = tot[3];
    }
}

// x entry i of N z; for a scaled incidence K1 gathers colv[i] * x_i instead,
// the product SciPy's csr_matvec forms for every entry of column i.
__device__ __forceinline__ void x_put(const bsls_bb_problem &P, int64_t i, double v) {
    P.x[i] = P.colv ? colv_at(P, i) * v : v;
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
// sc = scal[STOP], scal[SUMDG], scal[DZDG], scal[DGDG], loaded by the caller
// together with its other first loads (one round trip, not three)
__device__ __forceinline__ bool bb_step_t(const bsls_bb_problem &P, int64_t iter,
                                          const double (&sc)[4], double &t) {
    double *s = P.scal;
    if (sc[0] != 0.0) return false;
    if (P.early_exit && sc[1] == 0.0) {  // BB.py:22
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            s[BSLS_S_STOP] = (double)BSLS_STOP_NOCHANGE;
            s[BSLS_S_ITER] = (double)iter;
            s[BSLS_S_ZBUF] = (double)((iter - 1) & 1);
        }
        return false;
    }
    t = sc[2] / sc[3];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s[BSLS_S_T] = t;
        if (fabs(t) <= 1e-10 || fabs(t) > 1e10) s[BSLS_S_WARN] += 1.0;
    }
    return true;
}

// 8-B write-through (sc1) store through a buffer resource: the line leaves L2
// at once instead of as a dirty line at the kernel's end (as proj.hip's
// store-out).  Lanes whose offset is past `bytes` are dropped by the hardware.
__device__ __forceinline__ void wt_store_f64(const __amdgpu_buffer_rsrc_t &rs, int off,
                                             double v) {
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(HIP_vector_type<unsigned, 2>::Native_vec_, v), rs, off, 0, 16);
}

#ifndef BSLS_K3_SGPRS
#define BSLS_K3_SGPRS 80
#endif
#ifndef BSLS_DZ_PLAIN
#define BSLS_DZ_PLAIN 0   // 1: dz through an ordinary store (A/B variant)
#endif

// Each wave takes K3_PPW packs (w, w + W, ...; W = waves in the grid) and
// issues every load of all of them -- metadata, then z, g and the column
// scales -- before the first PAVA.  MERGE (K3_PPW = 2): the two packs' PAVA
// share the wave after their first passes (pava_v1_wave_pair).
// (at most 80 SGPRs: 256-thread blocks are admitted 8 per CU only up to 80,
// MI355X_MICROARCH.md "Residency"; the merged form otherwise takes 83 and 7)
template <int K3_PPW, bool MERGE, int CV = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(BSLS_K3_SGPRS)))
void bb_k3(bsls_bb_problem P, int64_t iter,
                                             const double *__restrict__ zc,
                                             const double *__restrict__ g,
                                             double *__restrict__ zn,
                                             double *__restrict__ dzo,
                                             int32_t *__restrict__ wsc, int rec,
                                             uint64_t *__restrict__ hd, int kinit) {
    const double sc[4] = {P.scal[BSLS_S_STOP], P.scal[BSLS_S_SUMDG], P.scal[BSLS_S_DZDG],
                          P.scal[BSLS_S_DGDG]};
    // kinit (stage 15): the next K1's r initialisation folded in (its atomic
    // group sums add into r): r = target on the shard_role 1 rank, 0 on the
    // others; once stopped, role 1 keeps its r and the others write 0 -- as
    // bb_k1_init, one launch fewer
    auto init_r = [&](bool stopped) {
        const int64_t gs = (int64_t)gridDim.x * blockDim.x;
        const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (stopped) {
            k1_stopped_rows(P, 0, P.m, t0, gs);
            return;
        }
        const bool add = P.shard_role == 1;
        for (int64_t row = t0; row < P.m; row += gs) {
            const double v = add ? P.target[row] : 0.0;
            P.r[row] = (P.r_fx > 0.0) ? r_fx_of(P, v) : v;
        }
    };
    // rec (stage 13, the sliced sharded schedule): stage 12 folded in -- f and
    // the stopping test of iter - 1 from the all-reduced scal[RR] and the kept
    // scal[PGG] / scal[PDGDG], decided alike by every workgroup (the same
    // inputs), recorded by workgroup 0; on a stop every workgroup returns
    if (rec && !(iter - 1 > 0 && sc[0] != 0.0)) {
        double *s = P.scal;
        const int64_t it = iter - 1;
        const double nr = sqrt(s[BSLS_S_RR]);
        const double fx = 0.5 * (nr * nr);
        const int reason = it > 0 ? bb_stop_reason(P, it, fx, s[BSLS_S_PGG], s[BSLS_S_PDGDG]) : 0;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            s[BSLS_S_FX] = fx;
            if (it > 0) {
                s[BSLS_S_ITER] = (double)it;
                s[BSLS_S_ZBUF] = (double)(it & 1);
            }
            if (reason) {
                s[BSLS_S_STOP] = (double)reason;
                for (int q = 0; q < 4; ++q) s[BSLS_S_SUMDG + q] = s[BSLS_S_PSUMDG + q];
            }
        }
        if (reason) {
            if (kinit) init_r(true);
            return;
        }
    }
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t w0 = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wv);   // wave-uniform
    __shared__ double pv_y[4][64];
    __shared__ int pv_p[4][128];
    __shared__ int pv_c[4][65];
    int64_t z0[K3_PPW], b0[K3_PPW];
    int L[K3_PPW];
    uint64_t B[K3_PPW], H[K3_PPW];
#pragma unroll
    for (int q = 0; q < K3_PPW; ++q) {
        // unconditional loads at a clamped index (straight-line, one round trip)
        const int64_t pk = w0 + q * nw;
        const int64_t pc = pk < P.npacks ? pk : P.npacks - 1;
        z0[q] = P.pk_z0[pc];
        b0[q] = P.pk_b0[pc];
        L[q] = pk < P.npacks ? P.pk_len[pc] : 0;
        B[q] = (uint64_t)P.pk_mask[pc];
        H[q] = hd ? hd[pc] : 0ull;
    }
    double zv[K3_PPW], gv[K3_PPW], cv[K3_PPW], cv2[K3_PPW];
#pragma unroll
    for (int q = 0; q < K3_PPW; ++q) {
        const bool act = l < L[q] && L[q] <= WAVE;
        const bool bend = (l == L[q] - 1) || (l < 63 && ((B[q] >> (l + 1)) & 1ull));
        const int64_t xi = z0[q] + l + b0[q] + __popcll(B[q] & mask_le(l)) - 1;
        cv[q] = cv2[q] = 1.0;
        if (P.colv) {
            // the column scales of this lane's x entries, loaded before the
            // PAVA so their round trip overlaps it (x_put's products)
            cv[q] = act ? colv_t<CV>(P, xi) : 1.0;
            cv2[q] = (act && bend) ? colv_t<CV>(P, xi + 1) : 1.0;
        }
        zv[q] = act ? zc[z0[q] + l] : 0.0;
        gv[q] = act ? g[z0[q] + l] : 0.0;
    }
    double t;
    const bool go = bb_step_t(P, iter, sc, t);
    if (kinit) init_r(!go);
    if (!go) return;
    double yv[K3_PPW];
#pragma unroll
    for (int q = 0; q < K3_PPW; ++q)   // x_next = x - t g (BB.py:29)
        yv[q] = (l < L[q] && L[q] <= WAVE) ? zv[q] - t * gv[q] : 0.0;
    if (BSLS_K3_KO != 1) {
        // warm start: the last run partition of each pack, tested first
        // (pava_warm); a pack that passes needs no reference pass
        // (BSLS_K3_REPAIR, the default: a partition that fails is repaired
        // -- its unsplittable runs kept pooled -- and the reference passes
        // continue from it, pava_warm_repair)
        bool need[K3_PPW], store[K3_PPW];
        uint64_t Hn[K3_PPW];
#pragma unroll
        for (int q = 0; q < K3_PPW; ++q) {
            need[q] = L[q] > 0 && L[q] <= WAVE;
            store[q] = need[q];
            if (hd && need[q] && (H[q] & B[q]) == B[q] && (H[q] & ~mask_lt(L[q])) == 0ull) {
#if BSLS_K3_REPAIR
                store[q] = pava_warm_repair(yv[q], L[q], B[q], H[q], pv_y[wv], pv_p[wv],
                                            pv_c[wv], &Hn[q]);
                need[q] = false;
#else
                need[q] = store[q] = !pava_warm(yv[q], L[q], B[q], H[q]);
#endif
            }
        }
        if (MERGE && K3_PPW == 2 && need[0] && need[K3_PPW - 1]) {
            pava_v1_wave_pair(yv[0], L[0], B[0], yv[K3_PPW - 1], L[K3_PPW - 1], B[K3_PPW - 1],
                              pv_y[wv], pv_p[wv], pv_c[wv], &Hn[0], &Hn[K3_PPW - 1]);
        } else {
#pragma unroll
            for (int q = 0; q < K3_PPW; ++q)
                if (need[q])
                    pava_v1_wave_c(yv[q], L[q], B[q], pv_y[wv], pv_p[wv], pv_c[wv], &Hn[q]);
        }
        if (hd) {
#pragma unroll
            for (int q = 0; q < K3_PPW; ++q)   // the new partition for the next call
                if (store[q] && l == 0) hd[w0 + q * nw] = Hn[q];
        }
    }
#pragma unroll
    for (int q = 0; q < K3_PPW; ++q) {
        if (L[q] == 0) break;
        if (L[q] <= WAVE) {
            const bool act = l < L[q];
            const bool bstart = (B[q] >> l) & 1ull;
            const int bl = __popcll(B[q] & mask_le(l)) - 1;   // block within the pack
            const bool bend = (l == L[q] - 1) || (l < 63 && ((B[q] >> (l + 1)) & 1ull));
            const double v = clip01(yv[q]);
            const double vprev = shfl_d(v, l > 0 ? l - 1 : 0);
            const int nb = __popcll(B[q]);
            const __amdgpu_buffer_rsrc_t rz =
                __builtin_amdgcn_make_buffer_rsrc(zn + z0[q], 0, L[q] * 8, 0x00020000);
            const __amdgpu_buffer_rsrc_t rd =
                __builtin_amdgcn_make_buffer_rsrc(dzo + z0[q], 0, L[q] * 8, 0x00020000);
            const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
                P.x + z0[q] + b0[q], 0, (L[q] + nb) * 8, 0x00020000);
            if (act) {
                wt_store_f64(rz, l * 8, v);
#if BSLS_DZ_PLAIN
                dzo[z0[q] + l] = v - zv[q];
#else
                wt_store_f64(rd, l * 8, v - zv[q]);   // next K2's z - z_prev
#endif
                const double d = v - (bstart ? 0.0 : vprev);
                const int xo = (l + bl) * 8;
                wt_store_f64(rx, xo, P.colv ? cv[q] * d : d);
                if (bend) wt_store_f64(rx, xo + 8, P.colv ? cv2[q] * (0.0 - v) : (0.0 - v));
            }
        } else if (!P.long_packs && l == 0) {
            // one block longer than a wave: serial PAVA in global memory
            // (with P.long_packs bb_k3_long takes it, a workgroup per block)
            const int64_t xs = P.xstarts[b0[q]];
            for (int64_t j = z0[q]; j < z0[q] + L[q]; ++j) {
                zn[j] = zc[j] - t * g[j];
                wsc[j] = 1;
            }
            pava_v1(zn, wsc, z0[q], z0[q] + L[q], 1);
            double prev = 0.0;
            int64_t xo = xs;
            for (int64_t j = z0[q]; j < z0[q] + L[q]; ++j) {
                const double v = clip01(zn[j]);
                zn[j] = v;
                dzo[j] = v - zc[j];
                x_put(P, xo++, v - prev);
                prev = v;
            }
            x_put(P, xo, 0.0 - prev);
        }
    }
}

// K3 for one z-block longer than a wave, one 1024-thread workgroup per block
// (after bb_k3 in the same stream): z - t g, PAVA v1 by the whole workgroup
// (pava_long.hpp, bit-identical), clip, dz and x as bb_k3's serial path.
// t as bb_step_t, without its writes (bb_k3 made them).
__global__ __launch_bounds__(LONG_T) void bb_k3_long(bsls_bb_problem P, int64_t iter,
                                                     const double *__restrict__ zc,
                                                     const double *__restrict__ g,
                                                     double *__restrict__ zn,
                                                     double *__restrict__ dzo) {
    __shared__ int64_t sh[LONG_T / 64 + 1];
    __shared__ int flag;
    const double *s = P.scal;
    if (s[BSLS_S_STOP] != 0.0) return;
    if (P.early_exit && s[BSLS_S_SUMDG] == 0.0) return;
    const double t = s[BSLS_S_DZDG] / s[BSLS_S_DGDG];
    const int64_t q = P.long_packs[blockIdx.x];
    const int64_t z0 = P.pk_z0[q], b0 = P.pk_b0[q], L = P.pk_len[q];
    const int64_t off = P.long_off[blockIdx.x], tot = P.long_off[P.nlong];
    double *Y0 = (double *)P.long_scratch + off;
    double *Y1 = (double *)P.long_scratch + tot + off;
    int32_t *W = (int32_t *)((double *)P.long_scratch + 2 * tot);
    int32_t *W0 = W + off, *W1 = W + tot + off, *CH = W + 2 * tot + blockIdx.x + off;
    for (int64_t j = threadIdx.x; j < L; j += LONG_T) zn[z0 + j] = zc[z0 + j] - t * g[z0 + j];
    __syncthreads();
    pava_v1_long(zn + z0, L, Y0, Y1, W0, W1, CH, sh, &flag);
    for (int64_t j = threadIdx.x; j < L; j += LONG_T) {
        const double v = clip01(zn[z0 + j]);
        zn[z0 + j] = v;
        dzo[z0 + j] = v - zc[z0 + j];
    }
    __syncthreads();
    const int64_t xs = P.xstarts[b0];
    for (int64_t j = threadIdx.x; j <= L; j += LONG_T) {
        const double v = (j < L) ? zn[z0 + j] : 0.0;
        const double prev = (j > 0) ? zn[z0 + j - 1] : 0.0;
        x_put(P, xs + j, v - prev);
    }
}

// Prologue helpers (BB.py:14-15: x_prev = x + 1); bb_z2x writes N z.
__global__ __launch_bounds__(256) void bb_plus_one(const double *__restrict__ a,
                                                   double *__restrict__ o,
                                                   double *__restrict__ dz, int64_t nz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nz) {
        const double v = a[i], w = v + 1;
        o[i] = w;
        dz[i] = v - w;   // iteration 1's z - z_prev
    }
}

// one thread per x entry (coalesced; C5 418 -> ~20 us against a thread per
// block): xz[i] is entry i's z index, -1 for a block's last entry (blocks
// have >= 2 routes); the same differences K3 forms (v - prev, prev = 0.0 at a
// block's first entry, 0.0 - z_last at its last)
__global__ __launch_bounds__(256) void bb_z2x(bsls_bb_problem P, const double *__restrict__ z) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const int32_t j = P.xz[i];
    const int32_t jp = (i > 0) ? P.xz[i - 1] : -1;
    double v;
    if (j >= 0) v = z[j] - (jp >= 0 ? z[jp] : 0.0);
    else v = 0.0 - z[jp];
    x_put(P, i, v);
}

// Up to ~160 KB of dynamic LDS (panel_lds_bytes): opt in once per kernel instance.
constexpr int PANEL_LDS_MAX = 163840 - 512;
template <typename K>
static void allow_lds(K kernel) {
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  PANEL_LDS_MAX);
        done = true;
    }
}

// K1's row blocks: panels 16 panels each, tiles H rows each
static int64_t k1_row_blocks(const bsls_bb_problem &P) {
    return P.At.ent ? P.At.nrb : (P.A.npanels + PANEL_WAVES - 1) / PANEL_WAVES;
}

// row blocks [rb0, rb1) of K1 (the whole matrix unless a multi-GPU driver
// all-reduces r part by part behind it); REDUCE needs the whole matrix
template <int MODE, bool ADD, bool REDUCE, bool ITER>
static void launch_k1_mode(const bsls_bb_problem &P, int64_t iter, const BBWork &w,
                           hipStream_t st, int64_t rb0, int64_t rb1) {
    allow_lds(bb_k1<MODE, ITER, ADD, REDUCE>);
    bb_k1<MODE, ITER, ADD, REDUCE><<<(int)(P.A.ngroups * (rb1 - rb0)), 1024, panel_lds_bytes(P.A),
                                     st>>>(P, iter, w.tkrb, w.p1, w.tk1, rb0);
}

// Several-group K1 without the partials: r initialised (bb_k1_init), every
// group's sums added by global f64 atomics, ||r||^2 and the stop test
// (REDUCE) by bb_r_finish.  The default on a column shard's partial residual
// (stage 1): the rehearsed 8-way C5 rank-0 iteration 162.6 -> 148.4 us -- no
// bb_k1_sum, and no 4 x 8 MB of partials through the Infinity Cache ahead of
// K2.  On one GPU it measured no faster (C3 83.0 / 85.7 us, C5 800 / 801: the
// ||r||^2 pass reads r again), and the atomics' varying order moves the exact
// zero sum(dg) exit of BB.py:22 (a tests/fast problem stopped at 967 instead
// of ~770), so one GPU keeps the group sums.  bsls_bb_problem.k1_atomic
// (the engine's BSLS_K1_ATOMIC, read once): 1 = never, 2 = wherever K1 has
// several groups, 0 = the default above.
static bool k1_atomic(const bsls_bb_problem &P, bool reduce) {
    if (P.k1_atomic) return P.k1_atomic == 2;
    return P.shard_role != 0 && !reduce;
}

// stage 15 / 14: the atomic K1's r initialisation done by the K3 before it
// (bb_k3 kinit) -- whole matrix only
static bool k1_init_folded(const bsls_bb_problem &P) {
    return P.At.ent && P.At.ngroups > 1 && k1_atomic(P, false);
}

template <int MODE, bool ADD, bool REDUCE, bool ITER>
static void launch_k1t_mode(const bsls_bb_problem &P, int64_t iter, const BBWork &w,
                            hipStream_t st, int64_t rb0, int64_t rb1, bool skip_init) {
    if (P.At.ngroups > 1 && k1_atomic(P, REDUCE)) {
        const int64_t r0 = rb0 * P.At.H, r1 = (rb1 * P.At.H < P.m) ? rb1 * P.At.H : P.m;
        const int gi = grid_for(r1 - r0, 256);
        // one row per thread (the grid-stride form at 1024 workgroups gave each
        // thread 4 rows at m = 1M; the rehearsed iteration measured the same
        // either way, 149.3-149.8 us)
        if (!skip_init)
            bb_k1_init<ITER, ADD><<<gi < 16384 ? gi : 16384, 256, 0, st>>>(P, r0, r1);
        allow_lds(bb_k1t<MODE, ITER, ADD, false, true>);
        bb_k1t<MODE, ITER, ADD, false, true><<<(int)((rb1 - rb0) * P.At.ngroups),
                                               BSLS_TILE_THREADS, tile_lds_doubles(P.At, false) * 8,
                                               st>>>(P, iter, w.tkrb, w.p1, w.tk1, rb0);
        if (REDUCE)
            bb_r_finish<<<(grid_for(P.m, 256) < R_FINISH_GRID ? grid_for(P.m, 256) : R_FINISH_GRID),
                          256, 0, st>>>(P, iter, w.pf, w.tkf, 0);
        return;
    }
    allow_lds(bb_k1t<MODE, ITER, ADD, REDUCE>);
    bb_k1t<MODE, ITER, ADD, REDUCE><<<(int)((rb1 - rb0) * P.At.ngroups), BSLS_TILE_THREADS,
                                      tile_lds_doubles(P.At, false) * 8, st>>>(P, iter, w.tkrb,
                                                                                w.p1, w.tk1, rb0);
    if (BSLS_K1_SPLIT && P.At.ngroups > 1) {
        const int64_t r0 = rb0 * P.At.H, r1 = (rb1 * P.At.H < P.m) ? rb1 * P.At.H : P.m;
        constexpr int K1_SUM_GRID = 1024;
        const int gk = grid_for(r1 - r0, 256);
        bb_k1_sum<ITER, ADD, REDUCE><<<(REDUCE && gk > K1_SUM_GRID) ? K1_SUM_GRID : gk, 256, 0, st>>>(
            P, iter, P.At.ngroups, r0, r1, w.pf, w.tkf);
    }
}

template <bool ADD, bool REDUCE, bool ITER>
static void launch_k1(const bsls_bb_problem &P, int64_t iter, const BBWork &w, hipStream_t st,
                      int64_t rb0 = 0, int64_t rb1 = -1, bool skip_init = false) {
    if (rb1 < 0) rb1 = k1_row_blocks(P);
    if (P.At.ent) {
        if (P.colv) launch_k1t_mode<0, ADD, REDUCE, ITER>(P, iter, w, st, rb0, rb1, skip_init);
        else launch_k1t_mode<1, ADD, REDUCE, ITER>(P, iter, w, st, rb0, rb1, skip_init);
    } else if (P.colv) {
        launch_k1_mode<0, ADD, REDUCE, ITER>(P, iter, w, st, rb0, rb1);
    } else {
        launch_k1_mode<1, ADD, REDUCE, ITER>(P, iter, w, st, rb0, rb1);
    }
}

// (dz: the vector the ITER sums dot with delta_g -- the workspace's z - z_prev
// unless given: the line search passes its direction d, with g_prev = 0)
template <int MODE, bool ITER, int FUSE>
static void launch_k2_mode(const bsls_bb_problem &P, const double *gp, double *gout,
                           const BBWork &w, hipStream_t st, int64_t iter, const double *dz) {
    allow_lds(bb_k2<MODE, ITER, FUSE>);
    bb_k2<MODE, ITER, FUSE><<<grid_for(P.AT.npanels, PANEL_WAVES), 1024, panel_lds_bytes(P.AT),
                              st>>>(P, dz, gp, gout, w.p2, w.tk2, iter);
}

template <int MODE, bool ITER, int FUSE, int CV>
static void launch_k2t_cv(const bsls_bb_problem &P, const double *gp, double *gout,
                          const BBWork &w, hipStream_t st, int64_t iter, const double *dz,
                          int gsel) {
    allow_lds(bb_k2t<MODE, ITER, FUSE, CV>);
    bb_k2t<MODE, ITER, FUSE, CV><<<(int)(gsel >= 0 ? P.ATt.nrb : P.ATt.nrb * P.ATt.ngroups),
                                   BSLS_TILE_THREADS, tile_lds_doubles(P.ATt, MODE == 2) * 8, st>>>(
        P, dz, gp, gout, w.p2, w.tk2, w.tk2rb, iter, gsel);
}

template <int MODE, bool ITER, int FUSE>
static void launch_k2t_mode(const bsls_bb_problem &P, const double *gp, double *gout,
                            const BBWork &w, hipStream_t st, int64_t iter, const double *dz,
                            int gsel) {
    if (MODE != 1 && P.colv_codec == 2)
        launch_k2t_cv<MODE, ITER, FUSE, 2>(P, gp, gout, w, st, iter, dz, gsel);
    else if (MODE != 1 && P.colv_codec == 1)
        launch_k2t_cv<MODE, ITER, FUSE, 1>(P, gp, gout, w, st, iter, dz, gsel);
    else launch_k2t_cv<MODE, ITER, FUSE, 0>(P, gp, gout, w, st, iter, dz, gsel);
}

template <bool ITER, int FUSE = 0>
static void launch_k2(const bsls_bb_problem &P, const double *gp, double *gout,
                      const BBWork &w, hipStream_t st, int64_t iter = 0,
                      const double *dz = nullptr, int gsel = -1) {
    if (!dz) dz = w.dz;
    if (P.ATt.ent) {
        if (!P.colv) launch_k2t_mode<1, ITER, FUSE>(P, gp, gout, w, st, iter, dz, gsel);
        else if (P.ATt.ngroups == 1 && P.ATt.layout == 0)
            launch_k2t_mode<2, ITER, FUSE>(P, gp, gout, w, st, iter, dz, gsel);
        else launch_k2t_mode<3, ITER, FUSE>(P, gp, gout, w, st, iter, dz, gsel);
    } else if (P.colv) {
        launch_k2_mode<2, ITER, FUSE>(P, gp, gout, w, st, iter, dz);
    } else {
        launch_k2_mode<1, ITER, FUSE>(P, gp, gout, w, st, iter, dz);
    }
}

// Two packs per wave sharing their passes after the first
// (pava_v1_wave_pair) pay where the grid runs many rounds of resident waves:
// C5 (172k packs) K3 153 -> 141 us; C3 (16.7k packs, two rounds of 8 waves
// per SIMD) 18.8 -> 20.6 us, the longer wave outlasting its rounds.  So from
// 64k packs (8 rounds); bsls_bb_problem.k3_merge (the engine's
// BSLS_K3_MERGE, read once) forces one (1) or two (2).
static bool k3_merge(const bsls_bb_problem &P) {
    return P.k3_merge ? P.k3_merge == 2 : P.npacks >= 65536;
}

template <int CV>
static void launch_k3_cv(const bsls_bb_problem &P, int64_t iter, const double *zc,
                         const double *g, double *zn, const BBWork &w, hipStream_t st, int rec,
                         int slot, int kinit) {
    // (bsls_bb_problem.pava_warm; a second set of masks for a second
    // projection whose inputs alternate with the first's)
    uint64_t *hd = P.pava_warm ? w.hd + (slot ? w.hd_stride : 0) : nullptr;
    if (k3_merge(P))
        bb_k3<2, true, CV><<<grid_for(P.npacks, 8), 256, 0, st>>>(P, iter, zc, g, zn, w.dz, w.wsc,
                                                                   rec, hd, kinit);
    else
        bb_k3<1, false, CV><<<grid_for(P.npacks, 4), 256, 0, st>>>(P, iter, zc, g, zn, w.dz,
                                                                    w.wsc, rec, hd, kinit);
}

static void launch_k3(const bsls_bb_problem &P, int64_t iter, const double *zc, const double *g,
                      double *zn, const BBWork &w, hipStream_t st, int rec = 0, int slot = 0,
                      int kinit = 0) {
    if (P.colv && P.colv_codec == 2) launch_k3_cv<2>(P, iter, zc, g, zn, w, st, rec, slot, kinit);
    else if (P.colv && P.colv_codec == 1)
        launch_k3_cv<1>(P, iter, zc, g, zn, w, st, rec, slot, kinit);
    else launch_k3_cv<0>(P, iter, zc, g, zn, w, st, rec, slot, kinit);
    if (P.long_packs && P.nlong > 0)
        bb_k3_long<<<(int)P.nlong, LONG_T, 0, st>>>(P, iter, zc, g, zn, w.dz);
}

static bool panels_ok(const bsls_panels &M, int64_t rows, int64_t cols, int64_t halo,
                      bool need_val) {
    if (M.rows != rows || M.cols != cols || M.halo != halo) return false;
    if (M.prow < 1 || M.prow + halo > 256 || M.npanels != (rows + M.prow - 1) / M.prow)
        return false;
    if (M.nchunks < 1 || M.ngroups < 1 || M.ngroups > M.nchunks) return false;
    if (M.tab_cap < 64 || M.tab_cap > BSLS_PANEL_CHUNK || panel_lds_bytes(M) > (size_t)PANEL_LDS_MAX)
        return false;
    if (!M.chunk_col || !M.group_chunk || !M.ent_off || !M.cnt_off || !M.seg_info || !M.cnt ||
        !M.ent)
        return false;
    return need_val ? M.val != nullptr : true;
}

static int check_problem(const bsls_bb_problem *p) {
    if (!p || p->m <= 0 || p->n <= 0 || p->nblocks <= 0 || p->nz != p->n - p->nblocks) return BSLS_E_ARG;
    if (p->shard_role < 0 || p->shard_role > 2) return BSLS_E_ARG;
    if (p->k1_atomic < 0 || p->k1_atomic > 2 || p->k3_merge < 0 || p->k3_merge > 2)
        return BSLS_E_ARG;
    // the fixed-point r: every writer of r is the atomic K1 (+ its init) and
    // every K2 reader the dealt walk
    if (!(p->r_fx >= 0.0) || p->r_fx > 1e300) return BSLS_E_ARG;
    if (p->r_fx > 0.0 && !(k1_init_folded(*p) && p->ATt.ent && (p->ATt.layout & 3) != 0))
        return BSLS_E_ARG;
    if (p->colv_codec < 0 || p->colv_codec > 2 || (p->colv_codec && (!p->colv_n || !p->colv)))
        return BSLS_E_ARG;
    // (sy_dr, dz . dg as ||r - r_prev||^2, retired in round 6: it moved where
    // the reference's exact-zero sum(delta_g) exit fires, BB.py:22)
    if (p->sy_dr != 0) return BSLS_E_ARG;
    const bool general = p->colv == nullptr;
    if (p->At.ent) {
        if (!tiles_valid(p->At, p->m, p->n, 0, general, false, PANEL_LDS_MAX)) return BSLS_E_ARG;
        if (p->At.ngroups > 1 && !p->rpart) return BSLS_E_ARG;
    } else if (!panels_ok(p->A, p->m, p->n, 0, general) || !p->rpart) {
        return BSLS_E_ARG;
    }
    if (p->ATt.ent) {
        if (!tiles_valid(p->ATt, p->n, p->m, 1, general,
                         !general && p->ATt.ngroups == 1 && p->ATt.layout == 0, PANEL_LDS_MAX))
            return BSLS_E_ARG;
        if (p->ATt.ngroups > 1 && !p->wpart) return BSLS_E_ARG;
    } else if (!panels_ok(p->AT, p->n, p->m, 1, general) || p->AT.ngroups != 1) {
        return BSLS_E_ARG;
    }
    if (p->work_bytes < bb_layout(nullptr, p->m, p->n, p->nz).bytes) return BSLS_E_WORKSPACE;
    if (!p->target || !p->xstarts || !p->zstarts || !p->xz) return BSLS_E_ARG;
    if (!p->pk_z0 || !p->pk_b0 || !p->pk_mask || !p->pk_len || p->npacks < 1) return BSLS_E_ARG;
    if (!p->z[0] || !p->z[1] || !p->g[0] || !p->g[1] || !p->x || !p->r || !p->scal || !p->work)
        return BSLS_E_ARG;
    if (p->long_packs && (p->nlong < 0 || (p->nlong > 0 && (!p->long_off || !p->long_scratch))))
        return BSLS_E_ARG;
    return BSLS_OK;
}

// ---- LBFGS.solve's weak Wolfe line search on the device -------------------------
// (python/LBFGS.py:9-53; include/bsls_hip.h bsls_lbfgs_ls_*).  One trial =
//   K3 on S1:  pt = clip01(PAVA(x - (-t) d)) = proj(x + t d) (the reference's
//              roundings: (-t) d = -(t d)), x_engine = colv N pt
//   K1 on S1:  r = A x + target, S1[FX] = f(pt)
//   armijo:    f(pt) >= fx + c1 t slope -> beta = t, t = (alpha + beta) / 2;
//              else open S2 for the curvature test
//   K2 on S2:  g(pt) = N'A'r -> gpt; the sums with g_prev = 0 and dz = d give
//              S2[DZDG] = d . g(pt)
//   curvature: d . g(pt) < c2 slope -> alpha = t, t = 2 alpha or (alpha +
//              beta) / 2; else accepted
// then the reference's two exits (|alpha - beta| <= 1e-14, ||t d|| <= 1e-8,
// the norm as |t| ||d||).  Every kernel of a trial is gated by the state, so
// the host enqueues trials in chunks and reads the state once per chunk.
// st[]: BSLS_LS_* slots.
__device__ __forceinline__ void ls_stop(double *st, double *S1, double *S2, double why) {
    st[BSLS_LS_STOP] = why;
    S1[BSLS_S_STOP] = 1.0;
    S2[BSLS_S_STOP] = 1.0;
}

// the exits after a new t (LBFGS.py:45-49), else the next trial's K3 step
__device__ __forceinline__ void ls_next(double *st, double *S1, double *S2, double tn) {
    st[BSLS_LS_T] = tn;
    if (fabs(st[BSLS_LS_LO] - st[BSLS_LS_HI]) <= 1e-14) ls_stop(st, S1, S2, BSLS_LS_BRACKET);
    else if (fabs(tn) * st[BSLS_LS_DNORM] <= 1e-8) ls_stop(st, S1, S2, BSLS_LS_SMALL);
    else S1[BSLS_S_DZDG] = -tn;
}

__global__ __launch_bounds__(256) void ls_begin_kernel(const double *__restrict__ d,
                                                       const double *__restrict__ gx, int64_t nz,
                                                       const double *fx, double *st,
                                                       double *S1, double *S2, double *part,
                                                       unsigned *tickets) {
    __shared__ double red[2 * 4];
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double v[2] = {0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nz; i += gs) {
        const double di = d[i];
        v[0] += di * gx[i];
        v[1] += di * di;
    }
    block_sum<2>(v, red);
    double tot[2];
    if (last_block_sum<2>(v, part, tickets, tot, red) && threadIdx.x == 0) {
        const double f0 = *fx;    // (fx may point into st: the last search's st[FT])
        for (int k = 0; k < BSLS_LS_COUNT; ++k) st[k] = 0.0;
        for (int k = 0; k < BSLS_S_COUNT; ++k) S1[k] = S2[k] = 0.0;
        st[BSLS_LS_T] = 1.0;
        st[BSLS_LS_HI] = INFINITY;
        st[BSLS_LS_SLOPE] = tot[0];
        st[BSLS_LS_DNORM] = sqrt(tot[1]);
        st[BSLS_LS_FX] = f0;
        S1[BSLS_S_SUMDG] = 1.0;      // K3's t = S1[DZDG] / S1[DGDG] = -t
        S1[BSLS_S_DZDG] = -1.0;
        S1[BSLS_S_DGDG] = 1.0;
        S2[BSLS_S_STOP] = 1.0;
    }
}

__global__ void ls_armijo_kernel(double *st, double *S1, double *S2, double c1) {
    if (threadIdx.x != 0 || st[BSLS_LS_STOP] != 0.0) return;
    const double t = st[BSLS_LS_T], ft = S1[BSLS_S_FX];
    st[BSLS_LS_NTRIAL] += 1.0;
    st[BSLS_LS_TLAST] = t;
    st[BSLS_LS_FT] = ft;
    if (ft >= st[BSLS_LS_FX] + c1 * t * st[BSLS_LS_SLOPE]) {   // Armijo violated (LBFGS.py:26)
        st[BSLS_LS_HI] = t;
        S2[BSLS_S_STOP] = 1.0;
        ls_next(st, S1, S2, 0.5 * (st[BSLS_LS_LO] + t));
    } else {
        S2[BSLS_S_STOP] = 0.0;     // the curvature test needs g(pt)
    }
}

__global__ void ls_curv_kernel(double *st, double *S1, double *S2, double c2) {
    if (threadIdx.x != 0 || st[BSLS_LS_STOP] != 0.0 || S2[BSLS_S_STOP] != 0.0) return;
    const double t = st[BSLS_LS_T];
    S2[BSLS_S_STOP] = 1.0;
    st[BSLS_LS_DGT] = S2[BSLS_S_DZDG];
    if (S2[BSLS_S_DZDG] < c2 * st[BSLS_LS_SLOPE]) {            // curvature violated (:33)
        st[BSLS_LS_LO] = t;
        const double hi = st[BSLS_LS_HI];
        ls_next(st, S1, S2, (hi == INFINITY) ? 2 * t : 0.5 * (t + hi));
    } else {
        ls_stop(st, S1, S2, BSLS_LS_ACCEPTED);                  // both conditions pass (:39)
    }
}

// after an accepted search: y = g(pt) - gx, s = t d (LBFGS.py:100-106, the
// same elementwise roundings), y.s and g(pt).g(pt); gated on the state
__global__ __launch_bounds__(256) void ls_finish_kernel(const double *__restrict__ d,
                                                        const double *__restrict__ gx,
                                                        const double *__restrict__ gpt, int64_t nz,
                                                        double *st, double *y_out, double *s_out,
                                                        double *part, unsigned *tickets) {
    __shared__ double red[2 * 4];
    if (st[BSLS_LS_STOP] != (double)BSLS_LS_ACCEPTED || st[BSLS_LS_DONE] != 0.0) return;
    const double t = st[BSLS_LS_T];
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double v[2] = {0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nz; i += gs) {
        const double gi = gpt[i];
        const double y = gi - gx[i], s = t * d[i];
        if (y_out) y_out[i] = y;
        if (s_out) s_out[i] = s;
        v[0] += y * s;
        v[1] += gi * gi;
    }
    block_sum<2>(v, red);
    double tot[2];
    if (last_block_sum<2>(v, part, tickets, tot, red) && threadIdx.x == 0) {
        st[BSLS_LS_YS] = tot[0];
        st[BSLS_LS_GG] = tot[1];
        st[BSLS_LS_DONE] = 1.0;
    }
}

// ---- DORE on the fused images (include/bsls_hip.h bsls_dore_iterate) --------
// Vector steps of python/DORE.py:31-80 with the reference's elementwise
// roundings; dot products as fixed-order block sums; every branch decided by
// the last block of a reduction and read by the kernels after it.

// Ax = linop(x), err = b - Ax; norm_change = ||x - x_prev||^2 (la.norm(.)**2:
// the square of the rooted sum) and the break test.  Ax is scale * r of this
// launch's K1 at iteration 0 (axs == nullptr); after that x is the previous
// iteration's x_select, whose linop the previous iteration already formed
// (axs: its Ax, = scale * r of K1 on the same x -- the reference recomputes
// it at DORE.py:33, here it is reused, one K1 and one z2x fewer per iteration)
__global__ __launch_bounds__(256) void dore_top(bsls_bb_problem P, bsls_dore_state D, int64_t it,
                                                const double *__restrict__ x,
                                                const double *__restrict__ xp,
                                                const double *__restrict__ axs) {
    __shared__ double red[4];
    if (D.S[BSLS_S_STOP] != 0.0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        D.S2[BSLS_S_STOP] = 1.0;     // the extrapolated path stays off unless dore_mid opens it
        D.dsc[BSLS_DORE_SEL] = 0.0;
    }
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < P.m; i += gs) {
        const double ax = axs ? axs[i] : P.r[i] * D.scale;
        D.err[i] = D.b[i] - ax;
    }
    double v[1] = {0.0};
    for (int64_t i = i0; i < P.nz; i += gs) {
        const double t = x[i] - xp[i];
        v[0] += t * t;
    }
    block_sum<1>(v, red);
    double tot[1];
    if (last_block_sum<1>(v, D.part, D.tickets, tot, red) && threadIdx.x == 0) {
        const double nr = sqrt(tot[0]);
        const double nc = nr * nr;
        D.dsc[BSLS_DORE_NC] = nc;
        if (it > 0 && nc <= D.eps) {
            D.S[BSLS_S_STOP] = 1.0;
            D.dsc[BSLS_DORE_STOPIT] = (double)it;
        }
    }
}

// Ax = linop(x_new) -> axo; err; ||err||^2; i > 2: dAx = Ax - Ax_prev, dp, dAx.err
__global__ __launch_bounds__(256) void dore_mid(bsls_bb_problem P, bsls_dore_state D, int64_t it,
                                                double *__restrict__ axo,
                                                const double *__restrict__ axp) {
    __shared__ double red[3 * 4];
    if (D.S[BSLS_S_STOP] != 0.0) return;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double v[3] = {0.0, 0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P.m; i += gs) {
        const double ax = P.r[i] * D.scale;
        axo[i] = ax;
        const double e = D.b[i] - ax;
        D.err[i] = e;
        v[0] += e * e;
        if (it > 2) {
            const double d = ax - axp[i];
            v[1] += d * d;
            v[2] += d * e;
        }
    }
    block_sum<3>(v, red);
    double tot[3];
    if (last_block_sum<3>(v, D.part, D.tickets, tot, red) && threadIdx.x == 0) {
        D.dsc[BSLS_DORE_EE] = tot[0];
        const bool ext = it > 2 && tot[1] > 0;
        if (ext) D.dsc[BSLS_DORE_A1] = tot[2] / tot[1];
        D.S2[BSLS_S_STOP] = ext ? 0.0 : 1.0;
    }
}

// first extrapolation: Ax_1 = (1 + a1) Ax - a1 Ax_prev, err_1 = b - Ax_1,
// dAx = Ax_1 - Ax_prev_prev (dp, dAx.err_1); x_1 = x_new + a1 (x_new - x) and
// x_1 - x_prev for the second; a2 and the K3 step t = -a2 into S2
__global__ __launch_bounds__(256) void dore_ext(bsls_bb_problem P, bsls_dore_state D,
                                                const double *__restrict__ ax,
                                                const double *__restrict__ axp,
                                                const double *__restrict__ axpp,
                                                const double *__restrict__ x,
                                                const double *__restrict__ xp,
                                                const double *__restrict__ xn) {
    __shared__ double red[2 * 4];
    if (D.S[BSLS_S_STOP] != 0.0 || D.S2[BSLS_S_STOP] != 0.0) return;
    const double a1 = D.dsc[BSLS_DORE_A1];
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double v[2] = {0.0, 0.0};
    for (int64_t i = i0; i < P.m; i += gs) {
        const double ax1 = (1 + a1) * ax[i] - a1 * axp[i];
        const double e1 = D.b[i] - ax1;
        const double d = ax1 - axpp[i];
        v[0] += d * d;
        v[1] += d * e1;
    }
    for (int64_t i = i0; i < P.nz; i += gs) {
        const double x1 = xn[i] + a1 * (xn[i] - x[i]);
        D.X1[i] = x1;
        D.D[i] = x1 - xp[i];
    }
    block_sum<2>(v, red);
    double tot[2];
    if (last_block_sum<2>(v, D.part, D.tickets, tot, red) && threadIdx.x == 0) {
        if (tot[0] > 0) {
            const double a2 = tot[1] / tot[0];
            D.dsc[BSLS_DORE_A2] = a2;
            D.S2[BSLS_S_SUMDG] = 1.0;
            D.S2[BSLS_S_DZDG] = -a2;    // K3: x_1 - (-a2) (x_1 - x_prev) = x_1 + a2 (...)
            D.S2[BSLS_S_DGDG] = 1.0;
        } else {
            D.S2[BSLS_S_STOP] = 1.0;
        }
    }
}

// Ax_2 = linop(x_2), err_2; keep x_2 when ||err_2||^2 / ||err||^2 < 1
__global__ __launch_bounds__(256) void dore_sel(bsls_bb_problem P, bsls_dore_state D) {
    __shared__ double red[4];
    if (D.S[BSLS_S_STOP] != 0.0 || D.S2[BSLS_S_STOP] != 0.0) return;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    double v[1] = {0.0};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P.m; i += gs) {
        const double ax2 = P.r[i] * D.scale;
        D.AX2[i] = ax2;
        const double e = D.b[i] - ax2;
        v[0] += e * e;
    }
    block_sum<1>(v, red);
    double tot[1];
    if (last_block_sum<1>(v, D.part, D.tickets, tot, red) && threadIdx.x == 0)
        D.dsc[BSLS_DORE_SEL] = (tot[0] / D.dsc[BSLS_DORE_EE] < 1) ? 1.0 : 0.0;
}

// x_select = x_2, Ax = Ax_2 when selected
__global__ __launch_bounds__(256) void dore_copy(bsls_bb_problem P, bsls_dore_state D,
                                                 double *__restrict__ xn,
                                                 double *__restrict__ axo) {
    if (D.S[BSLS_S_STOP] != 0.0 || D.S2[BSLS_S_STOP] != 0.0 || D.dsc[BSLS_DORE_SEL] == 0.0)
        return;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < P.nz; i += gs) xn[i] = D.X2[i];
    for (int64_t i = i0; i < P.m; i += gs) axo[i] = D.AX2[i];
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_dore_work_size(int64_t nz, int64_t m) {
    const int64_t n = (nz > m ? nz : m);
    return (size_t)((n + 255) / 256 + 1) * 3 * sizeof(double);
}

extern "C" int bsls_dore_iterate(const bsls_bb_problem *p, const bsls_dore_state *d,
                                 int64_t first_iter, int64_t count, void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    if (!d || first_iter < 0 || count < 0 || !d->X1 || !d->D || !d->X2 || !d->AX2 || !d->err ||
        !d->b || !d->S || !d->S2 || !d->dsc || !d->part || !d->tickets)
        return BSLS_E_ARG;
    for (int k = 0; k < 3; ++k)
        if (!d->X[k] || !d->AX[k]) return BSLS_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const BBWork w = bb_layout(*p);
    bsls_bb_problem PS = *p, P2 = *p, PE = *p;
    PS.scal = d->S;
    PE.scal = d->S;
    PE.r = d->err;                       // K2 reads err as its r
    P2.scal = d->S2;
    const bsls_dore_state D = *d;
    const int64_t big = (p->nz > p->m ? p->nz : p->m);
    // grid-stride elementwise steps: a fixed grid of at most DORE_GRID blocks
    // (two per CU), each thread summing its elements in stride order, so the
    // reductions' fan-in is DORE_GRID arrivals instead of one per 256
    // elements (C3: 3.7k workgroups made dore_top / dore_ext ~17 us for
    // ~18 / ~40 MB)
    constexpr int DORE_GRID = 512;
    const int gb0 = grid_for(big, 256), gm0 = grid_for(p->m, 256);
    const int gb = gb0 < DORE_GRID ? gb0 : DORE_GRID, gm = gm0 < DORE_GRID ? gm0 : DORE_GRID;
    for (int64_t i = first_iter; i < first_iter + count; ++i) {
        double *x = d->X[i % 3], *xp = d->X[(i + 2) % 3], *xn = d->X[(i + 1) % 3];
        double *axo = d->AX[i % 3], *axp = d->AX[(i + 2) % 3], *axpp = d->AX[(i + 1) % 3];
        // Ax = linop(x), err, norm_change (DORE.py:31-37); from iteration 1 on
        // x is the last x_select and Ax its linop, kept in axp (dore_top)
        static const bool recompute = [] {   // BSLS_DORE_RECOMPUTE=1: the reference's K1 (A/B)
            const char *e = getenv("BSLS_DORE_RECOMPUTE");
            return e && e[0] == '1';
        }();
        const bool top_k1 = i == 0 || recompute;
        if (top_k1) {
            bb_z2x<<<grid_for(p->n, 256), 256, 0, st>>>(PS, x);
            launch_k1<false, false, true>(PS, i, w, st);
        }
        dore_top<<<gb, 256, 0, st>>>(PS, D, i, x, xp, top_k1 ? nullptr : axp);
        // x_new = proj(x + linop_T(err)) (DORE.py:38-40; K3 with t = -scale)
        launch_k2<false>(PE, nullptr, p->g[0], w, st);
        launch_k3(PS, i, x, p->g[0], xn, w, st);
        // Ax = linop(x_new), err (DORE.py:41-42) and the first extrapolation
        launch_k1<false, false, true>(PS, i, w, st);
        dore_mid<<<gm, 256, 0, st>>>(PS, D, i, axo, axp);
        dore_ext<<<gb, 256, 0, st>>>(PS, D, axo, axp, axpp, x, xp, xn);
        // x_2 = proj(x_1 + a2 (x_1 - x_prev)), Ax_2 = linop(x_2), selection (DORE.py:55-69)
        launch_k3(P2, i, d->X1, d->D, d->X2, w, st, 0, 1);
        launch_k1<false, false, true>(P2, i, w, st);
        dore_sel<<<gm, 256, 0, st>>>(P2, D);
        dore_copy<<<gb, 256, 0, st>>>(P2, D, xn, axo);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

extern "C" size_t bsls_lbfgs_ls_work_size(int64_t nz) {
    return (size_t)(((nz > 0 ? nz : 1) + 255) / 256 + 1) * 2 * sizeof(double);
}

static int check_ls(const bsls_ls_state *s) {
    if (!s || !s->x || !s->d || !s->gx || !s->pt || !s->gpt || !s->zero || !s->fx || !s->st ||
        !s->S1 || !s->S2 || !s->part || !s->tickets)
        return BSLS_E_ARG;
    return BSLS_OK;
}

extern "C" int bsls_lbfgs_ls_begin(const bsls_bb_problem *p, const bsls_ls_state *s, void *stream) {
    int rc = check_problem(p);
    if (rc != BSLS_OK || (rc = check_ls(s)) != BSLS_OK) return rc;
    constexpr int LS_GRID = 512;
    const int g = grid_for(p->nz, 256);
    ls_begin_kernel<<<g < LS_GRID ? g : LS_GRID, 256, 0, (hipStream_t)stream>>>(
        s->d, s->gx, p->nz, s->fx, s->st, s->S1, s->S2, s->part, s->tickets);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_lbfgs_ls_trials(const bsls_bb_problem *p, const bsls_ls_state *s,
                                    int64_t count, void *stream) {
    int rc = check_problem(p);
    if (rc != BSLS_OK || (rc = check_ls(s)) != BSLS_OK) return rc;
    if (count < 0) return BSLS_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const BBWork w = bb_layout(*p);
    // the trial's problems: S1 gates K3 / K1 (and takes f), S2 gates K2; no
    // stopping rule of their own (max_iter unreachable, no early exits)
    bsls_bb_problem P1 = *p, P2 = *p;
    P1.scal = s->S1;
    P2.scal = s->S2;
    P1.max_iter = P2.max_iter = INT64_MAX;
    P1.early_exit = P2.early_exit = 0;
    for (int64_t k = 0; k < count; ++k) {
        launch_k3(P1, 1, s->x, s->d, s->pt, w, st, 0, 1);
        BSLS_LAUNCH_CHECK();
        launch_k1<true, true, true>(P1, 1, w, st);
        BSLS_LAUNCH_CHECK();
        ls_armijo_kernel<<<1, 64, 0, st>>>(s->st, s->S1, s->S2, s->c1);
        launch_k2<true>(P2, s->zero, s->gpt, w, st, 1, s->d);
        BSLS_LAUNCH_CHECK();
        ls_curv_kernel<<<1, 64, 0, st>>>(s->st, s->S1, s->S2, s->c2);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

extern "C" int bsls_lbfgs_ls_finish(const bsls_bb_problem *p, const bsls_ls_state *s,
                                    double *y_out, double *s_out, void *stream) {
    int rc = check_problem(p);
    if (rc != BSLS_OK || (rc = check_ls(s)) != BSLS_OK) return rc;
    constexpr int LS_GRID = 512;
    const int g = grid_for(p->nz, 256);
    ls_finish_kernel<<<g < LS_GRID ? g : LS_GRID, 256, 0, (hipStream_t)stream>>>(
        s->d, s->gx, s->gpt, p->nz, s->st, y_out, s_out, s->part, s->tickets);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" size_t bsls_ticket_bytes(void) { return (size_t)TICKET_BYTES; }

extern "C" size_t bsls_bb_workspace_size(int64_t m, int64_t n, int64_t nz) {
    return bb_layout(nullptr, m, n, nz).bytes;
}

extern "C" size_t bsls_bb_long_scratch_size(int64_t total) {
    // Y0, Y1 (doubles), W0, W1, CH (int32; CH one more per block, <= total)
    return (size_t)(total > 0 ? total : 0) * 32 + 64;
}

extern "C" size_t bsls_bb_dz_offset(int64_t m, int64_t n, int64_t nz) {
    return (size_t)((char *)bb_layout(nullptr, m, n, nz).dz - (char *)nullptr);
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
            BSLS_CHECK(hipMemsetAsync(P.work, 0, (size_t)((char *)w.p1 - (char *)P.work), st));
            return BSLS_OK;
        case 1:  // r_partial = A_g x_g (+ target on the shard_role 1 rank)
            if (P.shard_role == 1) {
                if (iter > 0) launch_k1<true, false, true>(P, iter, w, st);
                else launch_k1<true, false, false>(P, iter, w, st);
            } else {
                if (iter > 0) launch_k1<false, false, true>(P, iter, w, st);
                else launch_k1<false, false, false>(P, iter, w, st);
            }
            break;
        case 2:  // r += target, ||r||^2, stop test
        case 9:  // ||r||^2, stop test (r already the residual)
            bb_r_finish<<<(grid_for(P.m, 256) < R_FINISH_GRID ? grid_for(P.m, 256) : R_FINISH_GRID),
                          256, 0, st>>>(P, iter, w.pf, w.tkf, stage == 2 ? 1 : 0);
            break;
        case 8:  // stage 3 with stage 9 of iteration iter - 1 folded in
            if (iter <= 0) return BSLS_E_ARG;
            launch_k2<true, 1>(P, P.g[zc], P.g[zn], w, st, iter);
            break;
        case 10:  // stage 3 with this rank's slice of ||r||^2 (sliced schedule)
            if (iter <= 0) return BSLS_E_ARG;
            if (P.rr_lo < 0 || P.rr_hi > P.m || P.rr_lo > P.rr_hi) return BSLS_E_ARG;
            launch_k2<true, 2>(P, P.g[zc], P.g[zn], w, st, iter);
            break;
        case 13:  // stage 12 folded into stage 4's K3 (one launch fewer)
            if (iter <= 0) return BSLS_E_ARG;
            launch_k3(P, iter, P.z[zc], P.g[zn], P.z[zn], w, st, 1);
            break;
        case 15:  // stage 13 with the next stage 14's r initialisation folded in
            if (iter <= 0) return BSLS_E_ARG;
            launch_k3(P, iter, P.z[zc], P.g[zn], P.z[zn], w, st, 1, 0,
                      k1_init_folded(P) ? 1 : 0);
            break;
        case 14:  // stage 1 after stage 15 (r already initialised when it folds)
            if (iter <= 0) return BSLS_E_ARG;
            if (P.shard_role == 1) launch_k1<true, false, true>(P, iter, w, st, 0, -1, k1_init_folded(P));
            else launch_k1<false, false, true>(P, iter, w, st, 0, -1, k1_init_folded(P));
            break;
        case 12:  // f / stopping test of iteration iter - 1 (after the sums' all-reduce)
            if (iter <= 0) return BSLS_E_ARG;
            bb_shard_record<<<1, 64, 0, st>>>(P, iter);
            break;
        case 3:  // g = N'A'r (+ sums)
            if (iter > 0) launch_k2<true>(P, P.g[zc], P.g[zn], w, st);
            else launch_k2<false>(P, nullptr, P.g[0], w, st);
            break;
        case 4:  // t, projection, x
            if (iter <= 0) return BSLS_E_ARG;
            launch_k3(P, iter, P.z[zc], P.g[zn], P.z[zn], w, st);
            break;
        case 5:  // z[1] = z[0] + 1; x = N z[1]
            bb_plus_one<<<grid_for(P.nz > 0 ? P.nz : 1, 256), 256, 0, st>>>(P.z[0], P.z[1], w.dz, P.nz);
            BSLS_LAUNCH_CHECK();
            bb_z2x<<<grid_for(P.n, 256), 256, 0, st>>>(P, P.z[1]);
            break;
        case 6:  // x = N z[0]
            bb_z2x<<<grid_for(P.n, 256), 256, 0, st>>>(P, P.z[0]);
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

extern "C" int64_t bsls_bb_row_blocks(const bsls_bb_problem *p, int64_t *rows_per_block) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    if (rows_per_block)
        *rows_per_block = p->At.ent ? p->At.H : (int64_t)PANEL_WAVES * p->A.prow;
    return k1_row_blocks(*p);
}

extern "C" int bsls_bb_residual_rows(const bsls_bb_problem *p, int64_t iter, int64_t rb0,
                                     int64_t rb1, void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    const bsls_bb_problem &P = *p;
    if (rb0 < 0 || rb1 <= rb0 || rb1 > k1_row_blocks(P)) return BSLS_E_ARG;
    const BBWork w = bb_layout(P);
    hipStream_t st = (hipStream_t)stream;
    if (P.shard_role == 1) {
        if (iter > 0) launch_k1<true, false, true>(P, iter, w, st, rb0, rb1);
        else launch_k1<true, false, false>(P, iter, w, st, rb0, rb1);
    } else {
        if (iter > 0) launch_k1<false, false, true>(P, iter, w, st, rb0, rb1);
        else launch_k1<false, false, false>(P, iter, w, st, rb0, rb1);
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
        launch_k2<true>(P, P.g[zc], P.g[zn], w, st);
        launch_k3(P, i, P.z[zc], P.g[zn], P.z[zn], w, st);
        launch_k1<true, true, true>(P, i, w, st);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

// ---- the link-part pipeline of the column-sharded schedule -------------------
// (include/bsls_hip.h bsls_bb_k2_part / bsls_bb_k1_rows; csrc/shard.hip
// bsls_bb_shard_iterate_parts drives them with the exchange of each part's
// rows of r on a second stream)
extern "C" int bsls_bb_k2_part(const bsls_bb_problem *p, int64_t iter, int part, void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    const bsls_bb_problem &P = *p;
    if (iter <= 0 || !P.ATt.ent || (P.ATt.layout & 3) == 0 || P.ATt.ngroups < 2 || part < 0 ||
        part >= P.ATt.ngroups || !P.wpart)
        return BSLS_E_ARG;
    if (P.rr_lo < 0 || P.rr_hi > P.m || P.rr_lo > P.rr_hi) return BSLS_E_ARG;
    const BBWork w = bb_layout(P);
    const int zc = (int)((iter - 1) & 1), zn = (int)(iter & 1);
    launch_k2<true, 2>(P, P.g[zc], P.g[zn], w, (hipStream_t)stream, iter, nullptr, part);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}

extern "C" int bsls_bb_k1_rows(const bsls_bb_problem *p, int64_t iter, int64_t rb0, int64_t rb1,
                               void *stream) {
    const int rc = check_problem(p);
    if (rc != BSLS_OK) return rc;
    const bsls_bb_problem &P = *p;
    if (iter <= 0 || rb0 < 0 || rb1 <= rb0 || rb1 > k1_row_blocks(P)) return BSLS_E_ARG;
    const BBWork w = bb_layout(P);
    hipStream_t st = (hipStream_t)stream;
    const bool folded = k1_init_folded(P);
    if (P.shard_role == 1) launch_k1<true, false, true>(P, iter, w, st, rb0, rb1, folded);
    else launch_k1<false, false, true>(P, iter, w, st, rb0, rb1, folded);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
