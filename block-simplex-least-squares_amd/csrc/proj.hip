// proj.hip -- per-block Euclidean projection onto the probability simplex and
// onto the l1 ball, bit-identical to the reference
// (python/c_extensions/proj_simplex.h:17-74).
//
// Reference arithmetic (proj_simplex.h:17-34): sort the block descending
// (u_0 >= u_1 >= ...), S_i = u_0 + ... + u_i accumulated left to right,
// tmp_i = (1 - S_i)/(i+1); lambda = tmp_i at the LAST i >= 1 with
// u_i + tmp_i > 0, else 1 - u_0; y <- max(lambda + y, 0).  Ties in the sort
// do not change the S_i bit patterns (equal values), so any correct
// descending sort reproduces them; the S_i chain itself is sequential.
//
// Three size classes (host passes max_block; the small kernel routes the rest):
//   k <= 64      one LANE per block: block in registers, bitonic network of
//                8/16/32/64 (wave-uniform, chosen by the wave's largest block),
//                the S_i chain in-lane -> 64 blocks progress per wave;
//   64 < k <= 8192   one WORKGROUP per block: LDS bitonic sort, S_i by one
//                thread into LDS, conditions + last-index search in parallel;
//   k > 8192     one workgroup, sort in a global workspace (rare: the
//                reference's stack VLA already segfaults near k = 1M).
#include "bsls_common.hpp"

namespace bsls {

constexpr int SMALL_MAX = 64;
constexpr int LDS_MAX = 8192;
constexpr int LARGE_THREADS = 256;
constexpr int HUGE_THREADS = 1024;
constexpr int SCRATCH_WORDS = 32;  // >= HUGE_THREADS / WAVE partial maxima

__host__ __device__ inline int64_t pow2_ceil(int64_t k) {
    int64_t p = 1;
    while (p < k) p <<= 1;
    return p;
}

// Descending bitonic sorting network on registers (all indices compile-time).
template <int N>
__device__ __forceinline__ void bitonic_desc(double (&v)[N]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    // in-place compare-exchange with one temporary: written as
                    // asm so the scheduler cannot stretch a stage's live ranges
                    // (plain fmax/fmin needed 255 VGPRs at N = 64, this 141)
                    double t;
                    if ((i & k) == 0)
                        asm volatile(
                            "v_max_f64 %0, %1, %2\n\tv_min_f64 %2, %1, %2\n\tv_mov_b64 %1, %0"
                            : "=&v"(t), "+v"(v[i]), "+v"(v[l]));
                    else
                        asm volatile(
                            "v_min_f64 %0, %1, %2\n\tv_max_f64 %2, %1, %2\n\tv_mov_b64 %1, %0"
                            : "=&v"(t), "+v"(v[i]), "+v"(v[l]));
                }
            }
        }
    }
}

template <int N>
__device__ __forceinline__ double lambda_sorted(const double (&u)[N], int k) {
    double run = u[0];
    double lam = 1. - run;
#pragma unroll
    for (int i = 1; i < N; ++i) {
        if (i < k) {
            run = run + u[i];
            const double cand = (1. - run) / ((double)i + 1.);
            if (u[i] + cand > 0) lam = cand;
        }
    }
    return lam;
}

template <int N, bool BALL>
__device__ __forceinline__ void lane_block(double *__restrict__ y, int64_t s, int k) {
    double v[N];
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = (j < k) ? y[s + j] : -INFINITY;
    if (BALL) {
        // proj_simplex.h:56-64: clamp negatives, sum the rest in order.
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (j < k) {
                if (v[j] < 0.0) v[j] = 0.0;
                else acc += v[j];
            }
        }
        if (!(acc > 1.0)) {
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < k) y[s + j] = v[j];
            return;
        }
    }
    bitonic_desc<N>(v);
    const double lam = lambda_sorted<N>(v, k);
    asm volatile("" ::: "memory");   // re-read y after the sort, do not hoist
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (j < k) {
            double o = y[s + j];
            if (BALL) o = (o < 0.0) ? 0.0 : o;
            y[s + j] = relu_ref(lam + o);
        }
    }
}

template <bool BALL>
__global__ __launch_bounds__(256) void proj_small_kernel(double *__restrict__ y,
                                                         const int64_t *__restrict__ starts,
                                                         int64_t nb, int64_t n,
                                                         int64_t *__restrict__ big_list,
                                                         unsigned *__restrict__ big_count) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int k = 0;
    int64_t s = 0;
    if (b < nb) {
        s = starts[b];
        const int64_t kk = block_end(starts, nb, b, n) - s;
        if (kk > SMALL_MAX) {
            unsigned slot = atomicAdd(big_count, 1u);
            big_list[slot] = b;
        } else {
            k = (int)kk;
        }
    }
    const int kmax = wave_max(k);
    if (kmax == 0) return;
    if (kmax <= 8) lane_block<8, BALL>(y, s, k);
    else if (kmax <= 16) lane_block<16, BALL>(y, s, k);
    else if (kmax <= 32) lane_block<32, BALL>(y, s, k);
    else lane_block<64, BALL>(y, s, k);
}

// In-place descending bitonic sort of u[0..P) by the whole workgroup
// (u in LDS or in global memory private to this workgroup).
template <typename Ptr>
__device__ void bitonic_desc_shared(Ptr u, int64_t P) {
    for (int64_t k = 2; k <= P; k <<= 1) {
        for (int64_t j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (int64_t i = threadIdx.x; i < P / 2; i += blockDim.x) {
                const int64_t a = 2 * j * (i / j) + (i % j);
                const int64_t c = a + j;
                const double va = u[a], vc = u[c];
                const double hi = fmax(va, vc), lo = fmin(va, vc);
                if ((a & k) == 0) { u[a] = hi; u[c] = lo; }
                else { u[a] = lo; u[c] = hi; }
            }
        }
    }
    __syncthreads();
}

// Shared tail of the large/huge paths: u sorted descending (k valid entries),
// S written by one thread, conditions in parallel, lambda at the last index.
template <typename Ptr>
__device__ double lambda_shared(Ptr u, Ptr S, int64_t k, int64_t *best_part) {
    if (threadIdx.x == 0) {
        double run = u[0];
        S[0] = run;
        for (int64_t i = 1; i < k; ++i) {
            run = run + u[i];
            S[i] = run;
        }
    }
    __syncthreads();
    int64_t best = 0;
    for (int64_t i = 1 + threadIdx.x; i < k; i += blockDim.x) {
        const double cand = (1. - S[i]) / ((double)i + 1.);
        if (u[i] + cand > 0) best = i;   // i increases per thread: keeps its last
    }
    best = wave_max(best);
    if (lane_id() == 0) best_part[threadIdx.x / WAVE] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t bb = best_part[0];
        for (int w = 1; w < (int)(blockDim.x / WAVE); ++w) bb = best_part[w] > bb ? best_part[w] : bb;
        best_part[0] = bb;
    }
    __syncthreads();
    const int64_t i = best_part[0];
    const double lam = (1. - S[i]) / ((double)i + 1.);
    __syncthreads();
    return lam;
}

// Ball pre-pass for one block staged in u (original order): clamp, sequential
// sum of the non-negatives; returns true if the block still needs projecting.
template <typename Ptr>
__device__ bool ball_prepass(Ptr u, int64_t k, int64_t *scr) {
    int64_t &need = scr[0];
    if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int64_t j = 0; j < k; ++j) {
            const double v = u[j];
            if (!(v < 0.0)) acc += v;
        }
        need = (acc > 1.0);
    }
    __syncthreads();
    for (int64_t j = threadIdx.x; j < k; j += blockDim.x) {
        const double v = u[j];
        if (v < 0.0) u[j] = 0.0;
    }
    __syncthreads();
    return need != 0;
}

template <bool BALL>
__global__ __launch_bounds__(LARGE_THREADS) void proj_large_kernel(
    double *__restrict__ y, const int64_t *__restrict__ starts, int64_t nb, int64_t n,
    const int64_t *__restrict__ big_list, const unsigned *__restrict__ big_count) {
    // dynamic LDS only (cdna_hip_programming.md Guideline 17): [scratch][u][S]
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int64_t *scr = (int64_t *)lds;
    const unsigned cnt = *big_count;
    for (unsigned idx = blockIdx.x; idx < cnt; idx += gridDim.x) {
        const int64_t b = big_list[idx];
        const int64_t s = starts[b];
        const int64_t k = block_end(starts, nb, b, n) - s;
        if (k > LDS_MAX) continue;
        const int64_t P = pow2_ceil(k);
        double *u = lds + SCRATCH_WORDS;
        double *S = u + LDS_MAX;
        for (int64_t j = threadIdx.x; j < P; j += blockDim.x) u[j] = (j < k) ? y[s + j] : -INFINITY;
        __syncthreads();
        if (BALL && !ball_prepass(u, k, scr)) {
            for (int64_t j = threadIdx.x; j < k; j += blockDim.x) y[s + j] = u[j];
            __syncthreads();
            continue;
        }
        bitonic_desc_shared(u, P);
        const double lam = lambda_shared(u, S, k, scr);
        for (int64_t j = threadIdx.x; j < k; j += blockDim.x) {
            double o = y[s + j];
            if (BALL) o = (o < 0.0) ? 0.0 : o;
            y[s + j] = relu_ref(lam + o);
        }
        __syncthreads();
    }
}

template <bool BALL>
__global__ __launch_bounds__(HUGE_THREADS) void proj_huge_kernel(
    double *__restrict__ y, const int64_t *__restrict__ starts, int64_t nb, int64_t n,
    const int64_t *__restrict__ big_list, const unsigned *__restrict__ big_count,
    double *__restrict__ U, double *__restrict__ S) {
    __shared__ int64_t scr[SCRATCH_WORDS];
    const unsigned cnt = *big_count;
    for (unsigned idx = 0; idx < cnt; ++idx) {
        const int64_t b = big_list[idx];
        const int64_t s = starts[b];
        const int64_t k = block_end(starts, nb, b, n) - s;
        if (k <= LDS_MAX) continue;
        const int64_t P = pow2_ceil(k);
        for (int64_t j = threadIdx.x; j < P; j += blockDim.x) U[j] = (j < k) ? y[s + j] : -INFINITY;
        __syncthreads();
        if (BALL && !ball_prepass(U, k, scr)) {
            for (int64_t j = threadIdx.x; j < k; j += blockDim.x) y[s + j] = U[j];
            __syncthreads();
            continue;
        }
        bitonic_desc_shared(U, P);
        const double lam = lambda_shared(U, S, k, scr);
        for (int64_t j = threadIdx.x; j < k; j += blockDim.x) {
            double o = y[s + j];
            if (BALL) o = (o < 0.0) ? 0.0 : o;
            y[s + j] = relu_ref(lam + o);
        }
        __syncthreads();
    }
}

struct ProjWork {
    unsigned *count;
    int64_t *list;
    double *U, *S;
    size_t bytes;
};

static size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

static ProjWork proj_layout(void *base, int64_t n, int64_t nb, int64_t max_block) {
    ProjWork w{};
    char *p = (char *)base;
    size_t off = 0;
    w.count = (unsigned *)(p + off);
    off += 16;
    int64_t nbig = nb < (n / (SMALL_MAX + 1) + 1) ? nb : (n / (SMALL_MAX + 1) + 1);
    w.list = (int64_t *)(p + off);
    off += align16((size_t)nbig * sizeof(int64_t));
    if (max_block > LDS_MAX) {
        const int64_t P = pow2_ceil(max_block);
        w.U = (double *)(p + off);
        off += align16((size_t)P * sizeof(double));
        w.S = (double *)(p + off);
        off += align16((size_t)max_block * sizeof(double));
    }
    w.bytes = off;
    return w;
}

template <bool BALL>
static int proj_launch(double *y, const int64_t *starts, int64_t nb, int64_t n,
                       int64_t max_block, void *work, size_t work_bytes, hipStream_t st) {
    if (nb <= 0 || n <= 0 || y == nullptr || starts == nullptr) return BSLS_E_ARG;
    if (max_block < 1) return BSLS_E_ARG;
    ProjWork w = proj_layout(work, n, nb, max_block);
    if (work == nullptr || work_bytes < w.bytes) return BSLS_E_WORKSPACE;
    BSLS_CHECK(hipMemsetAsync(w.count, 0, 16, st));
    proj_small_kernel<BALL><<<grid_for(nb, 256), 256, 0, st>>>(y, starts, nb, n, w.list, w.count);
    BSLS_LAUNCH_CHECK();
    if (max_block > SMALL_MAX) {
        int64_t nbig = nb < (n / (SMALL_MAX + 1) + 1) ? nb : (n / (SMALL_MAX + 1) + 1);
        int grid = (int)(nbig < 2048 ? nbig : 2048);
        const size_t lds = (SCRATCH_WORDS + 2 * LDS_MAX) * sizeof(double);
        static bool attr_set = false;
        if (!attr_set) {
            BSLS_CHECK(hipFuncSetAttribute((const void *)proj_large_kernel<BALL>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr_set = true;
        }
        proj_large_kernel<BALL><<<grid, LARGE_THREADS, lds, st>>>(y, starts, nb, n, w.list, w.count);
        BSLS_LAUNCH_CHECK();
    }
    if (max_block > LDS_MAX) {
        proj_huge_kernel<BALL><<<1, HUGE_THREADS, 0, st>>>(y, starts, nb, n, w.list, w.count, w.U, w.S);
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

}  // namespace bsls

using namespace bsls;

extern "C" size_t bsls_proj_workspace_size(int64_t n, int64_t nblocks, int64_t max_block) {
    return proj_layout(nullptr, n, nblocks, max_block).bytes;
}

extern "C" int bsls_proj_multi_simplex(double *d_y, const int64_t *d_starts, int64_t nblocks,
                                       int64_t n, int64_t max_block, void *d_work,
                                       size_t work_bytes, void *stream) {
    return proj_launch<false>(d_y, d_starts, nblocks, n, max_block, d_work, work_bytes,
                              (hipStream_t)stream);
}

extern "C" int bsls_proj_multi_ball(double *d_y, const int64_t *d_starts, int64_t nblocks,
                                    int64_t n, int64_t max_block, void *d_work,
                                    size_t work_bytes, void *stream) {
    return proj_launch<true>(d_y, d_starts, nblocks, n, max_block, d_work, work_bytes,
                             (hipStream_t)stream);
}
