// Knock-out microbenchmark for the k <= 64 projection kernel (proj.hip):
// where does proj_lds_kernel's time go?  Variants V:
//   0 full (same work as the product kernel)   1 no sort
//   2 no lambda chain                          3 LDS stage in/out only
//   4 regs in/out only (no sort, no lambda)    5 full, unpredicated LDS loads
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC -I include -I <csrc> tools/proj_ubench.hip
#include "../block-simplex-least-squares_amd/csrc/proj.hip"

namespace ub {
using namespace bsls;
constexpr int UCAP = PCAP + 64;

// descending "flip" bitonic network: every comparator puts the max at the
// lower index, so -inf padding at indices >= KB never moves and every
// comparator touching index >= KB is dropped at compile time.
template <int N, int KB, int CE2>
__device__ __forceinline__ void bitonic_flip(double (&v)[N]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                int l;
                if (j == (k >> 1)) {
                    const int blk = i & ~(k - 1);
                    l = ((i - blk) < (k >> 1)) ? blk + k - 1 - (i - blk) : -1;
                } else {
                    l = i ^ j;
                }
                if (l > i && l < KB) {
                    if (CE2) {
                        double hi, lo;
                        asm volatile("v_max_f64 %0, %2, %3\n\tv_min_f64 %1, %2, %3"
                                     : "=&v"(hi), "=v"(lo) : "v"(v[i]), "v"(v[l]));
                        v[i] = hi;
                        v[l] = lo;
                    } else {
                        double t;
                        asm volatile("v_max_f64 %0, %1, %2\n\tv_min_f64 %2, %1, %2\n\tv_mov_b64 %1, %0"
                                     : "=&v"(t), "+v"(v[i]), "+v"(v[l]));
                    }
                }
            }
        }
    }
}

template <int N>
__device__ __forceinline__ double lambda_stop2(const double (&u)[N], int k, double margin) {
    double run = u[0];
    const double D0 = 1. - run;
    double Drho = D0;
    int rho = 0;
    bool live = true;
#pragma unroll
    for (int i = 1; i < N; ++i) {
        live = live && (i < k);
        if (!__builtin_amdgcn_ballot_w64(live)) break;
        run = run + u[i];
        const double D = 1. - run;
        const double ip1 = (double)i + 1.;
        const double E = __builtin_fma(ip1, u[i], D);
        const double T = ip1 * (__builtin_fabs(u[i]) * 0x1p-51 + 0x1p-1070);
        bool cond = E > T;
        if (live && E > 0.0 && !cond) cond = (u[i] + D / ip1 > 0);
        if (live && cond) {
            rho = i;
            Drho = D;
        }
        live = live && !(E < -margin);
    }
    return rho == 0 ? D0 : Drho / ((double)rho + 1.);
}

template <int N>
__device__ __forceinline__ double lambda_stop(const double (&u)[N], int k, double margin);

template <int N, int KB, int V>
__device__ __forceinline__ void lane_block_w(double *y, int s, int k) {
    // V 11: 2-instr CE, full network; 12: + pruned flip network;
    // 13: + early-stop lambda (Mx bound); 14: 13 with lambda_stop2
    double v[N];
    uint32_t hx = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double t = y[s + j];
        v[j] = (j < k) ? t : -INFINITY;
        if (V >= 13) {
            const uint32_t h = (uint32_t)((uint64_t)__double_as_longlong(t) >> 32) & 0x7fffffffu;
            hx = max(hx, (j < k) ? h : 0u);
        }
    }
    if (V == 11) bitonic_flip<N, N, 1>(v);
    else bitonic_flip<N, KB, 1>(v);
    double lam;
    if (V >= 13) {
        const double Mx = __longlong_as_double((long long)(((uint64_t)hx << 32) | 0xffffffffull));
        const double kk = (double)k;
        const double margin = kk * 0x1p-49 * (1. + 2. * kk * Mx);
        lam = (V == 13) ? lambda_stop<N>(v, k, margin) : lambda_stop2<N>(v, k, margin);
    } else {
        lam = lambda_sorted<N>(v, k);
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (j < k) y[s + j] = relu_ref(lam + y[s + j]);
    }
}

template <int N, int V>
__device__ __forceinline__ void lane_block_v(double *y, int s, int k) {
    double v[N];
    if (V == 5) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double t = y[s + j];
            v[j] = (j < k) ? t : -INFINITY;
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) v[j] = (j < k) ? y[s + j] : -INFINITY;
    }
    if (V != 1 && V != 4) bitonic_desc<N>(v);
    double lam = 0.0;
    if (V == 2) lam = v[0] * 0.5;
    else if (V != 4) lam = lambda_sorted<N>(v, k);
    else {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) acc = fmax(acc, v[j]);
        lam = acc;
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (j < k) y[s + j] = relu_ref(lam + y[s + j]);
    }
}

template <int V>
__global__ __launch_bounds__(64) void proj_v(double *__restrict__ y, const int64_t *__restrict__ starts,
                                             int64_t nb, int64_t n) {
    __shared__ double buf[UCAP];
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * WAVE;
    const int64_t b = b0 + lane;
    int k = 0;
    int64_t s = 0, e = 0;
    if (b < nb) {
        s = starts[b];
        e = block_end(starts, nb, b, n);
        k = (int)(e - s);
    }
    const int kmax = wave_max(k);
    const int lastl = (int)((nb - b0 < WAVE ? nb - b0 : WAVE) - 1);
    const int64_t s0 = uni64(s, 0);
    const int64_t e1 = uni64(e, lastl);
    const int tot = (int)(e1 - s0);
    if (tot > PCAP) return;
    for (int i = lane; i < tot; i += WAVE) buf[i] = y[s0 + i];
    __syncthreads();
    const int off = (int)(s - s0);
    if (V >= 11) {
        if (kmax <= 8) lane_block_w<8, 8, V>(buf, off, k);
        else if (kmax <= 16) lane_block_w<16, 16, V>(buf, off, k);
        else if (kmax <= 32) lane_block_w<32, 32, V>(buf, off, k);
        else if (kmax <= 40) lane_block_w<64, 40, V>(buf, off, k);
        else if (kmax <= 44) lane_block_w<64, 44, V>(buf, off, k);
        else if (kmax <= 48) lane_block_w<64, 48, V>(buf, off, k);
        else if (kmax <= 52) lane_block_w<64, 52, V>(buf, off, k);
        else if (kmax <= 56) lane_block_w<64, 56, V>(buf, off, k);
        else lane_block_w<64, 64, V>(buf, off, k);
    } else if (V != 3) {
        if (kmax <= 8) lane_block_v<8, V>(buf, off, k);
        else if (kmax <= 16) lane_block_v<16, V>(buf, off, k);
        else if (kmax <= 32) lane_block_v<32, V>(buf, off, k);
        else lane_block_v<64, V>(buf, off, k);
    }
    __syncthreads();
    for (int i = lane; i < tot; i += WAVE) y[s0 + i] = buf[i];
}

// ---- transposed staging: column l of T holds block l (T[j*LD + l]) so the
// lane-per-block accesses are bank-conflict-free; element -> (owner, j) via a
// bitmap of block starts (popcount below the lane).
constexpr int LD = 65;

template <int N>
__device__ __forceinline__ double lambda_stop(const double (&u)[N], int k, double margin) {
    double run = u[0];
    const double D0 = 1. - run;
    double Drho = D0;
    int rho = 0;
    bool live = true;
#pragma unroll
    for (int i = 1; i < N; ++i) {
        live = live && (i < k);
        if (!__builtin_amdgcn_ballot_w64(live)) break;
        if (live) {
            run = run + u[i];
            const double D = 1. - run;
            const double ip1 = (double)i + 1.;
            const double E = __builtin_fma(ip1, u[i], D);
            if (E < -margin) {
                live = false;
            } else {
                const double T = ip1 * (__builtin_fabs(u[i]) * 0x1p-51 + 0x1p-1070);
                bool cond = E > T;
                if (E > 0.0 && !cond) cond = (u[i] + D / ip1 > 0);
                if (cond) {
                    rho = i;
                    Drho = D;
                }
            }
        }
    }
    return rho == 0 ? D0 : Drho / ((double)rho + 1.);
}

template <int N, int V>
__device__ __forceinline__ void lane_block_t(double *T, int lane, int k) {
    double v[N];
    double A = 0.0, Mx = 0.0;
    uint32_t hx = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double t = T[j * LD + lane];
        v[j] = (j < k) ? t : -INFINITY;
        if (V == 9) {
            const uint32_t h = (uint32_t)((uint64_t)__double_as_longlong(t) >> 32) & 0x7fffffffu;
            hx = max(hx, (j < k) ? h : 0u);
        }
        if (V == 7 || V == 8) {
            const double a = (j < k) ? __builtin_fabs(t) : 0.0;
            A += a;
            Mx = fmax(Mx, a);
        }
    }
    bitonic_desc<N>(v);
    double lam;
    if (V == 9) {
        // |u| <= Mx for every element (high word max, low word all ones);
        // sum |u| <= k * Mx.  Inf/NaN -> margin inf/NaN -> never stops early.
        const double Mx9 = __longlong_as_double((long long)(((uint64_t)hx << 32) | 0xffffffffull));
        const double kk = (double)k;
        const double margin = kk * 0x1p-49 * (1. + 2. * kk * Mx9);
        lam = lambda_stop<N>(v, k, margin);
    } else if (V == 7 || V == 8) {
        const double kk = (double)k;
        const double margin = kk * 0x1p-49 * (1. + A * (1. + 0x1p-40) + kk * Mx);
        lam = lambda_stop<N>(v, k, margin);
    } else {
        lam = lambda_sorted<N>(v, k);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) T[j * LD + lane] = relu_ref(lam + T[j * LD + lane]);
}

template <int V>
__global__ __launch_bounds__(64) void proj_t(double *__restrict__ y, const int64_t *__restrict__ starts,
                                             int64_t nb, int64_t n) {
    __shared__ double T[64 * LD];
    __shared__ uint64_t smap[PCAP / 64];
    const int lane = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * WAVE;
    const int64_t b = b0 + lane;
    int k = 0;
    int64_t s = 0, e = 0;
    if (b < nb) {
        s = starts[b];
        e = block_end(starts, nb, b, n);
        k = (int)(e - s);
    }
    const int kmax = wave_max(k);
    const int lastl = (int)((nb - b0 < WAVE ? nb - b0 : WAVE) - 1);
    const int64_t s0 = uni64(s, 0);
    const int64_t e1 = uni64(e, lastl);
    const int tot = (int)(e1 - s0);
    if (tot > PCAP) return;
    const int off = (int)(s - s0);
    const int nw = (tot + 63) >> 6;
    if (lane < nw) smap[lane] = 0;
    __syncthreads();
    if (k > 0) atomicOr((unsigned long long *)&smap[off >> 6], 1ull << (off & 63));
    __syncthreads();
    const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
    if (V == 6 || V == 7) {
        int base = -1;
#pragma unroll 4
        for (int c = 0; c < nw; ++c) {
            const int i = (c << 6) + lane;
            const uint64_t w = smap[c];
            const int own = base + __popcll(w & le);
            base += __popcll(w);
            const int oo = __shfl(off, own, WAVE);
            if (i < tot) T[(i - oo) * LD + own] = y[s0 + i];
        }
    } else {
        // batched: SB global loads in flight, then the scatter into columns
        constexpr int SB = 8;
        int base = -1;
        for (int c0 = 0; c0 < nw; c0 += SB) {
            double t[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int i = ((c0 + q) << 6) + lane;
                t[q] = y[s0 + (i < tot ? i : tot - 1)];
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int c = c0 + q;
                const int i = (c << 6) + lane;
                const uint64_t w = (c < nw) ? smap[c] : 0ull;
                const int own = base + __popcll(w & le);
                base += __popcll(w);
                const int oo = __shfl(off, own, WAVE);
                if (i < tot) T[(i - oo) * LD + own] = t[q];
            }
        }
    }
    __syncthreads();
    if (V == 10) {
    } else if (kmax <= 8) lane_block_t<8, V>(T, lane, k);
    else if (kmax <= 16) lane_block_t<16, V>(T, lane, k);
    else if (kmax <= 32) lane_block_t<32, V>(T, lane, k);
    else lane_block_t<64, V>(T, lane, k);
    __syncthreads();
    {
        int base = -1;
#pragma unroll 4
        for (int c = 0; c < nw; ++c) {
            const int i = (c << 6) + lane;
            const uint64_t w = smap[c];
            const int own = base + __popcll(w & le);
            base += __popcll(w);
            const int oo = __shfl(off, own, WAVE);
            if (i < tot) y[s0 + i] = T[(i - oo) * LD + own];
        }
    }
}

static int64_t *g_list = nullptr;
static unsigned *g_count = nullptr;

template <int V>
static void launch(double *y, const int64_t *st, int64_t nb, int64_t n) {
    if (V == 15) {
        if (!g_list) {
            (void)hipMalloc(&g_list, 1 << 20);
            (void)hipMalloc(&g_count, 64);
            (void)hipMemset(g_count, 0, 64);
        }
        proj_lds_kernel<false><<<grid_for(nb, WAVE), WAVE>>>(y, st, nb, n, g_list, g_count, 0, nullptr);
        return;
    }
    if (V >= 6 && V <= 10) proj_t<V><<<grid_for(nb, WAVE), WAVE>>>(y, st, nb, n);
    else proj_v<V><<<grid_for(nb, WAVE), WAVE>>>(y, st, nb, n);
}
}  // namespace ub

extern "C" float proj_ubench(int V, double *y, const int64_t *st, int64_t nb, int64_t n, int reps) {
    using namespace ub;
    void (*f)(double *, const int64_t *, int64_t, int64_t) = nullptr;
    switch (V) {
        case 0: f = launch<0>; break;
        case 1: f = launch<1>; break;
        case 2: f = launch<2>; break;
        case 3: f = launch<3>; break;
        case 4: f = launch<4>; break;
        case 5: f = launch<5>; break;
        case 6: f = launch<6>; break;
        case 7: f = launch<7>; break;
        case 8: f = launch<8>; break;
        case 9: f = launch<9>; break;
        case 10: f = launch<10>; break;
        case 11: f = launch<11>; break;
        case 12: f = launch<12>; break;
        case 13: f = launch<13>; break;
        case 14: f = launch<14>; break;
        case 15: f = launch<15>; break;
        default: return -1.f;
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f(y, st, nb, n);
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) f(y, st, nb, n);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms * 1000.f / reps;
}

extern "C" void proj_ubench_once(int V, double *y, const int64_t *st, int64_t nb, int64_t n) {
    (void)proj_ubench(V, y, st, nb, n, 0);
    (void)hipDeviceSynchronize();
}
