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
//   k <= 64      one LANE per block (proj_lds_kernel): a wave stages its 64
//                consecutive blocks in LDS (DMA), each lane sorts its block in
//                registers with a flip-bitonic network pruned at compile time
//                to the wave's largest block, runs the S_i chain (division-
//                free test, the reference's division only within ulps) and
//                writes back through LDS -- all straight-line code; two such
//                waves per workgroup, the second loading once the first's
//                loads have landed (lds_group);
//   64 < k <= 8192   one WORKGROUP per block: LDS bitonic sort, S_i by one
//                thread into LDS, conditions + last-index search in parallel;
//   k > 8192     one workgroup, sort in a global workspace (rare: the
//                reference's stack VLA already segfaults near k = 1M).
#include <rocprim/device/device_radix_sort.hpp>

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

// proj_simplex.h:22-30 on u sorted descending, literally: S_i = sequential
// sum, lambda = (1 - S_i)/(i + 1) at the LAST i with u_i + that > 0 (else
// 1 - u_0).  Entries i >= KB are -inf padding and never reached.
template <int N, int KB = N>
__device__ __forceinline__ double lambda_sorted(const double (&u)[N], int k) {
    double run = u[0];
    double lam = 1. - run;
#pragma unroll
    for (int i = 1; i < KB; ++i) {
        if (i < k) {
            run = run + u[i];
            const double cand = (1. - run) / ((double)i + 1.);
            if (u[i] + cand > 0) lam = cand;
        }
    }
    return lam;
}

// The same lambda without a division per i and without branches.  The test
// u_i + fl(D_i/(i+1)) > 0 (D_i = fl(1 - S_i)) is decided by the sign of
// E = fl((i+1) u_i + D_i) (one fma, sign-exact): E <= 0 -> false (the
// quotient rounds to <= -u_i); E > T = (i+1)(|u_i| 2^-51 + 2^-1070) -> true
// (the quotient clears -u_i by more than its rounding error).  In between
// (within a few ulps) the lane reports `amb` and the caller redoes the lane
// with lambda_sorted; one division per block remains (lambda itself).
template <int N, int KB>
__device__ __forceinline__ double lambda_fast(const double (&u)[N], int k, bool &amb) {
    double run = u[0];
    const double D0 = 1. - run;
    double Drho = D0;
    int rho = 0;
    int a = 0;
#pragma unroll
    for (int i = 1; i < KB; ++i) {
        run = run + u[i];
        const double D = 1. - run;
        const double ip1 = (double)i + 1.;
        const double E = __builtin_fma(ip1, u[i], D);
        const double T = ip1 * __builtin_fma(__builtin_fabs(u[i]), 0x1p-51, 0x1p-1070);
        const bool live = i < k;
        const bool c = live && (E > T);
        a |= (live && (E > 0.0) && !(E > T)) ? 1 : 0;
        rho = c ? i : rho;
        Drho = c ? D : Drho;
        // materialise the running selects every step: left alone, the
        // compiler keeps every D_i and mask live and spills them
        asm volatile("" : "+v"(Drho), "+v"(rho), "+v"(a), "+v"(run));
    }
    amb = a != 0;
    return rho == 0 ? D0 : Drho / ((double)rho + 1.);
}

// Descending "flip" bitonic network: every comparator puts the max at the
// lower index, so -inf padding at indices >= KB never moves and every
// comparator that touches an index >= KB is dropped at compile time (the
// wave's largest block picks KB).  Comparators are 2-instruction asm so the
// scheduler keeps a stage's live ranges short (plain fmax/fmin: 255 VGPRs).
template <int N, int KB>
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
                    double hi, lo;
                    asm volatile("v_max_f64 %0, %2, %3\n\tv_min_f64 %1, %2, %3"
                                 : "=&v"(hi), "=v"(lo)
                                 : "v"(v[i]), "v"(v[l]));
                    v[i] = hi;
                    v[l] = lo;
                }
            }
        }
    }
}

template <int N, bool BALL, typename Ptr>
__device__ __forceinline__ void lane_block(Ptr y, int64_t s, int k) {
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

// Blocks <= 64 with the wave's contiguous range staged in LDS: one wave per
// 64 consecutive blocks (one lane each).  The range is read and written with
// coalesced 8-B-per-lane accesses; the lanes then sort / project their own
// blocks out of LDS.  Without staging, every wave-instruction touched 64 cache
// lines (one per block) -- measured 2.6x write amplification.  A wave whose
// range exceeds PCAP doubles falls back to direct global access.
// PCAP 2400: PBUF * 8 B = 20.2 KB per wave, so 8 waves per CU (the VGPR
// limit too) -- 2048 resident waves; a grid beyond the resident set leaves a
// tail of late waves (measured: 27 of 1563 waves at 3072 doubled the time).
constexpr int PCAP = 2400;
constexpr int PBUF = PCAP + 2 * WAVE + 2;   // + read slack, + one dummy slot per lane

__device__ __forceinline__ int64_t uni64(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// Comparator of the generated top-16 selection networks (proj_net.hpp): max
// to the lower index, 2-instruction asm like bitonic_flip's.
#define PROJ_CE(i, l)                                                                \
    do {                                                                             \
        double hi_, lo_;                                                             \
        asm volatile("v_max_f64 %0, %2, %3\n\tv_min_f64 %1, %2, %3"                  \
                     : "=&v"(hi_), "=v"(lo_)                                         \
                     : "v"(v[i]), "v"(v[l]));                                        \
        v[i] = hi_;                                                                  \
        v[l] = lo_;                                                                  \
    } while (0)
}  // namespace bsls
#include "proj_net.hpp"
namespace bsls {
#undef PROJ_CE

// lambda_fast over a sorted prefix only, stopping each lane once its answer
// is settled.  The exact e_i = (i+1) u_i + 1 - S_i is non-increasing in i
// (e_{i+1} - e_i = (i+1)(u_{i+1} - u_i) <= 0) and the reference's test at i
// is e_i > 0 up to rounding; with every fl error of S_i, 1 - S_i and the test
// bounded by 2^-53 (2 k^2 Mx + 3 (1 + k Mx)) <= margin = k 2^-49 (1 + 2 k Mx)
// (Mx >= max |u|), a computed E_i < -margin makes the test false at i and at
// every later index.  A lane is settled at that point or when i reaches k.
struct Chain {
    double run, D0, Drho;
    int rho, a;
    bool live;
};

template <int N>
__device__ __forceinline__ Chain chain_begin(const double (&u)[N], int k) {
    Chain c;
    c.run = u[0];
    c.D0 = 1. - c.run;
    c.Drho = c.D0;
    c.rho = 0;
    c.a = 0;
    c.live = k > 1;
    return c;
}

// indices I0 .. I1 - 1 of the chain (u sorted there); the wave leaves as soon
// as every lane is settled
template <int I0, int I1, int N>
__device__ __forceinline__ void chain_steps(const double (&u)[N], int k, double margin, Chain &c) {
#pragma unroll
    for (int i = I0; i < I1; ++i) {
        if (((i - I0) & 3) == 0 && !__builtin_amdgcn_ballot_w64(c.live)) break;
        c.live = c.live && (i < k);
        c.run = c.run + u[i];
        const double D = 1. - c.run;
        const double ip1 = (double)i + 1.;
        const double E = __builtin_fma(ip1, u[i], D);
        const double T = ip1 * __builtin_fma(__builtin_fabs(u[i]), 0x1p-51, 0x1p-1070);
        const bool ok = c.live && (E > T);
        c.a |= (c.live && (E > 0.0) && !(E > T)) ? 1 : 0;
        c.rho = ok ? i : c.rho;
        c.Drho = ok ? D : c.Drho;
        c.live = c.live && !(E < -margin);
        asm volatile("" : "+v"(c.Drho), "+v"(c.rho), "+v"(c.a), "+v"(c.run));
    }
}

__device__ __forceinline__ double chain_lambda(const Chain &c) {
    return c.rho == 0 ? c.D0 : c.Drho / ((double)c.rho + 1.);
}

// One lane, one block of k <= KB entries at buf[off ..): straight-line code.
// Reads are unconditional (slack after the range), writes of j >= k go to the
// lane's dummy slot, so no per-entry branches or per-entry waits.
// KB > 16: top-16 selection networks (proj_net.hpp) + the early-settling
// chain; a wave with an unsettled lane sorts fully (the networks only
// permute, the -inf padding stays put).
// THR (the sort-free path, bsls_proj_multi_*_fast): no sort and no chain --
// Michelot's threshold iteration on the lane's registers: from the lower
// bound tau = max(M - 1, (S - 1) / k) (M the block max, S its sum) each pass
// sums the entries above tau and sets tau = (sum - 1) / count; the active
// set only shrinks, and once its count repeats tau is the projection's
// threshold.  Within ulps of the sorted chain (the north star's 1e-12).
template <int N, int KB, bool BALL, bool THR = false>
__device__ __forceinline__ void lane_block_lds(double *buf, int off, int k, int lane) {
    double v[N];
    double acc = 0.0;
    uint32_t hx = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double t = -INFINITY;
        if (j < KB) t = buf[off + j];
        if (BALL) {
            // proj_simplex.h:56-64: clamp negatives, sum the rest in order
            // (adding the clamped 0.0 leaves acc's bits unchanged: acc >= +0)
            t = (t < 0.0) ? 0.0 : t;
            acc += (j < k) ? t : 0.0;
        }
        if (KB > 16 && j < KB) {
            const uint32_t h = (uint32_t)((uint64_t)__double_as_longlong(t) >> 32) & 0x7fffffffu;
            hx = (j < k && h > hx) ? h : hx;
        }
        v[j] = (j < k) ? t : -INFINITY;
    }
    const bool need = BALL ? (acc > 1.0) : true;
    double lam = 0.0;
    if constexpr (THR) {
        if (!BALL || __builtin_amdgcn_ballot_w64(need)) {
            double M = -INFINITY, S = 0.0;
#pragma unroll
            for (int j = 0; j < KB; ++j) {
                M = fmax(M, v[j]);
                S += (j < k) ? v[j] : 0.0;
            }
            double tau = fmax(M - 1.0, (S - 1.0) / (double)(k > 0 ? k : 1));
            bool done = (k == 0) || !need;
            int cp = -1;
            for (int it = 0; it <= KB + 1; ++it) {
                if (__builtin_amdgcn_ballot_w64(!done) == 0ull) break;
                double sa = 0.0;
                int c = 0;
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const bool a = v[j] > tau;
                    sa += a ? v[j] : 0.0;
                    c += a ? 1 : 0;
                }
                const double tn = (sa - 1.0) / (double)(c > 0 ? c : 1);
                if (!done) {
                    done = (c == cp);
                    tau = tn;
                    cp = c;
                }
            }
            lam = -tau;
        }
    } else if (!BALL || __builtin_amdgcn_ballot_w64(need)) {
        bool full = true;
        if constexpr (KB > 16) {
            // level 1: the 16 largest, sorted, and the chain over them;
            // level 2 (KB > 32): the next 16 of the rest, chain continued;
            // a wave with a lane still open after that sorts fully
            Top16<KB>::template run<0>(v);
            const double Mx =
                __longlong_as_double((long long)(((uint64_t)hx << 32) | 0xffffffffull));
            const double kk = (double)k;
            const double margin = kk * 0x1p-49 * (1. + 2. * kk * Mx);
            Chain c = chain_begin(v, k);
            chain_steps<1, 16>(v, k, margin, c);
            int depth = 16;
            if constexpr (KB > 32) {
                if (__builtin_amdgcn_ballot_w64(c.live && k > 16)) {
                    Top16<KB - 16>::template run<16>(v);
                    chain_steps<16, 32>(v, k, margin, c);
                    depth = 32;
                }
            }
            full = __builtin_amdgcn_ballot_w64(c.live && k > depth) != 0;
            if (!full) {
                lam = chain_lambda(c);
                if (__builtin_amdgcn_ballot_w64(c.a != 0)) {
                    if (c.a != 0) lam = lambda_sorted<N, (KB > 32 ? 32 : 16)>(v, k < depth ? k : depth);
                }
            }
        }
        if (full) {
            bitonic_flip<N, KB>(v);
            bool amb;
            lam = lambda_fast<N, KB>(v, k, amb);
            if (__builtin_amdgcn_ballot_w64(amb)) {
                if (amb) lam = lambda_sorted<N, KB>(v, k);
            }
        }
    }
    if constexpr (THR) {
        // nothing was sorted: v[j] (clamped for the ball, as the output wants)
        // is still entry j, so no second read of the block
#pragma unroll
        for (int j = 0; j < KB; ++j) {
            const double t = v[j];
            const double r = need ? relu_ref(lam + t) : t;
            buf[(j < k) ? off + j : PCAP + WAVE + 2 + lane] = r;
        }
        return;
    }
    asm volatile("" ::: "memory");   // keep the o[] loads after the sort (VGPRs)
    double o[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) o[j] = buf[off + j];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
        double t = o[j];
        if (BALL) t = (t < 0.0) ? 0.0 : t;
        const double r = need ? relu_ref(lam + t) : t;
        buf[(j < k) ? off + j : PCAP + WAVE + 2 + lane] = r;
    }
}

// One wave's group of 64 consecutive blocks (one lane each), staged in its
// own LDS buffer.  W > 1 (proj_lds_kernel<BALL, W>, W waves per workgroup):
// wave w issues its range's loads only once wave w - 1's have landed
// (`landed`, an LDS counter), so the waves of a CU pass through the load /
// sort / store phases staggered instead of all together -- wave w's loads
// stream while wave w - 1 sorts.  Every wave bumps the counter exactly once,
// whatever path it takes, so no wave waits forever.
template <bool BALL, int W, bool THR = false>
__device__ __forceinline__ void lds_group(double *__restrict__ y,
                                          const int64_t *__restrict__ starts, int64_t nb,
                                          int64_t n, int64_t *__restrict__ big_list,
                                          unsigned *__restrict__ big_count, int allow_big,
                                          double *buf, int *landed, int64_t grp, int wv,
                                          int lane) {
    auto wait_turn = [&]() {
        if constexpr (W > 1) {
            if (wv > 0)
                while (__atomic_load_n(landed, __ATOMIC_RELAXED) < wv) __builtin_amdgcn_s_sleep(1);
        }
    };
    auto pass_turn = [&]() {
        if constexpr (W > 1) {
            if (lane == 0) __atomic_store_n(landed, wv + 1, __ATOMIC_RELAXED);
        }
    };
    const int64_t b0 = grp * WAVE;
    const int64_t b = b0 + lane;
    int k = 0;
    int64_t s = 0, e = 0;
    if (b < nb) {
        s = starts[b];
        e = block_end(starts, nb, b, n);
        const int64_t kk = e - s;
        if (kk > SMALL_MAX) {
            if (allow_big) {   // (a block > max_block breaks the contract: left as is)
                unsigned slot = atomicAdd(big_count, 1u);
                big_list[slot] = b;
            }
        } else {
            k = (int)kk;
        }
    }
    const int kmax = wave_max(k);
    if (kmax == 0) {
        wait_turn();
        pass_turn();
        return;
    }
    const int lastl = (int)((nb - b0 < WAVE ? nb - b0 : WAVE) - 1);
    const int64_t s0 = uni64(s, 0);
    const int64_t e1 = uni64(e, lastl);
    const int64_t total = e1 - s0;
    if (total > PCAP) {
        wait_turn();
        pass_turn();
        if (kmax <= 8) lane_block<8, BALL>(y, s, k);
        else if (kmax <= 16) lane_block<16, BALL>(y, s, k);
        else if (kmax <= 32) lane_block<32, BALL>(y, s, k);
        else lane_block<64, BALL>(y, s, k);
        return;
    }
    const int tot = (int)total;
    // buf[sh + i] = y[s0 + i]: the 16-B pairs inside the range by LDS DMA
    // (all in flight at once, no VGPRs), the unaligned head / odd tail by
    // lane 0.  sh = 1 when y + s0 is not 16-B aligned.
    const double *src = y + s0;
    const int sh = (int)(((uintptr_t)src >> 3) & 1);
    const int npair = (tot - sh) >> 1;
    wait_turn();
    {
        const char *gs = (const char *)(src + sh);
        char *ls = (char *)(buf + 2 * sh);
        for (int p = 0; p * WAVE < npair; ++p) {
            const int i = p * WAVE + lane;
            if (i < npair)
                __builtin_amdgcn_global_load_lds((const void *)(gs + 16 * i),
                                                 (__attribute__((address_space(3))) void *)(ls + 1024 * p),
                                                 16, 0, 0);
        }
        if (lane == 0) {
            if (sh) buf[1] = src[0];
            if ((tot - sh) & 1) buf[sh + tot - 1] = src[tot - 1];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (W == 1) {
        __syncthreads();
    } else {
        // the wave reads only its own buffer: its DMA writes are complete at
        // vmcnt(0), and its own LDS accesses execute in order
        pass_turn();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const int off = (k > 0) ? (int)(s - s0) + sh : 0;
    if (kmax <= 8) lane_block_lds<8, 8, BALL, THR>(buf, off, k, lane);
    else if (kmax <= 16) lane_block_lds<16, 16, BALL, THR>(buf, off, k, lane);
    else if (kmax <= 32) lane_block_lds<32, 32, BALL, THR>(buf, off, k, lane);
    else if (kmax <= 40) lane_block_lds<64, 40, BALL, THR>(buf, off, k, lane);
    else if (kmax <= 48) lane_block_lds<64, 48, BALL, THR>(buf, off, k, lane);
    else if (kmax <= 56) lane_block_lds<64, 56, BALL, THR>(buf, off, k, lane);
    else lane_block_lds<64, 64, BALL, THR>(buf, off, k, lane);
    if constexpr (W == 1) __syncthreads();
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // out: 16-B write-through (sc1) stores of the aligned pairs -- the bytes
    // leave L2 while other waves still compute, instead of as dirty lines at
    // the kernel's end (measured -2.8 us at C2) -- and the unaligned head /
    // odd tail by lane 0
    double *dst = y + s0 + sh;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(dst, 0, npair * 16, 0x00020000);
    constexpr int SB = 8;   // LDS reads in flight per lane before the stores
    for (int c0 = 0; c0 < npair; c0 += SB * WAVE) {
        double2 t[SB];
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const int p = c0 + q * WAVE + lane;
            t[q] = *(const double2 *)&buf[2 * sh + 2 * (p < npair ? p : 0)];
        }
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const int p = c0 + q * WAVE + lane;
            if (p < npair)
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(HIP_vector_type<unsigned, 4>::Native_vec_, t[q]), rs,
                    16 * p, 0, 16);
        }
    }
    if (lane == 0) {
        if (sh) y[s0] = buf[1];
        if ((tot - sh) & 1) y[s0 + tot - 1] = buf[sh + tot - 1];
    }
}

// (64 W, 2): at most 256 VGPRs so two waves fit per SIMD -- the whole C2 grid
// (~6 waves per CU) is then resident at once.
template <bool BALL, int W, bool THR = false>
__global__ __launch_bounds__(64 * W, 2) void proj_lds_kernel(double *__restrict__ y,
                                                          const int64_t *__restrict__ starts,
                                                          int64_t nb, int64_t n,
                                                          int64_t *__restrict__ big_list,
                                                          unsigned *__restrict__ big_count,
                                                          int allow_big,
                                                          const double *__restrict__ gate) {
    __shared__ __attribute__((aligned(16))) double buf[W][PBUF];
    __shared__ int landed;
    // gated launch (the x-space BB engine, xbb.hip): run only when *gate == 1
    // (its STEP mode); the big-block kernels then find an empty list too
    if (gate && *gate != 1.0) return;
    const int wv = (W == 1) ? 0 : (int)(threadIdx.x / WAVE);
    const int lane = (W == 1) ? (int)threadIdx.x : (int)(threadIdx.x % WAVE);
    if constexpr (W > 1) {
        if (threadIdx.x == 0) landed = 0;
        __syncthreads();
    }
    lds_group<BALL, W, THR>(y, starts, nb, n, big_list, big_count, allow_big, buf[wv], &landed,
                            (int64_t)blockIdx.x * W + wv, wv, lane);
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

// Blocks longer than LDS_MAX (the reference's stress shapes go to 1e6 in one
// block, python/experiments/test_stress_proj_simplex.py:24-44): the whole
// chip sorts them -- every element of such a block keyed (value, block id),
// sorted by value descending then stably by block id (rocPRIM radix sorts:
// each block's values contiguous, in the reference's std::sort(greater)
// order) -- then one workgroup per block runs the reference's chain on its
// sorted run (S_i += u_i in order, the test at every i with the reference's
// division) only until it is settled: the exact e_i = (i+1) u_i + 1 - S_i is
// non-increasing, so once the computed e_i < -margin (margin >= every rounding
// error of the chain, as chain_steps) no later i passes; and writes
// y = max(lambda + y, 0).  The ball variant clamps first (ball_prepass,
// python/c_extensions/proj_simplex.h:50-74) and skips a block whose clamped
// sum is <= 1.
template <bool BALL>
__global__ __launch_bounds__(HUGE_THREADS) void proj_huge_fill(
    double *__restrict__ y, const int64_t *__restrict__ starts, int64_t nb, int64_t n,
    const int64_t *__restrict__ big_list, const unsigned *__restrict__ big_count,
    double *__restrict__ keys, int32_t *__restrict__ ids) {
    __shared__ int64_t scr[SCRATCH_WORDS];
    // (every other element: key 0.0, id 0x7F7F7F7F by the launcher's memsets,
    // so it sorts after every huge block)
    const unsigned cnt = *big_count;
    for (unsigned idx = blockIdx.x; idx < cnt; idx += gridDim.x) {
        const int64_t b = big_list[idx];
        const int64_t s = starts[b];
        const int64_t k = block_end(starts, nb, b, n) - s;
        if (k <= LDS_MAX) continue;
        if (BALL && !ball_prepass(y + s, k, scr)) continue;   // clamped in place, done
        for (int64_t j = threadIdx.x; j < k; j += HUGE_THREADS) {
            keys[s + j] = y[s + j];
            ids[s + j] = (int32_t)b;
        }
    }
}

template <bool BALL>
__global__ __launch_bounds__(HUGE_THREADS) void proj_huge_apply(
    double *__restrict__ y, const int64_t *__restrict__ starts, int64_t nb, int64_t n,
    const int64_t *__restrict__ big_list, const unsigned *__restrict__ big_count,
    const double *__restrict__ u_all, const int32_t *__restrict__ ids) {
    __shared__ double lam_sh;
    __shared__ int64_t pos_sh;
    const unsigned cnt = *big_count;
    for (unsigned idx = blockIdx.x; idx < cnt; idx += gridDim.x) {
        const int64_t b = big_list[idx];
        const int64_t s = starts[b];
        const int64_t k = block_end(starts, nb, b, n) - s;
        if (k <= LDS_MAX) continue;
        if (threadIdx.x == 0) {
            // this block's sorted run: the first id >= b
            int64_t lo = 0, hi = n;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ids[mid] < (int32_t)b) lo = mid + 1;
                else hi = mid;
            }
            pos_sh = lo;
        }
        __syncthreads();
        const int64_t pos = pos_sh;
        const bool active = pos < n && ids[pos] == (int32_t)b;   // ball: not skipped
        if (active && threadIdx.x == 0) {
            const double *u = u_all + pos;
            const double Mx = fmax(fabs(u[0]), fabs(u[k - 1]));
            const double kk = (double)k;
            const double margin = kk * 0x1p-49 * (1. + 2. * kk * Mx);
            double run = u[0];
            double lam = 1. - run;                      // proj_simplex.h:27-28
            for (int64_t i = 1; i < k; ++i) {
                run = run + u[i];
                const double tmp = (1. - run) / ((double)i + 1.);
                if (u[i] + tmp > 0) lam = tmp;          // the last i that passes wins
                const double E = __builtin_fma((double)i + 1., u[i], 1. - run);
                if (E < -margin) break;                 // settled: no later i passes
            }
            lam_sh = lam;
        }
        __syncthreads();
        if (active) {
            const double lam = lam_sh;
            for (int64_t j = threadIdx.x; j < k; j += HUGE_THREADS) {
                double o = y[s + j];
                if (BALL) o = (o < 0.0) ? 0.0 : o;
                y[s + j] = relu_ref(lam + o);
            }
        }
        __syncthreads();
    }
}

// ---- sort-free path (bsls_proj_multi_*_fast: 1e-12 contract, not bit-identical) ----
//
// With tau = -lambda the reference's result solves sum_j max(y_j - tau, 0) = 1,
// and for ANY subset A of the block tau >= (sum_A y - 1)/|A| (since
// sum_A (y - tau) <= sum max(y - tau, 0) = 1), with equality at the
// reference's top-(rho + 1) set.  Newton from the left on that convex,
// piecewise-linear function: tau_0 = max - 1 (the set {max}),
// A_{t+1} = {y in A_t : y > tau_t} (the max always stays),
// tau_{t+1} = (sum_{A_{t+1}} y - 1)/|A_{t+1}|.  The sets only shrink and tau
// never overshoots, so the first pass that removes nothing has the
// reference's set: lambda = (1 - sum_A y)/|A|, the reference's expression at
// rho = |A| - 1 (proj_simplex.h:27-31), its members summed in another order
// (per lane, then a DPP tree) -- ulps of the sum, no sort, no S_i chain.
// Passes (C2): 5 * N(0,1) blocks 1-2 (tau_0 is usually exact), U[0,1) ~5.
// A set of one element (rho = 0) reproduces 1 - u_0 bit for bit.
//
// Lane mapping: LPB lanes per block, 64 / LPB consecutive blocks per wave;
// lane (g, j) holds entries j, j + LPB, ... of block g in registers (EB
// slots, the wave's bucket), so the reductions are DPP steps inside a quad /
// half-row and a C2 wave (16 blocks) is ~4 KB of contiguous input: 6250 waves,
// one resident round at <= 64 VGPRs.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    return __hiloint2double(dpp_i<CTRL>(__double2hiint(v)), dpp_i<CTRL>(__double2loint(v)));
}
// sum / max over the LPB lanes of a group (xor 1, xor 2 in the quad, then the
// half-row mirror); every lane ends with the same bits (a + b == b + a)
// (16: then the row mirror, lane i <-> 15 - i, adds the other half-row)
template <int LPB>
__device__ __forceinline__ double grp_sum_d(double v) {
    if constexpr (LPB >= 2) v += dpp_d<0xB1>(v);
    if constexpr (LPB >= 4) v += dpp_d<0x4E>(v);
    if constexpr (LPB >= 8) v += dpp_d<0x141>(v);
    if constexpr (LPB >= 16) v += dpp_d<0x140>(v);
    return v;
}
template <int LPB>
__device__ __forceinline__ int grp_sum_i(int v) {
    if constexpr (LPB >= 2) v += dpp_i<0xB1>(v);
    if constexpr (LPB >= 4) v += dpp_i<0x4E>(v);
    if constexpr (LPB >= 8) v += dpp_i<0x141>(v);
    if constexpr (LPB >= 16) v += dpp_i<0x140>(v);
    return v;
}
template <int LPB>
__device__ __forceinline__ double grp_max_d(double v) {
    double u;
    if constexpr (LPB >= 2) { u = dpp_d<0xB1>(v); v = (u > v) ? u : v; }
    if constexpr (LPB >= 4) { u = dpp_d<0x4E>(v); v = (u > v) ? u : v; }
    if constexpr (LPB >= 8) { u = dpp_d<0x141>(v); v = (u > v) ? u : v; }
    if constexpr (LPB >= 16) { u = dpp_d<0x140>(v); v = (u > v) ? u : v; }
    return v;
}

// the largest double below x (finite x)
__device__ __forceinline__ double next_down(double x) {
    const long long b = __double_as_longlong(x);
    if (x == 0.0) return -4.9406564584124654e-324;
    return __longlong_as_double(x > 0.0 ? b - 1 : b + 1);
}

__device__ __forceinline__ double buf_ld(const __amdgpu_buffer_rsrc_t &rs, int off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
}

template <int LPB, int EB, bool BALL>
__device__ __forceinline__ void thr_solve(int64_t s, int64_t s0, int k, int j,
                                          const __amdgpu_buffer_rsrc_t &rs) {
    constexpr double PAD = -1.7976931348623157e308;   // below every entry, finite
    // every access through the wave's buffer resource: one offset register
    // (the block's start + j), slot e at + 8 LPB e (folded into the
    // instruction); ne = this lane's live slots
    const int base = (int)(s - s0 + j) * 8;
    const int ne = (k > j) ? (k - j + LPB - 1) / LPB : 0;
    double v[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) {
        const double t = buf_ld(rs, base + 8 * LPB * e);   // past the range: 0
        v[e] = (e < ne) ? t : PAD;
    }
    bool need = true;
    if constexpr (BALL) {
        // proj_simplex.h:56-64: clamp the negatives, project iff the rest sums > 1
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < EB; ++e) {
            const bool ok = e < ne;
            v[e] = (ok & (v[e] < 0.0)) ? 0.0 : v[e];
            acc += ok ? v[e] : 0.0;
        }
        need = grp_sum_d<LPB>(acc) > 1.0;
    }
    double lam = 0.0;
    if (!BALL || __builtin_amdgcn_ballot_w64(need && k > 0)) {
        double M = v[0];
#pragma unroll
        for (int e = 1; e < EB; ++e) M = (v[e] > M) ? v[e] : M;
        M = grp_max_d<LPB>(M);
        // tau stays below the max (clamped to the next double down: only a
        // |y| ~ 1e12+ rounding could reach it), so the max never leaves the set
        const double Mdn = next_down(M);
        double tau = fmin(M - 1.0, Mdn);
        double cprev = 1.0;   // tau_0 is the tau of the set {max}
        double S = M, c = 1.0;
        for (int pass = 0; pass <= LPB * EB; ++pass) {
            double sl = 0.0, cl = 0.0;
#pragma unroll
            for (int e = 0; e < EB; ++e) {
                // branch-free and mask-free: an entry leaving the set becomes
                // PAD in v (the sets only shrink, and PAD never passes again);
                // sum and count by a 0 / 1 factor (fma: one rounding, = the add)
                const bool keep = v[e] > tau;
                v[e] = keep ? v[e] : PAD;
                const double f = keep ? 1.0 : 0.0;
                sl = __builtin_fma(f, v[e], sl);
                cl += f;
            }
            S = grp_sum_d<LPB>(sl);
            c = grp_sum_d<LPB>(cl);
            const bool more = (k > 0) & need & (c != cprev);
            cprev = c;
            tau = fmin((S - 1.0) / c, Mdn);
            if (!__builtin_amdgcn_ballot_w64(more)) break;
        }
        lam = (1. - S) / c;
    }
    // out: the entries read again (the passes overwrote the dropped ones; the
    // lines are still in the caches), padding slots' offsets past the end so
    // the hardware drops their stores (no per-slot branch)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int e = 0; e < EB; ++e) {
        double o = buf_ld(rs, base + 8 * LPB * e);
        if (BALL) o = (o < 0.0) ? 0.0 : o;
        const double r = need ? relu_ref(lam + o) : o;
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(HIP_vector_type<unsigned, 2>::Native_vec_, r), rs,
            (e < ne) ? base + 8 * LPB * e : 0x7FFFFFF0, 0, 0);
    }
}

// One wave: blocks b0 .. b0 + 64/LPB - 1 (block ends from the same coalesced
// read of starts); blocks > SMALL_MAX go to the big list as in lds_group.
// at least BSLS_PROJ_MINW waves per SIMD (<= 512 / MINW VGPRs): the C2 grid
// (6250 waves at LPB 4) must be resident in one round -- at 73 VGPRs (six
// waves per SIMD, 6144 slots) 106 waves ran as a second round
#ifndef BSLS_PROJ_MINW
#define BSLS_PROJ_MINW 8
#endif
template <bool BALL, int LPB>
__global__ __launch_bounds__(256, BSLS_PROJ_MINW) void proj_thr_kernel(double *__restrict__ y,
                                                      const int64_t *__restrict__ starts,
                                                      int64_t nb, int64_t n,
                                                      int64_t *__restrict__ big_list,
                                                      unsigned *__restrict__ big_count,
                                                      int allow_big,
                                                      const double *__restrict__ gate) {
    static_assert(LPB == 2 || LPB == 4 || LPB == 8, "lanes per block");
    constexpr int BPW = WAVE / LPB;
    if (gate && *gate != 1.0) return;
    const int lane = lane_id();
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    const int64_t b0 = wave * BPW;
    if (b0 >= nb) return;
    const int g = lane / LPB, j = lane % LPB;
    long long st = (long long)n;
    if (lane <= BPW && b0 + lane < nb) st = (long long)starts[b0 + lane];
    const int64_t s = (int64_t)__shfl(st, g, WAVE);
    const int64_t e = (int64_t)__shfl(st, g + 1, WAVE);
    const int64_t b = b0 + g;
    int k = 0;
    if (b < nb) {
        const int64_t kk = e - s;
        if (kk > SMALL_MAX) {
            if (allow_big && j == 0) {   // (a block > max_block breaks the contract: left as is)
                const unsigned slot = atomicAdd(big_count, 1u);
                big_list[slot] = b;
            }
        } else {
            k = (int)kk;
        }
    }
    const int kmax = wave_max(k);
    if (kmax == 0) return;
    // the wave's range [s0, e1): its first block's start to its last block's end
    // (read into scalar registers: a buffer resource built from VGPRs becomes
    // a waterfall loop around every store)
    const int64_t s0 = uni64((int64_t)st, 0);
    const int nbw = __builtin_amdgcn_readfirstlane((int)((nb - b0 < BPW) ? nb - b0 : BPW));
    const int64_t e1 = uni64((int64_t)st, nbw);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(y + s0, 0, (int)((e1 - s0) * 8), 0x00020000);
    const int E = (kmax + LPB - 1) / LPB;
    if (E <= 4) thr_solve<LPB, 4, BALL>(s, s0, k, j, rs);
    else if (E <= 8) thr_solve<LPB, 8, BALL>(s, s0, k, j, rs);
    else if constexpr (LPB <= 4) {
        if (E <= 12) thr_solve<LPB, 12, BALL>(s, s0, k, j, rs);
        else if (E <= 16) thr_solve<LPB, 16, BALL>(s, s0, k, j, rs);
        else if constexpr (LPB == 2) {
            if (E <= 24) thr_solve<LPB, 24, BALL>(s, s0, k, j, rs);
            else thr_solve<LPB, 32, BALL>(s, s0, k, j, rs);
        }
    }
}

// ---- the pipelined sort-free kernel (the default fast form, round 5) --------
//
// The lane-per-block kernels above load, compute and store in lockstep: C2's
// 100k blocks make 1563 waves, ~1.5 per SIMD, each one long serial chain, so
// nothing overlaps the memory phases (with the compute knocked out the exact
// kernel still takes ~14 us to stream C2, a copy 8).  Here a block gets
// PIPE_LPB = 8 lanes (entry j + 8 e of the block in slot e of its lane j,
// PIPE_EB = 8 slots: blocks of <= 64; longer ones go to the big list as in
// lds_group), a GROUP of 8 consecutive blocks is one wave's unit, and a
// persistent wave walks groups w, w + W, w + 2 W, ... with the next group's
// entries and the block starts of the group after it already in flight while
// it runs Michelot's passes on the current group and stores it: every wave
// keeps loads outstanding through its compute, so HBM stays busy.  A load
// instruction reads 8 runs of 8 consecutive doubles (one per block), a store
// writes them back from registers: no LDS, ~60 VGPRs.
//
// Per pass a lane tests its 8 slots against tau, and the block's sum and
// count of {v > tau} come from three DPP steps inside the 8-lane group
// (grp_sum_*: every lane of the group ends with the same bits).  tau starts
// at max(M - 1, (S - 1) / k) -- the thresholds of the sets {max} and of the
// whole block, both lower bounds of the projection's (thr_solve's comment) --
// so U[0,1) blocks of ~32 take ~3-4 passes and 5 N(0,1) blocks 1-2.  The
// entries stay unchanged in registers (tau only grows, so {v > tau} shrinks
// by itself) and the output is relu(lambda + v) from them: lambda = (1 -
// S) / c, the reference's expression at rho = c - 1 with its members summed
// in another order (1e-12 contract, as thr_solve).
#ifndef BSLS_PIPE_LPB
#define BSLS_PIPE_LPB 8   // lanes per block (4, 8 or 16; A/B variant builds)
#endif
#ifndef BSLS_PIPE_STORE_AUX
#define BSLS_PIPE_STORE_AUX 16   // the stores' cache policy: sc1 (write-through); 0 plain
#endif
#ifndef BSLS_PIPE_LDS_TRIM
#define BSLS_PIPE_LDS_TRIM 0   // 1: the LDS variant skips its loads past the group's range
#endif
#ifndef BSLS_PIPE_KO
#define BSLS_PIPE_KO 0    // 1: no threshold passes (knock-out timing build, results wrong)
#endif
constexpr int PIPE_LPB = BSLS_PIPE_LPB, PIPE_EB = 64 / PIPE_LPB, PIPE_BPG = WAVE / PIPE_LPB;

struct PipeGroup {
    __amdgpu_buffer_rsrc_t rs;   // the group's range [s0, e1) of y (scalar registers)
    int base;                    // this lane's byte offset of its slot 0
    int k;                       // this lane's block length (0: none, or a big block)
    int len;                     // e1 - s0 (wave-uniform; clamped to 2^30)
};

// lanes 0 .. PIPE_BPG: the starts of group q's blocks and the end of its last
// (n past the last block).  One unconditional load per lane at a clamped
// index: a load under a branch would make the count of outstanding memory
// operations path-dependent, and the compiler's waits then conservative.
__device__ __forceinline__ long long pipe_meta(const int64_t *__restrict__ starts, int64_t nb,
                                               int64_t n, int64_t q, int lane) {
    const int64_t b = q * PIPE_BPG + lane;
    const long long v = (long long)starts[b < nb ? b : nb - 1];
    return (lane <= PIPE_BPG && b < nb) ? v : (long long)n;
}

// group q's blocks from its starts (BIG: blocks > SMALL_MAX go to the big
// list, once -- `real` is false for the clamped copy a wave loads past its
// last group)
template <bool BIG>
__device__ __forceinline__ PipeGroup pipe_setup(double *y, long long st, int64_t q, int64_t nb,
                                                int64_t *__restrict__ big_list,
                                                unsigned *__restrict__ big_count, bool real,
                                                int lane) {
    const int g = lane / PIPE_LPB, j = lane % PIPE_LPB;
    const int64_t s = (int64_t)__shfl(st, g, WAVE);
    const int64_t e = (int64_t)__shfl(st, g + 1, WAVE);
    const int64_t b = q * PIPE_BPG + g;
    const int64_t kk = e - s;
    const bool big = kk > SMALL_MAX;
    if constexpr (BIG) {
        if (big && real && b < nb && j == 0) {   // (a block > max_block breaks the contract: left as is)
            const unsigned slot = atomicAdd(big_count, 1u);
            big_list[slot] = b;
        }
    }
    // the range in scalar registers (a resource built from VGPRs becomes a
    // waterfall loop around every access); the host keeps it < 2 GB
    const int64_t s0 = uni64((int64_t)st, 0);
    const int nbw = __builtin_amdgcn_readfirstlane(
        (int)((nb - q * PIPE_BPG < PIPE_BPG) ? nb - q * PIPE_BPG : PIPE_BPG));
    const int64_t e1 = uni64((int64_t)st, nbw);
    PipeGroup G;
    G.rs = __builtin_amdgcn_make_buffer_rsrc(y + s0, 0, (int)((e1 - s0) * 8), 0x00020000);
    G.base = (int)(s - s0 + j) * 8;
    G.k = (b < nb && !big) ? (int)kk : 0;
    G.len = (int)((e1 - s0) < ((int64_t)1 << 30) ? e1 - s0 : ((int64_t)1 << 30));
    return G;
}

// (slots past the block read the next block's entries or, past the range, 0:
// masked by pipe_solve)
__device__ __forceinline__ void pipe_load(const PipeGroup &G, double (&v)[PIPE_EB]) {
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e) v[e] = buf_ld(G.rs, G.base + 8 * PIPE_LPB * e);
}

struct PipeOut {
    bool need;     // project (the ball variant: the clamped block sums > 1)
    double lam;    // the reference's lambda: y <- max(lambda + y, 0)
    int ne;        // this lane's live slots
};

// Michelot's passes on this lane's slots of its block (v: the entries, slots
// past the block anything -- they become PAD; the ball variant clamps them)
template <bool BALL>
__device__ __forceinline__ PipeOut pipe_threshold(int k, double (&v)[PIPE_EB], int j) {
    constexpr double PAD = -1.7976931348623157e308;   // below every entry, finite
    const int ne = (k > j) ? (k - j + PIPE_LPB - 1) / PIPE_LPB : 0;
    double S = 0.0;
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e) {
        const bool ok = e < ne;
        if (BALL) v[e] = (ok & (v[e] < 0.0)) ? 0.0 : v[e];   // proj_simplex.h:56-64
        S += ok ? v[e] : 0.0;
        v[e] = ok ? v[e] : PAD;
    }
    S = grp_sum_d<PIPE_LPB>(S);
    const bool need = !BALL || S > 1.0;
    // the slots any lane of the wave holds (wave-uniform: past them every
    // slot is padding, skipped by a scalar branch instead of computed)
    int nslot = 0;
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e) nslot += __builtin_amdgcn_ballot_w64(ne > e) != 0;
    double lam = 0.0;
    if (__builtin_amdgcn_ballot_w64(need && k > 0)) {
        double M = v[0];
#pragma unroll
        for (int e = 1; e < PIPE_EB; ++e)
            if (e < nslot) M = (v[e] > M) ? v[e] : M;
        // a third lower bound: the threshold of the set of the lanes' maxima
        // (min(k, LPB) members -- any subset's threshold is one).  U[0,1)
        // blocks of ~32: ~0.68 where the whole block's is ~0.47, one pass less
        const double SL = grp_sum_d<PIPE_LPB>(ne > 0 ? M : 0.0);
        const double kl = (double)(k < PIPE_LPB ? k : PIPE_LPB);
        M = grp_max_d<PIPE_LPB>(M);
        // tau stays below the max (clamped to the next double down: only a
        // |y| ~ 1e12+ rounding could reach it), so the max never leaves the set
        const double Mdn = next_down(M);
        const double kd = (double)k;
        // (one division: the larger of the two set thresholds by a cross
        // product, kd and kl > 0 -- a rounding tie picks either, both bounds)
        const bool lm = (SL - 1.0) * kd > (S - 1.0) * kl;
        const double t_set = (lm ? SL - 1.0 : S - 1.0) / (lm ? kl : kd), t_max = M - 1.0;
        const bool from_set = t_set >= t_max;
        double tau = from_set ? t_set : t_max;
        // the set tau was taken from: the lanes' maxima need not be {v > t_lm},
        // so no stop after pass 1 from there
        double cprev = from_set ? (lm ? -1.0 : kd) : 1.0;
        tau = fmin(tau, Mdn);
        double c = cprev;
        for (int pass = 0; pass <= (BSLS_PIPE_KO ? -1 : PIPE_LPB * PIPE_EB); ++pass) {
            double sl = 0.0, cl = 0.0;
#pragma unroll
            for (int e = 0; e < PIPE_EB; ++e) {
                if (e >= nslot) break;
                // sum and count by a 0 / 1 factor (fma: one rounding, = the add)
                const double f = (v[e] > tau) ? 1.0 : 0.0;
                sl = __builtin_fma(f, v[e], sl);
                cl += f;
            }
            S = grp_sum_d<PIPE_LPB>(sl);
            c = grp_sum_d<PIPE_LPB>(cl);
            const bool more = (k > 0) & need & (c != cprev);
            cprev = c;
            tau = fmin((S - 1.0) / c, Mdn);
            if (!__builtin_amdgcn_ballot_w64(more)) break;
        }
        lam = (1. - S) / c;
    }
    return PipeOut{need, lam, ne};
}

template <bool BALL>
__device__ __forceinline__ void pipe_solve(const PipeGroup &G, double (&v)[PIPE_EB], int j) {
    const PipeOut o = pipe_threshold<BALL>(G.k, v, j);
    const bool need = o.need;
    const double lam = o.lam;
    const int ne = o.ne;
    // out from the registers, write-through (sc1: the lines leave L2 while
    // other waves still compute, instead of as ~26 MB of dirty lines the next
    // kernel boundary waits for -- as lds_group's store-out); padding slots'
    // offsets past the range, so the hardware drops their stores (no per-slot
    // branch)
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e) {
        const double r = need ? relu_ref(lam + v[e]) : v[e];
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(HIP_vector_type<unsigned, 2>::Native_vec_, r), G.rs,
            (e < ne) ? G.base + 8 * PIPE_LPB * e : 0x7FFFFFF0, 0, BSLS_PIPE_STORE_AUX);
    }
}

// One wave: PIPE_G consecutive groups, straight-line (unrolled at compile
// time): the starts of all of them in one load, then the entries of every
// group, then the passes and stores group by group -- so a wave has all its
// bytes in flight at once and computes on the first group while the others
// land (round 5, measured at C2: one group ahead per step was slower than no
// pipelining at all, 23.9 against 19.1 us -- what the kernel is short of is
// bytes in flight per CU, not overlap inside a wave).  Straight-line code keeps
// the compiler's vmcnt waits exact; every memory operation is unconditional:
// a group past the last is a clamped copy with k = 0, whose stores the
// hardware drops.
template <bool BALL, bool BIG, int PIPE_G>
__global__ __launch_bounds__(256, 2) void proj_pipe_kernel(double *__restrict__ y,
                                                          const int64_t *__restrict__ starts,
                                                          int64_t nb, int64_t n,
                                                          int64_t *__restrict__ big_list,
                                                          unsigned *__restrict__ big_count,
                                                          const double *__restrict__ gate) {
    if (gate && *gate != 1.0) return;
    const int lane = lane_id(), j = lane % PIPE_LPB;
    const int64_t ngrp = (nb + PIPE_BPG - 1) / PIPE_BPG;
    const int64_t q0 = (int64_t)__builtin_amdgcn_readfirstlane(
                           (int)(blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE)) * PIPE_G;
    if (q0 >= ngrp) return;
    long long st[PIPE_G];
#pragma unroll
    for (int h = 0; h < PIPE_G; ++h)
        st[h] = pipe_meta(starts, nb, n, (q0 + h < ngrp) ? q0 + h : ngrp - 1, lane);
    asm volatile("" ::: "memory");
    PipeGroup P[PIPE_G];
    double v[PIPE_G][PIPE_EB];
#pragma unroll
    for (int h = 0; h < PIPE_G; ++h) {
        const int64_t q = q0 + h;
        const bool real = q < ngrp;
        P[h] = pipe_setup<BIG>(y, st[h], real ? q : ngrp - 1, nb, big_list, big_count, real, lane);
        if (!real) P[h].k = 0;
        pipe_load(P[h], v[h]);
    }
    // (keeps the compiler from sinking those loads past the passes)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < PIPE_G; ++h) pipe_solve<BALL>(P[h], v[h], j);
}

// The same group through LDS (round 5 A/B, BSLS_PROJ_PIPE_LDS): the group's
// range [s0, e1) comes in by 8-B coalesced loads (lane l, load e: entry 64 e +
// l -- 512 contiguous bytes per wave instruction, where the block-aligned
// loads read 8 runs of 64 B), goes to the lanes' block slots through the
// wave's own 4-KB LDS buffer, and back out the same way (write-through).  A
// group longer than PIPE_STAGE entries (big blocks inside) takes the direct
// path.  Entries of big blocks inside the range go back unchanged (the big-
// block kernel that follows in the stream projects them).
// PIPE_STAGE: the LDS buffer's entries per wave (a group's range up to it
// goes through LDS); BSLS_PIPE_STAGE overrides it for the A/B builds
#ifndef BSLS_PIPE_STAGE
#define BSLS_PIPE_STAGE (PIPE_BPG * 64)
#endif
constexpr int PIPE_STAGE = BSLS_PIPE_STAGE, PIPE_NL = PIPE_STAGE / WAVE;
static_assert(PIPE_STAGE % WAVE == 0, "the LDS stage is whole wave rows");

// the group's range by coalesced 8-B loads (lane l, load e: entry 64 e + l;
// past the range the hardware returns 0)
__device__ __forceinline__ void lds_range_load(const PipeGroup &G, double (&t)[PIPE_NL], int lane) {
#pragma unroll
    for (int e = 0; e < PIPE_NL; ++e)
        t[e] = (BSLS_PIPE_LDS_TRIM && WAVE * e >= G.len) ? 0.0 : buf_ld(G.rs, (WAVE * e + lane) * 8);
}

// t to the wave's LDS buffer, the lanes' block slots out of it, Michelot,
// the results back into the slots and the range out by coalesced
// write-through stores (a wave's own LDS accesses execute in order: no
// barrier, and the next group may reuse the buffer right after)
template <bool BALL>
__device__ __forceinline__ void lds_group(const PipeGroup &G, const double (&t)[PIPE_NL],
                                          double *buf, int lane, int j) {
#pragma unroll
    for (int e = 0; e < PIPE_NL; ++e) buf[WAVE * e + lane] = t[e];
    double v[PIPE_EB];
    const int b0 = min(G.base / 8, PIPE_STAGE);
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e) v[e] = buf[b0 + PIPE_LPB * e];
    const PipeOut o = pipe_threshold<BALL>(G.k, v, j);
#pragma unroll
    for (int e = 0; e < PIPE_EB; ++e)
        if (e < o.ne) buf[b0 + PIPE_LPB * e] = o.need ? relu_ref(o.lam + v[e]) : v[e];
#pragma unroll
    for (int e = 0; e < PIPE_NL; ++e) {
        const int i = WAVE * e + lane;
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(HIP_vector_type<unsigned, 2>::Native_vec_, buf[i]), G.rs,
            i < G.len ? i * 8 : 0x7FFFFFF0, 0, BSLS_PIPE_STORE_AUX);
    }
}

// one group either way: through LDS when its range fits the buffer, else
// straight into the lanes' registers (pipe_load / pipe_solve)
template <bool BALL>
__device__ __forceinline__ void pipe_group_one(const PipeGroup &G, double *buf, int lane, int j) {
    if (G.len > PIPE_STAGE) {
        double v[PIPE_EB];
        pipe_load(G, v);
        pipe_solve<BALL>(G, v, j);
        return;
    }
    double t[PIPE_NL];
    lds_range_load(G, t, lane);
    lds_group<BALL>(G, t, buf, lane, j);
}

// The same group through LDS (round 5, the default fast form; BSLS_PROJ_PIPE_LDS):
// the group's range [s0, e1) comes in by 8-B coalesced loads (512 contiguous
// bytes per wave instruction, where the block-aligned loads read 8 runs of
// 64 B), goes to the lanes' block slots through the wave's own LDS buffer,
// and back out the same way (write-through).  A group longer than
// PIPE_STAGE entries (big blocks inside) takes the direct path.  Entries of
// big blocks inside the range go back unchanged (the big-block kernel that
// follows in the stream projects them).
template <bool BALL, bool BIG>
__global__ __launch_bounds__(256, 2) void proj_pipe_lds_kernel(double *__restrict__ y,
                                                              const int64_t *__restrict__ starts,
                                                              int64_t nb, int64_t n,
                                                              int64_t *__restrict__ big_list,
                                                              unsigned *__restrict__ big_count,
                                                              const double *__restrict__ gate) {
    // (PIPE_STAGE + 64 entries: a lane's slot reads b0 + 8 e, b0 <= PIPE_STAGE,
    // stay inside its wave's buffer with no per-slot clamp)
    __shared__ double stage[4][PIPE_STAGE + WAVE];
    if (gate && *gate != 1.0) return;
    const int lane = lane_id(), j = lane % PIPE_LPB, wv = (int)(threadIdx.x / WAVE);
    const int64_t ngrp = (nb + PIPE_BPG - 1) / PIPE_BPG;
    const int64_t q = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x / WAVE) + wv));
    if (q >= ngrp) return;
    const PipeGroup G = pipe_setup<BIG>(y, pipe_meta(starts, nb, n, q, lane), q, nb, big_list,
                                        big_count, true, lane);
    pipe_group_one<BALL>(G, stage[wv], lane, j);
}

struct ProjWork {
    unsigned *count;
    int64_t *list;
    double *K0, *K1;      // huge path: sort keys (values), double-buffered
    int32_t *I0, *I1;     // huge path: block ids
    void *tmp;            // rocPRIM temporary storage
    size_t tmp_bytes;
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
        w.K0 = (double *)(p + off);
        off += align16((size_t)n * 8);
        w.K1 = (double *)(p + off);
        off += align16((size_t)n * 8);
        w.I0 = (int32_t *)(p + off);
        off += align16((size_t)n * 4);
        w.I1 = (int32_t *)(p + off);
        off += align16((size_t)n * 4);
        w.tmp = (void *)(p + off);
        w.tmp_bytes = align16((size_t)n * 4 + ((size_t)1 << 20));
        off += w.tmp_bytes;
    }
    w.bytes = off;
    return w;
}

template <bool BALL>
static int proj_launch(double *y, const int64_t *starts, int64_t nb, int64_t n,
                       int64_t max_block, void *work, size_t work_bytes, hipStream_t st,
                       const double *gate = nullptr, bool fast = false) {
    if (nb <= 0 || n <= 0 || y == nullptr || starts == nullptr) return BSLS_E_ARG;
    if (max_block < 1) return BSLS_E_ARG;
    ProjWork w = proj_layout(work, n, nb, max_block);
    if (work == nullptr || work_bytes < w.bytes) return BSLS_E_WORKSPACE;
    // the big-block list is only used when some block can exceed SMALL_MAX
    // (max_block is the caller's bound on every block length, like the
    // workspace size derived from it): otherwise no reset launch at all
    if (max_block > SMALL_MAX) BSLS_CHECK(hipMemsetAsync(w.count, 0, 16, st));
    // waves per workgroup (BSLS_PROJ_WAVES, A/B): 2, staggered, by default --
    // C2 20.7 -> 20.2 us per launch (HBM-fed batch); 3 is slower (27.9 us:
    // 60 KB of LDS per workgroup leave 512 slots for 521 workgroups, a tail)
    static const int pw = [] {
        const char *e = getenv("BSLS_PROJ_WAVES");
        const int v = e ? atoi(e) : 2;
        return (v == 1 || v == 3) ? v : 2;
    }();
    // the sort-free path: one lane per block (Michelot on the staged block,
    // proj_lds_kernel<BALL, 2, true>) unless BSLS_PROJ_LPB (A/B) asks for
    // proj_thr_kernel's 2 / 4 / 8 lanes per block
    static const int lpb = [] {
        const char *e = getenv("BSLS_PROJ_LPB");
        const int v = e ? atoi(e) : 0;
        return (v == 2 || v == 4 || v == 8) ? v : 0;
    }();
    // the pipelined kernel's groups per wave (BSLS_PROJ_PIPE = 1, 2, 4 or 8,
    // A/B; 0 = the lane-per-block Michelot form below)
    static const int pipe = [] {
        const char *e = getenv("BSLS_PROJ_PIPE");
        const int v = e ? atoi(e) : 1;
        return (v == 0 || v == 1 || v == 2 || v == 4 || v == 8) ? v : 1;
    }();
    const int64_t ngrp = (nb + WAVE - 1) / WAVE;
    // (its group ranges must stay below 2 GB of y: max_block bounds them)
    if (fast && lpb == 0 && pipe > 0 && max_block <= ((int64_t)1 << 24)) {
        const int64_t groups = (nb + PIPE_BPG - 1) / PIPE_BPG;
        const int64_t waves = (groups + pipe - 1) / pipe;
        const unsigned grid = (unsigned)((waves + 3) / 4);
        const bool big = max_block > SMALL_MAX;
#define BSLS_PIPE_LAUNCH(G)                                                                     \
    do {                                                                                        \
        if (big)                                                                                \
            proj_pipe_kernel<BALL, true, G><<<grid, 256, 0, st>>>(y, starts, nb, n, w.list,     \
                                                                  w.count, gate);               \
        else                                                                                    \
            proj_pipe_kernel<BALL, false, G><<<grid, 256, 0, st>>>(y, starts, nb, n, w.list,    \
                                                                   w.count, gate);              \
    } while (0)
        // through LDS (coalesced in and out) by default: C2 17.1 against 20.5
        // us for the direct form (round 5, HBM-fed batch); BSLS_PROJ_PIPE_LDS=0
        // selects the direct form (A/B)
        static const int via_lds = [] {
            const char *e = getenv("BSLS_PROJ_PIPE_LDS");
            return e ? atoi(e) : 1;
        }();
        if (via_lds) {
            const unsigned g1 = (unsigned)((groups + 3) / 4);
            if (big)
                proj_pipe_lds_kernel<BALL, true><<<g1, 256, 0, st>>>(y, starts, nb, n, w.list,
                                                                     w.count, gate);
            else
                proj_pipe_lds_kernel<BALL, false><<<g1, 256, 0, st>>>(y, starts, nb, n, w.list,
                                                                      w.count, gate);
        } else if (pipe == 1) BSLS_PIPE_LAUNCH(1);
        else if (pipe == 2) BSLS_PIPE_LAUNCH(2);
        else if (pipe == 8) BSLS_PIPE_LAUNCH(8);
        else BSLS_PIPE_LAUNCH(4);
#undef BSLS_PIPE_LAUNCH
    } else if (fast && lpb == 0) {
        proj_lds_kernel<BALL, 2, true><<<(unsigned)((ngrp + 1) / 2), 2 * WAVE, 0, st>>>(
            y, starts, nb, n, w.list, w.count, max_block > SMALL_MAX, gate);
    } else if (fast) {
        const int64_t waves = (nb + WAVE / lpb - 1) / (WAVE / lpb);
        const unsigned grid = (unsigned)((waves + 3) / 4);
        if (lpb == 2)
            proj_thr_kernel<BALL, 2><<<grid, 256, 0, st>>>(y, starts, nb, n, w.list, w.count,
                                                          max_block > SMALL_MAX, gate);
        else if (lpb == 8)
            proj_thr_kernel<BALL, 8><<<grid, 256, 0, st>>>(y, starts, nb, n, w.list, w.count,
                                                          max_block > SMALL_MAX, gate);
        else
            proj_thr_kernel<BALL, 4><<<grid, 256, 0, st>>>(y, starts, nb, n, w.list, w.count,
                                                          max_block > SMALL_MAX, gate);
    } else if (pw == 3)
        proj_lds_kernel<BALL, 3><<<(unsigned)((ngrp + 2) / 3), 3 * WAVE, 0, st>>>(
            y, starts, nb, n, w.list, w.count, max_block > SMALL_MAX, gate);
    else if (pw == 2)
        proj_lds_kernel<BALL, 2><<<(unsigned)((ngrp + 1) / 2), 2 * WAVE, 0, st>>>(
            y, starts, nb, n, w.list, w.count, max_block > SMALL_MAX, gate);
    else
        proj_lds_kernel<BALL, 1><<<grid_for(nb, WAVE), WAVE, 0, st>>>(
            y, starts, nb, n, w.list, w.count, max_block > SMALL_MAX, gate);
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
        const int64_t most = n / (LDS_MAX + 1) + 1;
        const int grid = (int)(most < 1024 ? most : 1024);
        BSLS_CHECK(hipMemsetAsync(w.K0, 0, (size_t)n * 8, st));
        BSLS_CHECK(hipMemsetAsync(w.I0, 0x7F, (size_t)n * 4, st));
        proj_huge_fill<BALL><<<grid, HUGE_THREADS, 0, st>>>(y, starts, nb, n, w.list, w.count,
                                                            w.K0, w.I0);
        BSLS_LAUNCH_CHECK();
        // by value (descending), then stably by block id: each huge block's
        // values contiguous and in std::sort(greater) order
        rocprim::double_buffer<double> keys(w.K0, w.K1);
        rocprim::double_buffer<int32_t> ids(w.I0, w.I1);
        size_t need = 0;
        BSLS_CHECK(rocprim::radix_sort_pairs_desc(nullptr, need, keys, ids, (size_t)n, 0, 64, st));
        if (need > w.tmp_bytes) return BSLS_E_WORKSPACE;
        BSLS_CHECK(rocprim::radix_sort_pairs_desc(w.tmp, need, keys, ids, (size_t)n, 0, 64, st));
        const unsigned idbits = 31;   // block ids < 2^31, the filler 0x7F7F7F7F
        need = 0;
        BSLS_CHECK(rocprim::radix_sort_pairs(nullptr, need, ids, keys, (size_t)n, 0, idbits, st));
        if (need > w.tmp_bytes) return BSLS_E_WORKSPACE;
        BSLS_CHECK(rocprim::radix_sort_pairs(w.tmp, need, ids, keys, (size_t)n, 0, idbits, st));
        proj_huge_apply<BALL><<<grid, HUGE_THREADS, 0, st>>>(y, starts, nb, n, w.list, w.count,
                                                             keys.current(), ids.current());
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

int proj_launch_gated(bool ball, double *y, const int64_t *starts, int64_t nb, int64_t n,
                      int64_t max_block, void *work, size_t work_bytes, hipStream_t st,
                      const double *gate, bool fast) {
    return ball ? proj_launch<true>(y, starts, nb, n, max_block, work, work_bytes, st, gate, fast)
                : proj_launch<false>(y, starts, nb, n, max_block, work, work_bytes, st, gate, fast);
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

extern "C" int bsls_proj_multi_simplex_fast(double *d_y, const int64_t *d_starts, int64_t nblocks,
                                            int64_t n, int64_t max_block, void *d_work,
                                            size_t work_bytes, void *stream) {
    return proj_launch<false>(d_y, d_starts, nblocks, n, max_block, d_work, work_bytes,
                              (hipStream_t)stream, nullptr, true);
}

extern "C" int bsls_proj_multi_ball_fast(double *d_y, const int64_t *d_starts, int64_t nblocks,
                                         int64_t n, int64_t max_block, void *d_work,
                                         size_t work_bytes, void *stream) {
    return proj_launch<true>(d_y, d_starts, nblocks, n, max_block, d_work, work_bytes,
                             (hipStream_t)stream, nullptr, true);
}
