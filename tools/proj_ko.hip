// Knock-out timing of the k <= 64 projection kernel after the top-16 change
// (diagnostic build; outputs are wrong for KO != 0).  KO bits:
//   1 no selection network   2 no lambda chain   4 no fallback full sort
//   8 conflict-free (transposed-index) LDS reads instead of buf[off + j]
//  16 no output pass (o[] reads + LDS writes)   32 no staging (skip DMA+stores)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC
//        -I include -I block-simplex-least-squares_amd/csrc tools/proj_ko.hip
#include "../block-simplex-least-squares_amd/csrc/proj.hip"

namespace ko {
using namespace bsls;

template <int N, int KB, int KO>
__device__ __forceinline__ void lane_block(double *buf, int off, int k, int lane) {
    double v[N];
    uint32_t hx = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double t = -INFINITY;
        if (j < KB) t = (KO & 8) ? buf[(j * 64 + lane) % PCAP] : buf[off + j];
        if (KB > 16 && j < KB) {
            const uint32_t h = (uint32_t)((uint64_t)__double_as_longlong(t) >> 32) & 0x7fffffffu;
            hx = (j < k && h > hx) ? h : hx;
        }
        v[j] = (j < k) ? t : -INFINITY;
    }
    double lam = 0.0;
    bool full = true;
    if constexpr (KB > 16) {
        if (!(KO & 1)) Top16<KB>::template run<0>(v);
        const double Mx = __longlong_as_double((long long)(((uint64_t)hx << 32) | 0xffffffffull));
        const double kk = (double)k;
        const double margin = kk * 0x1p-49 * (1. + 2. * kk * Mx);
        Chain c = chain_begin(v, k);
        int depth = 16;
        if (!(KO & 2)) {
            chain_steps<1, 16>(v, k, margin, c);
            if constexpr (KB > 32) {
                if (__builtin_amdgcn_ballot_w64(c.live && k > 16)) {
                    if (!(KO & 1)) Top16<KB - 16>::template run<16>(v);
                    chain_steps<16, 32>(v, k, margin, c);
                    depth = 32;
                }
            }
            lam = chain_lambda(c);
        } else {
            c.live = false;
            lam = v[0] * 0.5 + v[15];
        }
        full = __builtin_amdgcn_ballot_w64(c.live && k > depth) != 0;
    }
    if (full && !(KO & 4)) {
        bitonic_flip<N, KB>(v);
        bool amb;
        lam = lambda_fast<N, KB>(v, k, amb);
        if (__builtin_amdgcn_ballot_w64(amb)) {
            if (amb) lam = lambda_sorted<N, KB>(v, k);
        }
    }
    asm volatile("" ::: "memory");
    if (KO & 16) {
        buf[PCAP + WAVE + 2 + lane] = lam;
        return;
    }
    double o[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) o[j] = (KO & 8) ? buf[(j * 64 + lane) % PCAP] : buf[off + j];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
        const double r = relu_ref(lam + o[j]);
        buf[(j < k) ? ((KO & 8) ? (j * 64 + lane) % PCAP : off + j) : PCAP + WAVE + 2 + lane] = r;
    }
}

template <int KO>
__global__ __launch_bounds__(64, 2) void proj_ko_kernel(double *__restrict__ y,
                                                     const int64_t *__restrict__ starts,
                                                     int64_t nb, int64_t n) {
    __shared__ __attribute__((aligned(16))) double buf[PBUF];
    if (KO & 2048) return;
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
    if (tot > PCAP || kmax > 64) return;
    if (KO & 512) {
        if (KO & 1024) {   // plain streaming copy of the range through registers (x4, sc1 out)
            double *dst = y + s0 + (((uintptr_t)(y + s0) >> 3) & 1);
            const int np = (tot - 1) >> 1;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, np * 16, 0x00020000);
            for (int c0 = 0; c0 < np; c0 += 8 * WAVE) {
                double2 t[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int p = c0 + q * WAVE + lane;
                    t[q] = *(const double2 *)(dst + 2 * (p < np ? p : 0));
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int p = c0 + q * WAVE + lane;
                    t[q].x += 1.0;
                    if (p < np)
                        __builtin_amdgcn_raw_buffer_store_b128(
                            __builtin_bit_cast(HIP_vector_type<unsigned, 4>::Native_vec_, t[q]), rs, 16 * p, 0, 16);
                }
            }
        }
        return;
    }
    const double *src = y + s0;
    const int sh = (int)(((uintptr_t)src >> 3) & 1);
    const int npair = (tot - sh) >> 1;
    if (!(KO & 32)) {
        const char *gs = (const char *)(src + sh);
        char *ls = (char *)(buf + 2 * sh);
        for (int p = 0; p * WAVE < npair; ++p) {
            const int i = p * WAVE + lane;
            if (i < npair)
                __builtin_amdgcn_global_load_lds((const void *)(gs + 16 * i),
                                                 (__attribute__((address_space(3))) void *)(ls + 1024 * p),
                                                 16, 0, (KO & 256) ? 2 : 0);
        }
        if (lane == 0) {
            if (sh) buf[1] = src[0];
            if ((tot - sh) & 1) buf[sh + tot - 1] = src[tot - 1];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int i = lane; i < PBUF; i += 64) buf[i] = (double)(i & 255) * 0.01;
    }
    __syncthreads();
    const int off = (k > 0) ? (int)(s - s0) + sh : 0;
    if (kmax <= 8) lane_block<8, 8, KO>(buf, off, k, lane);
    else if (kmax <= 16) lane_block<16, 16, KO>(buf, off, k, lane);
    else if (kmax <= 32) lane_block<32, 32, KO>(buf, off, k, lane);
    else if (kmax <= 40) lane_block<64, 40, KO>(buf, off, k, lane);
    else if (kmax <= 48) lane_block<64, 48, KO>(buf, off, k, lane);
    else if (kmax <= 56) lane_block<64, 56, KO>(buf, off, k, lane);
    else lane_block<64, 64, KO>(buf, off, k, lane);
    __syncthreads();
    if (KO & 32) {
        if (lane == 0) y[s0] = buf[sh];
        return;
    }
    if (KO & (64 | 128)) {
        // 16-B stores of the aligned pairs (plain, or sc1 write-through by a
        // buffer store), the unaligned head / odd tail by lane 0
        double *dst = y + s0 + sh;
        const int np = (tot - sh) >> 1;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(dst, 0, np * 16, 0x00020000);
        constexpr int SB = 8;
        for (int c0 = 0; c0 < np; c0 += SB * WAVE) {
            double2 t[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int p = c0 + q * WAVE + lane;
                t[q] = *(const double2 *)&buf[2 * sh + 2 * (p < np ? p : 0)];
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int p = c0 + q * WAVE + lane;
                if (p < np) {
                    if (KO & 128) {
                        __builtin_amdgcn_raw_buffer_store_b128(
                            __builtin_bit_cast(HIP_vector_type<unsigned, 4>::Native_vec_, t[q]), rs, 16 * p, 0, 16);
                    } else {
                        *(double2 *)(dst + 2 * p) = t[q];
                    }
                }
            }
        }
        if (lane == 0) {
            if (sh) y[s0] = buf[1];
            if ((tot - sh) & 1) y[s0 + tot - 1] = buf[sh + tot - 1];
        }
        return;
    }
    constexpr int SB = 16;
    for (int c0 = 0; c0 < tot; c0 += SB * WAVE) {
        double t[SB];
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const int i = c0 + q * WAVE + lane;
            t[q] = buf[sh + (i < tot ? i : 0)];
        }
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const int i = c0 + q * WAVE + lane;
            if (i < tot) y[s0 + i] = t[q];
        }
    }
}

__global__ __launch_bounds__(256) void empty256(double *y) {
    __shared__ double buf[4 * PBUF];
    if (threadIdx.x == 999) y[0] = buf[threadIdx.x];
}
__global__ __launch_bounds__(64) void empty64(double *y) {
    __shared__ double buf[PBUF];
    if (threadIdx.x == 999) y[0] = buf[threadIdx.x];
}
__global__ __launch_bounds__(64) void empty64nolds(double *y) {
    if (threadIdx.x == 999) y[0] = 1.0;
}

template <int KO>
static float run(double *y, const double *y0, const int64_t *st, int64_t nb, int64_t n) {
    if (KO >= 4096) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        float best = 1e9f;
        for (int r = 0; r < 10; ++r) {
            (void)hipMemcpyAsync(y, y0, n * 8, hipMemcpyDeviceToDevice, 0);
            (void)hipEventRecord(a, 0);
            if (KO == 4096) empty64<<<1, 64>>>(y);
            if (KO == 8192) empty256<<<391, 256>>>(y);
            if (KO == 12288) empty64nolds<<<1563, 64>>>(y);
            if (KO == 16384) empty64<<<1563, 64>>>(y);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        return best * 1000.f;
    }
    const int grid = (int)((nb + 63) / 64);
    hipEvent_t a[10], b[10];
    float tot = 0.f;
    for (int r = 0; r < 12; ++r) {
        (void)hipMemcpyAsync(y, y0, n * 8, hipMemcpyDeviceToDevice, 0);
        if (r >= 2) { (void)hipEventCreate(&a[r - 2]); (void)hipEventCreate(&b[r - 2]); (void)hipEventRecord(a[r - 2], 0); }
        proj_ko_kernel<KO><<<grid, 64>>>(y, st, nb, n);
        if (r >= 2) (void)hipEventRecord(b[r - 2], 0);
    }
    (void)hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 10; ++r) {
        float ms;
        (void)hipEventElapsedTime(&ms, a[r], b[r]);
        best = ms < best ? ms : best;
        tot += ms;
    }
    return best * 1000.f;
}
}  // namespace ko

extern "C" float proj_ko(int KO, double *y, const double *y0, const int64_t *st, int64_t nb,
                         int64_t n) {
    using namespace ko;
    switch (KO) {
        case 0: return run<0>(y, y0, st, nb, n);
        case 1: return run<1>(y, y0, st, nb, n);
        case 2: return run<2>(y, y0, st, nb, n);
        case 3: return run<3>(y, y0, st, nb, n);
        case 4: return run<4>(y, y0, st, nb, n);
        case 7: return run<7>(y, y0, st, nb, n);
        case 8: return run<8>(y, y0, st, nb, n);
        case 12: return run<12>(y, y0, st, nb, n);
        case 16: return run<16>(y, y0, st, nb, n);
        case 23: return run<23>(y, y0, st, nb, n);
        case 32: return run<32>(y, y0, st, nb, n);
        case 36: return run<36>(y, y0, st, nb, n);
        case 55: return run<55>(y, y0, st, nb, n);
        case 64: return run<64>(y, y0, st, nb, n);
        case 512: return run<512>(y, y0, st, nb, n);
        case 2048: return run<2048>(y, y0, st, nb, n);
        case 4096: return run<4096>(y, y0, st, nb, n);
        case 8192: return run<8192>(y, y0, st, nb, n);
        case 12288: return run<12288>(y, y0, st, nb, n);
        case 16384: return run<16384>(y, y0, st, nb, n);
        case 1536: return run<1536>(y, y0, st, nb, n);
        case 384: return run<384>(y, y0, st, nb, n);
        case 407: return run<407>(y, y0, st, nb, n);
        case 128: return run<128>(y, y0, st, nb, n);
        case 87: return run<87>(y, y0, st, nb, n);
        case 151: return run<151>(y, y0, st, nb, n);
        default: return -1.f;
    }
}
