// Diagnostic build (never the product): proj_lds_kernel<false>'s LDS path with
// s_memrealtime stamps (100 MHz, chip-global) per wave at
//   T0 start, T1 staged (DMA landed + barrier), T2 sorted + lambda + written
//   to LDS, T3 stores issued, T4 stores complete (extra vmcnt(0) wait)
// plus HW_ID / XCC_ID, to read where a wave's time goes and how the phases of
// different waves overlap.  Read SHARES, not the length (the stamps fence).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC
//        -I include -I block-simplex-least-squares_amd/csrc tools/proj_trace.hip
#include "../block-simplex-least-squares_amd/csrc/proj.hip"

namespace tr {
using namespace bsls;

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ __launch_bounds__(64, 2) void proj_trace_kernel(double *__restrict__ y,
                                                        const int64_t *__restrict__ starts,
                                                        int64_t nb, int64_t n,
                                                        uint64_t *__restrict__ trace) {
    __shared__ __attribute__((aligned(16))) double buf[PBUF];
    const uint64_t t0 = stamp();
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
    const double *src = y + s0;
    const int sh = (int)(((uintptr_t)src >> 3) & 1);
    const int npair = (tot - sh) >> 1;
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
    __syncthreads();
    const uint64_t t1 = stamp();
    const int off = (k > 0) ? (int)(s - s0) + sh : 0;
    if (kmax <= 8) lane_block_lds<8, 8, false>(buf, off, k, lane);
    else if (kmax <= 16) lane_block_lds<16, 16, false>(buf, off, k, lane);
    else if (kmax <= 32) lane_block_lds<32, 32, false>(buf, off, k, lane);
    else if (kmax <= 40) lane_block_lds<64, 40, false>(buf, off, k, lane);
    else if (kmax <= 48) lane_block_lds<64, 48, false>(buf, off, k, lane);
    else if (kmax <= 56) lane_block_lds<64, 56, false>(buf, off, k, lane);
    else lane_block_lds<64, 64, false>(buf, off, k, lane);
    __syncthreads();
    const uint64_t t2 = stamp();
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
    const uint64_t t3 = stamp();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t4 = stamp();
    if (lane == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t *o = trace + 8 * blockIdx.x;
        o[0] = t0; o[1] = t1; o[2] = t2; o[3] = t3; o[4] = t4;
        o[5] = hw; o[6] = xcc; o[7] = (uint64_t)kmax | ((uint64_t)tot << 16);
    }
}
}  // namespace tr

extern "C" float proj_trace(double *y, const double *y0, const int64_t *st, int64_t nb,
                            int64_t n, uint64_t *trace) {
    // each launch on a fresh copy of the input (a projected vector re-projected
    // is the degenerate case: nothing settles early)
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = (int)((nb + 63) / 64);
    (void)hipMemcpyAsync(y, y0, n * 8, hipMemcpyDeviceToDevice, 0);
    tr::proj_trace_kernel<<<grid, 64>>>(y, st, nb, n, trace);
    (void)hipMemcpyAsync(y, y0, n * 8, hipMemcpyDeviceToDevice, 0);
    (void)hipEventRecord(a, 0);
    tr::proj_trace_kernel<<<grid, 64>>>(y, st, nb, n, trace);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f;
}
