// ubench_gather.hip -- gather-rate ceilings for the BB SpMVs (design aid, not product).
// G gathers of 8-B elements x[idx[e]] with idx streamed (4 B, coalesced) and summed
// per lane, from (a) global memory (L2-resident table), (b) a table staged into LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

// (a) each lane: PER gathers, idx stored [k][lane] per wave
template <int PER, int U>
__global__ __launch_bounds__(256) void gather_global(const int32_t *__restrict__ idx,
                                                      const double *__restrict__ x,
                                                      double *__restrict__ out, int64_t nlanes) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nlanes) return;
    const int64_t wbase = (t / 64) * 64 * PER + (t % 64);
    double s = 0.0;
    for (int k0 = 0; k0 < PER; k0 += U) {
        int32_t c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = __builtin_nontemporal_load(&idx[wbase + (int64_t)(k0 + u) * 64]);
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = x[c[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u];
    }
    out[t] = s;
}

// (b) table chunk of T doubles staged in LDS by each WG (1024 threads), then PER gathers per lane
template <int PER, int U>
__global__ __launch_bounds__(1024) void gather_lds(const int32_t *__restrict__ idx,
                                                   const double *__restrict__ x, int T,
                                                   double *__restrict__ out, int64_t nlanes) {
    extern __shared__ double tab[];
    for (int i = threadIdx.x; i < T; i += 1024) tab[i] = x[i];
    __syncthreads();
    const int64_t t = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    if (t >= nlanes) return;
    const int64_t wbase = (t / 64) * 64 * PER + (t % 64);
    double s = 0.0;
    for (int k0 = 0; k0 < PER; k0 += U) {
        int32_t c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = __builtin_nontemporal_load(&idx[wbase + (int64_t)(k0 + u) * 64]);
#pragma unroll
        for (int u = 0; u < U; ++u) s += tab[c[u]];
    }
    out[t] = s;
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main() {
    const int64_t G = 16 << 20;        // gathers
    int32_t *d_idx; double *d_x, *d_out;
    CK(hipMalloc(&d_idx, G * 4));
    CK(hipMalloc(&d_x, (64 << 20) * 8));
    CK(hipMalloc(&d_out, G * 8));
    CK(hipMemset(d_x, 0, (64 << 20) * 8));
    std::vector<int32_t> h(G);
    const int tabs[] = {4096, 8192, 16384, 19456, 100000};
    for (int T : tabs) {
        srand(1);
        for (int64_t i = 0; i < G; ++i) h[i] = (int32_t)(((uint64_t)rand() * 2654435761ull) % (uint64_t)T);
        CK(hipMemcpy(d_idx, h.data(), G * 4, hipMemcpyHostToDevice));
        {
            constexpr int PER = 16;
            const int64_t nl = G / PER;
            float us8 = timeit([&] { gather_global<PER, 8><<<(nl + 255) / 256, 256>>>(d_idx, d_x, d_out, nl); }, 20);
            float us16 = timeit([&] { gather_global<PER, 16><<<(nl + 255) / 256, 256>>>(d_idx, d_x, d_out, nl); }, 20);
            printf("global T=%9d doubles  PER=16: U8 %8.1f us  U16 %8.1f us  (%.1f Ggather/s)\n", T, us8, us16,
                   G / (us16 < us8 ? us16 : us8) * 1e-3);
        }
        if (T * 8 <= 160 * 1024 - 1024) {
            constexpr int PER = 64;
            const int64_t nl = G / PER;
            CK(hipFuncSetAttribute((const void *)gather_lds<PER, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, T * 8));
            float us = timeit([&] { gather_lds<PER, 8><<<(nl + 1023) / 1024, 1024, T * 8>>>(d_idx, d_x, T, d_out, nl); }, 20);
            printf("lds    T=%9d doubles  PER=64 grid %lld: %8.1f us (%.1f Ggather/s, staging %.1f MB)\n", T,
                   (long long)((nl + 1023) / 1024), us, G / us * 1e-3, (nl + 1023) / 1024 * T * 8e-6);
        }
    }
    // pure stream of the idx array for reference
    return 0;
}
