// coal_ubench.hip -- design probe (not product): do column-sorted gathers
// coalesce?  Each 1024-thread workgroup gathers E 8-B elements of one slice of
// T doubles (slice = blockIdx % 8: one slice per XCD, as the tile images'
// column groups) and sums them per lane.  mode 0: indices uniformly random
// (the tile walk: every lane's k-th entry somewhere in the slice); mode 1: the
// workgroup's E indices sorted and dealt in order, wave-instruction i of wave
// w taking entries [(i * 16 + w) * 64, +64) -- so one instruction's 64 gathers
// fall in ~64 T / E consecutive elements and the 16 waves sweep the slice
// together; mode 2: as mode 1, then every gathered value is added into an
// LDS row table at a random row with ds_add_f64 (the accumulation such a
// dealing needs); mode 3: rows split over the 16 waves (row % 16), each
// wave's entries sorted by column and dealt over its lanes, ds_add_f64 into
// the rows -- every add to a row then comes from one wave in column order
// (deterministic); the waves' streams padded to the longest (dummy row);
// mode 4: mode 1's dealing, each value turned into a 64-bit fixed-point
// integer and added with ds_add_u64 (order-free, so deterministic).
//
//   hipcc -O3 --offload-arch=gfx950 -o build/coal_ubench tools/coal_ubench.hip
//   build/coal_ubench T E nwg mode [rows]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void gather(const uint32_t *__restrict__ idx,
                                               const uint16_t *__restrict__ rowsel,
                                               const double *__restrict__ x, int64_t T,
                                               int64_t E, int rows, double *__restrict__ out) {
    extern __shared__ double acc[];
    unsigned long long *iacc = reinterpret_cast<unsigned long long *>(acc);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (MODE >= 2) {
        for (int i = threadIdx.x; i < rows + 1; i += 1024) acc[i] = 0.0;
        __syncthreads();
    }
    const double *xs = x + (int64_t)(blockIdx.x & 7) * T;
    const uint32_t *I = idx + (int64_t)blockIdx.x * E;
    const uint16_t *R = rowsel + (int64_t)blockIdx.x * E;
    const int64_t ninst = E / 1024;
    double s = 0.0;
    constexpr int U = 8;
    for (int64_t i0 = 0; i0 < ninst; i0 += U) {
        uint32_t c[U];
        uint16_t r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = ((i0 + u) * 16 + w) * 64 + lane;
            c[u] = (i0 + u < ninst) ? I[e] : 0u;
            if (MODE >= 2) r[u] = (i0 + u < ninst) ? R[e] : 0;
        }
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = xs[c[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE >= 2) {
                if (i0 + u < ninst) {
                    if (MODE == 4) {
                        const double q = v[u] * 0x1p40;
                        const double hi = __builtin_floor(q * 0x1p-32);
                        const uint32_t lo = (uint32_t)(q - hi * 0x1p32);
                        const long long iv = ((long long)(int)hi << 32) | lo;
                        atomicAdd(&iacc[r[u]], (unsigned long long)iv);
                    } else {
                        atomicAdd(&acc[r[u]], v[u]);
                    }
                }
            } else {
                s += v[u];
            }
        }
    }
    if (MODE >= 2) {
        __syncthreads();
        for (int i = threadIdx.x; i < rows; i += 1024)
            s += (MODE == 4) ? (double)(long long)iacc[i] * 0x1p-40 : acc[i];
    }
    out[(int64_t)blockIdx.x * 1024 + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        printf("usage: T E nwg mode [rows]\n");
        return 1;
    }
    const int64_t T = atoll(argv[1]), E = atoll(argv[2]);
    const int nwg = atoi(argv[3]), mode = atoi(argv[4]);
    const int rows = argc > 5 ? atoi(argv[5]) : 16384;
    std::mt19937_64 rng(5);
    std::vector<uint32_t> idx((size_t)nwg * E);
    std::vector<uint16_t> rs((size_t)nwg * E);
    for (int b = 0; b < nwg; ++b) {
        uint32_t *I = idx.data() + (size_t)b * E;
        for (int64_t e = 0; e < E; ++e) {
            I[e] = (uint32_t)(rng() % T);
            rs[(size_t)b * E + e] = (uint16_t)(rng() % rows);
        }
        if (mode == 3) {
            // rows over waves; per wave sort by column, deal; pad to E / 16
            std::vector<std::vector<std::pair<uint32_t, uint16_t>>> wl(16);
            for (int64_t e = 0; e < E; ++e) {
                const uint16_t r = rs[(size_t)b * E + e];
                wl[r % 16].push_back({I[e], r});
            }
            size_t mx = 0;
            for (auto &v : wl) {
                std::sort(v.begin(), v.end());
                mx = std::max(mx, v.size());
            }
            if (mx * 16 > (size_t)E) mx = E / 16;   // (drop the overflow: timing only)
            for (int w = 0; w < 16; ++w)
                for (size_t k = 0; k < mx; ++k) {
                    const size_t pos = ((k / 64) * 16 + w) * 64 + (k % 64);
                    if ((int64_t)pos >= E) continue;
                    const bool ok = k < wl[w].size();
                    I[pos] = ok ? wl[w][k].first : 0u;
                    rs[(size_t)b * E + pos] = ok ? wl[w][k].second : (uint16_t)rows;
                }
        } else if (mode >= 1) {   // (1, 2, 4)
            // sorted, dealt in order: entry j of the sorted list -> position
            // ((i * 16 + w) * 64 + lane) with j = (i * 16 + w) * 64 + lane: the
            // same index, so the sorted list is the layout
            std::sort(I, I + E);
        } else {
            // random: each lane's stream in column order (the tile walk's
            // property), streams interleaved
            std::vector<uint32_t> tmp(I, I + E);
            const int64_t per = E / 1024;
            for (int t = 0; t < 1024; ++t) {
                std::vector<uint32_t> st(per);
                for (int64_t k = 0; k < per; ++k) st[k] = tmp[t * per + k];
                std::sort(st.begin(), st.end());
                const int w = t >> 6, lane = t & 63;
                for (int64_t k = 0; k < per; ++k) I[(k * 16 + w) * 64 + lane] = st[k];
            }
        }
    }
    uint32_t *d_idx;
    uint16_t *d_rs;
    double *d_x, *d_out;
    CK(hipMalloc(&d_idx, idx.size() * 4));
    CK(hipMalloc(&d_rs, rs.size() * 2));
    CK(hipMalloc(&d_x, 8 * T * 8));
    CK(hipMalloc(&d_out, (size_t)nwg * 1024 * 8));
    CK(hipMemcpy(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_rs, rs.data(), rs.size() * 2, hipMemcpyHostToDevice));
    std::vector<double> xh(8 * T, 1.0);
    CK(hipMemcpy(d_x, xh.data(), xh.size() * 8, hipMemcpyHostToDevice));
    const size_t lds = mode >= 2 ? (size_t)(rows + 1) * 8 : 0;
    auto run = [&]() {
        if (mode == 0)
            gather<0><<<nwg, 1024, 0>>>(d_idx, d_rs, d_x, T, E, rows, d_out);
        else if (mode == 1)
            gather<1><<<nwg, 1024, 0>>>(d_idx, d_rs, d_x, T, E, rows, d_out);
        else if (mode == 4)
            gather<4><<<nwg, 1024, lds>>>(d_idx, d_rs, d_x, T, E, rows, d_out);
        else
            gather<2><<<nwg, 1024, lds>>>(d_idx, d_rs, d_x, T, E, rows, d_out);   // (3: same kernel)
    };
    run();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double G = (double)nwg * E / (us * 1e-6) / 1e9;
    printf("{\"T\": %lld, \"E\": %lld, \"nwg\": %d, \"mode\": %d, \"rows\": %d, \"us\": %.1f, "
           "\"Ggathers_s\": %.1f}\n",
           (long long)T, (long long)E, nwg, mode, rows, us, G);
    return 0;
}
