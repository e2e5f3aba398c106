// bank_ubench.hip -- design probe (not product), round 6: the dealt tile
// walk's LDS-atomic row sums lose most LDS cycles to bank conflicts (PMC:
// SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS 0.69 in K2, 0.88 in K1).  The
// lanes of one wave-instruction hold 64 column-sorted entries whose rows are
// random, so a ds_add_f64 lane group hits the same bank several times.  The
// host builder is free to permute the 64 entries over the lanes of their
// instruction (the instruction gathers the same cache lines whatever the lane
// order): does that remove the conflicts, and does the gather keep its rate?
//
// Each 1024-thread workgroup walks E column-sorted entries of one slice of T
// doubles (slice = blockIdx % 8, as coal_ubench), instruction i of wave w
// taking entries [(i * 16 + w) * 64, +64), and (add = 1) adds each gathered
// value into an LDS row table at the entry's row with ds_add_f64.
//   perm 0: lanes in column order (the shipped dealing)
//   perm 1: lanes randomly permuted within each instruction (gather rate vs
//           lane order)
//   perm 2: lanes assigned so each group of G lanes holds distinct row
//           residues mod K (greedy over the column-sorted entries; entries
//           stay in their instruction)
//   perm 4: round robin -- the entries ordered by row residue mod K, item k
//           to group k % (64 / G), each group's lanes in column order (the
//           residues spread as evenly as counts allow)
//   perm 3: synthetic rows: lane l's row = (random high bits) * K + l % K
//           (the conflict-free bound for that (K, G) guess)
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/bank_ubench tools/bank_ubench.hip
//   tools/bank_ubench T E nwg add perm [rows K G]
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

template <int ADD>
__global__ __launch_bounds__(1024) void walk(const uint32_t *__restrict__ idx,
                                             const uint16_t *__restrict__ rowsel,
                                             const double *__restrict__ x, int64_t T, int64_t E,
                                             int rows, double *__restrict__ out) {
    extern __shared__ double acc[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (ADD) {
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
            if (ADD) r[u] = (i0 + u < ninst) ? R[e] : 0;
        }
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = xs[c[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ADD) {
                if (i0 + u < ninst) atomicAdd(&acc[r[u]], v[u]);
            } else {
                s += v[u];
            }
        }
    }
    if (ADD) {
        __syncthreads();
        for (int i = threadIdx.x; i < rows; i += 1024) s += acc[i];
    }
    out[(int64_t)blockIdx.x * 1024 + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        printf("usage: T E nwg add perm [rows K G]\n");
        return 1;
    }
    const int64_t T = atoll(argv[1]), E = atoll(argv[2]);
    const int nwg = atoi(argv[3]), add = atoi(argv[4]), perm = atoi(argv[5]);
    const int rows = argc > 6 ? atoi(argv[6]) : 16384;
    const int K = argc > 7 ? atoi(argv[7]) : 16, G = argc > 8 ? atoi(argv[8]) : 16;
    std::mt19937_64 rng(5);
    std::vector<uint32_t> idx((size_t)nwg * E);
    std::vector<uint16_t> rs((size_t)nwg * E);
    std::vector<std::pair<uint32_t, uint16_t>> tmp(E);
    for (int b = 0; b < nwg; ++b) {
        uint32_t *I = idx.data() + (size_t)b * E;
        uint16_t *Rw = rs.data() + (size_t)b * E;
        for (int64_t e = 0; e < E; ++e) tmp[e] = {(uint32_t)(rng() % T), (uint16_t)(rng() % rows)};
        std::sort(tmp.begin(), tmp.end());
        for (int64_t i = 0; i < E / 64; ++i) {
            std::pair<uint32_t, uint16_t> *in = tmp.data() + i * 64;
            std::pair<uint32_t, uint16_t> o[64];
            if (perm == 1) {
                int p[64];
                for (int l = 0; l < 64; ++l) p[l] = l;
                std::shuffle(p, p + 64, rng);
                for (int l = 0; l < 64; ++l) o[l] = in[p[l]];
            } else if (perm == 2) {
                // greedy: each entry (column order) to the first group with a
                // free lane and without its residue, else the first free group
                const int ng = 64 / G;
                std::vector<std::vector<std::pair<uint32_t, uint16_t>>> grp(ng);
                std::vector<std::vector<char>> used(ng, std::vector<char>(K, 0));
                for (int l = 0; l < 64; ++l) {
                    const int res = in[l].second % K;
                    int gsel = -1;
                    for (int g = 0; g < ng && gsel < 0; ++g)
                        if ((int)grp[g].size() < G && !used[g][res]) gsel = g;
                    for (int g = 0; g < ng && gsel < 0; ++g)
                        if ((int)grp[g].size() < G) gsel = g;
                    grp[gsel].push_back(in[l]);
                    used[gsel][res] = 1;
                }
                int l = 0;
                for (int g = 0; g < ng; ++g)
                    for (auto &e : grp[g]) o[l++] = e;
            } else if (perm == 4) {
                const int ng = 64 / G;
                int ord[64];
                for (int l = 0; l < 64; ++l) ord[l] = l;
                std::stable_sort(ord, ord + 64, [&](int x, int y) {
                    return in[x].second % K < in[y].second % K;
                });
                std::vector<std::vector<int>> grp(ng);
                for (int k = 0; k < 64; ++k) grp[k % ng].push_back(ord[k]);
                int l = 0;
                for (int g = 0; g < ng; ++g) {
                    std::sort(grp[g].begin(), grp[g].end());
                    for (int x : grp[g]) o[l++] = in[x];
                }
            } else {
                for (int l = 0; l < 64; ++l) o[l] = in[l];
                if (perm == 3)
                    for (int l = 0; l < 64; ++l)
                        o[l].second = (uint16_t)(((rng() % (rows / K)) * K + l % K) % rows);
            }
            for (int l = 0; l < 64; ++l) {
                I[i * 64 + l] = o[l].first;
                Rw[i * 64 + l] = o[l].second;
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
    const size_t lds = add ? (size_t)(rows + 1) * 8 : 0;
    auto run = [&]() {
        if (add)
            walk<1><<<nwg, 1024, lds>>>(d_idx, d_rs, d_x, T, E, rows, d_out);
        else
            walk<0><<<nwg, 1024, 0>>>(d_idx, d_rs, d_x, T, E, rows, d_out);
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
    const double Gs = (double)nwg * E / (us * 1e-6) / 1e9;
    printf("{\"T\": %lld, \"E\": %lld, \"nwg\": %d, \"add\": %d, \"perm\": %d, \"rows\": %d, "
           "\"K\": %d, \"G\": %d, \"us\": %.1f, \"Ggathers_s\": %.1f}\n",
           (long long)T, (long long)E, nwg, add, perm, rows, K, G, us, Gs);
    return 0;
}
