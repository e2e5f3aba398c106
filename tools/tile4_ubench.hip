// tile4_ubench.hip -- design probe for the sparse-regime SpMV, thread-owned
// rows (not product code; tile3_ubench.hip measured the stepped form).
//
// Row block of H rows, running sums in LDS; thread t of the 1024-thread
// workgroup owns the local rows lr with lr % 1024 == t (LDS address lr: every
// lane of a wave hits its own bank pair, so the read-modify-write is free of
// bank conflicts and of races).  A thread walks ONE linear stream: the entries
// of its rows in the workgroup's column group, sorted by column (so a row's
// entries stay in CSR order -- bit-identical to SciPy with G = 1 -- and all
// threads sweep the columns together: the gathers stay in L1/L2).  The
// gathered vector is not staged; column group g = blockIdx % G (G | 8: one
// slice per XCD L2).  Entry (4 B): (lr / 1024) << 24 | column offset in the
// group; streams interleaved in 16-B quads, quad k of lane l of wave w at
// wave_off[w] + (k * 64 + l) * 4; padded to the wave's longest stream with
// entries for a dummy row.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o build/tile4_ubench tools/tile4_ubench.hip
//   build/tile4_ubench m n per_col H G [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../block-simplex-least-squares_amd/csrc/bsls_common.hpp"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

using namespace bsls;

constexpr int NT = 1024;

struct Tiles {
    int64_t rows, cols;
    int H, nrb, ngroups;
    const int64_t *group_col;   // ngroups + 1
    const int64_t *wave_off;    // nrb * ngroups * 16 + 1 (in quads)
    const uint32_t *ent;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// OP 0: full; 1: no gathers; 2: no row update
template <int P, int OP>
__global__ __launch_bounds__(NT) void tile4_k(Tiles T, const double *__restrict__ x,
                                              double *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double rows[];
    const int HR = ((T.H + NT - 1) / NT + 1) * NT;   // + one dummy slot row per thread
    const int64_t G = T.ngroups;
    const int64_t g = blockIdx.x % G, rb = blockIdx.x / G;
    const int t = threadIdx.x, lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(t / 64);
    for (int i = t; i < HR; i += NT) rows[i] = 0.0;
    __syncthreads();
    const int64_t sg = (rb * G + g) * 16 + wv;
    const int64_t q0 = T.wave_off[sg], nq = (T.wave_off[sg + 1] - q0) / 64;
    const u32x4 *Q = reinterpret_cast<const u32x4 *>(T.ent) + q0 + lane;
    const double *xb = x + T.group_col[g];
    u32x4 ring[P];
#pragma unroll
    for (int k = 0; k < P; ++k) ring[k] = (k < nq) ? Q[(int64_t)k * 64] : u32x4{0, 0, 0, 0};
    double acc = 0.0;
    double v[4], vn[4];
    auto gat = [&](const u32x4 &u, double (&o)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (OP == 1) ? 1.0 : xb[u[j] & 0xFFFFFFu];
    };
    gat(ring[0], v);
    for (int64_t q = 0; q < nq; q += P) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const u32x4 cur = ring[k];
            const u32x4 nxt = ring[(k + 1) % P];
            if (q + k + 1 < nq) gat(nxt, vn);
            ring[k] = (q + k + P < nq) ? Q[(q + k + P) * 64] : u32x4{0, 0, 0, 0};
            if (q + k < nq) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int lr = (int)(cur[j] >> 24) * NT + t;
                    if (OP == 2) acc += v[j];
                    else rows[lr] += v[j];
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = vn[j];
        }
    }
    __syncthreads();
    if (OP == 2 && acc == 12345.678) rows[lane] = acc;
    const int64_t r0 = rb * T.H;
    for (int i = t; i < T.H; i += NT)
        if (r0 + i < T.rows) part[g * T.rows + r0 + i] = rows[i];
}

// host -----------------------------------------------------------------------
struct HostTiles {
    int H, nrb, ngroups;
    std::vector<int64_t> group_col, wave_off;
    std::vector<uint32_t> ent;
};

static HostTiles build(int64_t R, int64_t C, const std::vector<int64_t> &ip,
                       const std::vector<int32_t> &ix, int H, int G) {
    HostTiles t;
    t.H = H;
    t.nrb = (int)((R + H - 1) / H);
    t.ngroups = G;
    t.group_col.resize(G + 1);
    for (int g = 0; g <= G; ++g) t.group_col[g] = (C * g / G) & ~1LL;
    t.group_col[G] = C;
    std::vector<int32_t> group_of(C);
    for (int g = 0; g < G; ++g)
        for (int64_t j = t.group_col[g]; j < t.group_col[g + 1]; ++j) group_of[j] = g;
    const int dummy_slot = (H + NT - 1) / NT;
    // per (rb, g, thread): entries keyed (col offset, slot)
    const int64_t nthr = (int64_t)t.nrb * G * NT;
    std::vector<int64_t> cnt(nthr + 1, 0);
    auto th_of = [&](int64_t i, int64_t col) {
        const int64_t rb = i / H, lr = i % H;
        return (rb * G + group_of[col]) * NT + lr % NT;
    };
    for (int64_t i = 0; i < R; ++i)
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) cnt[th_of(i, ix[k]) + 1]++;
    for (int64_t s = 0; s < nthr; ++s) cnt[s + 1] += cnt[s];
    std::vector<uint64_t> flat(ip[R]);
    {
        std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < R; ++i)
            for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
                const int64_t th = th_of(i, ix[k]);
                const int64_t off = ix[k] - t.group_col[group_of[ix[k]]];
                const int64_t slot = (i % H) / NT;
                flat[cur[th]++] = ((uint64_t)off << 8) | (uint64_t)slot;
            }
    }
    const int64_t nwav = (int64_t)t.nrb * G * 16;
    t.wave_off.assign(nwav + 1, 0);
    for (int64_t w = 0; w < nwav; ++w) {
        int64_t mx = 0;
        for (int l = 0; l < 64; ++l) {
            const int64_t th = w * 64 + l;
            std::sort(flat.begin() + cnt[th], flat.begin() + cnt[th + 1]);
            mx = std::max(mx, cnt[th + 1] - cnt[th]);
        }
        const int64_t nq = (mx + 3) / 4;
        t.wave_off[w + 1] = t.wave_off[w] + nq * 64;
    }
    t.ent.assign((size_t)t.wave_off[nwav] * 4, ((uint32_t)dummy_slot << 24));
    for (int64_t w = 0; w < nwav; ++w) {
        for (int l = 0; l < 64; ++l) {
            const int64_t th = w * 64 + l;
            for (int64_t k = cnt[th]; k < cnt[th + 1]; ++k) {
                const int64_t e = k - cnt[th];
                const int64_t quad = t.wave_off[w] + (e / 4) * 64 + l;
                t.ent[quad * 4 + e % 4] = ((uint32_t)(flat[k] & 0xFF) << 24) | (uint32_t)(flat[k] >> 8);
            }
        }
    }
    return t;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        printf("usage: %s m n per_col H G [reps]\n", argv[0]);
        return 1;
    }
    const int64_t m = atoll(argv[1]), n = atoll(argv[2]);
    const int pc = atoi(argv[3]), H = atoi(argv[4]), G = atoi(argv[5]);
    const int reps = argc > 6 ? atoi(argv[6]) : 20;
    auto t0 = std::chrono::steady_clock::now();
    std::mt19937_64 rng(237423433);
    std::vector<int64_t> ip(m + 1, 0);
    std::vector<int32_t> ix;
    auto draw = [&](int32_t *r, int k, int64_t range) {
        for (int q = 0; q < k; ++q) {
            for (;;) {
                const int32_t v = (int32_t)(rng() % (uint64_t)range);
                bool dup = false;
                for (int z = 0; z < q; ++z) dup |= r[z] == v;
                if (!dup) { r[q] = v; break; }
            }
        }
    };
    if (pc > 0) {
        std::vector<int32_t> crow((size_t)n * pc);
        for (int64_t j = 0; j < n; ++j) draw(&crow[(size_t)j * pc], pc, m);
        for (size_t k = 0; k < crow.size(); ++k) ip[crow[k] + 1]++;
        for (int64_t i = 0; i < m; ++i) ip[i + 1] += ip[i];
        ix.resize(ip[m]);
        std::vector<int64_t> cur(ip.begin(), ip.end() - 1);
        for (int64_t j = 0; j < n; ++j)
            for (int k = 0; k < pc; ++k) ix[cur[crow[(size_t)j * pc + k]]++] = (int32_t)j;
    } else {
        const int k = -pc;
        ix.resize((size_t)m * k);
        for (int64_t i = 0; i < m; ++i) {
            draw(&ix[(size_t)i * k], k, n);
            std::sort(ix.begin() + (size_t)i * k, ix.begin() + (size_t)(i + 1) * k);
            ip[i + 1] = (i + 1) * k;
        }
    }
    std::vector<double> x(n);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (auto &v : x) v = U(rng);
    std::vector<double> ref(m);
    for (int64_t i = 0; i < m; ++i) {
        double s = 0.0;
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) s += x[ix[k]];
        ref[i] = s;
    }
    HostTiles ht = build(m, n, ip, ix, H, G);
    auto t1 = std::chrono::steady_clock::now();
    const double util = (double)ip[m] / (double)ht.ent.size();
    printf("m %ld n %ld nnz %ld H %d G %d: %d row blocks -> %d workgroups, stream %.0f MB "
           "(lane use %.2f), host %.1f s\n",
           (long)m, (long)n, (long)ip[m], H, G, ht.nrb, ht.nrb * G, ht.ent.size() * 4e-6, util,
           std::chrono::duration<double>(t1 - t0).count());
    int64_t *d_gc, *d_wo;
    uint32_t *d_ent;
    double *d_x, *d_part;
    CK(hipMalloc(&d_gc, ht.group_col.size() * 8));
    CK(hipMalloc(&d_wo, ht.wave_off.size() * 8));
    CK(hipMalloc(&d_ent, ht.ent.size() * 4 + 1024));
    CK(hipMalloc(&d_x, n * 8 + 64));
    CK(hipMalloc(&d_part, (size_t)G * m * 8));
    CK(hipMemcpy(d_gc, ht.group_col.data(), ht.group_col.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_wo, ht.wave_off.data(), ht.wave_off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ent, ht.ent.data(), ht.ent.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), n * 8, hipMemcpyHostToDevice));
    Tiles T{m, n, H, ht.nrb, ht.ngroups, d_gc, d_wo, d_ent};
    const int grid = ht.nrb * G;
    auto run = [&](auto kern, const char *name) {
        const size_t lds = (size_t)(((H + NT - 1) / NT + 1) * NT) * 8;
        if (lds > 163840) {
            printf("  %-10s LDS %zu too big\n", name, lds);
            return;
        }
        CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
        CK(hipMemset(d_part, 0, (size_t)G * m * 8));
        kern<<<grid, NT, lds>>>(T, d_x, d_part);
        CK(hipDeviceSynchronize());
        std::vector<double> p((size_t)G * m);
        CK(hipMemcpy(p.data(), d_part, p.size() * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        double mx = 0;
        for (int64_t i = 0; i < m; ++i) {
            double s = p[i];
            for (int g = 1; g < G; ++g) s += p[(size_t)g * m + i];
            if (s != ref[i]) ++bad;
            mx = std::max(mx, std::fabs(s - ref[i]) / (std::fabs(ref[i]) + 1e-300));
        }
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) kern<<<grid, NT, lds>>>(T, d_x, d_part);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        const double alg = 12.0 * ip[m] + 4.0 * (m + 1) + 8.0 * n + 8.0 * m;
        const double fmt = 4.0 * ht.ent.size();
        printf("  %-10s %9.1f us  alg %.0f MB -> %.2f TB/s (stream %.0f MB)  mismatch-vs-CSR %ld "
               "(max rel %.2e)\n",
               name, us, alg / 1e6, alg / (us * 1e-6) / 1e12, fmt / 1e6, (long)bad, mx);
    };
    run(tile4_k<4, 0>, "p4");
    run(tile4_k<8, 0>, "p8");
    run(tile4_k<8, 1>, "p8-nogath");
    run(tile4_k<8, 2>, "p8-norow");
    return 0;
}
