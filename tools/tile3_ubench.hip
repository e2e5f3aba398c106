// tile3_ubench.hip -- design probe for the sparse-regime SpMV, streamed form
// (not product code; tools/tile2_ubench.hip measured the staged form).
//
// Row block of H rows: running sums in LDS (the whole LDS is available for
// rows: the gathered vector is NOT staged, it is read through L1/L2 -- the
// column group g of a workgroup is blockIdx % G, so with G | 8 every workgroup
// on one XCD reads the same slice and the XCD's L2 holds it).  Wave w owns
// local rows lr with (lr >> 4) % 16 == w and walks ONE linear stream of steps
// over its group's columns (window by window, W columns each, for L1
// locality): no barriers between windows, so entries and gathers are
// prefetched batches ahead.  A step holds at most one entry per lane, lane l
// only rows with lr % 16 == l % 16 (the row read-modify-write is free of LDS
// bank conflicts), never two entries of one row, a row's entries in column
// order (CSR order: bit-identical to SciPy with G = 1).  Entry (4 B):
// (lr >> 8) << 24 | column offset in the group; per step a 64-bit lane mask.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o build/tile3_ubench tools/tile3_ubench.hip
//   build/tile3_ubench m n per_col H W G [reps]
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

constexpr int NW = 16;

struct Tiles {
    int64_t rows, cols;
    int H, nrb, ngroups;
    const int64_t *group_col;   // ngroups + 1
    const int64_t *msk_off;     // nrb * ngroups * NW + 1
    const int64_t *ent_off;
    const uint64_t *mask;
    const uint32_t *ent;
};

__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

template <int B>
struct Batch {
    uint64_t m[B];
    uint32_t u[B];
    double v[B];
};

// OP 0: full; 1: no gathers (adds 1.0); 2: no row update
template <int B, int OP>
__global__ __launch_bounds__(NW * 64) void tile3_k(Tiles T, const double *__restrict__ x,
                                                   double *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double rows[];
    const int HR = (T.H + 255) & ~255;
    const int64_t G = T.ngroups;
    const int64_t g = blockIdx.x % G, rb = blockIdx.x / G;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = lane_id();
    for (int i = threadIdx.x; i < HR; i += blockDim.x) rows[i] = 0.0;
    __syncthreads();
    const int64_t sg = (rb * G + g) * NW + wv;
    const int64_t s0 = T.msk_off[sg], S = T.msk_off[sg + 1] - s0;
    const uint64_t *M = T.mask + s0;
    const uint32_t *E = T.ent + T.ent_off[sg];
    const double *xb = x + T.group_col[g];
    const int rlo = (wv << 4) | (lane & 15);
    int64_t e = 0;
    auto masks = [&](int64_t b, Batch<B> &q) {
#pragma unroll
        for (int k = 0; k < B; ++k) q.m[k] = (b * B + k < S) ? M[b * B + k] : 0ull;
    };
    auto ents = [&](Batch<B> &q) {
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const bool on = (q.m[k] >> lane) & 1ull;
            const int64_t p = e + mbcnt64(q.m[k]);
            q.u[k] = on ? E[p] : 0u;
            e += __popcll(q.m[k]);
        }
    };
    auto gathers = [&](Batch<B> &q) {
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const bool on = (q.m[k] >> lane) & 1ull;
            if (OP == 1) q.v[k] = 1.0;
            else q.v[k] = on ? xb[q.u[k] & 0xFFFFFFu] : 0.0;
        }
    };
    double acc = 0.0;
    auto rmw = [&](const Batch<B> &q) {
#pragma unroll
        for (int k = 0; k < B; ++k) {
            if ((q.m[k] >> lane) & 1ull) {
                const int lr = (int)((q.u[k] >> 24) << 8) | rlo;
                if (OP == 2) acc += q.v[k];
                else rows[lr] += q.v[k];
            }
        }
    };
    const int64_t nb = (S + B - 1) / B;
    Batch<B> A, Bq, C;
    // pipeline: gathers one batch ahead of the row updates, entries two, masks three
    masks(0, A);
    masks(1, Bq);
    masks(2, C);
    ents(A);
    ents(Bq);
    gathers(A);
    for (int64_t b = 0; b < nb; ++b) {
        gathers(Bq);
        ents(C);
        rmw(A);
        A = Bq;
        Bq = C;
        masks(b + 3, C);
    }
    __syncthreads();
    if (OP == 2 && acc == 12345.678) rows[lane] = acc;
    const int64_t r0 = rb * T.H;
    for (int i = threadIdx.x; i < T.H; i += blockDim.x)
        if (r0 + i < T.rows) part[g * T.rows + r0 + i] = rows[i];
}

// host -----------------------------------------------------------------------
struct HostTiles {
    int H, nrb, ngroups;
    std::vector<int64_t> group_col, msk_off, ent_off;
    std::vector<uint64_t> mask;
    std::vector<uint32_t> ent;
};

static HostTiles build(int64_t R, int64_t C, const std::vector<int64_t> &ip,
                       const std::vector<int32_t> &ix, int H, int W, int G) {
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
    const int64_t nseg = (int64_t)t.nrb * G * NW;
    std::vector<int64_t> cnt(nseg + 1, 0);
    auto seg_of = [&](int64_t i, int64_t col) {
        const int64_t rb = i / H, lr = i % H, w = (lr >> 4) % NW;
        return (rb * G + group_of[col]) * NW + w;
    };
    for (int64_t i = 0; i < R; ++i)
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) cnt[seg_of(i, ix[k]) + 1]++;
    for (int64_t s = 0; s < nseg; ++s) cnt[s + 1] += cnt[s];
    // per segment: (window, lr, col) keys; rows ascending then columns ascending
    std::vector<uint64_t> flat(ip[R]);
    {
        std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < R; ++i)
            for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
                const int64_t sg = seg_of(i, ix[k]);
                const int64_t off = ix[k] - t.group_col[group_of[ix[k]]];
                flat[cur[sg]++] = ((uint64_t)(off / W) << 48) | ((uint64_t)(i % H) << 24) | (uint64_t)off;
            }
    }
    t.msk_off.assign(nseg + 1, 0);
    t.ent_off.assign(nseg + 1, 0);
    t.ent.reserve(ip[R]);
    std::vector<std::vector<uint64_t>> cls(16);
    std::vector<std::vector<std::vector<uint64_t>>> sched(16);
    for (int64_t sg = 0; sg < nseg; ++sg) {
        t.msk_off[sg] = (int64_t)t.mask.size();
        t.ent_off[sg] = (int64_t)t.ent.size();
        std::sort(flat.begin() + cnt[sg], flat.begin() + cnt[sg + 1]);
        for (int64_t a = cnt[sg]; a < cnt[sg + 1];) {
            int64_t z = a;
            const uint64_t win = flat[a] >> 48;
            while (z < cnt[sg + 1] && (flat[z] >> 48) == win) ++z;
            for (auto &v : cls) v.clear();
            for (int64_t k = a; k < z; ++k) cls[((flat[k] >> 24) & 0xFFFFFF) & 15].push_back(flat[k]);
            size_t nst = 0;
            for (int q = 0; q < 16; ++q) {
                auto &L = cls[q];
                auto &Sd = sched[q];
                Sd.clear();
                std::vector<std::pair<int, uint64_t>> seq;
                for (size_t p = 0; p < L.size();) {
                    size_t y = p;
                    while (y < L.size() && ((L[y] >> 24) & 0xFFFFFF) == ((L[p] >> 24) & 0xFFFFFF)) ++y;
                    for (size_t j = p; j < y; ++j) seq.push_back({(int)(j - p), L[j]});
                    p = y;
                }
                std::stable_sort(seq.begin(), seq.end(),
                                 [](const std::pair<int, uint64_t> &p1, const std::pair<int, uint64_t> &p2) {
                                     return p1.first < p2.first;
                                 });
                std::vector<char> used(seq.size(), 0);
                size_t left = seq.size(), start = 0;
                while (left) {
                    std::vector<uint64_t> step;
                    for (size_t j = start; j < seq.size() && step.size() < 4; ++j) {
                        if (used[j]) continue;
                        const uint64_t row = (seq[j].second >> 24) & 0xFFFFFF;
                        bool bad = false;
                        for (uint64_t s2 : step) bad |= ((s2 >> 24) & 0xFFFFFF) == row;
                        for (size_t jj = start; jj < j && !bad; ++jj)
                            bad |= !used[jj] && ((seq[jj].second >> 24) & 0xFFFFFF) == row;
                        if (bad) continue;
                        step.push_back(seq[j].second);
                        used[j] = 1;
                        --left;
                    }
                    while (start < seq.size() && used[start]) ++start;
                    Sd.push_back(step);
                }
                nst = std::max(nst, Sd.size());
            }
            for (size_t s = 0; s < nst; ++s) {
                uint64_t m = 0;
                uint32_t le[64];
                for (int q = 0; q < 16; ++q) {
                    if (s >= sched[q].size()) continue;
                    const auto &st = sched[q][s];
                    for (size_t j = 0; j < st.size(); ++j) {
                        const int l = q + 16 * (int)j;
                        m |= 1ull << l;
                        const uint64_t lr = (st[j] >> 24) & 0xFFFFFF;
                        le[l] = (uint32_t)((lr >> 8) << 24) | (uint32_t)(st[j] & 0xFFFFFF);
                    }
                }
                t.mask.push_back(m);
                for (int l = 0; l < 64; ++l)
                    if ((m >> l) & 1) t.ent.push_back(le[l]);
            }
            a = z;
        }
    }
    t.msk_off[nseg] = (int64_t)t.mask.size();
    t.ent_off[nseg] = (int64_t)t.ent.size();
    return t;
}

int main(int argc, char **argv) {
    if (argc < 7) {
        printf("usage: %s m n per_col H W G [reps]\n", argv[0]);
        return 1;
    }
    const int64_t m = atoll(argv[1]), n = atoll(argv[2]);
    const int pc = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]), G = atoi(argv[6]);
    const int reps = argc > 7 ? atoi(argv[7]) : 20;
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
    HostTiles ht = build(m, n, ip, ix, H, W, G);
    auto t1 = std::chrono::steady_clock::now();
    const double util = (double)ht.ent.size() / (64.0 * ht.mask.size());
    printf("m %ld n %ld nnz %ld H %d W %d G %d: %d row blocks -> %d workgroups, %zu steps (lane "
           "use %.2f), host %.1f s\n",
           (long)m, (long)n, (long)ip[m], H, W, G, ht.nrb, ht.nrb * G, ht.mask.size(), util,
           std::chrono::duration<double>(t1 - t0).count());
    int64_t *d_gc, *d_mo, *d_eo;
    uint64_t *d_mask;
    uint32_t *d_ent;
    double *d_x, *d_part;
    CK(hipMalloc(&d_gc, ht.group_col.size() * 8));
    CK(hipMalloc(&d_mo, ht.msk_off.size() * 8));
    CK(hipMalloc(&d_eo, ht.ent_off.size() * 8));
    CK(hipMalloc(&d_mask, ht.mask.size() * 8 + 1024));
    CK(hipMalloc(&d_ent, ht.ent.size() * 4 + 1024));
    CK(hipMalloc(&d_x, n * 8 + 64));
    CK(hipMalloc(&d_part, (size_t)G * m * 8));
    CK(hipMemset(d_mask, 0, ht.mask.size() * 8 + 1024));
    CK(hipMemcpy(d_gc, ht.group_col.data(), ht.group_col.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mo, ht.msk_off.data(), ht.msk_off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_eo, ht.ent_off.data(), ht.ent_off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mask, ht.mask.data(), ht.mask.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ent, ht.ent.data(), ht.ent.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), n * 8, hipMemcpyHostToDevice));
    Tiles T{m, n, H, ht.nrb, ht.ngroups, d_gc, d_mo, d_eo, d_mask, d_ent};
    const int grid = ht.nrb * G;
    auto run = [&](auto kern, const char *name) {
        const size_t lds = (size_t)((H + 255) & ~255) * 8;
        if (lds > 163840) {
            printf("  %-10s LDS %zu too big\n", name, lds);
            return;
        }
        CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
        CK(hipMemset(d_part, 0, (size_t)G * m * 8));
        kern<<<grid, NW * 64, lds>>>(T, d_x, d_part);
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
        for (int r = 0; r < reps; ++r) kern<<<grid, NW * 64, lds>>>(T, d_x, d_part);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        const double alg = 12.0 * ip[m] + 4.0 * (m + 1) + 8.0 * n + 8.0 * m;
        const double fmt = 4.0 * ht.ent.size() + 8.0 * ht.mask.size();
        printf("  %-10s %9.1f us  alg %.0f MB -> %.2f TB/s (stream %.0f MB)  mismatch-vs-CSR %ld "
               "(max rel %.2e)\n",
               name, us, alg / 1e6, alg / (us * 1e-6) / 1e12, fmt / 1e6, (long)bad, mx);
    };
    run(tile3_k<4, 0>, "b4");
    run(tile3_k<8, 0>, "b8");
    run(tile3_k<8, 1>, "b8-nogath");
    run(tile3_k<8, 2>, "b8-norow");
    return 0;
}
