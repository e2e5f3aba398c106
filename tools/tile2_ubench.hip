// tile2_ubench.hip -- design probe for the sparse-regime SpMV, stepped form
// (not product code; tools/tile_ubench.hip measured the first form).
//
// Row block of H rows (running sums in LDS) x column chunk of <= W columns
// (staged by LDS-DMA, double-buffered).  Wave w owns local rows lr with
// (lr / 16) % 16 == w.  A wave walks its tile entries in STEPS: a step holds at
// most one entry per lane, lane l only entries whose row has lr % 16 == l % 16
// (4 lanes per class), never two entries of one row, and a row's entries in
// column order over the steps.  So the row read-modify-write of a step is free
// of LDS bank conflicts (ds_write_b64: 16-lane groups, bank (2 lr) mod 32) and
// of races, and each row is summed in CSR order (bit-identical to SciPy when
// one workgroup sees every chunk).  Per step: a 64-bit lane mask; the step's
// entries are stored compactly (lane position = mbcnt of the mask).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o build/tile2_ubench tools/tile2_ubench.hip
//   build/tile2_ubench m n per_col H W G [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../block-simplex-least-squares_amd/csrc/panels.hpp"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

using namespace bsls;

struct Tiles {
    int64_t rows, cols;
    int H, W, nrb, nchunks, ngroups;
    const int64_t *chunk_col, *group_chunk, *step_off, *ent_off;
    const uint64_t *mask;
    const uint32_t *ent;
};

constexpr int NW = 16;

__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// OP 0: full; 1: no row update (gathers summed in a register); 2: x gathered
// from global memory (L1/L2), no LDS staging and no barriers
template <int B, int OP>
__global__ __launch_bounds__(NW * 64) void tile2_k(Tiles T, const double *__restrict__ x,
                                                   double *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int HR = (T.H + 255) & ~255;
    double *rows = lds;
    double *tab[2] = {lds + HR, lds + HR + T.W};
    const int64_t G = T.ngroups;
    const int64_t g = blockIdx.x % G, rb = blockIdx.x / G;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = lane_id();
    for (int i = threadIdx.x; i < HR; i += blockDim.x) rows[i] = 0.0;
    const int64_t c0 = T.group_chunk[g], c1 = T.group_chunk[g + 1];
    if (OP != 2)
        panel_stage(tab[0], x + T.chunk_col[c0], (int)(T.chunk_col[c0 + 1] - T.chunk_col[c0]));
    else
        __syncthreads();
    double acc = 0.0;
    for (int64_t c = c0; c < c1; ++c) {
        const int b = (int)((c - c0) & 1);
        if (OP != 2) {
            __syncthreads();
            if (c + 1 < c1)
                panel_stage(tab[b ^ 1], x + T.chunk_col[c + 1],
                            (int)(T.chunk_col[c + 2] - T.chunk_col[c + 1]));
        }
        const double *tb = OP == 2 ? x + T.chunk_col[c] : tab[b];
        const int64_t sg = (rb * T.nchunks + c) * NW + wv;
        const int64_t s0 = T.step_off[sg], s1 = T.step_off[sg + 1];
        int64_t e = T.ent_off[sg];
        for (int64_t st = s0; st < s1; st += B) {
            uint64_t mk[B];
#pragma unroll
            for (int k = 0; k < B; ++k) mk[k] = (st + k < s1) ? T.mask[st + k] : 0ull;
            uint32_t u[B];
#pragma unroll
            for (int k = 0; k < B; ++k) {
                const bool on = (mk[k] >> lane) & 1ull;
                const int64_t p = e + mbcnt64(mk[k]);
                u[k] = on ? T.ent[p] : 0u;
                e += __popcll(mk[k]);
            }
            double v[B];
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = tb[u[k] & 0xFFFFu];
#pragma unroll
            for (int k = 0; k < B; ++k) {
                if ((mk[k] >> lane) & 1ull) {
                    if (OP != 1) rows[u[k] >> 16] += v[k];
                    else acc += v[k];
                }
            }
        }
    }
    __syncthreads();
    if (OP == 1 && acc == 12345.678) rows[lane] = acc;
    const int64_t r0 = rb * T.H;
    for (int i = threadIdx.x; i < T.H; i += blockDim.x)
        if (r0 + i < T.rows) part[g * T.rows + r0 + i] = rows[i];
}

// host -----------------------------------------------------------------------
struct HostTiles {
    int H, W, nrb, nchunks, ngroups;
    std::vector<int64_t> chunk_col, group_chunk, step_off, ent_off;
    std::vector<uint64_t> mask;
    std::vector<uint32_t> ent;
};

static HostTiles build(int64_t R, int64_t C, const std::vector<int64_t> &ip,
                       const std::vector<int32_t> &ix, int H, int W, int G) {
    HostTiles t;
    t.H = H;
    t.W = W;
    t.nrb = (int)((R + H - 1) / H);
    int64_t nch = (C + W - 1) / W;
    if (nch < G) nch = G;
    t.chunk_col.resize(nch + 1);
    for (int64_t c = 0; c <= nch; ++c) t.chunk_col[c] = std::min<int64_t>(C, (C * c / nch + 1) & ~1LL);
    t.chunk_col[0] = 0;
    t.chunk_col[nch] = C;
    t.nchunks = (int)nch;
    t.ngroups = G;
    t.group_chunk.resize(G + 1);
    for (int g = 0; g <= G; ++g) t.group_chunk[g] = nch * g / G;
    std::vector<int32_t> chunk_of(C);
    for (int64_t c = 0; c < nch; ++c)
        for (int64_t j = t.chunk_col[c]; j < t.chunk_col[c + 1]; ++j) chunk_of[j] = (int32_t)c;
    // bucket the entries by segment (rb, c, w), rows ascending, columns ascending
    const int64_t nseg = (int64_t)t.nrb * nch * NW;
    std::vector<int64_t> cnt(nseg + 1, 0);
    auto seg_of = [&](int64_t i, int64_t col) {
        const int64_t rb = i / H, lr = i % H, w = (lr >> 4) % NW;
        return (rb * nch + chunk_of[col]) * NW + w;
    };
    for (int64_t i = 0; i < R; ++i)
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) cnt[seg_of(i, ix[k]) + 1]++;
    for (int64_t s = 0; s < nseg; ++s) cnt[s + 1] += cnt[s];
    std::vector<uint32_t> flat(ip[R]);
    {
        std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < R; ++i)
            for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
                const int64_t sg = seg_of(i, ix[k]);
                const int64_t c = chunk_of[ix[k]];
                flat[cur[sg]++] = ((uint32_t)(i % H) << 16) | (uint32_t)(ix[k] - t.chunk_col[c]);
            }
    }
    // per segment: schedule steps
    t.step_off.assign(nseg + 1, 0);
    t.ent_off.assign(nseg + 1, 0);
    t.ent.reserve(ip[R]);
    std::vector<std::vector<uint32_t>> cls(16);
    std::vector<std::vector<std::vector<uint32_t>>> sched(16);   // [class][step] entries
    for (int64_t sg = 0; sg < nseg; ++sg) {
        t.step_off[sg] = (int64_t)t.mask.size();
        t.ent_off[sg] = (int64_t)t.ent.size();
        for (auto &v : cls) v.clear();
        for (int64_t k = cnt[sg]; k < cnt[sg + 1]; ++k) cls[(flat[k] >> 16) & 15].push_back(flat[k]);
        size_t nst = 0;
        for (int q = 0; q < 16; ++q) {
            auto &L = cls[q];   // rows ascending, columns ascending inside a row
            auto &S = sched[q];
            S.clear();
            // pending entries in order of (k-th entry of the row, row)
            std::vector<std::pair<int, uint32_t>> seq;   // (k, entry)
            for (size_t a = 0; a < L.size();) {
                size_t z = a;
                while (z < L.size() && (L[z] >> 16) == (L[a] >> 16)) ++z;
                for (size_t j = a; j < z; ++j) seq.push_back({(int)(j - a), L[j]});
                a = z;
            }
            std::stable_sort(seq.begin(), seq.end(),
                             [](const std::pair<int, uint32_t> &p, const std::pair<int, uint32_t> &r) {
                                 return p.first < r.first;
                             });
            std::vector<char> used(seq.size(), 0);
            size_t left = seq.size(), start = 0;
            while (left) {
                std::vector<uint32_t> step;
                for (size_t j = start; j < seq.size() && step.size() < 4; ++j) {
                    if (used[j]) continue;
                    const uint32_t row = seq[j].second >> 16;
                    bool dup = false;
                    for (uint32_t s2 : step) dup |= (s2 >> 16) == row;
                    if (dup) continue;
                    // a row's earlier entry must already be placed in an earlier step
                    bool ok = true;
                    for (size_t jj = start; jj < j; ++jj)
                        if (!used[jj] && (seq[jj].second >> 16) == row) { ok = false; break; }
                    if (!ok) continue;
                    step.push_back(seq[j].second);
                    used[j] = 1;
                    --left;
                }
                while (start < seq.size() && used[start]) ++start;
                S.push_back(step);
            }
            nst = std::max(nst, S.size());
        }
        for (size_t s = 0; s < nst; ++s) {
            uint64_t m = 0;
            uint32_t lane_ent[64];
            for (int q = 0; q < 16; ++q) {
                if (s >= sched[q].size()) continue;
                const auto &st = sched[q][s];
                for (size_t j = 0; j < st.size(); ++j) {
                    const int l = q + 16 * (int)j;
                    m |= 1ull << l;
                    lane_ent[l] = st[j];
                }
            }
            t.mask.push_back(m);
            for (int l = 0; l < 64; ++l)
                if ((m >> l) & 1) t.ent.push_back(lane_ent[l]);
        }
    }
    t.step_off[nseg] = (int64_t)t.mask.size();
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
    printf("m %ld n %ld nnz %ld H %d W %d G %d: %d row blocks x %d chunks -> %d workgroups, "
           "%zu steps (lane use %.2f, %.1f steps per wave-tile), host %.1f s\n",
           (long)m, (long)n, (long)ip[m], H, W, G, ht.nrb, ht.nchunks, ht.nrb * G,
           ht.mask.size(), util, (double)ht.mask.size() / ((double)ht.nrb * ht.nchunks * NW),
           std::chrono::duration<double>(t1 - t0).count());
    int64_t *d_cc, *d_gc, *d_so, *d_eo;
    uint64_t *d_mask;
    uint32_t *d_ent;
    double *d_x, *d_part;
    CK(hipMalloc(&d_cc, ht.chunk_col.size() * 8));
    CK(hipMalloc(&d_gc, ht.group_chunk.size() * 8));
    CK(hipMalloc(&d_so, ht.step_off.size() * 8));
    CK(hipMalloc(&d_eo, ht.ent_off.size() * 8));
    CK(hipMalloc(&d_mask, ht.mask.size() * 8 + 256));
    CK(hipMalloc(&d_ent, ht.ent.size() * 4 + 256));
    CK(hipMalloc(&d_x, n * 8 + 64));
    CK(hipMalloc(&d_part, (size_t)G * m * 8));
    CK(hipMemcpy(d_cc, ht.chunk_col.data(), ht.chunk_col.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_gc, ht.group_chunk.data(), ht.group_chunk.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_so, ht.step_off.data(), ht.step_off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_eo, ht.ent_off.data(), ht.ent_off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mask, ht.mask.data(), ht.mask.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ent, ht.ent.data(), ht.ent.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), n * 8, hipMemcpyHostToDevice));
    Tiles T{m, n, H, W, ht.nrb, ht.nchunks, ht.ngroups, d_cc, d_gc, d_so, d_eo, d_mask, d_ent};
    const int grid = ht.nrb * G;
    auto run = [&](auto kern, const char *name) {
        const size_t lds = ((size_t)((H + 255) & ~255) + 2 * (size_t)W) * 8;
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
        const double fmt = 4.0 * ht.ent.size() + 8.0 * ht.mask.size() + 8.0 * n * ht.nrb;
        printf("  %-10s %9.1f us  alg %.0f MB -> %.2f TB/s (format %.0f MB)  mismatch-vs-CSR %ld "
               "(max rel %.2e)\n",
               name, us, alg / 1e6, alg / (us * 1e-6) / 1e12, fmt / 1e6, (long)bad, mx);
    };
    run(tile2_k<4, 0>, "b4");
    run(tile2_k<8, 1>, "b8-norow");
    run(tile2_k<4, 2>, "b4-glob");
    run(tile2_k<8, 2>, "b8-glob");
    return 0;
}
