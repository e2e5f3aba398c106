// tile_ubench.hip -- design probe for the sparse-regime SpMV (not product code).
//
// Tile format: row blocks of H rows x column chunks of <= W columns.  A
// workgroup owns one row block (and one of G column groups): its H running
// row sums live in LDS for the whole launch, the x chunk is staged into LDS by
// LDS-DMA, and every entry of the tile -- (local row << 16 | local column),
// 4 B -- is one LDS gather plus one LDS f64 atomic add.  Wave w owns the local
// rows lr with lr % NW == w, so no two waves add to one row (deterministic).
// Question this answers: how fast, and is a row summed in entry order (lane
// order inside one ds_add instruction), i.e. bit-identical to CSR order?
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o build/tile_ubench tools/tile_ubench.hip
//   build/tile_ubench m n per_col H W G [reps]
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
    const int64_t *chunk_col, *group_chunk, *off;
    const uint32_t *ent;
};

constexpr int NW = 16;

// OP 0: LDS f64 atomic add; 1: plain read-modify-write (racy inside an
// instruction: timing only); 2: gathers only (summed in a register); 3: entry
// loads only
template <int U, bool DB, int OP = 0>
__global__ __launch_bounds__(NW * 64) void tile_k(Tiles T, const double *__restrict__ x,
                                                  double *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int HR = (T.H + 1) & ~1;
    double *rows = lds;
    double *tab[2] = {lds + HR, lds + HR + (DB ? T.W : 0)};
    const int64_t G = T.ngroups;
    const int64_t g = blockIdx.x % G, rb = blockIdx.x / G;
    const int wv = threadIdx.x / 64, lane = lane_id();
    for (int i = threadIdx.x; i < HR; i += blockDim.x) rows[i] = 0.0;
    const int64_t c0 = T.group_chunk[g], c1 = T.group_chunk[g + 1];
    panel_stage(tab[0], x + T.chunk_col[c0], (int)(T.chunk_col[c0 + 1] - T.chunk_col[c0]));
    for (int64_t c = c0; c < c1; ++c) {
        const int b = DB ? (int)((c - c0) & 1) : 0;
        __syncthreads();
        if (DB && c + 1 < c1)
            panel_stage(tab[b ^ 1], x + T.chunk_col[c + 1],
                        (int)(T.chunk_col[c + 2] - T.chunk_col[c + 1]));
        const double *tb = tab[b];
        const int64_t sg = (rb * T.nchunks + c) * NW + wv;
        const int64_t s = T.off[sg], e = T.off[sg + 1];
        double acc = 0.0;
        for (int64_t i0 = s; i0 < e; i0 += 64 * U) {
            uint32_t u[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int64_t i = i0 + 64 * k + lane;
                u[k] = i < e ? T.ent[i] : 0xFFFFFFFFu;
            }
            double v[U];
#pragma unroll
            for (int k = 0; k < U; ++k) v[k] = tb[u[k] == 0xFFFFFFFFu ? 0 : (u[k] & 0xFFFFu)];
#pragma unroll
            for (int k = 0; k < U; ++k)
                if (u[k] != 0xFFFFFFFFu) {
                    if (OP == 0)
                        __hip_atomic_fetch_add(&rows[u[k] >> 16], v[k], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                    else if (OP == 1)
                        rows[u[k] >> 16] += v[k];
                    else if (OP == 2)
                        acc += v[k];
                    else
                        acc += (double)u[k];
                }
        }
        if (OP >= 2 && acc == 12345.678) rows[lane] = acc;
        if (!DB && c + 1 < c1) {
            __syncthreads();
            panel_stage(tab[0], x + T.chunk_col[c + 1],
                        (int)(T.chunk_col[c + 2] - T.chunk_col[c + 1]));
        }
    }
    __syncthreads();
    const int64_t r0 = rb * T.H;
    for (int i = threadIdx.x; i < T.H; i += blockDim.x)
        if (r0 + i < T.rows) part[g * T.rows + r0 + i] = rows[i];
}

// host -----------------------------------------------------------------------
struct HostTiles {
    int H, W, nrb, nchunks, ngroups;
    std::vector<int64_t> chunk_col, group_chunk, off;
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
    // equal chunks, even starts
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
    const int64_t nseg = (int64_t)t.nrb * nch * NW;
    std::vector<int64_t> cnt(nseg + 1, 0);
    for (int64_t i = 0; i < R; ++i) {
        const int64_t rb = i / H, lr = i % H, w = lr % NW;
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) cnt[(rb * nch + chunk_of[ix[k]]) * NW + w + 1]++;
    }
    for (int64_t s = 0; s < nseg; ++s) cnt[s + 1] += cnt[s];
    t.off = cnt;
    t.ent.resize(ip[R]);
    std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
    for (int64_t i = 0; i < R; ++i) {
        const int64_t rb = i / H, lr = i % H, w = lr % NW;
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
            const int64_t c = chunk_of[ix[k]];
            const int64_t sg = (rb * nch + c) * NW + w;
            t.ent[cur[sg]++] = ((uint32_t)lr << 16) | (uint32_t)(ix[k] - t.chunk_col[c]);
        }
    }
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
    // pc > 0: every column has pc distinct uniform rows (A); pc < 0: every row
    // has -pc distinct uniform columns (A')
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
    printf("m %ld n %ld nnz %ld H %d W %d G %d: %d row blocks x %d chunks -> %d workgroups, "
           "host %.1f s\n",
           (long)m, (long)n, (long)ip[m], H, W, G, ht.nrb, ht.nchunks, ht.nrb * G,
           std::chrono::duration<double>(t1 - t0).count());
    int64_t *d_cc, *d_gc, *d_off;
    uint32_t *d_ent;
    double *d_x, *d_part;
    CK(hipMalloc(&d_cc, ht.chunk_col.size() * 8));
    CK(hipMalloc(&d_gc, ht.group_chunk.size() * 8));
    CK(hipMalloc(&d_off, ht.off.size() * 8));
    CK(hipMalloc(&d_ent, ht.ent.size() * 4 + 256));
    CK(hipMalloc(&d_x, n * 8 + 64));
    CK(hipMalloc(&d_part, (size_t)G * m * 8));
    CK(hipMemcpy(d_cc, ht.chunk_col.data(), ht.chunk_col.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_gc, ht.group_chunk.data(), ht.group_chunk.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, ht.off.data(), ht.off.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ent, ht.ent.data(), ht.ent.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), n * 8, hipMemcpyHostToDevice));
    Tiles T{m, n, H, W, ht.nrb, ht.nchunks, ht.ngroups, d_cc, d_gc, d_off, d_ent};
    const int grid = ht.nrb * G;
    auto run = [&](auto kern, bool db, const char *name) {
        const size_t lds = ((size_t)((H + 1) & ~1) + (db ? 2 : 1) * (size_t)W) * 8;
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
        // determinism: a second run must match bit for bit
        std::vector<double> p2((size_t)G * m);
        kern<<<grid, NW * 64, lds>>>(T, d_x, d_part);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(p2.data(), d_part, p2.size() * 8, hipMemcpyDeviceToHost));
        const bool det = memcmp(p.data(), p2.data(), p.size() * 8) == 0;
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
        printf("  %-10s %9.1f us  alg %.0f MB -> %.2f TB/s  mismatch-vs-CSR-order %ld (max rel "
               "%.2e)  deterministic %d\n",
               name, us, alg / 1e6, alg / (us * 1e-6) / 1e12, (long)bad, mx, (int)det);
    };
    run(tile_k<4, false, 0>, false, "atomic");
    run(tile_k<4, false, 1>, false, "rmw");
    run(tile_k<4, false, 2>, false, "gather");
    run(tile_k<4, false, 3>, false, "loads");
    run(tile_k<4, true, 0>, true, "atomic-db");
    run(tile_k<4, true, 1>, true, "rmw-db");
    run(tile_k<4, true, 2>, true, "gather-db");
    return 0;
}
