// panel_ubench.hip -- design experiments on the panel SpMV loop (not product code).
// Variants of K2's chunk loop over a real panel image (device.plan_panels):
//   0 full: stage chunk + walk segments (block DMA path if blk_cap > 0)
//   1 stage only
#include "../block-simplex-least-squares_amd/csrc/panels.hpp"

using namespace bsls;

// Knock-out copy of panel_chunks (MODE 2, csrc/panels.hpp):
//   KO & 1: no LDS gathers (add the column offset instead)
//   KO & 2: no entry loads (column = lane + k)
//   KO & 4: no count loads (every row 3 entries)
//   KO & 8: no staging (chunk 0 staged once, no per-chunk barriers)
template <int KO>
__global__ __launch_bounds__(1024) void k2_ko(bsls_panels M, const double *__restrict__ r,
                                              const double *__restrict__ colv,
                                              double *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = lane_id();
    const int64_t panel = (int64_t)blockIdx.x * PANEL_WAVES + wv;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, sc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
        const int64_t i = panel * M.prow + 64 * q + lane;
        if (panel < M.npanels && 64 * q + lane <= M.prow && i < M.rows) sc[q] = colv[i];
    }
    const bool live = panel < M.npanels;
    const int64_t seg0 = ((int64_t)blockIdx.x * M.nchunks) * PANEL_WAVES + wv;
    auto seg = [&](int64_t c) { return seg0 + c * PANEL_WAVES; };
    struct Body {
        int D[4], cnt[4];
        uint32_t base[4];
        uint32_t c2[4][4];
    };
    auto head = [&](int64_t sg, int (&D)[4], int (&incl)[4], int64_t &e0) {
        const int64_t info = live ? M.seg_info[sg] : 0;
        int64_t co = live ? M.cnt_off[sg] : 0;
        e0 = live ? M.ent_off[sg] : 0;
        for (int q = 0; q < 4; ++q) {
            D[q] = (int)((info >> (16 * q)) & 0xFFFF);
            incl[q] = 0;
            if (D[q] > 0) {
                incl[q] = (KO & 4) ? 6 * (lane + 1) : (int)M.cnt[co + lane];
                co += 64;
            }
        }
    };
    auto body = [&](Body &b, const int (&D)[4], const int (&incl)[4], int64_t e0) {
        const char *ent = (const char *)(M.ent + e0);
        uint32_t e = 0;
        for (int q = 0; q < 4; ++q) {
            b.D[q] = D[q];
            b.cnt[q] = 0;
            b.base[q] = 0;
            if (D[q] > 0) {
                const int inc = incl[q] & ~1;
                const int ex = wave_shr1(incl[q]) & ~1;
                b.cnt[q] = inc - ex - (incl[q] & 1);
                b.base[q] = e + (uint32_t)ex;
                e += (uint32_t)(readlane_i(incl[q], 63) & ~1);
                for (int j = 0; j < 4; ++j)
                    if (2 * j < D[q])
                        b.c2[q][j] = (KO & 2) ? (uint32_t)((lane * 37 + j * 101) % 19000) * 0x10001u
                                              : *(const uint32_t *)(ent + (b.base[q] + 2 * j) * 2u);
            }
        }
    };
    auto walk = [&](const Body &b) {
        for (int q = 0; q < 4; ++q) {
            if (b.D[q] == 0) continue;
            for (int k = 0; k < 8; ++k) {
                if (k < b.D[q] && k < b.cnt[q]) {
                    const uint32_t w = b.c2[q][k >> 1];
                    const uint32_t ci = (k & 1) ? (w >> 16) : (w & 0xFFFFu);
                    const double a = (KO & 1) ? (double)ci : lds[ci];
                    s[q] += sc[q] * a;
                }
            }
        }
    };
    int Da[4], Ia[4], Db[4], Ib[4];
    int64_t ea, eb;
    Body ba, bb;
    head(seg(0), Da, Ia, ea);
    body(ba, Da, Ia, ea);
    if (1 < M.nchunks) head(seg(1), Db, Ib, eb);
    if (KO & 8) {
        __syncthreads();
        panel_stage(lds, r, (int)(M.chunk_col[1] - M.chunk_col[0]));
        __syncthreads();
    }
    auto step = [&](int64_t c, const Body &cur, int (&Dn)[4], int (&In)[4], int64_t &en,
                    Body &bn, int (&Dn2)[4], int (&In2)[4], int64_t &en2) {
        if (!(KO & 8)) {
            const int64_t col0 = M.chunk_col[c];
            __syncthreads();
            panel_stage(lds, r + col0, (int)(M.chunk_col[c + 1] - col0));
            __syncthreads();
        }
        if (c + 1 < M.nchunks) body(bn, Dn, In, en);
        if (c + 2 < M.nchunks) head(seg(c + 2), Dn2, In2, en2);
        if (live) walk(cur);
    };
    for (int64_t c = 0; c < M.nchunks; c += 2) {
        step(c, ba, Db, Ib, eb, bb, Da, Ia, ea);
        if (c + 1 < M.nchunks) step(c + 1, bb, Da, Ia, ea, ba, Db, Ib, eb);
    }
    if (panel >= M.npanels) return;
    for (int q = 0; q < 4; ++q) {
        const int i = 64 * q + lane;
        const int64_t row = panel * M.prow + i;
        if (i < M.prow && row < M.rows) out[row] = s[q];
    }
}

template <int KO>
static float run_ko(const bsls_panels *M, const double *r, const double *colv, double *out, int reps) {
    auto k = k2_ko<KO>;
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 512);
    const int grid = (int)((M->npanels + PANEL_WAVES - 1) / PANEL_WAVES);
    const size_t lds = panel_lds_bytes(*M);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<<<grid, 1024, lds>>>(*M, r, colv, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) k<<<grid, 1024, lds>>>(*M, r, colv, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

extern "C" float panel_ko(int ko, const bsls_panels *M, const double *r, const double *colv,
                          double *out, int reps) {
    switch (ko) {
        case 0: return run_ko<0>(M, r, colv, out, reps);
        case 1: return run_ko<1>(M, r, colv, out, reps);
        case 2: return run_ko<2>(M, r, colv, out, reps);
        case 3: return run_ko<3>(M, r, colv, out, reps);
        case 4: return run_ko<4>(M, r, colv, out, reps);
        case 7: return run_ko<7>(M, r, colv, out, reps);
        case 8: return run_ko<8>(M, r, colv, out, reps);
        case 9: return run_ko<9>(M, r, colv, out, reps);
        case 10: return run_ko<10>(M, r, colv, out, reps);
        case 11: return run_ko<11>(M, r, colv, out, reps);
        case 15: return run_ko<15>(M, r, colv, out, reps);
    }
    return -1.f;
}

template <int VAR>
__global__ __launch_bounds__(1024) void k2_var(bsls_panels M, const double *__restrict__ r,
                                               const double *__restrict__ colv,
                                               double *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = lane_id();
    const int64_t panel = (int64_t)blockIdx.x * PANEL_WAVES + wv;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, sc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
        const int64_t i = panel * M.prow + 64 * q + lane;
        if (panel < M.npanels && 64 * q + lane <= M.prow && i < M.rows) sc[q] = colv[i];
    }
    if (VAR == 0) {
        panel_chunks<2>(M, blockIdx.x, wv, 0, M.nchunks, r, lds, s, sc);
    } else {
        for (int64_t c = 0; c < M.nchunks; ++c) {
            const int64_t col0 = M.chunk_col[c];
            __syncthreads();
            panel_stage(lds, r + col0, (int)(M.chunk_col[c + 1] - col0));
            __syncthreads();
        }
    }
    if (panel >= M.npanels) return;
    for (int q = 0; q < 4; ++q) {
        const int i = 64 * q + lane;
        const int64_t row = panel * M.prow + i;
        if (i < M.prow && row < M.rows) out[row] = s[q];
    }
}

// Timeline of the product chunk loop (copy of panel_chunks<2> with s_memtime
// stamps): per chunk step, for wave 0 of every workgroup: [0] before loads,
// [1] after body/head issue, [2] after the walk, [3] after barrier A,
// [4] after the DMA issue, [5] after barrier B.
__global__ __launch_bounds__(1024) void k2_trace(bsls_panels M, const double *__restrict__ r,
                                                 const double *__restrict__ colv,
                                                 double *__restrict__ out, long long *T) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = lane_id();
    const int64_t panel = (int64_t)blockIdx.x * PANEL_WAVES + wv;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, sc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
        const int64_t i = panel * M.prow + 64 * q + lane;
        if (panel < M.npanels && 64 * q + lane <= M.prow && i < M.rows) sc[q] = colv[i];
    }
    long long *t = T + (int64_t)blockIdx.x * 64;
    const bool rec = (wv == 0 && lane == 0);
    if (rec) t[0] = wall_clock64();
    const bool live = panel < M.npanels;
    const int64_t c0 = 0, c1 = M.nchunks;
    const int64_t seg0 = ((int64_t)blockIdx.x * M.nchunks) * PANEL_WAVES + wv;
    auto seg = [&](int64_t c) { return seg0 + c * PANEL_WAVES; };
    SegHead ha, hb;
    SegBody<2> ba, bb;
    {
        int64_t a, b;
        sload2(M.chunk_col + c0, M.chunk_col + c0 + 1, a, b);
        panel_stage(lds, r + a, (int)(b - a));
    }
    ha.load(M, seg(c0), live);
    ba.load(M, ha);
    if (c0 + 1 < c1) hb.load(M, seg(c0 + 1), live);
    if (rec) t[1] = wall_clock64();
    int ti = 2;
    auto step = [&](int64_t c, const SegBody<2> &cur, SegHead &hn, SegBody<2> &bn, SegHead &hn2) {
        if (c > c0) {
            int64_t a, b;
            sload2(M.chunk_col + c, M.chunk_col + c + 1, a, b);
            __syncthreads();
            if (rec) t[ti++] = wall_clock64();
            panel_stage(lds, r + a, (int)(b - a));
        } else if (rec) {
            t[ti++] = wall_clock64();
        }
        __syncthreads();
        if (rec) t[ti++] = wall_clock64();
        const long long tw0 = wall_clock64();
        if (live) cur.walk(M, lds, s, sc);
        {
            double z = s[0] + s[1] + s[2] + s[3];
            const long long tw1 = wall_clock64() + (z == 12345.678 ? 1 : 0);
            int deep = 0;
            for (int q = 0; q < 4; ++q) deep |= (cur.D[q] > 8) << q;
            if (lane == 0 && c < 5) {
                long long *u = T + 4096 * 64 + ((int64_t)blockIdx.x * 16 + wv) * 16;
                u[2 * c] = tw1 - tw0;
                u[2 * c + 1] = deep;
            }
        }
        if (c + 1 < c1) bn.load(M, hn);
        if (c + 2 < c1) hn2.load(M, seg(c + 2), live);
        if (rec) {
            // the walk's adds are done when s is: force it
            double z = s[0] + s[1] + s[2] + s[3];
            t[ti++] = wall_clock64() + (z == 12345.678 ? 1 : 0);
        }
    };
    for (int64_t c = c0; c < c1; c += 2) {
        step(c, ba, hb, bb, ha);
        if (c + 1 < c1) step(c + 1, bb, ha, ba, hb);
    }
    if (rec) t[63] = wall_clock64();
    if (panel >= M.npanels) return;
    for (int q = 0; q < 4; ++q) {
        const int i = 64 * q + lane;
        const int64_t row = panel * M.prow + i;
        if (i < M.prow && row < M.rows) out[row] = s[q];
    }
}

extern "C" int panel_trace(const bsls_panels *M, const double *r, const double *colv, double *out,
                           long long *T) {
    hipFuncSetAttribute((const void *)k2_trace, hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 512);
    const int grid = (int)((M->npanels + PANEL_WAVES - 1) / PANEL_WAVES);
    const size_t lds = panel_lds_bytes(*M);
    for (int i = 0; i < 3; ++i) k2_trace<<<grid, 1024, lds>>>(*M, r, colv, out, T);
    hipDeviceSynchronize();
    return grid;
}

template <int VAR>
static float run(const bsls_panels *M, const double *r, const double *colv, double *out, int reps) {
    auto k = k2_var<VAR>;
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 512);
    const int grid = (int)((M->npanels + PANEL_WAVES - 1) / PANEL_WAVES);
    const size_t lds = panel_lds_bytes(*M);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<<<grid, 1024, lds>>>(*M, r, colv, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) k<<<grid, 1024, lds>>>(*M, r, colv, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms * 1000.f / reps;
}

extern "C" float panel_ubench(int var, const bsls_panels *M, const double *r, const double *colv,
                              double *out, int reps) {
    switch (var) {
        case 0: return run<0>(M, r, colv, out, reps);
        case 1: return run<1>(M, r, colv, out, reps);
    }
    return -1.f;
}
