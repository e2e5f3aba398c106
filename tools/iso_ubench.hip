// iso_ubench.hip -- design probe (not product), round 6: where the standalone
// PAVA (iso_packs_kernel<1,false>, 17.0 us at the C3/C4 z layout, 950k
// entries / 50k blocks / 17.4k packs) spends its time.  The same pack plan
// and pava_wave.hpp passes as the product, with knobs:
//   mode 0: one pack per wave, at most `maxpass` + 1 passes (-1: none --
//           load, expand, store), the product at maxpass >= 64
//   mode 1: two packs per wave, passes after the first shared
//           (pava_v1_wave_pair, the product's MERGE form)
//   mode 2: two packs per wave, one after the other
//   mode 3: four packs per workgroup, runs merged across waves (iso_quad)
//   mode 4: pairs of waves, the odd one hands over after `maxpass` passes
//           and exits (iso_pairx)
//   mode 5 / 6: modes 0 / 4 with wave_pass_s (chain bounds by DPP scan)
//   frac:   run only the first frac of the packs (issue- vs latency-bound)
//   wg:     threads per workgroup (64 or 256)
// Prints the median per-launch time over `copies` distinct inputs launched
// back to back (as bench.py's iso leg) and, at maxpass >= 64, whether the
// result equals mode 0's.
//
//   hipcc -O3 --offload-arch=gfx950 -I block-simplex-least-squares_amd/csrc \
//       -o tools/iso_ubench tools/iso_ubench.hip
//   tools/iso_ubench mode maxpass frac wg
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pava_wave.hpp"

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

using namespace bsls;

// mode 5 / 6: wave_pass with the chain bounds from registers: the chain-start
// table (an LDS write and read) and the bpermutes of the chain's first, last
// and folded values (three more LDS round trips) give way to a DPP max-scan
// that hands every lane its chain head (lane, first element, block-start
// flag), a ballot of "this run differs from the previous one of its chain"
// (a non-increasing chain pools iff its first and last values differ iff
// some member differs from its predecessor), and the pooled run kept by the
// chain's LAST lane, which holds the fold; its length is the chain's element
// span.  Same passes, same fold order, same division: bit-identical to
// wave_pass, with one LDS round trip per pass (the survivors' packing)
// instead of four -- and 36 % more VALU (the scan and the 64-bit mask
// searches), measured slower: not in the product.
__device__ __forceinline__ int max_scan_i(int v) {
    // inclusive prefix max over the wave for v >= 0 (identity 0: DPP reads
    // outside a row, and rows a broadcast does not target, give 0)
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ bool wave_pass_s(WaveRuns &s, double *ys, int *ps) {
    const int t = lane_id();
    const bool act = t < s.nh;
    const double yp = dpp_shr1_d(s.Y);
    const bool cs = act & ((s.BS != 0) | !(s.Y <= yp));   // lane 0 is always a block start
    // members after a chain's first that differ from their predecessor: no
    // such member, no chain pools (the converged pack's check pass)
    const uint64_t D = ballot_b(act & !cs & (s.Y != yp));
    if (!D) return false;
    const uint64_t CS = ballot_b(cs);
    // chain head of every lane: (lane, block-start flag, first element)
    const int key = max_scan_i(cs ? ((t << 16) | (s.BS << 15) | s.O) : 0);
    const int mycs = key >> 16;
    const uint64_t above = CS & ~mask_le(t);
    const int nxt = above ? lo_bit(above) : s.nh;       // the next chain's first run
    const bool pool = act & ((D & mask_lt(nxt) & ~mask_le(mycs)) != 0ull);
    const double pr = s.Y * (double)s.W;
    double num = 0.0 + pr;
    // the in-order fold of wave_pass (see there), over pooled chains only
    const int dk = pool ? t - mycs : 0;
    for (int k = 1;; ++k) {
        const bool step = dk >= k;
        if (!ballot_b(step)) break;
        const double np = dpp_shr1_d(num);
        if (step) num = np + pr;
    }
    const bool last = t == nxt - 1;
    if (pool & last) {
        const int oh = key & 0x7FFF;
        const int den = s.O + s.W - oh;                 // the chain's element span
        s.Y = num / (double)den;
        s.W = den;
        s.O = oh;
        s.BS = (key >> 15) & 1;
    }
    // pack the surviving runs into lanes 0 .. nh-1
    const bool surv = act & (!pool | last);
    const uint64_t S = ballot_b(surv);
    if (surv) {
        const int idx = mbcnt64(S);
        ys[idx] = s.Y;
        ps[idx] = s.W | (s.BS << 8) | (s.O << 9);
    }
    s.nh = __popcll(S);
    if (t < s.nh) {
        s.Y = ys[t];
        const int pk = ps[t];
        s.W = pk & 255;
        s.BS = (pk >> 8) & 1;
        s.O = pk >> 9;
    }
    return true;
}


// PS: wave_pass_s (chain bounds by DPP scan) instead of wave_pass
template <bool PS>
__device__ __forceinline__ bool pass_fn(WaveRuns &s, double *ys, int *ps, int *cst) {
    return PS ? wave_pass_s(s, ys, ps) : wave_pass(s, ys, ps, cst);
}

template <int MODE, int WG, bool PS>
__global__ __launch_bounds__(WG) void iso_probe(double *__restrict__ y,
                                                const int64_t *__restrict__ pk_start,
                                                const int64_t *__restrict__ pk_mask,
                                                const int32_t *__restrict__ pk_len,
                                                int64_t npacks, int maxpass) {
    constexpr int NW = WG / WAVE;
    constexpr int PPW = MODE == 0 ? 1 : 2;
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t nw = (int64_t)gridDim.x * NW;
    const int64_t w0 = __builtin_amdgcn_readfirstlane((int)blockIdx.x * NW + wv);
    __shared__ double pv_y[NW][64];
    __shared__ int pv_p[NW][128];
    __shared__ int pv_c[NW][65];
    int64_t s0[PPW];
    int L[PPW];
    uint64_t B[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int64_t pk = w0 + q * nw;
        const int64_t pc = pk < npacks ? pk : npacks - 1;
        s0[q] = pk_start[pc];
        B[q] = (uint64_t)pk_mask[pc];
        L[q] = pk < npacks ? pk_len[pc] : 0;
    }
    double v[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) v[q] = (l < L[q]) ? y[s0[q] + l] : 0.0;
    if (MODE == 1 && L[0] > 0 && L[PPW - 1] > 0) {
        pava_v1_wave_pair(v[0], L[0], B[0], v[PPW - 1], L[PPW - 1], B[PPW - 1], pv_y[wv],
                          pv_p[wv], pv_c[wv]);
    } else {
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            if (L[q] <= 0) continue;
            WaveRuns s = wave_runs(v[q], L[q], B[q], 0);
            for (int pass = 0; pass <= maxpass; ++pass)
                if (!pass_fn<PS>(s, pv_y[wv], pv_p[wv], pv_c[wv])) break;
            v[q] = wave_expand(s, v[q], L[q], 0, pv_p[wv]);
        }
    }
#pragma unroll
    for (int q = 0; q < PPW; ++q)
        if (l < L[q]) y[s0[q] + l] = v[q];
}


// mode 3: a workgroup of four waves takes four packs; passes 1-2 per wave,
// then the two pairs' runs merged into waves 0 and 2 for pass 3 (when each
// pair's runs fit 64 lanes), then all four packs' runs into wave 0 (when
// they fit) for the passes to convergence -- waves whose runs were taken
// idle at the barriers and issue nothing, so later passes cost one wave
// instead of four.  Chains never cross a pack (a pack starts a block), as in
// pava_v1_wave_pair.
__device__ __forceinline__ int run_pack(const WaveRuns &s) { return s.W | (s.BS << 8) | (s.O << 9); }
__device__ __forceinline__ void run_unpack(WaveRuns &s, double y, int pk) {
    s.Y = y;
    s.W = pk & 255;
    s.BS = (pk >> 8) & 1;
    s.O = pk >> 9;
}

__global__ __launch_bounds__(256) void iso_quad(double *__restrict__ y,
                                                const int64_t *__restrict__ pk_start,
                                                const int64_t *__restrict__ pk_mask,
                                                const int32_t *__restrict__ pk_len,
                                                int64_t npacks, int maxpass) {
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t q = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wv);
    __shared__ double sc_y[4][64];
    __shared__ int sc_p[4][64];
    __shared__ int sc_c[4][65];
    __shared__ double xY[256], val[256];
    __shared__ int xP[256], hd[256];
    __shared__ int xn1[4], xm1[4], xn2[4], xm2[4];
    int L = 0;
    int64_t s0 = 0;
    uint64_t B = 0;
    if (q < npacks) {
        s0 = pk_start[q];
        B = (uint64_t)pk_mask[q];
        L = pk_len[q];
        if (L > WAVE) L = 0;
    }
    const double v = (l < L) ? y[s0 + l] : 0.0;
    hd[WAVE * wv + l] = 0;
    WaveRuns s = wave_runs(v, L, B, WAVE * wv);
    double *ys = sc_y[wv];
    int *ps = sc_p[wv], *cst = sc_c[wv];
    bool more = L > 0;
    if (more) more = wave_pass(s, ys, ps, cst);
    if (more) more = wave_pass(s, ys, ps, cst);
    if (l < s.nh) {
        xY[WAVE * wv + l] = s.Y;
        xP[WAVE * wv + l] = run_pack(s);
    }
    if (l == 0) {
        xn1[wv] = s.nh;
        xm1[wv] = more;
    }
    __syncthreads();
    // pairs (0, 1) and (2, 3)
    const bool fit01 = xn1[0] + xn1[1] <= WAVE, fit23 = xn1[2] + xn1[3] <= WAVE;
    const bool fitp = (wv < 2) ? fit01 : fit23;
    bool alive = true;
    if (fitp) {
        if (wv & 1) {
            alive = false;
        } else {
            const int n0 = s.nh, n1 = xn1[wv + 1];
            if (l >= n0 && l < n0 + n1)
                run_unpack(s, xY[WAVE * (wv + 1) + l - n0], xP[WAVE * (wv + 1) + l - n0]);
            s.nh = n0 + n1;
            more = more || xm1[wv + 1] != 0;
        }
    }
    if (alive && more) more = wave_pass(s, ys, ps, cst);
    if (alive && !(wv & 1)) {
        if (l < s.nh) {
            xY[WAVE * wv + l] = s.Y;
            xP[WAVE * wv + l] = run_pack(s);
        }
        if (l == 0) {
            xn2[wv] = s.nh;
            xm2[wv] = more;
        }
    }
    __syncthreads();
    // quad: wave 0 takes wave 2's runs when both pairs merged and all fit
    const bool quad = fit01 && fit23 && xn2[0] + xn2[2] <= WAVE;
    if (quad) {
        if (wv == 2) {
            alive = false;
        } else if (wv == 0) {
            const int n0 = s.nh, n1 = xn2[2];
            if (l >= n0 && l < n0 + n1) run_unpack(s, xY[2 * WAVE + l - n0], xP[2 * WAVE + l - n0]);
            s.nh = n0 + n1;
            more = more || xm2[2] != 0;
        }
    }
    if (alive)
        for (int pass = 0; more && pass <= 4 * WAVE; ++pass) more = wave_pass(s, ys, ps, cst);
    if (alive && l < s.nh) {
        val[s.O] = s.Y;
        hd[s.O] = 1;
    }
    __syncthreads();
    const uint64_t RS = ballot_b((l < L) & (hd[WAVE * wv + l] != 0));
    const uint64_t below = RS & mask_le(l);
    const int h = below ? hi_bit(below) : 0;
    const double r = val[WAVE * wv + h];
    if (l < L) y[s0 + l] = r;
}


// mode 4: pairs of waves; pass 1 per wave, then (when the pair's runs fit
// 64 lanes) the odd wave hands its runs and its pack's place to the even
// wave and exits -- one barrier, no wave idles at a later one -- and the even
// wave runs the remaining passes and expands and stores both packs
template <bool PS>
__global__ __launch_bounds__(256) void iso_pairx(double *__restrict__ y,
                                                 const int64_t *__restrict__ pk_start,
                                                 const int64_t *__restrict__ pk_mask,
                                                 const int32_t *__restrict__ pk_len,
                                                 int64_t npacks, int npre) {
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t q = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wv);
    __shared__ double sc_y[4][64];
    __shared__ int sc_p[4][64];
    __shared__ int sc_c[4][65];
    __shared__ double xY[256];
    __shared__ int xP[256];
    __shared__ int xn[4], xm[4], xL[4];
    __shared__ int64_t xs[4];
    int L = 0;
    int64_t s0 = 0;
    uint64_t B = 0;
    if (q < npacks) {
        s0 = pk_start[q];
        B = (uint64_t)pk_mask[q];
        L = pk_len[q];
        if (L > WAVE) L = 0;
    }
    const double v = (l < L) ? y[s0 + l] : 0.0;
    WaveRuns s = wave_runs(v, L, B, WAVE * (wv & 1));
    double *ys = sc_y[wv];
    int *ps = sc_p[wv], *cst = sc_c[wv];
    bool more = L > 0;
    for (int k = 0; k < npre && more; ++k) more = pass_fn<PS>(s, ys, ps, cst);
    if (l < s.nh) {
        xY[WAVE * wv + l] = s.Y;
        xP[WAVE * wv + l] = run_pack(s);
    }
    if (l == 0) {
        xn[wv] = s.nh;
        xm[wv] = more;
        xL[wv] = L;
        xs[wv] = s0;
    }
    __syncthreads();
    const int pa = wv & ~1;
    const bool fit = xn[pa] + xn[pa + 1] <= WAVE;
    if (fit && (wv & 1)) return;
    int Lb = 0;
    int64_t sb = 0;
    if (fit) {
        const int n0 = s.nh, n1 = xn[wv + 1];
        if (l >= n0 && l < n0 + n1) run_unpack(s, xY[WAVE * (wv + 1) + l - n0], xP[WAVE * (wv + 1) + l - n0]);
        s.nh = n0 + n1;
        more = more || xm[wv + 1] != 0;
        Lb = xL[wv + 1];
        sb = xs[wv + 1];
    }
    for (int pass = 0; more && pass <= 2 * WAVE; ++pass) more = pass_fn<PS>(s, ys, ps, cst);
    if (!fit) {
        const double r = wave_expand(s, v, L, WAVE * (wv & 1), ps);
        if (l < L) y[s0 + l] = r;
        return;
    }
    // expand over the 128 element slots (a's at 0.., b's at 64..), as
    // pava_v1_wave_pair; xP is free again (only this wave reads its pair's)
    int *pf = xP + WAVE * pa;
    pf[l] = 0;
    pf[WAVE + l] = 0;
    if (l < s.nh) pf[s.O] = 1;
    const uint64_t RA = __ballot(l < L && pf[l] != 0);
    const uint64_t RB = __ballot(l < Lb && pf[WAVE + l] != 0);
    const int ia = mbcnt64(RA) + (int)((RA >> l) & 1ull) - 1;
    const int ib = __popcll(RA) + mbcnt64(RB) + (int)((RB >> l) & 1ull) - 1;
    const double va = shfl_d(s.Y, ia < 0 ? 0 : ia);
    const double vb = shfl_d(s.Y, ib < 0 ? 0 : ib);
    if (l < L) y[s0 + l] = va;
    if (l < Lb) y[sb + l] = vb;
}

template <int MODE, int WG, bool PS = false>
static void launch(double *y, const int64_t *ps, const int64_t *pm, const int32_t *pl,
                   int64_t np, int maxpass) {
    constexpr int NW = WG / WAVE;
    const int64_t waves = MODE == 0 ? np : (np + 1) / 2;
    const int grid = (int)((waves + NW - 1) / NW);
    iso_probe<MODE, WG, PS><<<grid, WG>>>(y, ps, pm, pl, np, maxpass);
}

int main(int argc, char **argv) {
    if (argc < 5) {
        printf("usage: iso_ubench mode maxpass frac wg\n");
        return 2;
    }
    const int mode = atoi(argv[1]), maxpass = atoi(argv[2]), wg = atoi(argv[4]);
    const double frac = atof(argv[3]);
    if (mode < 0 || mode > 6 || (wg != 64 && wg != 256) || !(frac > 0 && frac <= 1)) return 2;
    // the bench's layout: 1M routes in 50k blocks (every block >= 1 route),
    // z entries = routes - 1 per block
    const int64_t n = 1000000, p = 50000;
    std::mt19937_64 rng(7);
    std::vector<int64_t> sizes(p, 1);
    for (int64_t i = 0; i < n - p; ++i) sizes[rng() % p] += 1;
    std::vector<int64_t> zs(p);
    int64_t nz = 0;
    for (int64_t b = 0; b < p; ++b) {
        zs[b] = nz;
        nz += sizes[b] - 1;
    }
    // the product's pack plan (bsls_isotonic_pack_plan): runs of whole
    // consecutive blocks with <= 64 elements
    std::vector<int64_t> pst, pmk;
    std::vector<int32_t> pln;
    for (int64_t b = 0; b < p;) {
        int64_t tot = 0, e = b;
        uint64_t m = 0;
        while (e < p) {
            const int64_t k = sizes[e] - 1;
            if (k > 64 || tot + k > 64) break;
            if (k > 0) m |= 1ull << tot;
            tot += k;
            ++e;
        }
        if (e == b) {
            printf("block longer than a wave\n");
            return 1;
        }
        pst.push_back(zs[b]);
        pmk.push_back((int64_t)m);
        pln.push_back((int32_t)tot);
        b = e;
    }
    const int64_t np_all = (int64_t)pst.size();
    const int64_t np = std::max<int64_t>(1, (int64_t)(np_all * frac));
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> G(0.0, 1.0);
    std::vector<double> y0(nz);
    for (auto &v : y0) v = U(rng) - 0.3 * G(rng);
    const int copies = 16;
    double *dy, *dref;
    int64_t *dps, *dpm;
    int32_t *dpl;
    CK(hipMalloc(&dy, (size_t)copies * nz * 8));
    CK(hipMalloc(&dref, (size_t)nz * 8));
    CK(hipMalloc(&dps, np_all * 8));
    CK(hipMalloc(&dpm, np_all * 8));
    CK(hipMalloc(&dpl, np_all * 4));
    CK(hipMemcpy(dps, pst.data(), np_all * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpm, pmk.data(), np_all * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpl, pln.data(), np_all * 4, hipMemcpyHostToDevice));
    auto run = [&](double *y) {
        if (mode == 0) {
            if (wg == 64) launch<0, 64>(y, dps, dpm, dpl, np, maxpass);
            else launch<0, 256>(y, dps, dpm, dpl, np, maxpass);
        } else if (mode == 1) {
            if (wg == 64) launch<1, 64>(y, dps, dpm, dpl, np, maxpass);
            else launch<1, 256>(y, dps, dpm, dpl, np, maxpass);
        } else if (mode == 4 || mode == 6) {
            if (mode == 4) iso_pairx<false><<<(int)((np + 3) / 4), 256>>>(y, dps, dpm, dpl, np, maxpass);
            else iso_pairx<true><<<(int)((np + 3) / 4), 256>>>(y, dps, dpm, dpl, np, maxpass);
        } else if (mode == 5) {
            if (wg == 64) launch<0, 64, true>(y, dps, dpm, dpl, np, maxpass);
            else launch<0, 256, true>(y, dps, dpm, dpl, np, maxpass);
        } else if (mode == 3) {
            iso_quad<<<(int)((np + 3) / 4), 256>>>(y, dps, dpm, dpl, np, maxpass);
        } else {
            if (wg == 64) launch<2, 64>(y, dps, dpm, dpl, np, maxpass);
            else launch<2, 256>(y, dps, dpm, dpl, np, maxpass);
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int rep = 0; rep < 7; ++rep) {
        for (int c = 0; c < copies; ++c)
            CK(hipMemcpy(dy + (size_t)c * nz, y0.data(), nz * 8, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int c = 0; c < copies; ++c) run(dy + (size_t)c * nz);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f / copies);
    }
    std::sort(ts.begin(), ts.end());
    // reference result: mode 0, all passes
    CK(hipMemcpy(dref, y0.data(), nz * 8, hipMemcpyHostToDevice));
    launch<0, 256>(dref, dps, dpm, dpl, np, 1 << 20);
    CK(hipDeviceSynchronize());
    std::vector<double> got(nz), ref(nz);
    CK(hipMemcpy(got.data(), dy, nz * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref.data(), dref, nz * 8, hipMemcpyDeviceToHost));
    const bool same = memcmp(got.data(), ref.data(), nz * 8) == 0;
    printf("mode %d maxpass %d frac %.2f wg %d packs %ld/%ld nz %ld: %.2f us (min %.2f) %s\n",
           mode, maxpass, frac, wg, (long)np, (long)np_all, (long)nz, ts[ts.size() / 2], ts[0],
           (maxpass >= 64 || mode == 4 || mode == 6) ? (same ? "same" : "DIFFERS") : "-");
    return 0;
}
