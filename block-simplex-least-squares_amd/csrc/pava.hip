// pava.hip -- multi-block isotonic regression entry point
// (replaces isotonic_regression_multi{,_2,_3}, isotonic_regression.h:85-102,157-164).
//
// Layout: one 64-lane workgroup per 64 consecutive blocks, one lane per block.
// The wave's contiguous element range is staged into LDS with coalesced loads
// (y as fp64, run lengths as int32), every lane runs the serial PAVA of its own
// block in LDS, and the range is written back coalesced.  A wave whose range
// exceeds ISO_CAP elements runs the same code on global memory instead (run
// lengths then live in the caller's weight array or in the workspace).
//
// The path main.py takes (variant 1, weight=None, update=1 -- fresh unit run
// lengths, c_extensions.pyx:84-85) runs wave-parallel instead (iso_pack_kernel,
// the compacted PAVA of pava_wave.hpp that K3 runs, bit-identical): a planning
// pass maps every 32-element window to the blocks starting in it; wave q takes
// windows 2q and 2q + 1 as one pack when their blocks span at most 64
// elements, else each window's blocks as a pack of at most 63 elements (every
// block but a window's last is shorter than 32, the last is taken on its own
// when it is longer; one longer than a wave goes to iso_long_kernel, a
// workgroup per block, pava_long.hpp), so no host plan is needed.
#include "pava.hpp"
#include "pava_long.hpp"
#include "pava_wave.hpp"

namespace bsls {

constexpr int ISO_CAP = 2048;

template <int VARIANT>
__global__ __launch_bounds__(WAVE) void iso_kernel(double *__restrict__ y,
                                                   const int64_t *__restrict__ starts,
                                                   int64_t nb, int64_t n,
                                                   int32_t *__restrict__ wio, int expand,
                                                   int32_t *__restrict__ wscratch,
                                                   int32_t *__restrict__ status) {
    __shared__ double ly[ISO_CAP];
    __shared__ int32_t lw[ISO_CAP];
    const int lane = lane_id();
    const int64_t b0 = (int64_t)blockIdx.x * WAVE;
    const int64_t b = b0 + lane;
    const bool valid = b < nb;
    const int64_t s = valid ? starts[b] : 0;
    const int64_t e = valid ? block_end(starts, nb, b, n) : 0;
    const int64_t blast = (b0 + WAVE - 1 < nb) ? b0 + WAVE - 1 : nb - 1;
    const int64_t R0 = starts[b0];
    const int64_t R = block_end(starts, nb, blast, n) - R0;
    bool ok = true;
    if (R <= ISO_CAP) {
        const int r = (int)R;
        for (int j = lane; j < r; j += WAVE) {
            ly[j] = y[R0 + j];
            if (VARIANT != 2) lw[j] = wio ? wio[R0 + j] : 1;
        }
        __syncthreads();
        if (valid) {
            const int lo = (int)(s - R0), hi = (int)(e - R0);
            if (VARIANT == 1) ok = pava_v1(ly, lw, lo, hi, expand);
            else if (VARIANT == 2) pava_v2(ly, lo, hi);
            else ok = pava_v3(ly, lw, lo, hi, expand);
        }
        __syncthreads();
        for (int j = lane; j < r; j += WAVE) {
            y[R0 + j] = ly[j];
            if (VARIANT != 2 && wio) wio[R0 + j] = lw[j];
        }
    } else if (valid) {
        if (VARIANT == 2) {
            pava_v2(y, s, e);
        } else {
            int32_t *W = wio ? wio : wscratch;
            if (!wio)
                for (int64_t j = s; j < e; ++j) W[j] = 1;
            ok = (VARIANT == 1) ? pava_v1(y, W, s, e, expand) : pava_v3(y, W, s, e, expand);
        }
    }
    if (!ok && status) atomicOr(status, 1);
}

constexpr int ISO_WIN = 32;   // pack window (elements)

inline int64_t iso_nwin(int64_t n) { return (n + ISO_WIN - 1) / ISO_WIN; }

// workspace: [Y0 n][Y1 n] doubles, [wscratch n][W0 n][W1 n][CH n+1][plan nwin+1]
// [long count 4][long list n/65+1] int32 (long-block runs indexed by element)
struct IsoWork {
    double *Y0, *Y1;
    int32_t *ws, *W0, *W1, *CH, *plan, *lcnt, *llist;
    size_t bytes;
};

static IsoWork iso_layout(void *base, int64_t n) {
    IsoWork w{};
    char *p = (char *)base;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *q = p + off;
        off += (bytes + 15) & ~(size_t)15;
        return q;
    };
    w.Y0 = (double *)take((size_t)n * 8);
    w.Y1 = (double *)take((size_t)n * 8);
    w.ws = (int32_t *)take((size_t)n * 4);
    w.W0 = (int32_t *)take((size_t)n * 4);
    w.W1 = (int32_t *)take((size_t)n * 4);
    w.CH = (int32_t *)take((size_t)(n + 1) * 4);
    w.plan = (int32_t *)take((size_t)(iso_nwin(n) + 1) * 4);
    w.lcnt = (int32_t *)take(16);
    w.llist = (int32_t *)take((size_t)(n / (WAVE + 1) + 1) * 4);
    w.bytes = off;
    return w;
}

// win_first[w] = first block starting at or after element 32 w (w = 0 .. nwin)
__global__ __launch_bounds__(256) void iso_plan_kernel(const int64_t *__restrict__ starts,
                                                       int64_t nb, int64_t nwin,
                                                       int32_t *__restrict__ win_first,
                                                       int32_t *__restrict__ lcnt) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0 && lcnt) *lcnt = 0;
    if (b > nb) return;
    const int64_t lo = (b == 0) ? 0 : (starts[b - 1] / ISO_WIN) + 1;
    const int64_t hi = (b == nb) ? nwin : starts[b] / ISO_WIN;
    for (int64_t w = lo; w <= hi; ++w) win_first[w] = (int32_t)b;
}

// one wave-parallel PAVA v1 (unit weights, expand) over y[s0, s0 + L), L <= 64,
// blocks starting at the set bits of B
__device__ __forceinline__ void iso_wave_pack(double *__restrict__ y, int64_t s0, int L,
                                              uint64_t B, double *ys, int *ps, int *cst) {
    const int l = lane_id();
    double v = (l < L) ? y[s0 + l] : 0.0;
    pava_v1_wave_c(v, L, B, ys, ps, cst);
    if (l < L) y[s0 + l] = v;
}

// window blocks [f, e): one pack of <= 63 elements, the last block on its own
// when it is longer than the window
__device__ __forceinline__ void iso_window(double *__restrict__ y,
                                           const int64_t *__restrict__ starts, int64_t nb,
                                           int64_t n, int64_t f, int64_t e,
                                           int32_t *__restrict__ lcnt,
                                           int32_t *__restrict__ llist, double *ys, int *ps,
                                           int *cst) {
    const int l = lane_id();
    if (f >= e) return;
    const int64_t s0 = starts[f], sl = starts[e - 1];
    const int64_t el = block_end(starts, nb, e - 1, n);
    const bool big = el - sl > ISO_WIN;          // only the window's last block can be
    const int64_t nsm = (e - f) - (big ? 1 : 0);
    if (nsm > 0) {
        const int L = (int)((big ? sl : el) - s0);  // <= 63
        ps[l] = 0;
        if (l < nsm) ps[(int)(starts[f + l] - s0)] = 1;
        const uint64_t B = __ballot(l < L && ps[l] != 0);
        iso_wave_pack(y, s0, L, B, ys, ps, cst);
    }
    if (big) {
        const int64_t len = el - sl;
        if (len <= WAVE) {
            iso_wave_pack(y, sl, (int)len, 1ull, ys, ps, cst);
        } else if (l == 0) {
            llist[atomicAdd(lcnt, 1)] = (int32_t)(e - 1);   // iso_long_kernel's
        }
    }
}

// wave q: windows 2q and 2q + 1 -- as one pack when their blocks span <= 64
// elements (the common case), else window by window
__global__ __launch_bounds__(256) void iso_pack_kernel(double *__restrict__ y,
                                                       const int64_t *__restrict__ starts,
                                                       int64_t nb, int64_t n, int64_t nwin,
                                                       const int32_t *__restrict__ win_first,
                                                       int32_t *__restrict__ lcnt,
                                                       int32_t *__restrict__ llist) {
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t q = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wv);
    __shared__ double pv_y[4][64];
    __shared__ int pv_p[4][128];
    __shared__ int pv_c[4][65];
    const int64_t p0 = 2 * q;
    if (p0 >= nwin) return;
    const int64_t f = win_first[p0];
    const int64_t m = win_first[p0 + 1];
    const int64_t e = win_first[p0 + 2 <= nwin ? p0 + 2 : nwin];
    if (f >= e) return;
    const int64_t s0 = starts[f];
    const int64_t span = block_end(starts, nb, e - 1, n) - s0;
    int *ps = pv_p[wv];
    if (span <= WAVE) {
        const int64_t nbk = e - f;               // <= 64 blocks (each >= 1 element)
        ps[l] = 0;
        if (l < nbk) ps[(int)(starts[f + l] - s0)] = 1;
        const uint64_t B = __ballot(l < span && ps[l] != 0);
        iso_wave_pack(y, s0, (int)span, B, pv_y[wv], ps, pv_c[wv]);
    } else {
        // two packs, one per window; with no long last block (the common
        // case) both run in the wave together, sharing their passes after
        // the first (pava_v1_wave_pair) instead of one after the other
        const int64_t ea = (m > f) ? block_end(starts, nb, m - 1, n) : 0;
        const int64_t eb = (e > m) ? block_end(starts, nb, e - 1, n) : 0;
        const bool pair = m > f && e > m && ea - starts[m - 1] <= ISO_WIN &&
                          eb - starts[e - 1] <= ISO_WIN;
        if (pair) {
            const int64_t sa = s0, sb = starts[m];
            const int La = (int)(ea - sa), Lb = (int)(eb - sb);   // <= 63 each
            ps[l] = 0;
            if (l < m - f) ps[(int)(starts[f + l] - sa)] = 1;
            const uint64_t Ba = __ballot(l < La && ps[l] != 0);
            ps[l] = 0;
            if (l < e - m) ps[(int)(starts[m + l] - sb)] = 1;
            const uint64_t Bb = __ballot(l < Lb && ps[l] != 0);
            double va = (l < La) ? y[sa + l] : 0.0;
            double vb = (l < Lb) ? y[sb + l] : 0.0;
            pava_v1_wave_pair(va, La, Ba, vb, Lb, Bb, pv_y[wv], ps, pv_c[wv]);
            if (l < La) y[sa + l] = va;
            if (l < Lb) y[sb + l] = vb;
        } else {
            iso_window(y, starts, nb, n, f, m, lcnt, llist, pv_y[wv], ps, pv_c[wv]);
            iso_window(y, starts, nb, n, m, e, lcnt, llist, pv_y[wv], ps, pv_c[wv]);
        }
    }
}

// one workgroup per listed long block (> 64 elements), grid-strided
__global__ __launch_bounds__(LONG_T) void iso_long_kernel(double *__restrict__ y,
                                                          const int64_t *__restrict__ starts,
                                                          int64_t nb, int64_t n, IsoWork w) {
    __shared__ int64_t sh[LONG_T / 64 + 1];
    __shared__ int flag;
    const int cnt = *w.lcnt;
    for (int idx = blockIdx.x; idx < cnt; idx += gridDim.x) {
        const int64_t b = w.llist[idx];
        const int64_t s = starts[b], k = block_end(starts, nb, b, n) - s;
        pava_v1_long(y + s, k, w.Y0 + s, w.Y1 + s, w.W0 + s, w.W1 + s, w.CH + s, sh, &flag);
    }
}

// ---- planned packs (bsls_isotonic_pack_plan / bsls_isotonic_packs) ----------
// The packs are planned once per block layout (host, bsls_isotonic_pack_plan:
// runs of whole consecutive blocks with <= 64 elements, or one longer block),
// so a call is one launch whose waves read their pack's (start, mask, length)
// in one round trip and then y -- as K3 does -- instead of the window plan's
// three dependent rounds (window bounds, block starts, the starts of every
// block of the window).  Wave w takes packs w and w + W (W = waves in the
// grid); with MERGE their passes after the first are shared
// (pava_v1_wave_pair), which pays once the grid runs several rounds of waves.
template <int PPW, bool MERGE>
__global__ __launch_bounds__(256) void iso_packs_kernel(double *__restrict__ y,
                                                        const int64_t *__restrict__ pk_start,
                                                        const int64_t *__restrict__ pk_mask,
                                                        const int32_t *__restrict__ pk_len,
                                                        int64_t npacks) {
    const int l = lane_id();
    const int wv = threadIdx.x / WAVE;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t w0 = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wv);
    __shared__ double pv_y[4][64];
    __shared__ int pv_p[4][128];
    __shared__ int pv_c[4][65];
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
    for (int q = 0; q < PPW; ++q) v[q] = (l < L[q] && L[q] <= WAVE) ? y[s0[q] + l] : 0.0;
    if (MERGE && PPW == 2 && L[0] > 0 && L[0] <= WAVE && L[PPW - 1] > 0 && L[PPW - 1] <= WAVE) {
        pava_v1_wave_pair(v[0], L[0], B[0], v[PPW - 1], L[PPW - 1], B[PPW - 1], pv_y[wv], pv_p[wv],
                          pv_c[wv]);
    } else {
#pragma unroll
        for (int q = 0; q < PPW; ++q)
            if (L[q] > 0 && L[q] <= WAVE) pava_v1_wave_c(v[q], L[q], B[q], pv_y[wv], pv_p[wv], pv_c[wv]);
    }
#pragma unroll
    for (int q = 0; q < PPW; ++q)
        if (l < L[q] && L[q] <= WAVE) y[s0[q] + l] = v[q];
}

// one workgroup per long block of the plan (> 64 elements), grid-strided
__global__ __launch_bounds__(LONG_T) void iso_long_planned(double *__restrict__ y,
                                                           const int64_t *__restrict__ pk_start,
                                                           const int32_t *__restrict__ pk_len,
                                                           const int32_t *__restrict__ longs,
                                                           int64_t nlong, IsoWork w) {
    __shared__ int64_t sh[LONG_T / 64 + 1];
    __shared__ int flag;
    for (int64_t idx = blockIdx.x; idx < nlong; idx += gridDim.x) {
        const int64_t q = longs[idx];
        const int64_t s = pk_start[q], k = pk_len[q];
        pava_v1_long(y + s, k, w.Y0 + s, w.Y1 + s, w.W0 + s, w.W1 + s, w.CH + s, sh, &flag);
    }
}

}  // namespace bsls

using namespace bsls;

extern "C" int64_t bsls_isotonic_pack_plan(const int64_t *starts, int64_t nblocks, int64_t n,
                                           int64_t *pk_start, int64_t *pk_mask, int32_t *pk_len,
                                           int32_t *long_packs, int64_t *nlong, int64_t cap) {
    if (!starts || nblocks <= 0 || n <= 0 || starts[0] < 0 || starts[nblocks - 1] >= n)
        return BSLS_E_ARG;
    for (int64_t b = 1; b < nblocks; ++b)
        if (starts[b] <= starts[b - 1]) return BSLS_E_ARG;
    int64_t np = 0, nl = 0, b = 0;
    auto len_of = [&](int64_t k) { return ((k + 1 < nblocks) ? starts[k + 1] : n) - starts[k]; };
    while (b < nblocks) {
        const int64_t k0 = len_of(b);
        int64_t tot = 0, e = b;
        uint64_t m = 0;
        if (k0 > WAVE) {
            tot = k0;
            m = 1;
            e = b + 1;
            if (long_packs && np < cap) long_packs[nl] = (int32_t)np;
            ++nl;
        } else {
            while (e < nblocks) {
                const int64_t k = len_of(e);
                if (k > WAVE || tot + k > WAVE) break;
                m |= 1ull << tot;
                tot += k;
                ++e;
            }
        }
        if (pk_start && np < cap) {
            pk_start[np] = starts[b];
            pk_mask[np] = (int64_t)m;
            pk_len[np] = (int32_t)tot;
        }
        ++np;
        b = e;
    }
    if (nlong) *nlong = nl;
    return np;
}

extern "C" int bsls_isotonic_packs(double *d_y, const int64_t *d_pk_start, const int64_t *d_pk_mask,
                                   const int32_t *d_pk_len, int64_t npacks,
                                   const int32_t *d_long_packs, int64_t nlong, int64_t n,
                                   void *d_work, size_t work_bytes, void *stream) {
    if (!d_y || !d_pk_start || !d_pk_mask || !d_pk_len || npacks < 1 || n <= 0 || nlong < 0)
        return BSLS_E_ARG;
    if (nlong > 0 && (!d_long_packs || !d_work || work_bytes < bsls_isotonic_workspace_size(n)))
        return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    // two packs per wave from 64k packs (several rounds of resident waves), as
    // K3; BSLS_K3_MERGE = 0 / 1 forces either form (A/B), read once per process
    static const int env_merge = [] {
        const char *e = getenv("BSLS_K3_MERGE");
        return e ? (atoi(e) != 0 ? 1 : 0) : -1;
    }();
    const bool merge = env_merge >= 0 ? env_merge == 1 : npacks >= 65536;
    if (merge)
        iso_packs_kernel<2, true><<<grid_for(npacks, 8), 256, 0, st>>>(d_y, d_pk_start, d_pk_mask,
                                                                       d_pk_len, npacks);
    else
        iso_packs_kernel<1, false><<<grid_for(npacks, 4), 256, 0, st>>>(d_y, d_pk_start, d_pk_mask,
                                                                        d_pk_len, npacks);
    BSLS_LAUNCH_CHECK();
    if (nlong > 0) {
        iso_long_planned<<<(int)(nlong < 1024 ? nlong : 1024), LONG_T, 0, st>>>(
            d_y, d_pk_start, d_pk_len, d_long_packs, nlong, iso_layout(d_work, n));
        BSLS_LAUNCH_CHECK();
    }
    return BSLS_OK;
}

extern "C" size_t bsls_isotonic_workspace_size(int64_t n) {
    return iso_layout(nullptr, n).bytes;
}

extern "C" int bsls_isotonic_multi(int variant, double *d_y, const int64_t *d_starts,
                                   int64_t nblocks, int64_t n, int32_t *d_weight, int expand,
                                   int64_t max_block, void *d_work, size_t work_bytes,
                                   int32_t *d_status, void *stream) {
    if (nblocks <= 0 || n <= 0 || !d_y || !d_starts) return BSLS_E_ARG;
    if (variant < 1 || variant > 3) return BSLS_E_ARG;
    if (variant != 2 && !d_weight && (!d_work || work_bytes < bsls_isotonic_workspace_size(n)))
        return BSLS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const int grid = grid_for(nblocks, WAVE);
    const IsoWork w = iso_layout(d_work, n);
    int32_t *ws = w.ws;
    if (variant == 1 && !d_weight && expand) {
        const int64_t nwin = iso_nwin(n);
        iso_plan_kernel<<<grid_for(nblocks + 1, 256), 256, 0, st>>>(d_starts, nblocks, nwin,
                                                                    w.plan, w.lcnt);
        BSLS_LAUNCH_CHECK();
        iso_pack_kernel<<<grid_for((nwin + 1) / 2, 4), 256, 0, st>>>(d_y, d_starts, nblocks, n, nwin,
                                                                    w.plan, w.lcnt, w.llist);
        BSLS_LAUNCH_CHECK();
        if (max_block > WAVE) {
            const int64_t most = n / (WAVE + 1) + 1;
            iso_long_kernel<<<(int)(most < 1024 ? most : 1024), LONG_T, 0, st>>>(d_y, d_starts,
                                                                              nblocks, n, w);
            BSLS_LAUNCH_CHECK();
        }
        return BSLS_OK;
    }
    if (variant == 1)
        iso_kernel<1><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, d_weight, expand, ws, d_status);
    else if (variant == 2)
        iso_kernel<2><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, nullptr, 0, nullptr, d_status);
    else
        iso_kernel<3><<<grid, WAVE, 0, st>>>(d_y, d_starts, nblocks, n, d_weight, expand, ws, d_status);
    BSLS_LAUNCH_CHECK();
    return BSLS_OK;
}
