// panels.hpp -- the fused SpMVs' matrix format: LDS-chunked jagged diagonals.
//
// Why: a random 8-B gather served by L2 costs a TA/L2 request per lane
// (~0.24 T gathers/s chip-wide measured, tools/ubench_gather.hip), the same
// gather from LDS ~1.3 T/s.  So the gathered vector is staged, one column
// chunk (<= BSLS_PANEL_CHUNK doubles, ~120 KB) at a time, into the LDS of the
// workgroup, and the matrix is stored so every chunk's entries of a wave's
// rows can be walked without padding:
//   panel   = prow consecutive rows (+1 halo row for K2), one wave;
//   segment = (panel, chunk): the panel's rows having entries in the chunk,
//             sorted by that count (descending; perm[] = row in panel per
//             position), then "diagonal" d = the d-th entry of each of those
//             rows, at positions 0 .. dlen[d]-1 (a prefix, since sorted);
//   entry   = uint16 column offset inside the chunk (+ f64 value unless the
//             matrix is a scaled incidence, where the column's scale is applied
//             outside: K1 gathers colv*x, K2 multiplies by colv of its row).
// A lane owns positions lane + 64q (q < 4); its row's running sum lives in LDS
// across chunks, so every row is summed in CSR order, entry after entry,
// exactly like SciPy's csr_matvec (bit-identical when one workgroup sees all
// chunks, as K2 does).
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int PANEL_WAVES = 16;                 // panels per workgroup (1024 threads)
constexpr int PANEL_ACC = 256;                  // LDS row sums per wave (prow + halo <= 256)
constexpr size_t PANEL_LDS = (size_t)BSLS_PANEL_CHUNK * 8 + (size_t)PANEL_WAVES * PANEL_ACC * 8;

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Stage src[0, w) into tab (w <= BSLS_PANEL_CHUNK); src 16-B aligned (chunk
// starts are even columns).  LDS-DMA (global_load_lds_dwordx4): wave-instruction
// k of wave v moves the 1-KB piece p = 16 k + v straight into LDS, no VGPRs.
// The caller brackets it with barriers (__syncthreads drains the DMA).
__device__ __forceinline__ void panel_stage(double *tab, const double *__restrict__ src, int w) {
    const int lane = lane_id(), wv = threadIdx.x / WAVE;
    const int w2 = w >> 1;                       // 16-B units
    const int npieces = (w2 + 63) >> 6;
    for (int p = wv; p < npieces; p += PANEL_WAVES) {
        const int i = p * 64 + lane;
        if (i < w2)
            __builtin_amdgcn_global_load_lds((const void *)(src + 2 * (int64_t)i),
                                             (__attribute__((address_space(3))) void *)(tab + p * 128),
                                             16, 0, 0);
    }
    if ((w & 1) && threadIdx.x == 0) tab[w - 1] = src[w - 1];
}

// One segment by one wave.  acc: the wave's row sums (LDS); tab: the staged
// chunk; rowscale: colv of the panel's row 0 (MODE 2 only).
// MODE 0: s += tab[c]                (K1, scaled incidence: tab = colv * x)
// MODE 1: s += val[e] * tab[c]       (general matrix)
// MODE 2: s += rowscale[row] * tab[c] (K2, scaled incidence)
// Diagonals go in blocks of DB: the entry loads of all DB diagonals and 4
// position slices are issued before the first gather (one memory round trip
// per block; a segment rarely has more than DB diagonals).  Diagonal lengths
// never increase, so whole (slice, diagonal) pairs drop out uniformly.
template <int MODE>
__device__ __forceinline__ void panel_segment(const bsls_panels &M, int64_t seg,
                                              const double *tab, double *acc,
                                              const double *__restrict__ rowscale) {
    const int64_t d0 = M.dl_off[seg], d1 = M.dl_off[seg + 1];
    if (d0 == d1) return;
    constexpr int DB = (MODE == 1) ? 4 : 8;
    const int lane = lane_id();
    // wave-uniform bases + 32-bit lane offsets (saddr + voffset addressing)
    const int64_t e0 = M.ent_off[seg];
    const uint16_t *__restrict__ ent = M.ent + e0;
    const double *__restrict__ val = M.val + e0;
    const int64_t pb = M.perm_off[seg];
    uint32_t e = 0;
    const int n0 = (int)M.dlen[d0];
    int row[4];
    double s[4], sc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int pos = lane + 64 * q;
        row[q] = (pos < n0) ? (int)M.perm[pb + pos] : 0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int pos = lane + 64 * q;
        s[q] = (pos < n0) ? acc[row[q]] : 0.0;
        sc[q] = (MODE == 2 && pos < n0) ? rowscale[row[q]] : 0.0;
    }
    for (int64_t dg = d0; dg < d1; dg += 64) {
        const int nd = (int)((d1 - dg) < 64 ? (d1 - dg) : 64);
        const int len = (lane < nd) ? (int)M.dlen[dg + lane] : 0;
        int incl = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, WAVE);
            if (lane >= o) incl += t;
        }
        const int excl = incl - len;
        for (int d = 0; d < nd; d += DB) {
            int ln[DB];
            uint32_t eo[DB];
#pragma unroll
            for (int k = 0; k < DB; ++k) {
                ln[k] = (d + k < nd) ? readlane_i(len, d + k) : 0;
                eo[k] = e + (uint32_t)((d + k < nd) ? readlane_i(excl, d + k) : 0);
            }
            int c[4][DB];
            double v[4][DB];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pos = lane + 64 * q;
#pragma unroll
                for (int k = 0; k < DB; ++k) {
                    c[q][k] = 0;
                    v[q][k] = 0.0;
                    if (64 * q < ln[k] && pos < ln[k]) {
                        c[q][k] = ent[eo[k] + (uint32_t)pos];
                        if (MODE == 1) v[q][k] = val[eo[k] + (uint32_t)pos];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pos = lane + 64 * q;
#pragma unroll
                for (int k = 0; k < DB; ++k) {
                    if (64 * q < ln[k] && pos < ln[k]) {
                        const double a = tab[c[q][k]];
                        if (MODE == 0) s[q] += a;
                        else if (MODE == 1) s[q] += v[q][k] * a;
                        else s[q] += sc[q] * a;
                    }
                }
            }
        }
        e += (uint32_t)readlane_i(incl, 63);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (lane + 64 * q < n0) acc[row[q]] = s[q];
}

}  // namespace bsls
