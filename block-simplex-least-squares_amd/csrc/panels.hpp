// panels.hpp -- the fused SpMVs' matrix format: LDS-chunked row panels.
//
// Why: a random 8-B gather served by L2 costs a TA/L2 request per lane
// (~0.24 T gathers/s chip-wide measured, tools/ubench_gather.hip), the same
// gather from LDS ~1.3 T/s.  So the gathered vector is staged, one column
// chunk (<= tab_cap doubles, ~158 KB) at a time, into the LDS of the
// workgroup, and the matrix is cut to match (include/bsls_hip.h, struct
// bsls_panels):
//   panel   = prow consecutive rows (+1 halo row for K2), one wave; row r in
//             lane r % 64 of slice r / 64, its running sum in a register of
//             that lane for the whole launch;
//   segment = (panel, chunk): per live slice, the 64 rows' entry counts in
//             the chunk and their entries, row after row in column order;
//   entry   = uint16 column offset inside the chunk (+ f64 value unless the
//             matrix is a scaled incidence, where the column's scale is applied
//             outside: K1 gathers colv*x, K2 multiplies by colv of its row).
// Lane l walks diagonal k of slice q (its row's k-th entry in the chunk) if
// k < cnt: one compare; the entry sits at slice_base + rowstart + k (rowstart
// and cnt from the stored running counts by one DPP shift), so the loads of a
// segment use one address register per slice and immediate offsets.  Every row is summed in CSR order, entry after entry, exactly like
// SciPy's csr_matvec (bit-identical when one workgroup sees all chunks, as K2
// does).  Measured before this layout (jagged diagonals sorted per chunk,
// sums in LDS): VALU-bound, ~1 VALU wave-instruction per entry; here ~4 per
// diagonal of 64 rows.
//
// Latency: the 16 waves move in lockstep between the per-chunk barriers, and
// a chunk's entries depend on its running counts (their addresses).  Counts
// are loaded two chunks ahead, entries one chunk ahead, issued right after a
// walk so they fly across the barrier and the LDS-DMA of the next chunk.  The
// prefetch loads are straight-line and unconditional so the compiler can
// count them in vmcnt; nothing is issued before a walk, whose own waits
// (vmcnt is in order) would otherwise drain the prefetch (measured with
// tools/panel_ubench.py's per-chunk timeline).
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int PANEL_WAVES = BSLS_PANEL_WAVES;   // panels per workgroup (1024 threads)

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// a wave-uniform value the compiler cannot prove uniform, moved to SGPRs
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// Dynamic LDS of a panel kernel: the chunk table (tab_cap doubles; K2 reuses
// it as reduction scratch, hence >= 64).
__host__ __device__ inline size_t panel_lds_bytes(const bsls_panels &M) {
    return (size_t)M.tab_cap * 8;
}

// LDS-DMA (global_load_lds_dwordx4) of n16 16-byte units from src to LDS dst:
// wave-instruction k of wave v moves the 1-KB piece p = nwaves k + v, no VGPRs.
// Completion: the next __syncthreads (it drains vmcnt).
__device__ __forceinline__ void lds_dma(void *dst, const void *src, int64_t n16) {
    const int lane = lane_id(), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    const int64_t npieces = (n16 + 63) >> 6;
    const char *s = (const char *)src;
    char *d = (char *)dst;
    for (int64_t p = wv; p < npieces; p += nw) {
        const int64_t i = p * 64 + lane;
        if (i < n16)
            __builtin_amdgcn_global_load_lds((const void *)(s + 16 * i),
                                             (__attribute__((address_space(3))) void *)(d + 1024 * p),
                                             16, 0, 0);
    }
}

// Stage src[0, w) into tab (w <= tab_cap); src 16-B aligned (chunk starts are
// even columns).
__device__ __forceinline__ void panel_stage(double *tab, const double *__restrict__ src, int w) {
    lds_dma(tab, src, w >> 1);
    if ((w & 1) && threadIdx.x == 0) tab[w - 1] = src[w - 1];
}

// lane l - 1's value (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ int wave_shr1(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
}

// Uniform int64 metadata through the scalar unit: s_load waits on lgkmcnt,
// not vmcnt.  As vector loads (what the compiler emits for pointers it cannot
// prove read-only), the wait for them would, vmcnt being in order, also wait
// for every prefetch issued before -- draining the entry loads of the next
// chunk right after issuing them.
__device__ __forceinline__ void sload2(const int64_t *a, const int64_t *b, int64_t &x, int64_t &y) {
    asm volatile(
        "s_load_dwordx2 %0, %2, 0x0\n\t"
        "s_load_dwordx2 %1, %3, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(x), "=&s"(y)
        : "s"(a), "s"(b)
        : "memory");
}

__device__ __forceinline__ void sload3(const int64_t *a, const int64_t *b, const int64_t *c,
                                       int64_t &x, int64_t &y, int64_t &z) {
    asm volatile(
        "s_load_dwordx2 %0, %3, 0x0\n\t"
        "s_load_dwordx2 %1, %4, 0x0\n\t"
        "s_load_dwordx2 %2, %5, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(x), "=&s"(y), "=&s"(z)
        : "s"(a), "s"(b), "s"(c)
        : "memory");
}

// An empty asm that "uses" the gathered values: every gather is issued before
// it and none is sunk into the conditional adds after it (left alone, the
// compiler moves each load under its lane predicate and waits on it there)
__device__ __forceinline__ void pin8(double (&a)[8]) {
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                 "+v"(a[6]), "+v"(a[7]));
}
__device__ __forceinline__ void pin8(double (&a)[2]) { asm volatile("" : "+v"(a[0]), "+v"(a[1])); }

__device__ __forceinline__ void sload5(const int64_t *a, const int64_t *b, const int64_t *c,
                                       const int64_t *d, const int64_t *e, int64_t &x, int64_t &y,
                                       int64_t &z, int64_t &u, int64_t &v) {
    asm volatile(
        "s_load_dwordx2 %0, %5, 0x0\n\t"
        "s_load_dwordx2 %1, %6, 0x0\n\t"
        "s_load_dwordx2 %2, %7, 0x0\n\t"
        "s_load_dwordx2 %3, %8, 0x0\n\t"
        "s_load_dwordx2 %4, %9, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(x), "=&s"(y), "=&s"(z), "=&s"(u), "=&s"(v)
        : "s"(a), "s"(b), "s"(c), "s"(d), "s"(e)
        : "memory");
}

// A segment's first round trip: slice depths D_q (uniform) and each lane's
// running count per live slice (inclusive prefix over the slice's rows).
struct SegHead {
    int D[4];
    int incl[4];
    int64_t e0;

    __device__ __forceinline__ void load(const bsls_panels &M, int64_t seg, bool live) {
        // seg is wave-uniform (padded panels have empty segments): scalar loads.
        // Straight-line, unconditional vector loads (a dead slice reads the next
        // group of counts, ignored), so the compiler can count them in vmcnt.
        (void)live;
        int64_t info, co;
        sload3(M.seg_info + seg, M.cnt_off + seg, M.ent_off + seg, info, co, e0);
        load_counts(M, info, co);
    }

    // the vector half, from the segment's metadata (info, cnt_off)
    __device__ __forceinline__ void load_counts(const bsls_panels &M, int64_t info, int64_t co) {
        const int lane = lane_id();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            D[q] = (int)((info >> (16 * q)) & 0xFFFF);
            incl[q] = (int)M.cnt[co + lane];
            co += (D[q] > 0) ? 64 : 0;
        }
    }
};

// A segment's entries (second round trip) and the walk.
template <int MODE>
struct SegBody {
    static constexpr int DBK = (MODE == 1) ? 2 : 8;   // diagonals held per slice
    int D[4];            // uniform
    int cnt[4];          // this lane's row count per slice
    uint32_t base[4];    // this lane's first entry per slice (relative to e0)
    int64_t e0;
    uint32_t c2[4][DBK / 2];   // column offsets of diagonals 2j, 2j+1 (low, high half)
    double v[4][DBK];    // values (MODE 1)

    // DBK entries of one row from its (even, i.e. 4-B aligned) entry index i:
    // one 16-B load (dword alignment suffices for global dwordx4)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
    __device__ __forceinline__ static u32x4 ent8(const uint16_t *ent, uint32_t i) {
        return *reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(ent) + i * 2u);
    }

    __device__ __forceinline__ void load(const bsls_panels &M, const SegHead &h) {
        const uint16_t *ent = M.ent + h.e0;
        const double *val = M.val + h.e0;
        e0 = h.e0;
        uint32_t e = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // stored: running total of even-padded run lengths | (own count odd);
            // straight-line and unconditional (a dead slice reads at the running
            // offset: within the segments that follow, or the array's slack)
            D[q] = h.D[q];
            const bool on = D[q] > 0;
            const int inc = h.incl[q] & ~1;
            const int ex = wave_shr1(h.incl[q]) & ~1;
            cnt[q] = on ? inc - ex - (h.incl[q] & 1) : 0;
            base[q] = e + (on ? (uint32_t)ex : 0u);
            e += on ? (uint32_t)(readlane_i(h.incl[q], 63) & ~1) : 0u;
            // a row's run is even-padded; lanes past their row's end read the
            // next rows' entries (or the array's 64-entry slack): harmless
            if (DBK == 8) {
                const u32x4 w = ent8(ent, base[q]);
#pragma unroll
                for (int j = 0; j < 4; ++j) c2[q][j] = w[j];
            } else {
#pragma unroll
                for (int j = 0; j < DBK / 2; ++j) {
                    c2[q][j] = *reinterpret_cast<const uint32_t *>(
                        reinterpret_cast<const char *>(ent) + (base[q] + 2 * j) * 2u);
                    if (MODE == 1) {
                        v[q][2 * j] = val[base[q] + 2 * j];
                        v[q][2 * j + 1] = val[base[q] + 2 * j + 1];
                    }
                }
            }
        }
    }

    // MODE 0: s += tab[c]; 1: s += val * tab[c]; 2: s += sc * tab[c]
    __device__ __forceinline__ void walk(const bsls_panels &M, const double *tab, double (&s)[4],
                                         const double (&sc)[4]) const {
        const uint16_t *ent = M.ent + e0;
        const double *val = M.val + e0;
        // diagonals DBK .. 2 DBK - 1 of every slice deeper than DBK, issued
        // before any of the walk so their round trips overlap each other and
        // the shallow part of the walk (a deep slice in ~30 % of the waves of a
        // chunk made those waves the stragglers at the next barrier)
        u32x4 ext[4];
        if (DBK == 8) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (D[q] > DBK)
                    ext[q] = ent8(ent, base[q] + (DBK < cnt[q] ? (uint32_t)DBK : 0u));
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (D[q] == 0) continue;
            // all gathers of the slice first (every held offset is a valid
            // column of the chunk, or 0), then the adds in order; a lane past
            // its row's end adds 0.0, which leaves its sum bit-for-bit unchanged
            // (a sum started at +0.0 is never -0.0)
            // (gathers masked to the lanes whose row reaches diagonal k and to
            // k < D: measured slower, 41.8 -> 43.4 us for K2 -- the exec-mask
            // branches cost more than the lanes they leave out of the LDS)
            double a[DBK];
#pragma unroll
            for (int k = 0; k < DBK; ++k) {
                const uint32_t w = c2[q][k >> 1];
                a[k] = tab[(k & 1) ? (w >> 16) : (w & 0xFFFFu)];
            }
            pin8(a);
#pragma unroll
            for (int k = 0; k < DBK; ++k) {
                if (k < D[q]) {
                    double t;
                    if (MODE == 0) t = a[k];
                    else if (MODE == 1) t = v[q][k] * a[k];
                    else t = sc[q] * a[k];
                    if (k < cnt[q]) s[q] += t;
                }
            }
            // long rows (a slice deeper than DBK): further diagonals DBK at a time,
            // all loads of a batch in flight together
            for (int k0 = DBK; k0 < D[q]; k0 += DBK) {
                int cc[DBK];
                double vv[DBK];
                if (DBK == 8) {
                    // one 16-B load per 8 diagonals; a lane whose row has ended
                    // re-reads its first entries (any in-chunk offset will do)
                    const u32x4 w = (k0 == DBK)
                                        ? ext[q]
                                        : ent8(ent, base[q] + (k0 < cnt[q] ? (uint32_t)k0 : 0u));
#pragma unroll
                    for (int k = 0; k < DBK; ++k)
                        cc[k] = (int)((k & 1) ? (w[k >> 1] >> 16) : (w[k >> 1] & 0xFFFFu));
                } else {
#pragma unroll
                    for (int k = 0; k < DBK; ++k) {
                        const uint32_t i = base[q] + (uint32_t)(k0 + k);
                        const bool in = k0 + k < cnt[q];
                        cc[k] = in ? (int)ent[i] : 0;
                        if (MODE == 1) vv[k] = in ? val[i] : 0.0;
                    }
                }
                double a2[DBK];
#pragma unroll
                for (int k = 0; k < DBK; ++k) a2[k] = tab[cc[k]];
                pin8(a2);
#pragma unroll
                for (int k = 0; k < DBK; ++k) {
                    double t;
                    if (MODE == 0) t = a2[k];
                    else if (MODE == 1) t = vv[k] * a2[k];
                    else t = sc[q] * a2[k];
                    if (k0 + k < cnt[q]) s[q] += t;
                }
            }
        }
    }
};

// The chunk loop shared by K1a and K2: chunks [c0, c1) of panel 16 rb + wv,
// each staged from src (column chunk_col[c] at src[chunk_col[c]]) into tab,
// then walked by this wave into s[q] (row 64 q + lane).  Every wave of the
// workgroup calls it (barriers).  Pipeline: during the step of chunk c the
// wave holds chunk c's entries (walked now), loads chunk c+1's entries and
// chunk c+2's running counts; the loop is unrolled twice so the two register
// sets swap roles without copies.
template <int MODE>
__device__ __forceinline__ void panel_chunks(const bsls_panels &M, int64_t rb, int wv, int64_t c0,
                                             int64_t c1, const double *src, double *tab,
                                             double (&s)[4], const double (&sc)[4]) {
    wv = __builtin_amdgcn_readfirstlane(wv);              // uniform: scalar segment loads
    rb = uni64(rb);
    const bool live = rb * PANEL_WAVES + wv < M.npanels;
    const int64_t seg0 = (rb * M.nchunks) * PANEL_WAVES + wv;
    auto seg = [&](int64_t c) { return seg0 + c * PANEL_WAVES; };
    SegHead ha, hb;
    SegBody<MODE> ba, bb;
    // chunk c0's DMA goes first, so it overlaps the prologue's two round trips
    {
        int64_t a, b;
        sload2(M.chunk_col + c0, M.chunk_col + c0 + 1, a, b);
        panel_stage(tab, src + a, (int)(b - a));
    }
    ha.load(M, seg(c0), live);
    ba.load(M, ha);
    if (c0 + 1 < c1) hb.load(M, seg(c0 + 1), live);
    int64_t ca = 0, cb = 0;   // column bounds of the next chunk to stage
    auto step = [&](int64_t c, const SegBody<MODE> &cur, SegHead &hn, SegBody<MODE> &bn,
                    SegHead &hn2) {
        if (c > c0) {
            // barrier A: every wave is done reading the table (its LDS reads
            // were consumed by its adds).  A bare s_barrier: __syncthreads'
            // fence would also wait vmcnt(0), i.e. for the prefetch just issued.
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) (gfx9 encoding)
            __builtin_amdgcn_s_barrier();
            panel_stage(tab, src + ca, (int)(cb - ca));
        }
        __syncthreads();
        // walk first: its long-row loads wait on vmcnt, which is in order, so
        // no prefetch may be outstanding yet; the prefetch issued after it flies
        // across the next barrier and DMA.  One scalar round trip per step:
        // chunk c+2's segment metadata with chunk c+1's column bounds.
        if (live) cur.walk(M, tab, s, sc);
        if (c + 1 < c1) bn.load(M, hn);
        {
            const int64_t sg = seg(c + 2 < c1 ? c + 2 : c1 - 1);
            const int64_t cn = c + 1 < c1 ? c + 1 : c;
            int64_t info, co;
            sload5(M.seg_info + sg, M.cnt_off + sg, M.ent_off + sg, M.chunk_col + cn,
                   M.chunk_col + cn + 1, info, co, hn2.e0, ca, cb);
            if (c + 2 < c1) hn2.load_counts(M, info, co);
        }
    };
    for (int64_t c = c0; c < c1; c += 2) {
        step(c, ba, hb, bb, ha);
        if (c + 1 < c1) step(c + 1, bb, ha, ba, hb);
    }
}

}  // namespace bsls
