// tiles.hpp -- the SpMV format for sparse row blocks: streamed tiles
// (include/bsls_hip.h, struct bsls_tiles).
//
// Why a second format.  The panel image (panels.hpp) stages a 20k-column chunk
// of the gathered vector into LDS and walks it row-per-lane with the row sums
// in registers; that pays while a 64-row slice holds several entries per chunk
// (config C3: ~3.2 per row).  Over C5's 1M links a row holds ~0.3 entries per
// chunk: the per-(slice, chunk) metadata and the mostly idle lanes make the
// panel K1 / K2 take 278 / 465 us on a 20M-entry C5 column shard.  Measured
// on that shard (tools/tile*_ubench.hip): staged-chunk variants were bound by
// the per-chunk round trips (a barrier per chunk, two dependent loads after
// it); this form, with no barrier at all, ~100 us, bound by the gathers.
//
// Form.  Workgroup (rb, g) of 1024 threads keeps row block rb's running sums
// in LDS (slot-major: local row lr at rows[lr], thread lr % 1024 owns it, so
// a wave's read-modify-write touches 64 consecutive doubles: no bank
// conflicts, no races).  Each thread walks ONE linear stream: its rows'
// entries of column group g sorted by column -- each row summed in CSR order
// (bit-identical to SciPy's csr_matvec when ngroups == 1), and all threads
// sweep the columns together.  The gathered vector is read straight through
// L1/L2 (no LDS staging): random 8-B gathers run at the L2 line rate (~0.27 T
// per second chip-wide, the same as the round-1 gather probe); the column
// groups keep each XCD on one slice so the slice stays in that XCD's L2
// (order 0 with ngroups | 8, order 1 for ngroups % 8 == 0).  The streams are
// interleaved in 16-B quads (one 1-KB load per wave per 4 entries), loaded P
// quads ahead, gathers one quad ahead of the row updates.
#pragma once
#include "bsls_common.hpp"

namespace bsls {

constexpr int TILE_T = BSLS_TILE_THREADS;

__host__ __device__ inline int64_t tile_nslots(const bsls_tiles &T) {
    return (T.H + T.halo + TILE_T - 1) / TILE_T;
}

// dynamic LDS doubles of a tile kernel: the row sums (+ the dummy slot), and
// with `colv` the rows' column scales (K2 on a scaled incidence)
__host__ __device__ inline size_t tile_lds_doubles(const bsls_tiles &T, bool colv) {
    if ((T.layout & 0xFF) >= 1) return (size_t)(T.H + T.halo + 1) * (colv ? 2 : 1);
    return (size_t)(tile_nslots(T) + 1) * TILE_T * (colv ? 2 : 1);
}

// workgroup b of a launch over `nrb` row blocks -> (row block, group)
__device__ __forceinline__ void tile_map(const bsls_tiles &T, int64_t b, int64_t nrb, int64_t &rb,
                                         int64_t &g) {
    if (T.order == 1) {
        const int64_t x = b & 7, i = b >> 3;
        rb = i % nrb;
        g = x + 8 * (i / nrb);
    } else {
        g = b % T.ngroups;
        rb = b / T.ngroups;
    }
}

typedef uint32_t tile_quad __attribute__((ext_vector_type(4)));

// BSLS_TILE_KO (timing knock-outs of the dealt walk, never in the product
// build; 4 = K2's epilogue skipped instead -- bb.hip)
// build): 1 = plain LDS add instead of ds_add_f64, 2 = no LDS accumulation,
// 3 = no walk at all (what is left: the LDS clear, the finish, the tail)
#ifndef BSLS_TILE_KO
#define BSLS_TILE_KO 0
#endif

// the dealt walk's entry stream: non-temporal loads when the image is larger
// than the Infinity Cache (layout flag BSLS_TILE_NT: the stream would only
// evict the gathered vector; C5 on one GPU K1 368 -> 357, K2 505 -> 492 us),
// plain loads when it stays resident across iterations (a C5 shard / 8:
// K1 60 vs 70, K2 79 vs 87 us with nt)
template <bool NT>
__device__ __forceinline__ tile_quad tq_load(const tile_quad *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// Walk this thread's stream of tile (rb, g) into rows[] (LDS, zeroed by the
// caller, barrier after):
//   MODE 0  rows[lr] += src[c]                 (pattern / scaled incidence, K1)
//   MODE 1  rows[lr] += val * src[c]           (stored values)
//   MODE 2  rows[lr] += rcol[lr] * src[c]      (scaled incidence, K2: rcol in LDS)
// src is indexed by the column relative to group_col[g].
template <int MODE, int P = 4>
__device__ __forceinline__ void tile_walk(const bsls_tiles &T, int64_t rb, int64_t g,
                                          const double *__restrict__ src, double *rows,
                                          const double *rcol) {
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t s = (rb * T.ngroups + g) * 16 + wv;
    const int64_t q0 = T.wave_off[s], nq = (T.wave_off[s + 1] - q0) >> 6;
    const tile_quad *Q = reinterpret_cast<const tile_quad *>(T.ent) + q0 + lane;
    const double *V = (MODE == 1) ? T.val + 4 * (q0 + lane) : nullptr;
    const double *xb = src + T.group_col[g];
    tile_quad ring[P];
#pragma unroll
    for (int k = 0; k < P; ++k) ring[k] = (k < nq) ? Q[(int64_t)k * 64] : tile_quad{0, 0, 0, 0};
    double v[4], vn[4], a[4], an[4];
    auto gat = [&](const tile_quad &u, int64_t q, double (&o)[4], double (&w)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = xb[u[j] & 0xFFFFFFu];
        if (MODE == 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = V[q * 256 + j];
        }
    };
    gat(ring[0], 0, v, a);
    for (int64_t q = 0; q < nq; q += P) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const tile_quad cur = ring[k];
            if (q + k + 1 < nq) gat(ring[(k + 1) % P], q + k + 1, vn, an);
            ring[k] = (q + k + P < nq) ? Q[(q + k + P) * 64] : tile_quad{0, 0, 0, 0};
            if (q + k < nq) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int lr = (int)(cur[j] >> 24) * TILE_T + t;
                    double term;
                    if (MODE == 0) term = v[j];
                    else if (MODE == 1) term = a[j] * v[j];
                    else term = rcol[lr] * v[j];
                    rows[lr] += term;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = vn[j];
                if (MODE == 1) a[j] = an[j];
            }
        }
    }
}

// Layout 2's entries: 3 uint32 per lane hold four 24-bit entries
typedef uint32_t tile_tri __attribute__((ext_vector_type(3)));

template <bool NT>
__device__ __forceinline__ tile_tri tt_load(const uint32_t *p) {
    const tile_tri *q = reinterpret_cast<const tile_tri *>(p);
    if (NT) return __builtin_nontemporal_load(q);
    return *q;
}

__device__ __forceinline__ uint32_t tri_entry(const tile_tri &t, int j) {
    switch (j) {
        case 0: return t[0] & 0xFFFFFFu;
        case 1: return (t[0] >> 24) | ((t[1] & 0xFFFFu) << 8);
        case 2: return (t[1] >> 16) | ((t[2] & 0xFFu) << 16);
        default: return t[2] >> 8;
    }
}

// Layout 1 (dealt, include/bsls_hip.h): wave w walks its instructions of tile
// (rb, g) quad-step by quad-step -- one 16-B entry load (4 slots) and one
// scalar 16-B base load per step, loaded P steps ahead, the gathers of step
// s + D issued before the LDS atomic adds of step s.  MODE as tile_walk.
// PK3 (layout 2): the step's entries are one 12-B load (four 24-bit entries:
// 25 % less stream), unpacked where they are used.
#ifndef BSLS_TILE_P
#define BSLS_TILE_P 4
#endif
#ifndef BSLS_TILE_D
#define BSLS_TILE_D 1
#endif
template <bool PK3>
struct TileEnt {
    typedef tile_quad type;
};
template <>
struct TileEnt<true> {
    typedef tile_tri type;
};

// the stored values (MODE 1) in the image's value type (VT 0: double, 1:
// float, 2: _Float16 -- BSLS_TILE_VAL32 / VAL16, exact conversions of the
// doubles): value e of the image as a double
template <int VT>
__device__ __forceinline__ double tile_val(const double *__restrict__ val, int64_t e) {
    if constexpr (VT == 1) return (double)reinterpret_cast<const float *>(val)[e];
    else if constexpr (VT == 2) return (double)reinterpret_cast<const _Float16 *>(val)[e];
    else return val[e];
}

// a lane's four stored values of one step (entries 4 l .. 4 l + 3 of the
// lane's quad, aligned): one or two vector loads, streaming (nt) with NT like
// the entries, so the value stream does not evict the gathered vector's lines
typedef double tile_d2 __attribute__((ext_vector_type(2)));
typedef float tile_f4 __attribute__((ext_vector_type(4)));
typedef _Float16 tile_h4 __attribute__((ext_vector_type(4)));
template <typename V, bool NT>
__device__ __forceinline__ V tile_vload(const V *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <int VT, bool NT>
__device__ __forceinline__ void tile_vals4(const double *__restrict__ val, int64_t e,
                                           double (&w)[4]) {
    if constexpr (VT == 1) {
        const tile_f4 f = tile_vload<tile_f4, NT>(reinterpret_cast<const tile_f4 *>(
            reinterpret_cast<const float *>(val) + e));
        w[0] = (double)f.x; w[1] = (double)f.y; w[2] = (double)f.z; w[3] = (double)f.w;
    } else if constexpr (VT == 2) {
        const tile_h4 h = tile_vload<tile_h4, NT>(reinterpret_cast<const tile_h4 *>(
            reinterpret_cast<const _Float16 *>(val) + e));
        w[0] = (double)h.x; w[1] = (double)h.y; w[2] = (double)h.z; w[3] = (double)h.w;
    } else {
        const tile_d2 *p = reinterpret_cast<const tile_d2 *>(val + e);
        const tile_d2 a = tile_vload<tile_d2, NT>(p), b = tile_vload<tile_d2, NT>(p + 1);
        w[0] = a.x; w[1] = a.y; w[2] = b.x; w[3] = b.y;
    }
}

// FX: the row sums in two-word fixed point instead (order-free: integer
// adds commute, so a row's sum is the same bits whatever order the atomics
// land in).  fxs = 2^k puts every term * fxs within [-2^50, 2^50]; the high
// word takes it rounded to an integer (the 1.5 * 2^52 trick: one add, one
// 64-bit subtract), the low word the exact remainder scaled by 2^50 and
// rounded (2^-s of the unit, s = fx_lo_shift: ~100 bits below the bound),
// two ds_add_u64 per entry.  The low words sit H + halo + 1 slots after the
// high ones (twice the LDS).
constexpr double FX_MAGIC = 6755399441055744.0;   // 1.5 * 2^52: ulp 1 over +-2^51

// The low word's scale 2^s: a row of N <= cols entries adds at most N 2^(s-1)
// to it (every remainder |v - h| <= 1/2, all of one sign at worst -- e.g.
// x = 1/3 on a dense link), so 2^s <= 2^62 / 2^bit_width(cols) keeps the sum
// inside int64 whatever the remainders: s = 50 up to 4095 columns, 38 at 10M
// (a term then rounds by 2^-(s+1) of the unit = bound 2^-(s+51), still ~2^-89).
__host__ __device__ inline int fx_lo_shift(int64_t cols) {
    const int bw = cols > 0 ? 64 - __builtin_clzll((unsigned long long)cols) : 0;
    return 62 - bw < 50 ? 62 - bw : 50;
}

__device__ __forceinline__ void fx_add(double *rows, int lr, int lo_off, double v, double los) {
    const double t = v + FX_MAGIC;
    const double h = t - FX_MAGIC;                  // v rounded to an integer, exactly
    const double l = (v - h) * los;                 // |v - h| <= 1/2: exact, then scaled
    const double tl = l + FX_MAGIC;
    atomicAdd(reinterpret_cast<unsigned long long *>(&rows[lr]),
              (unsigned long long)(__double_as_longlong(t) - __double_as_longlong(FX_MAGIC)));
    atomicAdd(reinterpret_cast<unsigned long long *>(&rows[lr + lo_off]),
              (unsigned long long)(__double_as_longlong(tl) - __double_as_longlong(FX_MAGIC)));
}

// a row's two words back to a double: hi 2^-k + lo 2^-(k+s), inv_lo = 2^-(k+s)
__device__ __forceinline__ double fx_value(const double *rows, int lr, int lo_off, double inv,
                                           double inv_lo) {
    const long long hi = reinterpret_cast<const long long *>(rows)[lr];
    const long long lo = reinterpret_cast<const long long *>(rows)[lr + lo_off];
    return (double)hi * inv + (double)lo * inv_lo;
}

// FXIN: the gathered vector is in 64-bit fixed point (a column shard's r,
// bsls_bb_problem.r_fx): each gathered word is an int64, its value that times
// fxin (the inverse scale)
template <int MODE, bool NT, bool PK3 = false, int VT = 0, int P = BSLS_TILE_P,
          int D = BSLS_TILE_D, bool FX = false, bool FXIN = false>
__device__ __forceinline__ void tile_walk_dealt(const bsls_tiles &T, int64_t rb, int64_t g,
                                                const double *__restrict__ src, double *rows,
                                                const double *rcol, double fxs = 1.0,
                                                double fxin = 1.0) {
    static_assert(D >= 1 && D < P, "gathers run ahead of the entry loads");
    if (BSLS_TILE_KO == 3) return;
    typedef typename TileEnt<PK3>::type ent_t;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t t = rb * T.ngroups + g;
    const int64_t q0 = T.wave_off[t], nq = T.wave_off[t + 1] - q0;
    // entries: lane (q0 * 16 + wv) * 64 + lane of the image, 1024 lanes per step
    const int64_t l0 = (q0 * 16 + wv) * 64 + lane;
    const uint32_t *E = T.ent + (PK3 ? 3 : 4) * l0;
    constexpr int64_t STEP = (PK3 ? 3 : 4) * 1024;   // uint32 per quad-step
    // layout 2: column offset in the low cb bits, the local row above
    const int cb = PK3 ? 24 - (32 - __builtin_clz((unsigned)(T.H + T.halo))) : 16;
    const uint32_t cmask = (1u << cb) - 1u;
    auto ld = [&](int64_t s) -> ent_t {
        if constexpr (PK3) return tt_load<NT>(E + s * STEP);
        else return tq_load<NT>(reinterpret_cast<const tile_quad *>(E + s * STEP));
    };
    auto ent = [&](const ent_t &u, int j) -> uint32_t {
        if constexpr (PK3) return tri_entry(u, j);
        else return u[j];
    };
    const int4 *Bq = reinterpret_cast<const int4 *>(T.base) + q0 * 16 + wv;
    const int64_t v0 = 4 * l0;   // first value of this lane (MODE 1)
    const double *xb = src + T.group_col[g];
    const int lo_off = (int)(T.H + T.halo + 1);     // FX: the low words
    const double fxl = FX ? ldexp(1.0, fx_lo_shift(T.cols)) : 0.0;
    ent_t ring[P];
    int4 bring[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        ring[k] = (k < nq) ? ld(k) : ent_t{};
        bring[k] = (k < nq) ? Bq[(int64_t)k * 16] : int4{0, 0, 0, 0};
    }
    // v[d] / a[d]: the gathered values (and stored values) of step s + d
    double v[D + 1][4], a[D + 1][4];
    double ko = 0.0;
    auto gat = [&](const ent_t &u, const int4 &b, int64_t q, double (&o)[4], double (&w)[4]) {
        o[0] = xb[b.x + (ent(u, 0) & cmask)];
        o[1] = xb[b.y + (ent(u, 1) & cmask)];
        o[2] = xb[b.z + (ent(u, 2) & cmask)];
        o[3] = xb[b.w + (ent(u, 3) & cmask)];
        if (MODE == 1) tile_vals4<VT, NT>(T.val, v0 + q * 4096, w);
    };
    // (FXIN: the int64 words to doubles where used, not where gathered, so
    // the conversion does not wait on the gathers in flight)
    auto gval = [&](double o) -> double {
        if constexpr (FXIN) return (double)__double_as_longlong(o) * fxin;
        else return o;
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nq) gat(ring[d], bring[d], d, v[d], a[d]);
    for (int64_t q = 0; q < nq; q += P) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const ent_t cur = ring[k];
            if (q + k + D < nq) gat(ring[(k + D) % P], bring[(k + D) % P], q + k + D, v[D], a[D]);
            if (q + k + P < nq) {
                ring[k] = ld(q + k + P);
                bring[k] = Bq[(q + k + P) * 16];
            }
            if (q + k < nq) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int lr = (int)(ent(cur, j) >> cb);
                    double term;
                    if (MODE == 0) term = gval(v[0][j]);
                    else if (MODE == 1) term = a[0][j] * gval(v[0][j]);
                    else term = rcol[lr] * gval(v[0][j]);
#if BSLS_TILE_KO == 1
                    rows[lr] += term;                 // (knock-out: racy plain add)
#elif BSLS_TILE_KO == 2
                    ko += term;                       // (knock-out: no LDS)
#else
                    if constexpr (FX) fx_add(rows, lr, lo_off, term * fxs, fxl);
                    else atomicAdd(&rows[lr], term);
#endif
                }
            }
#pragma unroll
            for (int d = 0; d < D; ++d)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[d][j] = v[d + 1][j];
                    if (MODE == 1) a[d][j] = a[d + 1][j];
                }
        }
    }
    if (BSLS_TILE_KO == 2) rows[threadIdx.x] += ko;
}

// the dealt walk with its value type (MODE 1 only: the other modes store none)
template <int MODE, bool NT, bool PK3, bool FX = false, bool FXIN = false>
__device__ __forceinline__ void tile_walk_dealt_vt(const bsls_tiles &T, int64_t rb, int64_t g,
                                                   const double *__restrict__ src, double *rows,
                                                   const double *rcol, double fxs = 1.0,
                                                   double fxin = 1.0) {
    constexpr int P = BSLS_TILE_P, D = BSLS_TILE_D;
    if constexpr (MODE == 1) {
        if (T.layout & BSLS_TILE_VAL16)
            tile_walk_dealt<MODE, NT, PK3, 2, P, D, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
        else if (T.layout & BSLS_TILE_VAL32)
            tile_walk_dealt<MODE, NT, PK3, 1, P, D, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
        else
            tile_walk_dealt<MODE, NT, PK3, 0, P, D, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    } else {
        tile_walk_dealt<MODE, NT, PK3, 0, P, D, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    }
}

// the walk of either layout (FX, FXIN: dealt layouts only)
template <int MODE, bool FX = false, bool FXIN = false>
__device__ __forceinline__ void tile_walk_any(const bsls_tiles &T, int64_t rb, int64_t g,
                                              const double *__restrict__ src, double *rows,
                                              const double *rcol, double fxs = 1.0,
                                              double fxin = 1.0) {
    const int64_t lay = T.layout & ~(int64_t)(BSLS_TILE_VAL32 | BSLS_TILE_VAL16);
    if (lay == 1)
        tile_walk_dealt_vt<MODE, false, false, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    else if (lay == (1 | BSLS_TILE_NT))
        tile_walk_dealt_vt<MODE, true, false, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    else if (lay == 2)
        tile_walk_dealt_vt<MODE, false, true, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    else if (lay == (2 | BSLS_TILE_NT))
        tile_walk_dealt_vt<MODE, true, true, FX, FXIN>(T, rb, g, src, rows, rcol, fxs, fxin);
    else if constexpr (!FX && !FXIN) tile_walk<MODE>(T, rb, g, src, rows, rcol);
}

// Host-side validation of a tile image against the matrix it claims to hold
// (bb.hip's K1 / K2 images, lsq.hip's x-space operator): shape, plan, LDS
// budget, layout flags and the bit widths the dealt entries assume.
inline bool tiles_valid(const bsls_tiles &T, int64_t rows, int64_t cols, int64_t halo,
                        bool need_val, bool colv_lds, int64_t lds_max) {
    if (T.rows != rows || T.cols != cols || T.halo != halo || T.H < 64) return false;
    if (T.nrb != (rows + T.H - 1) / T.H || T.ngroups < 1 || T.nquads < 0) return false;
    if (T.order != 0 && !(T.order == 1 && T.ngroups % 8 == 0)) return false;
    if (tile_lds_doubles(T, colv_lds) * 8 > (size_t)lds_max) return false;
    if (!T.group_col || !T.wave_off || !T.ent) return false;
    const int64_t lay = T.layout & ~(int64_t)(BSLS_TILE_NT | BSLS_TILE_VAL32 | BSLS_TILE_VAL16);
    if (T.layout != 0 && !((lay == 1 || lay == 2) && T.base && T.H + T.halo < 65536))
        return false;
    if ((T.layout & BSLS_TILE_VAL32) && (T.layout & BSLS_TILE_VAL16)) return false;
    if (lay == 2 && T.H + T.halo >= (1 << 18)) return false;   // >= 6 column bits
    return need_val ? T.val != nullptr : true;
}

}  // namespace bsls
