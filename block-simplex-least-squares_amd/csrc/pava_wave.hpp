// pava_wave.hpp -- wave-parallel PAVA v1, bit-identical to the serial reference
// (python/c_extensions/isotonic_regression.h:13-58).
//
// A wave holds a "pack": up to 64 consecutive elements forming whole blocks,
// one element per lane.  Run structure lives in two wave-uniform 64-bit masks:
//   H  run heads (initially every element; the run of head h is [h, next head))
//   B  block starts (forced chain starts; chains never cross blocks)
// One reference pass = split every block's run sequence into maximal
// non-increasing chains (the reference's `while (y[k] <= y[j])` walk: a chain
// breaks at the first head r with !(y[r] <= y[previous head])), then pool each
// chain whose first and last values differ: num = sum over its runs, in order,
// of y*w, den = sum of w, y = num / den -- the same sequence of roundings as the
// reference, computed by the chain's head lane from lane shuffles.  Passes
// repeat until no chain pools; a block that did not pool is unchanged by later
// passes, so running the wave to the slowest block's convergence is exact.
// Every shuffle runs with all lanes active (ds_bpermute reads only active lanes).
#pragma once
#include "bsls_common.hpp"

// BSLS_K3_KO (timing knock-outs, never in the product build): 1 = no PAVA in
// K3 (and no passes in pava_v1_wave_c), 2 = one pass, 3 = two passes.
#ifndef BSLS_K3_KO
#define BSLS_K3_KO 0
#endif
// BSLS_K3_REPAIR: K3's warm start repairs a failed partition
// (pava_warm_repair) instead of running the reference passes from scratch
#ifndef BSLS_K3_REPAIR
#define BSLS_K3_REPAIR 1
#endif

namespace bsls {

// bits [0, l); l may be 64 (a 64-bit shift by 64 is undefined, and wraps on the GPU)
__device__ __forceinline__ uint64_t mask_lt(int l) {
    return (l >= 64) ? ~0ull : ((1ull << l) - 1ull);
}
__device__ __forceinline__ uint64_t mask_le(int l) {
    return (l >= 63) ? ~0ull : ((2ull << l) - 1ull);
}
__device__ __forceinline__ int hi_bit(uint64_t m) { return 63 - __clzll((long long)m); }
__device__ __forceinline__ int lo_bit(uint64_t m) { return __ffsll((long long)m) - 1; }

__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, WAVE); }
__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, WAVE); }

// y / w: this lane's element value and run length (meaningful at run heads);
// L: active lanes (elements) in the pack; B: block-start mask.
// On return y holds the expanded isotonic fit of this lane's element
// (update = 1 semantics); w the run length if this lane heads a run, and
// `heads` the final run-head mask.
__device__ __forceinline__ void pava_v1_wave(double &y, int &w, int L, uint64_t B,
                                             uint64_t &heads) {
    const int l = lane_id();
    const bool act = l < L;
    uint64_t H = (L >= 64) ? ~0ull : mask_lt(L);
    for (int pass = 0; pass <= L; ++pass) {
        // previous head of every head lane, and the chain starts
        const uint64_t below = H & mask_lt(l);
        const int p = below ? hi_bit(below) : l;
        const double yp = shfl_d(y, p);
        const bool head = act && ((H >> l) & 1ull);
        const bool cs = head && (((B >> l) & 1ull) || !(y <= yp));
        const uint64_t CS = __ballot(cs);
        // chain of a chain start: heads in [l, next chain start)
        const uint64_t above = CS & ~mask_le(l);
        const int nxt = above ? lo_bit(above) : L;
        const uint64_t chain = H & mask_lt(nxt) & ~mask_lt(l);
        const int last = chain ? hi_bit(chain) : l;
        const double ylast = shfl_d(y, last);
        const bool pool = cs && (y != ylast);
        uint64_t cur = pool ? chain : 0ull;
        double num = 0.0;
        int den = 0;
        while (__ballot(cur != 0ull)) {
            const int src = cur ? lo_bit(cur) : l;
            const double ys = shfl_d(y, src);
            const int ws = shfl_i(w, src);
            if (cur) {
                num += ys * (double)ws;
                den += ws;
                cur &= cur - 1ull;
            }
        }
        const uint64_t POOL = __ballot(pool);
        if (!POOL) break;
        // heads absorbed into a pooled chain (every head of it but the first)
        const uint64_t cs_le = CS & mask_le(l);
        const int mycs = cs_le ? hi_bit(cs_le) : l;
        const bool absorbed = head && !cs && ((POOL >> mycs) & 1ull);
        const uint64_t ABS = __ballot(absorbed);
        if (pool) {
            y = num / (double)den;
            w = den;
        }
        H &= ~ABS;
    }
    heads = H;
    // expand: every element takes its run head's value (update = 1)
    const uint64_t hl = H & mask_le(l);
    const int myhead = hl ? hi_bit(hl) : l;
    const double yh = shfl_d(y, myhead);
    if (act) y = yh;
}

// ---------------------------------------------------------------------------
// Compacted form (what K3 runs).  The pass structure and every rounding are the
// same as above; the state is kept per RUN instead of per element: lane t holds
// run t of the pack (value Y, length W, block-start flag, first element O),
// runs packed into lanes 0 .. nh-1 after every pass (a 768-B LDS scatter per
// wave).  Then the previous run is lane t-1 (DPP shift), a chain is a range of
// consecutive lanes, and its in-order pooled sum  num = ((0 + y0 w0) + y1 w1)
// + ...  is a DPP scan, one step per chain member -- about half the VALU of
// the element-lane form (whose searches are 64-bit mask ops and bpermutes).
// Checked bit-for-bit against the reference PAVA (oracle) in
// tests/test_gpu_bb.py::test_k3_wave_pava_bit_exact.

// lane l - 1's value, DPP wave_shr:1 with bound_ctrl (lane 0 reads 0) and
// no `old` operand: one v_mov_b32_dpp per dword, no zero-initialised
// destination (wave_pass only uses the shifted value on lanes >= 1)
__device__ __forceinline__ int dpp_shr1_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ double dpp_shr1_d(double v) {
    const int lo = dpp_shr1_i(__double2loint(v));
    const int hi = dpp_shr1_i(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
// ballot of a bool computed with bitwise operators under the full exec mask
// (HIP's __ballot(int) after a short-circuit && materialises the predicate
// through a branch, a v_cndmask and a v_cmp)
__device__ __forceinline__ uint64_t ballot_b(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Run state of the compacted form: lane t < nh holds run t (value Y, length
// W, block-start flag BS, first element O).
struct WaveRuns {
    double Y;
    int W, BS, O, nh;
};

__device__ __forceinline__ WaveRuns wave_runs(double y, int L, uint64_t B, int obase) {
    const int t = lane_id();
    return WaveRuns{y, 1, (int)((B >> t) & 1ull), t + obase, L};
}

// One reference pass over the runs: false (state unchanged) when no chain
// pools, else the pooled chains merged and the survivors packed into lanes
// 0 .. nh-1.  ys / ps / cst: this wave's 64 doubles / 64 ints / 65 ints of LDS.
__device__ __forceinline__ bool wave_pass(WaveRuns &s, double *ys, int *ps, int *cst) {
    // (predicates with bitwise operators: no branches; the wave masks are
    // combined from ballots of single compares with scalar ops -- a ballot of
    // a compound predicate costs a v_cndmask and a v_cmp to rematerialise the
    // mask the compares already left in SGPRs; the scan counter is
    // wave-uniform)
    const int t = lane_id();
    const bool act = t < s.nh;
    const double yp = dpp_shr1_d(s.Y);
    const bool cs = act & ((s.BS != 0) | !(s.Y <= yp));   // lane 0 is always a block start
    const uint64_t ACT = ballot_b(act);
    const uint64_t CS = ACT & (ballot_b(s.BS != 0) | ballot_b(!(s.Y <= yp)));
    // every run starts a chain (the converged pack's check pass, usually):
    // no chain has two runs, so none pools -- leave before any LDS traffic
    if (!(ACT & ~CS)) return false;
    // chain c of this lane (lanes >= nh: the last chain, unused); the
    // table holds every chain's first run, then nh.  c = (chain starts at or
    // below this lane) - 1 = the chain starts in [1, t], as lane 0 always
    // starts one: the count of CS >> 1 below this lane
    const int c = mbcnt64(CS >> 1);
    if (cs) cst[c] = t;
    if (t == 0) cst[__popcll(CS)] = s.nh;
    const int mycs = cst[c], nxt = cst[c + 1];
    const int last = nxt - 1;                      // this chain's last run
    const double yfirst = shfl_d(s.Y, mycs);
    const double ylast = shfl_d(s.Y, last);
    // the chain pools iff its first and last values differ (the reference's
    // y[i] != y[j]); every member sees both
    const bool inpool = act & (yfirst != ylast);
    const bool pool = cs & inpool;
    if (!(CS & ballot_b(yfirst != ylast))) return false;
    const int depth = t - mycs;
    const double pr = s.Y * (double)s.W;
    double num = 0.0 + pr;
    // k = 1 .. the deepest pooled member (a ballot per step instead of a
    // six-round shuffle max up front: 2-4 steps are typical).  Every member
    // at depth >= k steps at k: after step k such a lane holds the left fold
    // ((0 + pr[t-k]) + pr[t-k+1]) + ... + pr[t] (by induction: lane t - 1,
    // at depth >= k - 1, held the fold over [t-k, t-1]), so at the end a
    // member at depth d holds the fold from its chain's first run -- the
    // reference's order.  The step test is the loop test (one compare per
    // step, no select on depth == k).  Lanes at depth >= 1 read lane t - 1
    // >= 0, so the bound_ctrl zero at lane 0 is never used; the shifts run
    // under the full exec mask (DPP reads of disabled lanes return 0).
    const int dk = inpool ? depth : 0;
    for (int k = 1;; ++k) {
        const bool step = dk >= k;
        if (!ballot_b(step)) break;
        const double np = dpp_shr1_d(num);
        if (step) {
            // (the empty asm keeps this a masked add: if-converted, the
            // update costs two v_cndmask per step)
            num = np + pr;
            asm volatile("" : "+v"(num));
        }
    }
    // the pooled length is the chain's element span (runs cover consecutive
    // elements): the last run's end minus the head's first element -- no
    // integer fold beside the value's (round 6: -7 VALU per pass)
    const double tn = shfl_d(num, last);
    const int tend = shfl_i(s.O + s.W, last);
    if (pool) {
        const int td = tend - s.O;
        s.Y = tn / (double)td;
        s.W = td;
    }
    // pack the surviving runs into lanes 0 .. nh-1
    const bool surv = act & !(dk > 0);
    const uint64_t S = ACT & ~ballot_b(dk > 0);
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

// expand: element e (< L) takes the value of the last run starting at or
// before it (runs with first elements O - obase in [0, L))
__device__ __forceinline__ double wave_expand(const WaveRuns &s, double y, int L, int obase,
                                              int *ps, uint64_t *heads = nullptr) {
    const int t = lane_id();
    ps[t] = 0;
    if (t < s.nh) ps[s.O - obase] = 1;
    const uint64_t RS = __ballot(t < L && ps[t] != 0);
    if (heads) *heads = RS;
    const int idx = mbcnt64(RS) + (int)((RS >> t) & 1ull) - 1;
    const double v = shfl_d(s.Y, idx < 0 ? 0 : idx);
    return (t < L) ? v : y;
}

// y: this lane's element (lanes < L); B: block starts (bit 0 set).  ys / ps /
// cst: this wave's 64 doubles / 64 ints / 65 ints of LDS.  On return y = the
// expanded fit.  (The pass is VALU-bound: chain bounds come from a chain-start
// table in LDS, not from 64-bit mask searches.)
__device__ __forceinline__ void pava_v1_wave_c(double &y, int L, uint64_t B, double *ys,
                                               int *ps, int *cst, uint64_t *heads = nullptr) {
    WaveRuns s = wave_runs(y, L, B, 0);
    const int maxpass = BSLS_K3_KO >= 2 ? BSLS_K3_KO - 2 : L;
    for (int pass = 0; pass <= maxpass && BSLS_K3_KO != 1; ++pass)
        if (!wave_pass(s, ys, ps, cst)) break;
    y = wave_expand(s, y, L, 0, ps, heads);
}

// Two packs in one wave (La, Lb <= 64 elements, one each per lane in ya /
// yb): the first pass of each on its own, then -- when their surviving runs
// fit one wave (C3-like inputs: ~30 of ~55 runs survive the first pass) --
// both run lists in one (b's after a's; chains never cross a block start, and
// a pack starts at one) for the remaining passes, which then cost one pass
// for the two packs.  Each pack's passes and roundings are the reference's:
// a pack that stopped pooling is left unchanged by the passes the other still
// needs.  ps: 128 ints.
__device__ __forceinline__ void pava_v1_wave_pair(double &ya, int La, uint64_t Ba, double &yb,
                                                  int Lb, uint64_t Bb, double *ys, int *ps,
                                                  int *cst, uint64_t *ha = nullptr,
                                                  uint64_t *hb = nullptr) {
    const int t = lane_id();
    WaveRuns a = wave_runs(ya, La, Ba, 0), b = wave_runs(yb, Lb, Bb, 64);
    bool pa = wave_pass(a, ys, ps, cst);
    bool pb = wave_pass(b, ys, ps, cst);
    if (a.nh + b.nh <= WAVE) {
        if (t < b.nh) {
            ys[a.nh + t] = b.Y;
            ps[a.nh + t] = b.W | (b.BS << 8) | (b.O << 9);
        }
        WaveRuns m = a;
        m.nh = a.nh + b.nh;
        if (t >= a.nh && t < m.nh) {
            m.Y = ys[t];
            const int pk = ps[t];
            m.W = pk & 255;
            m.BS = (pk >> 8) & 1;
            m.O = pk >> 9;
        }
        bool more = pa || pb;
        for (int pass = 0; more && pass <= 2 * WAVE; ++pass) more = wave_pass(m, ys, ps, cst);
        // expand over the 128 element slots (a's at 0.., b's at 64..)
        ps[t] = 0;
        ps[WAVE + t] = 0;
        if (t < m.nh) ps[m.O] = 1;
        const uint64_t RA = __ballot(t < La && ps[t] != 0);
        const uint64_t RB = __ballot(t < Lb && ps[WAVE + t] != 0);
        if (ha) *ha = RA;
        if (hb) *hb = RB;
        const int ia = mbcnt64(RA) + (int)((RA >> t) & 1ull) - 1;
        const int ib = __popcll(RA) + mbcnt64(RB) + (int)((RB >> t) & 1ull) - 1;
        const double va = shfl_d(m.Y, ia < 0 ? 0 : ia);
        const double vb = shfl_d(m.Y, ib < 0 ? 0 : ib);
        if (t < La) ya = va;
        if (t < Lb) yb = vb;
        return;
    }
    for (int pass = 0; pa && pass <= La; ++pass) pa = wave_pass(a, ys, ps, cst);
    for (int pass = 0; pb && pass <= Lb; ++pass) pb = wave_pass(b, ys, ps, cst);
    ya = wave_expand(a, ya, La, 0, ps, ha);
    yb = wave_expand(b, yb, Lb, WAVE, ps, hb);
}

// ---------------------------------------------------------------------------
// Warm start (K3 inside an iteration; the north star's 1e-12 contract, not
// bit-identity).  PAVA's fit is unique: a partition of the pack into runs
// (every block start a run start) IS the fit's partition iff, within each
// block, the runs' means do not decrease from run to run and no run can be
// split -- every proper prefix of a run has a mean >= the run's.  Between BB
// iterations the partition rarely changes (oracle replay on a C3-shaped
// problem, /tools/k3_warm.py: 75 % of packs keep it by iteration 20, 97 % by
// 200), so K3 keeps each pack's final run-head mask H and first tests the
// new input against it: one segmented scan (DPP, log steps) gives every
// lane its run's prefix sum, the run sum comes from the run's last lane, and
// two comparisons per lane decide.  If every lane passes, the fit is the run
// means (sums in a tree order: within ulps of the reference's pooled
// roundings); otherwise the pack runs the reference passes.  Comparisons that
// fail only by rounding send the pack to the reference passes (still exact);
// comparisons that pass only by rounding give a fit within ulps of the exact
// one.  H must contain B (bit 0 set) and no bit at or above L.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_mov_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RM, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RM, 0xF, true);
    return __hiloint2double(hi, lo);
}

// The test of a kept partition H, shared by both warm forms: this lane's run
// [h, e], the run's mean m, and the two conditions (split: the prefix of the
// run up to this lane has a mean >= m; order: a run head's mean is >= the
// previous run's within its block).
struct WarmTest {
    int h, e;
    double m;
    bool split_ok, ok;
};

__device__ __forceinline__ WarmTest warm_test(double y, int L, uint64_t B, uint64_t H) {
    const int l = lane_id();
    const bool act = l < L;
    const int h = hi_bit(H & mask_le(l));                    // this lane's run head
    const uint64_t Hg = H & ~mask_le(l);
    const int e = (Hg != 0ull && lo_bit(Hg) < L) ? lo_bit(Hg) - 1 : L - 1;   // its last lane
    // segmented inclusive scan: s = y_h + ... + y_l
    double s = act ? y : 0.0;
    double u;
    u = dpp_mov_d<0x111, 0xF>(s);                            // row_shr:1
    s += (l - 1 >= h) ? u : 0.0;
    u = dpp_mov_d<0x112, 0xF>(s);                            // row_shr:2
    s += (l - 2 >= h) ? u : 0.0;
    u = dpp_mov_d<0x114, 0xF>(s);                            // row_shr:4
    s += (l - 4 >= h) ? u : 0.0;
    u = dpp_mov_d<0x118, 0xF>(s);                            // row_shr:8
    s += (l - 8 >= h) ? u : 0.0;
    u = dpp_mov_d<0x142, 0xA>(s);                            // row_bcast:15 -> rows 1, 3
    s += ((l & 16) != 0 && h <= (l & ~15) - 1) ? u : 0.0;
    u = dpp_mov_d<0x143, 0xC>(s);                            // row_bcast:31 -> rows 2, 3
    s += (l >= 32 && h <= 31) ? u : 0.0;
    const double S = shfl_d(s, e);
    const double m = S / (double)(e - h + 1);
    const double mp = dpp_shr1_d(m);                         // the previous lane's run mean
    const bool split_ok = (l == e) | (s >= (double)(l - h + 1) * m);
    const bool order_ok = (l != h) | (((B >> l) & 1ull) != 0ull) | (mp <= m);
    const bool ok = !act | (split_ok & order_ok);
    return WarmTest{h, e, m, split_ok, ok};
}

__device__ __forceinline__ bool pava_warm(double &y, int L, uint64_t B, uint64_t H) {
    const WarmTest w = warm_test(y, L, B, H);
    if (ballot_b(!w.ok) != 0ull) return false;
    if (lane_id() < L) y = w.m;
    return true;
}

// The warm start with repair (round 5): as pava_warm, but a pack whose kept
// partition fails does not start over from single elements.  A kept run that
// still cannot be split (its every proper prefix mean >= its mean: alone it
// is one level of its own isotonic fit) is a state the reference's pooling
// can reach from single elements, and pooling adjacent violators from any
// such state ends at the one fit; so such runs stay pooled, the runs that can
// be split go back to their elements, and the reference passes run from
// there -- usually one or two instead of ~4 from scratch.  The fit is the
// unique PAVA fit up to the roundings of the kept runs' tree-order sums (the
// north star's 1e-12, as pava_warm).  Returns false when the kept partition
// held (y = its run means, nothing to store), true when the passes ran
// (y = the expanded fit, *heads = its run-head mask).  ys / ps / cst: as
// pava_v1_wave_c.  H as pava_warm.  CPU model over the oracle's weighted
// PAVA: tests/test_pava_repair_model.py.
__device__ __forceinline__ bool pava_warm_repair(double &y, int L, uint64_t B, uint64_t H,
                                                 double *ys, int *ps, int *cst, uint64_t *heads) {
    const int l = lane_id();
    const bool act = l < L;
    const WarmTest w = warm_test(y, L, B, H);
    if (ballot_b(!w.ok) == 0ull) {
        if (act) y = w.m;
        return false;
    }
    // runs holding a lane that fails the split test go back to their
    // elements; the others stay pooled (value m, weight e - h + 1)
    const uint64_t bad = ballot_b(act & !w.split_ok);
    const bool keep = (bad & mask_le(w.e) & ~mask_lt(w.h)) == 0ull;
    const uint64_t H2 = ballot_b(act & (!keep | (l == w.h)));
    if ((H2 >> l) & 1ull) {
        const int idx = mbcnt64(H2);
        ys[idx] = keep ? w.m : y;
        ps[idx] = (keep ? w.e - w.h + 1 : 1) | ((int)((B >> l) & 1ull) << 8) | (l << 9);
    }
    WaveRuns r{y, 1, 0, l, (int)__popcll(H2)};
    if (l < r.nh) {
        r.Y = ys[l];
        const int pk = ps[l];
        r.W = pk & 255;
        r.BS = (pk >> 8) & 1;
        r.O = pk >> 9;
    }
    for (int pass = 0; pass <= L; ++pass)
        if (!wave_pass(r, ys, ps, cst)) break;
    y = wave_expand(r, y, L, 0, ps, heads);
    return true;
}

}  // namespace bsls
