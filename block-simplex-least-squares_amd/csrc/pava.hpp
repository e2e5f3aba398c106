// pava.hpp -- per-block isotonic regression (pool-adjacent-violators), three
// variants with the reference's exact pooling order so results are
// bit-identical (python/c_extensions/isotonic_regression.h).
//
// Each function runs the whole block serially in ONE lane; the caller gives
// each lane its own block, so a wave advances 64 blocks at once.  y/w may point
// into LDS (the staged path) or global memory (the fallback for wide waves).
// w holds run lengths at run heads (the reference's int weight array).
// Returns false if a run length < 1 or a run crossing the block end is met
// (only possible with caller-supplied weights; the reference loops forever or
// reads out of bounds there); the block is then left partially processed.
#pragma once
#include "bsls_common.hpp"

namespace bsls {

// v1 "PAVA+": isotonic_regression.h:13-58
template <typename YP, typename WP, typename I>
__device__ __forceinline__ bool pava_v1(YP y, WP w, I lo, I hi, int expand) {
    const I span = hi - lo;
    for (I pass = 0;; ++pass) {
        if (pass > span) return false;
        bool changed = false;
        I h = lo;
        while (h < hi) {
            const int wh = w[h];
            if (wh < 1) return false;
            I last = h, nxt = h + wh;
            while (nxt < hi && y[nxt] <= y[last]) {
                last = nxt;
                const int wn = w[nxt];
                if (wn < 1) return false;
                nxt += wn;
            }
            if (nxt > hi) return false;
            if (y[h] != y[last]) {
                double num = 0.0;
                int den = 0;
                for (I r = h; r < nxt;) {
                    const int wr = w[r];
                    num += y[r] * (double)wr;
                    den += wr;
                    r += wr;
                }
                y[h] = num / (double)den;
                w[h] = den;
                changed = true;
            }
            h = nxt;
        }
        if (!changed) break;
    }
    if (expand) {
        for (I h = lo; h < hi;) {
            const int wh = w[h];
            const double v = y[h];
            for (I r = h + 1; r < h + wh; ++r) y[r] = v;
            h += wh;
        }
    }
    return true;
}

// v2: unweighted repeated sweeps, isotonic_regression.h:61-82
template <typename YP, typename I>
__device__ __forceinline__ void pava_v2(YP y, I lo, I hi) {
    const I last = hi - 1;
    for (;;) {
        bool changed = false;
        I a = lo;
        while (a < last) {
            I b = a;
            while (b < last && y[b] >= y[b + 1]) ++b;
            if (y[a] != y[b]) {
                double s = 0.0;
                for (I r = a; r <= b; ++r) s += y[r];
                const double mean = s / (double)(b + 1 - a);
                for (I r = a; r <= b; ++r) y[r] = mean;
                changed = true;
            }
            a = b + 1;
        }
        if (!changed) break;
    }
}

// v3: one sweep with backtracking, isotonic_regression.h:105-155
template <typename YP, typename WP, typename I>
__device__ __forceinline__ bool pava_v3(YP y, WP w, I lo, I hi, int expand) {
    I h = lo;
    int64_t guard = 0;
    const int64_t guard_max = 4 * (int64_t)(hi - lo) + 16;
    while (h < hi) {
        if (++guard > guard_max) return false;
        const int wh = w[h];
        if (wh < 1) return false;
        I last = h, nxt = h + wh;
        while (nxt < hi && y[nxt] <= y[last]) {
            last = nxt;
            const int wn = w[nxt];
            if (wn < 1) return false;
            nxt += wn;
        }
        if (nxt > hi) return false;
        if (y[h] != y[last]) {
            double num = 0.0;
            int den = 0;
            for (I r = h; r < nxt;) {
                const int wr = w[r];
                num += y[r] * (double)wr;
                den += wr;
                r += wr;
            }
            y[h] = num / (double)den;
            w[h] = den;
            w[nxt - 1] = den;
            if (h > lo) {
                I p = h - w[h - 1];
                while (p >= lo && y[p] >= y[h]) {
                    y[p] = ((double)w[h] * y[h] + (double)w[p] * y[p]) / (double)(w[h] + w[p]);
                    w[p] = w[h] + w[p];
                    h = p;
                    if (p == lo) break;
                    p -= w[p - 1];
                }
                w[nxt - 1] = w[h];
            }
        } else {
            h = nxt;
        }
    }
    if (expand) {
        for (I a = lo; a < hi;) {
            const int wa = w[a];
            const double v = y[a];
            for (I r = a + 1; r < a + wa && r < hi; ++r) y[r] = v;
            a += wa;
        }
    }
    return true;
}

}  // namespace bsls
