"""K3's warm-start repair (csrc/pava_wave.hpp `pava_warm_repair`) modelled on
the CPU over the oracle's PAVA v1 (python/c_extensions/isotonic_regression.h:
13-58, `oracle.isotonic_regression_multi_c`).  The reference's `weight`
argument already describes a pre-pooled state (a run head holds the run's
value and length, `isotonic_regression.h:22-24`), so the model hands the
oracle the repaired state directly: each run of a stale partition whose every
proper prefix mean is >= its mean stays pooled (value = its mean), every other
run goes back to its elements, and the reference passes run from there.  The
claim the kernel rests on -- pooling adjacent violators from any such state
ends at the one isotonic fit -- is checked here against the exact fit for
partitions kept from nearby inputs (what K3 sees between BB iterations) and
for arbitrary random partitions; and the split is shown to be needed."""
import numpy as np


def _runs(heads, n):
    h = np.flatnonzero(heads)
    return zip(h, np.append(h[1:], n))


def repaired_state(y, heads):
    """(values, weights) of the repaired state: kept runs pooled at their head."""
    n = y.shape[0]
    yy, w = y.copy(), np.ones(n, dtype=np.int32)
    for a, b in _runs(heads, n):
        seg = y[a:b]
        k = b - a
        m = seg.sum() / k
        pre = np.cumsum(seg)[:-1]
        if np.all(pre >= np.arange(1, k) * m):
            yy[a], w[a] = m, k
    return yy, w


def fit_heads(fit, starts):
    """Run heads of a fit: block starts and every change of value."""
    heads = np.zeros(fit.shape[0], dtype=bool)
    heads[starts] = True
    heads[1:] |= fit[1:] != fit[:-1]
    return heads


def _problem(rs, nblocks=400):
    sizes = rs.randint(1, 60, size=nblocks)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    return starts, int(sizes.sum())


def _exact(orc, y, starts):
    e = y.copy()
    orc.isotonic_regression_multi_c(e, starts)
    return e


def _from_state(orc, y, heads, starts):
    yy, w = repaired_state(y, heads)
    orc.isotonic_regression_multi_c(yy, starts, weight=w, update=1)
    return yy


def test_repair_from_nearby_partitions(orc):
    rs = np.random.RandomState(3)
    starts, n = _problem(rs)
    base = rs.randn(n)
    prev = _exact(orc, base, starts)
    heads = fit_heads(prev, starts)
    for scale in (0.0, 1e-9, 1e-4, 1e-2, 0.3, 3.0):
        y = base + scale * rs.randn(n)
        got = _from_state(orc, y, heads, starts)
        ref = _exact(orc, y, starts)
        assert np.max(np.abs(got - ref)) <= 1e-12, scale


def test_repair_from_random_partitions(orc):
    rs = np.random.RandomState(5)
    for trial in range(20):
        starts, n = _problem(rs, 200)
        y = rs.randn(n) * rs.choice([1e-3, 1.0, 1e3])
        heads = rs.rand(n) < rs.choice([0.05, 0.3, 0.7])
        heads[starts] = True
        got = _from_state(orc, y, heads, starts)
        ref = _exact(orc, y, starts)
        assert np.max(np.abs(got - ref)) <= 1e-12 * max(1.0, np.max(np.abs(y))), trial


def test_split_is_needed(orc):
    """Keeping every stale run pooled (no split test) misses the fit: the
    passes only merge, so a run the new input splits stays wrong."""
    rs = np.random.RandomState(7)
    starts, n = _problem(rs)
    prev = _exact(orc, rs.randn(n), starts)
    heads = fit_heads(prev, starts)
    y = rs.randn(n)
    yy, w = y.copy(), np.ones(n, dtype=np.int32)
    for a, b in _runs(heads, n):
        yy[a], w[a] = y[a:b].mean(), b - a
    orc.isotonic_regression_multi_c(yy, starts, weight=w, update=1)
    assert np.max(np.abs(yy - _exact(orc, y, starts))) > 1e-3


def test_repair_with_ties(orc):
    """Inputs on a coarse grid (many exact ties: equal runs pool or not as the
    passes meet them), kept partitions from a nearby tied input."""
    rs = np.random.RandomState(9)
    starts, n = _problem(rs)
    base = np.round(rs.randn(n) * 4) / 4
    heads = fit_heads(_exact(orc, base, starts), starts)
    for y in (base, base + 0.25 * (rs.rand(n) < 0.1), np.round(rs.randn(n) * 2) / 2):
        got = _from_state(orc, y, heads, starts)
        assert np.max(np.abs(got - _exact(orc, y, starts))) <= 1e-12


def test_repair_near_ties_over_many_warm_starts(orc):
    """a kept run that can be split only by a rounding margin
    stays pooled under the repair's floating-point prefix test.  Inputs on a
    coarse grid (exact ties) perturbed by ~1e-15 relative, 60 warm starts in a
    row, each keeping the previous result's partition (as K3 does between
    iterations): every fit within 1e-12 of the exact one."""
    rs = np.random.RandomState(13)
    starts, n = _problem(rs)
    grid = np.round(rs.randn(n) * 4) / 4
    heads = fit_heads(_exact(orc, grid, starts), starts)
    worst = 0.0
    for it in range(60):
        y = grid * (1.0 + 1e-15 * rs.randn(n)) + 1e-15 * rs.randn(n) * (it % 3 == 0)
        got = _from_state(orc, y, heads, starts)
        err = np.max(np.abs(got - _exact(orc, y, starts)))
        worst = max(worst, err)
        assert err <= 1e-12 * max(1.0, np.max(np.abs(y))), (it, err)
        heads = fit_heads(got, starts)
    assert worst < 1e-13, worst
