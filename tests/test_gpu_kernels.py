"""Parity of the HIP kernels (through the C ABI) with the oracle.  Needs an MI355X.

Bar: bit-exact for projections / PAVA / x<->z / dense QP (the reference's own
arithmetic order is reproduced); SpMV within 1e-13 relative (summation order
differs from SciPy's sequential row loop).
"""
import numpy as np
import pytest
import scipy.sparse as sps

from conftest import SEED

pytestmark = pytest.mark.gpu


def exact(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


@pytest.fixture(scope='module')
def cx(cuda):
    from c_extensions import c_extensions
    return c_extensions


@pytest.fixture
def exact_proj(monkeypatch):
    """c_extensions' projections on the bit-identical sorting kernels
    (BSLS_PROJ=exact, the default, set explicitly); fast_proj: the sort-free
    _fast path."""
    monkeypatch.setenv('BSLS_PROJ', 'exact')


@pytest.fixture
def fast_proj(monkeypatch):
    monkeypatch.setenv('BSLS_PROJ', 'fast')


def close12(a, ref):
    """The north star's projection contract: |a - ref| <= 1e-12 max(1, |ref|)."""
    a, ref = np.asarray(a, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    return a.shape == ref.shape and bool(np.all(np.abs(a - ref) <= 1e-12 * np.maximum(1.0, np.abs(ref))))


# ------------------------------------------------------------------ projections

def test_proj_golden_numpy(cx, golden, exact_proj):
    G = golden('proj_simplex.npz')
    for ci in range(int(G['ncases'])):
        y, b = G['c%d_y' % ci], G['c%d_blocks' % ci]
        ys = y.copy(); cx.proj_multi_simplex_c(ys, b)
        assert exact(ys, G['c%d_simplex' % ci]), ('simplex', ci)
        yb = y.copy(); cx.proj_multi_ball_c(yb, b)
        assert exact(yb, G['c%d_ball' % ci]), ('ball', ci)
    y = G['single_y'].copy(); cx.proj_simplex_c(y, 10, 40)
    assert exact(y, G['single_out'])


def test_proj_kats(cx, exact_proj):
    z = np.array([5.352, 3.23, 32.78, -1.234, 1.7, 104., 53.])
    for truth, s, e in [([5.352, 3.23, 1., 0., 1.7, 104., 53.], 2, 4),
                        ([0., 0., 0., 0., 0, 1., 0.], 0, 7), (list(z), 4, 4)]:
        y = z.copy(); cx.proj_simplex_c(y, s, e)
        assert list(y) == truth
    for b, truth in [([0, 2, 4], [1., 0., 1., 0., 0., 1., 0.]),
                     ([0], [0., 0., 0., 0., 0., 1., 0.]), ([0, 3], [0., 0., 1., 0., 0., 1., 0.])]:
        y = z.copy(); cx.proj_multi_simplex_c(y, np.array(b))
        assert list(y) == truth
    y = np.array([0.234, 0.5, 1.3, -1.234, 1.7, -1.0, 53.])
    cx.proj_multi_ball_c(y, np.array([0, 2, 4]))
    assert list(y) == [0.234, 0.5, 1., 0., 0., 0., 1.]


@pytest.mark.parametrize('kind', ['unif', 'gauss'])
def test_proj_c2_full_size_bit_exact(cx, orc, kind, exact_proj):
    """Config C2 (3.2M fp64, 100k blocks) on device tensors vs the oracle."""
    import torch
    from synthetic import proj_input
    y, starts = proj_input(kind=kind)
    ref = y.copy()
    orc.proj_multi_simplex_c(ref, starts)
    yd = torch.from_numpy(y).cuda()
    cx.proj_multi_simplex_c(yd, torch.from_numpy(starts).cuda())
    assert exact(yd.cpu().numpy(), ref)


def test_proj_size_classes(cx, orc, exact_proj):
    """Blocks straddling every path: lane (<=64), LDS (<=8192), global (>8192)."""
    rs = np.random.RandomState(SEED)
    sizes = np.array([1, 2, 3, 7, 8, 9, 16, 17, 31, 33, 63, 64, 65, 100, 1000, 4096, 8192, 8193,
                      20000, 5, 64, 1])
    for trial in range(3):
        perm = rs.permutation(sizes)
        starts = np.concatenate(([3], 3 + np.cumsum(perm)[:-1])).astype(np.int64)
        n = 3 + int(perm.sum())
        for scale in (1.0, 0.001, 100.0):
            y = rs.randn(n) * scale
            for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
                a = y.copy(); getattr(cx, name)(a, starts)
                r = y.copy(); getattr(orc, name)(r, starts)
                assert exact(a, r), (trial, scale, name)


def test_proj_ties_and_zeros(cx, orc, exact_proj):
    rs = np.random.RandomState(SEED + 3)
    n = 5000
    starts = np.sort(rs.choice(np.arange(1, n), 150, replace=False))
    starts = np.concatenate(([0], starts)).astype(np.int64)
    for y in (np.zeros(n), np.full(n, 0.25), np.round(rs.rand(n) * 3) / 3, -np.abs(rs.randn(n)),
              np.where(rs.rand(n) < 0.5, -0.0, 0.0)):
        a = y.copy(); cx.proj_multi_simplex_c(a, starts)
        r = y.copy(); orc.proj_multi_simplex_c(r, starts)
        assert exact(a, r)


def test_proj_borderline_decisions(cx, orc, exact_proj):
    """Values on coarse dyadic grids make u_i + (1 - S_i)/(i + 1) land exactly
    on, or within a few ulps of, zero for many i: the cases the kernel decides
    with the reference's own division instead of the fma sign test."""
    rs = np.random.RandomState(SEED + 5)
    n = 60_000
    sizes = rs.randint(1, 65, size=3000)
    sizes = sizes[np.cumsum(sizes) <= n]
    n = int(sizes.sum())
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    grids = [rs.randint(-16, 17, size=n) / 8.0,
             rs.randint(-64, 65, size=n) / 64.0,
             1.0 / rs.randint(1, 9, size=n) - rs.randint(0, 2, size=n) / 3.0,
             np.repeat(rs.randint(-4, 5, size=sizes.size) / 4.0, sizes)
             + rs.randint(-2, 3, size=n) * 2.0 ** -50]
    for gi, y in enumerate(grids):
        for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
            a = y.copy(); getattr(cx, name)(a, starts)
            r = y.copy(); getattr(orc, name)(r, starts)
            assert exact(a, r), (gi, name)


def test_proj_exact_pipe_verification_fallbacks(cx, orc, exact_proj):
    """The pipelined exact path (csrc/proj.hip pipe_exact_lambda) verifies
    Michelot's candidate set in the reference's arithmetic and redoes a block
    the reference's way where it cannot: blocks whose threshold lands exactly
    on an entry (0.75, 0.25, 0, ...: e_c = 0 at the boundary), ties across
    the boundary, all-equal blocks (every entry a member), single entries;
    ball blocks whose clamped sum is 1 to within a few ulps (the left-to-right
    sum decides, proj_simplex.h:56-66); mixed with blocks > 64 inside a wave's
    range (their entries must come back untouched for the big-block kernel).
    Bit-identical to the oracle."""
    rs = np.random.RandomState(SEED + 11)
    blocks = []
    for _ in range(400):
        kind = rs.randint(7)
        k = int(rs.randint(1, 65))
        if kind == 0:
            b = np.zeros(k); b[0] = 0.75
            if k > 1: b[1] = 0.25
        elif kind == 1:
            b = np.full(k, rs.choice([0.5, 1.0 / 3.0, 0.25, 2.0]))
        elif kind == 2:
            b = np.round(rs.rand(k) * 4) / 4
        elif kind == 3:
            r = rs.rand(k); b = r / r.sum()
            b[rs.rand(k) < 0.2] *= -1.0
        elif kind == 4:
            b = np.full(k, 1.0 / k) + rs.randint(-2, 3, size=k) * 2.0 ** -53
        elif kind == 5:
            b = rs.rand(int(rs.randint(65, 200)))
        else:
            b = rs.rand(k)
        blocks.append(b)
    y = np.concatenate(blocks)
    starts = np.concatenate(([0], np.cumsum([b.size for b in blocks])[:-1])).astype(np.int64)
    for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
        for scale in (1.0, 3.0):
            a = y * scale; getattr(cx, name)(a, starts)
            r = y * scale; getattr(orc, name)(r, starts)
            assert exact(a, r), (name, scale)


# ------------------------------------------------- sort-free projection (_fast)
# bsls_proj_multi_*_fast (c_extensions with BSLS_PROJ=fast): Newton on the threshold,
# no sort -- held to the north star's contract |d| <= 1e-12 max(1, |ref|)
# against the oracle (which is pinned to the reference), on the same inputs
# the bit-exact tests above use.

def test_fast_proj_golden_and_kats(cx, golden, fast_proj):
    G = golden('proj_simplex.npz')
    for ci in range(int(G['ncases'])):
        y, b = G['c%d_y' % ci], G['c%d_blocks' % ci]
        ys = y.copy(); cx.proj_multi_simplex_c(ys, b)
        assert close12(ys, G['c%d_simplex' % ci]), ('simplex', ci)
        yb = y.copy(); cx.proj_multi_ball_c(yb, b)
        assert close12(yb, G['c%d_ball' % ci]), ('ball', ci)
    y = G['single_y'].copy(); cx.proj_simplex_c(y, 10, 40)
    assert close12(y, G['single_out'])
    # tests/fast/test_proj_simplex.py:24-82: the reference's exact-equality KATs
    z = np.array([5.352, 3.23, 32.78, -1.234, 1.7, 104., 53.])
    for truth, s_, e_ in [([5.352, 3.23, 1., 0., 1.7, 104., 53.], 2, 4),
                          ([0., 0., 0., 0., 0, 1., 0.], 0, 7), (list(z), 4, 4)]:
        y = z.copy(); cx.proj_simplex_c(y, s_, e_)
        assert list(y) == truth
    for b, truth in [([0, 2, 4], [1., 0., 1., 0., 0., 1., 0.]),
                     ([0], [0., 0., 0., 0., 0., 1., 0.]), ([0, 3], [0., 0., 1., 0., 0., 1., 0.])]:
        y = z.copy(); cx.proj_multi_simplex_c(y, np.array(b))
        assert list(y) == truth
    y = np.array([0.234, 0.5, 1.3, -1.234, 1.7, -1.0, 53.])
    cx.proj_multi_ball_c(y, np.array([0, 2, 4]))
    assert list(y) == [0.234, 0.5, 1., 0., 0., 0., 1.]
    np.random.seed(SEED)
    y = np.random.rand(7)
    cx.proj_simplex_c(y, 0, 7)
    assert np.linalg.norm(y - np.array([0., .05006376, .54108944, 0., .38841272, 0.,
                                        .02043408])) < 1e-6


@pytest.mark.parametrize('kind', ['unif', 'gauss'])
def test_fast_proj_c2_full_size(cx, orc, kind, fast_proj):
    """Config C2 (3.2M fp64, 100k blocks), U[0,1) and 5 N(0,1), simplex and
    ball, device tensors, vs the oracle at 1e-12; and deterministic."""
    import torch
    from synthetic import proj_input
    y, starts = proj_input(kind=kind)
    st = torch.from_numpy(starts).cuda()
    for gpu, cpu in ((cx.proj_multi_simplex_c, orc.proj_multi_simplex_c),
                     (cx.proj_multi_ball_c, orc.proj_multi_ball_c)):
        ref = y.copy()
        cpu(ref, starts)
        yd = torch.from_numpy(y).cuda()
        gpu(yd, st)
        out = yd.cpu().numpy()
        assert close12(out, ref), (kind, gpu.__name__)
        yd2 = torch.from_numpy(y).cuda()
        gpu(yd2, st)
        assert exact(yd2.cpu().numpy(), out)            # fixed reduction order
        # the sums of the projected blocks (simplex: exactly the unit simplex)
        if gpu is cx.proj_multi_simplex_c:
            sums = np.add.reduceat(out, starts)
            assert np.max(np.abs(sums - 1.0)) < 1e-12


def test_fast_proj_size_classes_ties_borderline(cx, orc, fast_proj):
    """Every size class (lane groups <= 64, the exact workgroup / whole-chip
    paths beyond), scales 1e-3..1e2, ties, zeros, signed zeros, the dyadic
    borderline grids where u_i + (1 - S_i)/(i + 1) lands on or near zero."""
    rs = np.random.RandomState(SEED)
    sizes = np.array([1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 31, 33, 63, 64, 65, 100, 1000, 4096,
                      8193, 5, 64, 1])
    for trial in range(3):
        perm = rs.permutation(sizes)
        starts = np.concatenate(([3], 3 + np.cumsum(perm)[:-1])).astype(np.int64)
        n = 3 + int(perm.sum())
        for scale in (1.0, 0.001, 100.0):
            y = rs.randn(n) * scale
            for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
                a = y.copy(); getattr(cx, name)(a, starts)
                r = y.copy(); getattr(orc, name)(r, starts)
                assert close12(a, r), (trial, scale, name)
    n = 5000
    starts = np.sort(rs.choice(np.arange(1, n), 150, replace=False))
    starts = np.concatenate(([0], starts)).astype(np.int64)
    for y in (np.zeros(n), np.full(n, 0.25), np.round(rs.rand(n) * 3) / 3, -np.abs(rs.randn(n)),
              np.where(rs.rand(n) < 0.5, -0.0, 0.0), np.full(n, 1e6), np.full(n, -3.0)):
        for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
            a = y.copy(); getattr(cx, name)(a, starts)
            r = y.copy(); getattr(orc, name)(r, starts)
            assert close12(a, r), name
    n = 60_000
    sizes = rs.randint(1, 65, size=3000)
    sizes = sizes[np.cumsum(sizes) <= n]
    n = int(sizes.sum())
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    grids = [rs.randint(-16, 17, size=n) / 8.0,
             rs.randint(-64, 65, size=n) / 64.0,
             1.0 / rs.randint(1, 9, size=n) - rs.randint(0, 2, size=n) / 3.0,
             np.repeat(rs.randint(-4, 5, size=sizes.size) / 4.0, sizes)
             + rs.randint(-2, 3, size=n) * 2.0 ** -50]
    for gi, y in enumerate(grids):
        for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
            a = y.copy(); getattr(cx, name)(a, starts)
            r = y.copy(); getattr(orc, name)(r, starts)
            assert close12(a, r), (gi, name)


def test_fast_proj_group_ranges(cx, orc, fast_proj):
    """The group kernel's edges (8 consecutive blocks per wave; through LDS
    when the group's range fits the 512-entry stage, else straight to the
    lanes): eight blocks of 64
    (a full stage), a 65 among sevens (a big block inside an LDS range, left
    to the big-block kernel), ranges just past the stage (direct), a partial
    last group, an odd n, and entries before the first block that no block
    owns -- simplex and ball vs the oracle at 1e-12."""
    rs = np.random.RandomState(21)
    layouts = [[64] * 8, [7] * 7 + [65], [65] + [7] * 7, [64] * 7 + [65], [1] * 8,
               [64, 1, 64, 1, 64, 1, 64, 63], [100, 100, 100, 100, 50, 30, 20, 13],
               [33] * 8, [3, 5, 64]]
    sizes = np.array([v for lay in layouts for v in lay])
    for lead in (0, 3):
        starts = (lead + np.concatenate(([0], np.cumsum(sizes)[:-1]))).astype(np.int64)
        n = lead + int(sizes.sum())
        assert n % 2 == 1 or lead == 0
        for scale in (1.0, 5.0, 0.01):
            y = rs.randn(n) * scale
            for name in ('proj_multi_simplex_c', 'proj_multi_ball_c'):
                a = y.copy(); getattr(cx, name)(a, starts)
                r = y.copy(); getattr(orc, name)(r, starts)
                assert close12(a, r), (lead, scale, name)
                assert np.array_equal(a[:lead], y[:lead])


def test_fast_proj_c_abi_entry(cuda, orc):
    """bsls_proj_multi_simplex_fast through the C ABI directly (what bench.py
    times), on a wave-boundary layout: 16-block waves with the last wave
    partial, a first block starting past 0, blocks of 64 and 65."""
    import torch
    import _native
    from _native import ptr, stream_handle, check
    L = _native.lib()
    rs = np.random.RandomState(SEED + 11)
    sizes = np.concatenate((rs.randint(1, 65, size=16 * 37 + 5), [64, 65, 1]))
    starts = np.concatenate(([2], 2 + np.cumsum(sizes)[:-1])).astype(np.int64)
    n = 2 + int(sizes.sum())
    y = rs.rand(n) * 2 - 0.5
    mb = int(sizes.max())
    for fn, cpu in ((L.bsls_proj_multi_simplex_fast, orc.proj_multi_simplex_c),
                    (L.bsls_proj_multi_ball_fast, orc.proj_multi_ball_c)):
        yd = torch.from_numpy(y).cuda()
        sd = torch.from_numpy(starts).cuda()
        ws = torch.zeros(L.bsls_proj_workspace_size(n, sizes.size, mb), dtype=torch.uint8,
                         device='cuda')
        check(fn(ptr(yd), ptr(sd), sizes.size, n, mb, ptr(ws), ws.numel(), stream_handle()),
              'fast')
        r = y.copy()
        cpu(r, starts)
        out = yd.cpu().numpy()
        assert close12(out, r)
        assert out[0] == y[0] and out[1] == y[1]      # before the first block: untouched
    assert L.bsls_proj_multi_simplex_fast(None, None, 0, 0, 1, None, 0, None) == _native.BSLS_E_ARG


# ------------------------------------------------------------------ PAVA

def test_isotonic_golden(cx, golden):
    G = golden('isotonic.npz')
    for ci in range(int(G['ncases'])):
        y, b = G['c%d_y' % ci], G['c%d_blocks' % ci]
        for tag, fn in (('v1', cx.isotonic_regression_multi_c),
                        ('v3', cx.isotonic_regression_multi_c_3)):
            for upd in (1, 0):
                yy = y.copy()
                w = np.ones(len(y), dtype=np.int32)
                fn(yy, b, w, upd)
                assert exact(yy, G['c%d_%s_u%d' % (ci, tag, upd)]), (ci, tag, upd)
                assert np.array_equal(w, G['c%d_%s_u%d_w' % (ci, tag, upd)]), (ci, tag, upd)
        yy = y.copy(); cx.isotonic_regression_multi_c_2(yy, b)
        assert exact(yy, G['c%d_v2' % ci]), ci
    y = np.array([4., 5., 1., 6., 8., 7.])
    cx.isotonic_regression_c(y, 0, 6)
    assert exact(y, G['kat_single'])


def test_isotonic_wave_path_golden(cx, golden):
    """weight=None, update=1 (main.py's call) takes the wave-parallel pack path:
    same bits as the reference with fresh unit weights."""
    G = golden('isotonic.npz')
    for ci in range(int(G['ncases'])):
        yy = G['c%d_y' % ci].copy()
        cx.isotonic_regression_multi_c(yy, G['c%d_blocks' % ci])
        assert exact(yy, G['c%d_v1_u1' % ci]), ci


@pytest.mark.parametrize('kind', ['randn', 'ties', 'decreasing'])
def test_isotonic_wave_path_size_classes(cx, orc, kind):
    """Pack-window edge cases: blocks of 1..130 elements incl. 31/32/33 (the
    window), 63/64/65 (a wave), blocks[0] > 0, and long runs of 1-element
    blocks."""
    rs = np.random.RandomState(17)
    sizes = np.concatenate([rs.randint(1, 40, 3000), [31, 32, 33, 63, 64, 65, 130, 1, 1, 1],
                            np.ones(200, dtype=np.int64), rs.randint(30, 70, 300)])
    rs.shuffle(sizes)
    first = 7
    starts = (first + np.concatenate(([0], np.cumsum(sizes)[:-1]))).astype(np.int64)
    n = int(first + sizes.sum())
    if kind == 'randn':
        y = rs.randn(n)
    elif kind == 'ties':
        y = np.round(rs.randn(n), 0)
        y[rs.rand(n) < 0.1] = -0.0
    else:
        y = -np.arange(n, dtype=np.float64) + 0.25 * rs.randn(n)
    ref = y.copy(); orc.isotonic_regression_multi_c(ref, starts)
    got = y.copy(); cx.isotonic_regression_multi_c(got, starts)
    assert exact(got, ref)
    assert exact(got[:first], y[:first])


def test_isotonic_c3_full_size(cx, orc):
    """z-space PAVA at config C3 (950k entries, 50k blocks) vs the oracle."""
    import torch
    rs = np.random.RandomState(SEED)
    sizes = rs.multinomial(1_000_000 - 50_000, np.ones(50_000) / 50_000) + 1
    zst = np.concatenate(([0], np.cumsum(sizes - 1)[:-1])).astype(np.int64)
    nz = int((sizes - 1).sum())
    y = rs.randn(nz)
    ref = y.copy(); orc.isotonic_regression_multi_c(ref, zst)
    yd = torch.from_numpy(y).cuda()
    cx.isotonic_regression_multi_c(yd, torch.from_numpy(zst).cuda())
    assert exact(yd.cpu().numpy(), ref)


def test_isotonic_weight_semantics(cx):
    # an int32 contiguous weight array is updated in place; int64 is copied
    y = np.array([4., 5., 1., 6., 8., 7.])
    w32 = np.ones(6, dtype=np.int32)
    cx.isotonic_regression_multi_c(y, np.array([0]), w32, 0)
    assert list(w32[[0, 3, 4]]) == [3, 1, 2]
    w64 = np.ones(6, dtype=np.int64)
    cx.isotonic_regression_multi_c(np.array([4., 5., 1., 6., 8., 7.]), np.array([0]), w64, 0)
    assert list(w64) == [1] * 6


# ------------------------------------------------------------------ x<->z, QP

def test_xz_quad_golden(cx, golden):
    G = golden('xz_quad.npz')
    for ci in range(int(G['nxz'])):
        x, b, zt = G['c%d_x' % ci], G['c%d_blocks' % ci], G['c%d_z' % ci]
        z = np.zeros_like(zt)
        cx.x2z_c(x, z, b)
        assert exact(z, zt)
        xb = np.zeros_like(x)
        cx.z2x_c(xb, z, b)
        assert exact(xb, G['c%d_xback' % ci])
    for qi in range(int(G['nquad'])):
        x, Q, c = G['q%d_x' % qi], G['q%d_Q' % qi], G['q%d_c' % qi]
        g = np.zeros_like(x)
        f = cx.quad_obj_c(x, Q.flatten(), c, g)
        assert exact(g, G['q%d_g' % qi]) and f == float(G['q%d_f' % qi])


def test_line_search_vs_oracle(cx, orc):
    rs = np.random.RandomState(SEED)
    Q = (2 * np.array([[2, .5], [.5, 1]])).flatten()
    c = np.array([1.0, 1.0])
    for x, f, g in [((.5, .5), 2., (3.5, 2.5)), ((.25, .75), 1.875, (2.75, 2.75)),
                    ((.26, .74), 1.8752, (2.78, 2.74))]:
        outs = []
        for mod in (cx, orc):
            xn, gn = np.array([0., 1.]), np.array([2., 3.])
            fn = mod.line_search_quad_obj_c(np.array(x), f, np.array(g), xn, 2., gn, Q, c)
            outs.append((fn, xn, gn))
        assert outs[0][0] == outs[1][0] and exact(outs[0][1], outs[1][1]) and \
            exact(outs[0][2], outs[1][2])
    for n in (3, 17):
        M = rs.randn(n, n); Qn = (M @ M.T).flatten(); cn = rs.randn(n)
        x = rs.rand(n); g = np.zeros(n); f = orc.quad_obj_c(x, Qn, cn, g)
        xn0 = x + rs.randn(n); gn0 = np.zeros(n); fn0 = orc.quad_obj_c(xn0, Qn, cn, gn0)
        outs = []
        for mod in (cx, orc):
            xn, gn = xn0.copy(), gn0.copy()
            fo = mod.line_search_quad_obj_c(x, f, g, xn, fn0, gn, Qn, cn)
            outs.append((fo, xn, gn))
        assert outs[0][0] == outs[1][0] and exact(outs[0][1], outs[1][1])
        assert exact(outs[0][2], outs[1][2])


# ------------------------------------------------------------------ SpMV

@pytest.mark.parametrize('shape,per_row', [((1000, 3000), 40), ((5000, 800), 3), ((300, 300), 160)])
def test_spmv_vs_scipy(cuda, shape, per_row):
    import torch
    from device import DeviceCSR
    rs = np.random.RandomState(SEED)
    m, n = shape
    A = sps.random(m, n, density=min(1.0, per_row / n), random_state=rs, format='csr')
    A.data = rs.randn(A.nnz)
    x = rs.randn(n)
    add = rs.randn(m)
    D = DeviceCSR(A)
    out, sq = D.matvec(torch.from_numpy(x).cuda(), add=torch.from_numpy(add).cuda(), want_sq=True)
    ref = A.dot(x) + add
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-13, atol=1e-13)
    assert abs(float(sq.item()) - ref.dot(ref)) <= 1e-12 * ref.dot(ref)
    for G in (1, 2, 4, 8, 16, 32, 64):
        D.group = G
        o = D.matvec(torch.from_numpy(x).cuda())
        np.testing.assert_allclose(o.cpu().numpy(), A.dot(x), rtol=1e-13, atol=1e-13)


# ------------------------------------------------------------------ stress shapes

def test_proj_stress_shapes_bit_exact(cx, orc, exact_proj):
    """python/experiments/test_stress_proj_simplex.py:24-44: single U[0,1) blocks
    up to 1e6 and 1e6 elements in 10 / 100 / 1e4 random blocks (the whole-chip
    sort path for blocks > 8192), simplex and l1-ball, vs the oracle."""
    np.random.seed(SEED)
    for n in (20_000, 1_000_000):
        y = np.random.rand(n)
        a, r = y.copy(), y.copy()
        cx.proj_simplex_c(a, 0, n)
        orc.proj_simplex_c(r, 0, n)
        assert exact(a, r), n
    for nb in (10, 100, 10_000):
        y = np.random.rand(1_000_000)
        blocks = np.sort(np.random.choice(1_000_000, nb, replace=False)).astype(np.int64)
        for gpu, cpu in ((cx.proj_multi_simplex_c, orc.proj_multi_simplex_c),
                         (cx.proj_multi_ball_c, orc.proj_multi_ball_c)):
            a, r = y.copy(), y.copy()
            gpu(a, blocks)
            cpu(r, blocks)
            assert exact(a, r), nb
    # ball blocks whose clamped sum is <= 1 (left clamped, not projected)
    y = np.random.rand(100_000) * 1e-6 - 2e-7
    a, r = y.copy(), y.copy()
    cx.proj_multi_ball_c(a, np.array([0, 30_000]))
    orc.proj_multi_ball_c(r, np.array([0, 30_000]))
    assert exact(a, r)


def test_pava_stress_shapes_bit_exact(cx, orc):
    """python/experiments/PAVA_worst_case.py:12-40 on variant 1 (main.py's):
    the log-trend data up to 1e6 in one block and the worst case (arange with
    y[-1] = -1e12, one pooling per pass), one workgroup per long block."""
    rs = np.random.RandomState(0)
    for n in (1000, 100_000, 1_000_000):
        y = rs.randint(-50, 50, size=(n,)) + 50. * np.log(1 + np.arange(n))
        a, r = y.copy(), y.copy()
        cx.isotonic_regression_c(a, 0, n)
        orc.isotonic_regression_c(r, 0, n)
        assert exact(a, r), n
    for n in (100, 2000):
        y = np.arange(n).astype(float)
        y[-1] = -1e12
        a, r = y.copy(), y.copy()
        cx.isotonic_regression_c(a, 0, n)
        orc.isotonic_regression_c(r, 0, n)
        assert exact(a, r), n
    # several long blocks next to short ones, one pass
    y = rs.randn(300_000)
    blocks = np.sort(np.concatenate(([0], rs.choice(np.arange(1, 300_000), 40, replace=False))))
    a, r = y.copy(), y.copy()
    cx.isotonic_regression_multi_c(a, blocks)
    orc.isotonic_regression_multi_c(r, blocks)
    assert exact(a, r)
