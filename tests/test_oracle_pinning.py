"""Pin the CPU oracle to the reference (CPU only).

Every oracle function is checked bit-for-bit against
  * the golden fixtures captured from the reference itself
    (tests/golden/make_golden.py), and
  * the reference's own known-answer tests (tests/fast/test_proj_simplex.py,
    test_isotonic_regression.py, test_c_extensions.py, isotonic_regression.h
    self-test), restated here as data, and
  * oracle/_ref/libbsls_ref.so (reference headers compiled here) on fresh
    random inputs, when that library is present.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sps

from conftest import SEED


def exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


# --------------------------------------------------------------- KATs

def test_kat_proj_simplex_single(orc):
    # tests/fast/test_proj_simplex.py:24-34
    z = np.array([5.352, 3.23, 32.78, -1.234, 1.7, 104., 53.])
    cases = [([5.352, 3.23, 1., 0., 1.7, 104., 53.], 2, 4),
             ([0., 0., 0., 0., 0, 1., 0.], 0, 7),
             (list(z), 4, 4)]
    for truth, s, e in cases:
        y = z.copy()
        orc.proj_simplex_c(y, s, e)
        assert list(y) == truth
    np.random.seed(SEED)
    y = np.random.rand(7)
    orc.proj_simplex_c(y, 0, 7)
    truth = np.array([0., .05006376, .54108944, 0., .38841272, 0., .02043408])
    assert np.linalg.norm(y - truth) < 1e-6
    for s, e in [(2, 8), (-1, 7), (-1, 4)]:
        with pytest.raises(AssertionError):
            orc.proj_simplex_c(y, s, e)


def test_kat_proj_multi(orc):
    # tests/fast/test_proj_simplex.py:43-59,77-81
    z = np.array([5.352, 3.23, 32.78, -1.234, 1.7, 104., 53.])
    for b, truth in [([0, 2, 4], [1., 0., 1., 0., 0., 1., 0.]),
                     ([0], [0., 0., 0., 0., 0., 1., 0.]),
                     ([0, 3], [0., 0., 1., 0., 0., 1., 0.])]:
        y = z.copy()
        orc.proj_multi_simplex_c(y, np.array(b))
        assert list(y) == truth
    for b in ([-1, 2, 4], [1, 3, 7], [0, 4, 2]):
        with pytest.raises(AssertionError):
            orc.proj_multi_simplex_c(z.copy(), np.array(b))
    y = np.array([0.234, 0.5, 1.3, -1.234, 1.7, -1.0, 53.])
    orc.proj_multi_ball_c(y, np.array([0, 2, 4]))
    assert list(y) == [0.234, 0.5, 1., 0., 0., 0., 1.]


def test_kat_isotonic(orc, golden):
    # isotonic_regression.h:169-194 / check_extensions.py:11-22
    y = np.array([4., 5., 1., 6., 8., 7.])
    orc.isotonic_regression_multi_c(y, np.array([0]))
    assert np.allclose(y, [10 / 3, 10 / 3, 10 / 3, 6, 7.5, 7.5], atol=1e-12)
    assert exact(y, golden('isotonic.npz')['kat_single'])
    y = np.array([4., 5., 1., 6., 8., 7.])
    orc.isotonic_regression_multi_c(y, np.array([0, 2, 4]))
    assert list(y) == [4, 5, 1, 6, 7.5, 7.5]
    for fn in (orc.isotonic_regression_multi_c_2, orc.isotonic_regression_multi_c_3):
        y = np.array([4., 5., 1., 6., 8., 7.])
        fn(y, np.array([0, 2, 4]))
        assert list(y) == [4, 5, 1, 6, 7.5, 7.5]


def test_kat_isotonic_vs_sklearn(orc):
    # tests/fast/test_isotonic_regression.py:49-115 (sklearn at 1e-8)
    from sklearn.isotonic import IsotonicRegression
    from sklearn.utils import check_random_state
    np.random.seed(SEED)
    rs = check_random_state(0)
    n = 10
    for _ in range(10):
        y = rs.randint(-50, 50, size=(n,)) + 50. * np.log(1 + np.arange(n))
        blocks = np.sort(np.random.choice(n, 3, replace=False))
        truth = y.copy()
        for s, e in zip(blocks, np.append(blocks[1:], [n])):
            truth[s:e] = IsotonicRegression().fit_transform(np.arange(s, e), y[s:e])
        for fn in (orc.isotonic_regression_multi_c, orc.isotonic_regression_multi_c_2,
                   orc.isotonic_regression_multi_c_3):
            yy = y.copy()
            fn(yy, blocks)
            assert np.linalg.norm(yy - truth) < 1e-8


def test_kat_x2z_z2x(orc):
    # tests/fast/test_c_extensions.py:67-79
    xs = [[.6, .1, .3], [.5, .5, .2, .8], [1., .6, .1, .3]]
    zs = [[.6, .7], [.5, .2], [.6, .7]]
    bs = [[0], [0, 2], [0, 1]]
    for xt, zt, b in zip(xs, zs, bs):
        z = np.zeros(len(zt))
        orc.x2z_c(np.array(xt), z, np.array(b))
        assert np.linalg.norm(z - zt) < 1e-8
        x = np.zeros(len(xt))
        orc.z2x_c(x, z, np.array(b))
        assert np.linalg.norm(x - xt) < 1e-8


def test_kat_line_search(orc):
    # tests/fast/test_c_extensions.py:44-64
    Q = (2 * np.array([[2, .5], [.5, 1]])).flatten()
    c = np.array([1.0, 1.0])
    cases = [((.5, .5), 2., (3.5, 2.5), (.25, .75), 1.875, (2.75, 2.75)),
             ((.25, .75), 1.875, (2.75, 2.75), (.25, .75), 1.875, (2.75, 2.75)),
             ((.26, .74), 1.8752, (2.78, 2.74), (0.2559375, 0.7440625), 1.87507050781,
              (2.7678125, 2.7440625))]
    for x, f, g, xt, ft, gt in cases:
        x_new, g_new = np.array([0., 1.]), np.array([2., 3.])
        fn = orc.line_search_quad_obj_c(np.array(x), f, np.array(g), x_new, 2., g_new, Q, c)
        assert np.linalg.norm(x_new - xt) < 1e-8
        assert abs(fn - ft) < 1e-8
        assert np.linalg.norm(g_new - gt) < 1e-6


def test_kat_particular_x0(orc):
    # tests/fast/test_util.py:27-32
    assert list(orc.particular_x0(np.array([1, 2, 3, 4]))) == [1, 0, 1, 0, 0, 1, 0, 0, 0, 1]


# --------------------------------------------------------------- golden vectors

def test_golden_projection(orc, golden):
    G = golden('proj_simplex.npz')
    for ci in range(int(G['ncases'])):
        y, b = G['c%d_y' % ci], G['c%d_blocks' % ci]
        ys = y.copy(); orc.proj_multi_simplex_c(ys, b)
        yb = y.copy(); orc.proj_multi_ball_c(yb, b)
        assert exact(ys, G['c%d_simplex' % ci]), ci
        assert exact(yb, G['c%d_ball' % ci]), ci
    y = G['single_y'].copy(); orc.proj_simplex_c(y, 10, 40)
    assert exact(y, G['single_out'])


def test_golden_isotonic(orc, golden):
    G = golden('isotonic.npz')
    for ci in range(int(G['ncases'])):
        y, b = G['c%d_y' % ci], G['c%d_blocks' % ci]
        for tag, fn in (('v1', orc.isotonic_regression_multi_c),
                        ('v3', orc.isotonic_regression_multi_c_3)):
            for upd in (1, 0):
                yy = y.copy()
                w = fn(yy, b, None, upd)
                assert exact(yy, G['c%d_%s_u%d' % (ci, tag, upd)]), (ci, tag, upd)
                assert np.array_equal(w, G['c%d_%s_u%d_w' % (ci, tag, upd)]), (ci, tag, upd)
        yy = y.copy(); orc.isotonic_regression_multi_c_2(yy, b)
        assert exact(yy, G['c%d_v2' % ci]), ci


def test_golden_xz_quad(orc, golden):
    G = golden('xz_quad.npz')
    for ci in range(int(G['nxz'])):
        x, b, zt = G['c%d_x' % ci], G['c%d_blocks' % ci], G['c%d_z' % ci]
        z = np.zeros_like(zt)
        orc.x2z_c(x, z, b)
        assert exact(z, zt)
        xb = np.zeros_like(x)
        orc.z2x_c(xb, z, b)
        assert exact(xb, G['c%d_xback' % ci])
    for qi in range(int(G['nquad'])):
        x, Q, c = G['q%d_x' % qi], G['q%d_Q' % qi], G['q%d_c' % qi]
        g = np.zeros_like(x)
        f = orc.quad_obj_c(x, Q.flatten(), c, g)
        assert exact(g, G['q%d_g' % qi]) and f == float(G['q%d_f' % qi])


def _csr(G, tag):
    return sps.csr_matrix((G['%s_A_data' % tag], G['%s_A_indices' % tag],
                           G['%s_A_indptr' % tag]), shape=tuple(G['%s_A_shape' % tag]))


@pytest.mark.parametrize('tag', ['bbs', 'bbc'])
def test_golden_bb_trajectory(orc, golden, tag):
    """Oracle BB loop == reference BB.solve, every iteration, bit for bit."""
    G = golden('solvers.npz')
    A = _csr(G, tag)
    iters = G['%s_iters' % tag]
    rec = orc.bb_trace(A, G['%s_b' % tag], G['%s_block_sizes' % tag], int(iters[-1]))
    assert sorted(rec) == list(iters)
    for k, it in enumerate(iters):
        assert exact(rec[it], G['%s_states' % tag][k]), it


def test_golden_dore(orc, golden):
    G = golden('solvers.npz')
    A = _csr(G, 'dore')
    iters, states, lsv = orc.dore_run(A, G['dore_b'], G['dore_block_sizes'], 300)
    assert abs(lsv - float(G['dore_lsv'])) <= 1e-12 * abs(lsv)
    assert list(iters) == list(G['dore_iters'])
    for s, t in zip(states, G['dore_states']):
        np.testing.assert_allclose(s, t, rtol=1e-9, atol=1e-12)


def test_golden_mirror_descent(orc, golden):
    G = golden('solvers.npz')
    A = _csr(G, 'md')
    for it in (1, 5, 40):
        x = orc.md_least_squares(A, G['md_b'], list(G['md_blocks']), iters=it, tolerance=0.0)
        np.testing.assert_allclose(x, G['md_x_%d' % it], rtol=1e-10, atol=1e-14)


def test_golden_main_problems_converge(orc, golden):
    """tests/fast/test_main.py: BB on the generate_data problems reaches
    0.5||Ax-b||^2 < 1e-16 at the same final iteration as the reference."""
    G = golden('solvers.npz')
    for vi in range(3):
        A = _csr(G, 'main%d' % vi)
        b, bs = G['main%d_b' % vi], G['main%d_block_sizes' % vi]
        P = orc.solve_in_z_parts(A, b, bs)
        rec = {}

        def log(i, s, dt):
            rec[i] = np.array(s)
            return 0.0
        orc.bb_solve(P['z0'], P['f'], P['nabla_f'], orc.stopping, proj=P['proj'], log=log,
                     options={'max_iter': 300000, 'verbose': 1, 'opt_tol': 1e-30})
        ref_iters = list(G['main%d_iters' % vi])
        assert sorted(rec) == sorted(set(ref_iters))
        last = max(rec)
        assert exact(rec[last], G['main%d_states' % vi][-1])
        x = P['x0'] + P['N'].dot(rec[last])
        assert 0.5 * np.linalg.norm(A.dot(x) - b) ** 2 < 1e-16


@pytest.mark.parametrize('tag', ['grad8', 'noopt', 'maxit', 'vertex'])
def test_golden_stopping_exits(orc, golden, tag):
    """Oracle BB loop + stopping == the reference's GradientDescent('BB') runs
    ending at each exit of solvers.stopping / BB.py:22: same logged
    iterations (so the same exit iteration), same states bit for bit."""
    G = golden('plugins.npz')
    A = _csr(G, tag)
    opts = {'grad8': {'max_iter': 20000, 'verbose': 0, 'opt_tol': 1e-8},
            'noopt': {'max_iter': 20000, 'verbose': 0},
            'maxit': {'max_iter': 777, 'verbose': 0, 'opt_tol': 1e-30},
            'vertex': {'max_iter': 2000, 'verbose': 0, 'opt_tol': 1e-30}}[tag]
    P = orc.solve_in_z_parts(A, G['%s_b' % tag], G['%s_block_sizes' % tag])
    rec = {}

    def log(i, s, dt):
        rec[i] = np.array(s)
        return 0.0
    orc.bb_solve(P['z0'], P['f'], P['nabla_f'], orc.stopping, proj=P['proj'], log=log,
                 options=opts)
    assert sorted(rec) == list(G['%s_iters' % tag])
    for k, it in enumerate(G['%s_iters' % tag]):
        assert exact(rec[it], G['%s_states' % tag][k]), it


# --------------------------------------------------------------- vs compiled reference

def _ref_or_skip(orc):
    R = orc.ref_lib()
    if R is None:
        pytest.skip('oracle/_ref not built (no /root/reference here)')
    return R


def test_vs_ref_projection_random(orc):
    R = _ref_or_skip(orc)
    rs = np.random.RandomState(SEED)
    for trial in range(40):
        n = int(rs.randint(2, 4000))
        nb = int(rs.randint(1, max(2, n // 3)))
        starts = np.sort(rs.choice(np.arange(1, n), nb - 1, replace=False)) if nb > 1 else []
        first = int(rs.randint(0, 3)) if (nb == 1 or starts[0] > 3) else 0
        b = np.concatenate(([first], starts)).astype(np.int64)
        y = rs.randn(n) * rs.choice([0.01, 1, 10])
        b32 = b.astype(np.int32)
        for oname, rname in (('proj_multi_simplex_c', 'ref_proj_multi_simplex'),
                             ('proj_multi_ball_c', 'ref_proj_multi_ball')):
            a = y.copy(); getattr(orc, oname)(a, b)
            r = y.copy(); getattr(R, rname)(orc._pd(r), orc._p32(b32), len(b), n)
            assert exact(a, r), (trial, oname)
        for oname, rname in (('isotonic_regression_multi_c', 'ref_isotonic_regression_multi'),
                             ('isotonic_regression_multi_c_3', 'ref_isotonic_regression_multi_3')):
            for upd in (0, 1):
                a = y.copy(); wa = getattr(orc, oname)(a, b, None, upd)
                r = y.copy(); wr = np.ones(n, dtype=np.int32)
                getattr(R, rname)(orc._pd(r), orc._p32(b32), len(b), n, orc._p32(wr), upd)
                assert exact(a, r) and np.array_equal(wa, wr), (trial, oname, upd)
        a = y.copy(); orc.isotonic_regression_multi_c_2(a, b)
        r = y.copy(); R.ref_isotonic_regression_multi_2(orc._pd(r), orc._p32(b32), len(b), n)
        assert exact(a, r), trial


def test_vs_ref_quad(orc):
    R = _ref_or_skip(orc)
    rs = np.random.RandomState(SEED)
    for n in (1, 2, 7, 40):
        for _ in range(5):
            x = rs.randn(n); Q = rs.randn(n, n); Q = (Q @ Q.T).flatten(); c = rs.randn(n)
            g1, g2 = np.zeros(n), np.zeros(n)
            f1 = orc.quad_obj_c(x, Q, c, g1)
            f2 = R.ref_quad_obj(orc._pd(x), orc._pd(Q), orc._pd(c), orc._pd(g2), n)
            assert f1 == f2 and exact(g1, g2)
            xn = x + rs.randn(n)
            gn = np.zeros(n)
            fn = orc.quad_obj_c(xn, Q, c, gn)
            a_x, a_g = xn.copy(), gn.copy()
            r_x, r_g = xn.copy(), np.append(gn, 0.0)     # room for the reference's g_new[n]
            fa = orc.line_search_quad_obj_c(x, f1, g1, a_x, fn, a_g, Q, c)
            fr = R.ref_line_search(orc._pd(x), f1, orc._pd(g1), orc._pd(r_x), fn, orc._pd(r_g),
                                   orc._pd(Q), orc._pd(c), n)
            assert fa == fr and exact(a_x, r_x) and exact(a_g, r_g[:n])


# ------------------------------------------------ x-space batch solvers

def _batch_problem(golden, tag):
    d = golden('batch.npz')
    A = sps.csr_matrix((d['%s_A_data' % tag], d['%s_A_indices' % tag], d['%s_A_indptr' % tag]),
                       shape=tuple(d['%s_A_shape' % tag]))
    return d, A, d['%s_b' % tag], d['%s_starts' % tag], d['%s_x_init' % tag]


@pytest.mark.parametrize('tag,lasso', [('s', False), ('c', False), ('l', True)])
def test_golden_batch_solve_bb(orc, golden, tag, lasso):
    """BATCH.solve_BB over get_solver_parts(is_sparse=True) (python/BATCH.py:55-106):
    the restatement reproduces the reference bit for bit (same SciPy SpMV, same
    projection arithmetic, same NumPy reductions)."""
    d, A, b, starts, x0 = _batch_problem(golden, tag)
    obj, proj, ls = orc.sparse_parts(A, b, starts, lasso=lasso)
    for k in (2, 3, 6, 15, 40):
        sol = orc.batch_solve_bb(obj, proj, ls, x0.copy(), max_iter=k)
        assert exact(sol['x'], d['%s_bb%d_x' % (tag, k)]), (tag, k)
        assert sol['iterations'] == int(d['%s_bb%d_it' % (tag, k)])
        assert sol['stop'] == str(d['%s_bb%d_stop' % (tag, k)])
        assert exact(sol['progress'], d['%s_bb%d_prog' % (tag, k)])


LBFGS_RUNS = [(k, 50) for k in (2, 3, 6, 7, 10, 15, 40, 2000)] + [(30, 3)]


def _lbfgs_key(tag, k, corr):
    return '%s_lb%d' % (tag, k) + ('' if corr == 50 else '_c%d' % corr)


@pytest.mark.parametrize('tag', ['s', 'c'])
def test_golden_batch_solve_lbfgs(orc, golden, tag):
    """BATCH.solve_LBFGS over get_solver_parts(is_sparse=True)
    (python/BATCH.py:110-214, fixtures tests/golden/lbfgs.npz): the
    restatement's vector recursion reproduces the reference bit for bit,
    BB steps (i <= 5), LBFGS_helper (i >= 6), the queues' cap (corrections 3)
    and both exits (max_iter, the revert's |f_old - f| = 0)."""
    d = golden('lbfgs.npz')
    A = sps.csr_matrix((d['%s_A_data' % tag], d['%s_A_indices' % tag], d['%s_A_indptr' % tag]),
                       shape=tuple(d['%s_A_shape' % tag]))
    obj, proj, ls = orc.sparse_parts(A, d['%s_b' % tag], d['%s_starts' % tag])
    for k, corr in LBFGS_RUNS:
        key = _lbfgs_key(tag, k, corr)
        sol = orc.batch_solve_lbfgs(obj, proj, ls, d['%s_x_init' % tag].copy(), max_iter=k,
                                    corrections=corr)
        assert exact(sol['x'], d[key + '_x']), key
        assert sol['iterations'] == int(d[key + '_it'])
        assert sol['stop'] == str(d[key + '_stop'])
        assert exact(sol['progress'], d[key + '_prog'])


def test_golden_lbfgs_solve(orc, golden):
    """LBFGS.solve (python/LBFGS.py:56-123) from GradientDescent('LBFGS')'s
    start z0 + 1 over main.solve_in_z's closures, 60 iterations, every iterate
    (tests/golden/lbfgs.npz gd_*): the restatement reproduces the reference
    bit for bit (history of m = 50 zero pairs, weak Wolfe bisection)."""
    d = golden('lbfgs.npz')
    A = sps.csr_matrix((d['gd_A_data'], d['gd_A_indices'], d['gd_A_indptr']),
                       shape=tuple(d['gd_A_shape']))
    rec = orc.lbfgs_trace(A, d['gd_b'], d['gd_block_sizes'], int(d['gd_iters'][-1]))
    assert sorted(rec) == list(d['gd_iters'])
    for k, it in enumerate(d['gd_iters']):
        assert exact(rec[int(it)], d['gd_states'][k]), it


@pytest.mark.parametrize('tag', ['s', 'c'])
def test_golden_batch_solve_md(orc, golden, tag):
    """BATCH.solve_MD (python/BATCH.py:217-250), decreasing_step_size(i, 1, 1e8)."""
    d, A, b, starts, x0 = _batch_problem(golden, tag)
    obj, _, _ = orc.sparse_parts(A, b, starts)
    step = lambda i: 1.0 / (1e8 * i + 1.0)
    for k in (2, 10, 50):
        sol = orc.batch_solve_md(obj, starts, step, x0.copy(), max_iter=k)
        assert exact(sol['x'], d['%s_md%d_x' % (tag, k)]), (tag, k)
        assert exact(sol['progress'], d['%s_md%d_prog' % (tag, k)])


@pytest.mark.parametrize('threads', [1, 4])
def test_cpu_bb_port_follows_restatement(orc, threads):
    """bench.py's all-cores CPU baseline (oracle/bsls_cpu_bb.c, OpenMP) does the
    same iterations as the 1-thread restatement of BB.py (to rounding: its
    SpMV rows and dot products sum in another order)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)),
                                    'block-simplex-least-squares_amd'))
    from synthetic import make_shard, add_noise
    sh = make_shard(20_000, 1_000, 2_000, per_col=16, seed=5)
    b = add_noise(sh['Ax'], 0.02, seed=5)
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], 12, record_every=1)
    z, fx = orc.cpu_bb_run(sh['A'], b, sh['block_sizes'], 12, threads=threads)
    assert np.max(np.abs(z - ref[12])) <= 1e-9 * max(1.0, np.max(np.abs(ref[12])))
    assert np.isfinite(fx)
