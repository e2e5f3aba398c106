"""x-space batch solvers on the device (python/BATCH.py over
python/algorithm_utils.get_solver_parts), against the golden runs of the
reference itself (tests/golden/batch.npz, tests/golden/make_golden.py).

Tolerances (north star): iterates to 1e-6 relative; objective histories to
1e-6 relative.  The device sums (dots, ||r||^2, SpMV rows) run in a different
order than NumPy/BLAS/SciPy, so results agree to ~1e-12, not bit for bit; a
run that the reference ended by the line search's "step too small" revert can
end an iteration earlier or later, so converged runs are compared by f and x,
not by iteration count.
"""
import numpy as np
import pytest
import scipy.sparse as sps

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _problem(golden, tag):
    d = golden('batch.npz')
    A = sps.csr_matrix((d['%s_A_data' % tag], d['%s_A_indices' % tag], d['%s_A_indptr' % tag]),
                       shape=tuple(d['%s_A_shape' % tag]))
    return d, A, d['%s_b' % tag], d['%s_starts' % tag], d['%s_x_init' % tag]


@pytest.mark.parametrize('fused,panels', [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize('tag,lasso', [('s', False), ('c', False), ('l', True)])
def test_solve_bb_vs_reference(cuda, golden, monkeypatch, tag, lasso, fused, panels):
    import BATCH
    from algorithm_utils import SparseLSQ, get_solver_parts
    # panels: both products on the panel images (csrc/lsq.hip), forced on
    # these small problems; otherwise the CSR kernels
    monkeypatch.setattr(SparseLSQ, 'PANEL_MIN_NNZ', 0 if panels else 1 << 62)
    d, A, b, starts, x0 = _problem(golden, tag)
    step, proj, ls, obj = get_solver_parts((A, b), starts, 1.0, is_sparse=True, lasso=lasso)
    assert (obj.lsq is not None) == panels
    for k in (2, 3, 6, 15, 40):
        sol = BATCH.solve_BB(obj, proj, ls, x0.copy(), max_iter=k, fused=fused)
        ref_it = int(d['%s_bb%d_it' % (tag, k)])
        if str(d['%s_bb%d_stop' % (tag, k)]) == 'max_iter':
            assert sol['iterations'] == ref_it and sol['stop'] == 'max_iter', (k, sol['stop'])
            assert rel(sol['x'], d['%s_bb%d_x' % (tag, k)]) < 1e-6, k
            prog = np.array([q[1] for q in sol['progress']])
            ref = d['%s_bb%d_prog' % (tag, k)]
            assert prog.shape == ref.shape
            assert np.max(np.abs(prog - ref) / np.maximum(np.abs(ref), 1e-3)) < 1e-6, k
        else:
            # the reference stalled (revert of a too-small step) at f's floor:
            # the device run ends within a few ulps of that f, by the same test
            # or at max_iter
            ref_f = float(d['%s_bb%d_f' % (tag, k)])
            assert sol['stop'].endswith('< prog_tol') or sol['stop'] == 'max_iter'
            assert abs(sol['f'] - ref_f) <= 1e-9 * max(abs(ref_f), 1.0), (k, sol['f'], ref_f)
            assert rel(sol['x'], d['%s_bb%d_x' % (tag, k)]) < 1e-5, k
    # converged run (reference default max_iter = 2000)
    sol = BATCH.solve_BB(obj, proj, ls, x0.copy(), fused=fused)
    ref_f = float(d['%s_bb2000_f' % tag])
    assert sol['stop'].endswith('< prog_tol'), sol['stop']
    assert abs(sol['f'] - ref_f) <= 1e-6 * max(abs(ref_f), 1.0)
    assert rel(sol['x'], d['%s_bb2000_x' % tag]) < 1e-5


@pytest.mark.parametrize('tag,lasso', [('s', False), ('l', True)])
def test_solve_bb_fast_projection(cuda, golden, monkeypatch, tag, lasso):
    """BSLS_PROJ=fast: the fused x-space rounds take the sort-free projection
    (bsls_xbb_problem.ball bit 1; the closures the _fast c_extensions entries):
    the reference's runs within the same 1e-6, fused and closure loops alike."""
    import BATCH
    from algorithm_utils import SparseLSQ, get_solver_parts
    monkeypatch.setenv('BSLS_PROJ', 'fast')
    monkeypatch.setattr(SparseLSQ, 'PANEL_MIN_NNZ', 1 << 62)
    d, A, b, starts, x0 = _problem(golden, tag)
    step, proj, ls, obj = get_solver_parts((A, b), starts, 1.0, is_sparse=True, lasso=lasso)
    for k in (2, 6, 15):
        if str(d['%s_bb%d_stop' % (tag, k)]) != 'max_iter':
            continue
        for fused in (True, False):
            sol = BATCH.solve_BB(obj, proj, ls, x0.copy(), max_iter=k, fused=fused)
            assert sol['iterations'] == int(d['%s_bb%d_it' % (tag, k)]), (k, fused)
            assert rel(sol['x'], d['%s_bb%d_x' % (tag, k)]) < 1e-6, (k, fused)


@pytest.mark.parametrize('tag', ['s', 'c'])
def test_solve_md_vs_reference(cuda, golden, tag):
    import BATCH
    from algorithm_utils import get_solver_parts
    d, A, b, starts, x0 = _problem(golden, tag)
    step = get_solver_parts((A, b), starts, 1e8, is_sparse=True)[0]
    _, _, _, obj = get_solver_parts((A, b), starts, 1e8, is_sparse=True)
    for k in (2, 10, 50):
        sol = BATCH.solve_MD(obj, starts, step, x0.copy(), max_iter=k)
        assert sol['iterations'] == k
        assert rel(sol['x'], d['%s_md%d_x' % (tag, k)]) < 1e-10, k
        prog = np.array([q[1] for q in sol['progress']])
        assert rel(prog / d['%s_md%d_prog' % (tag, k)], np.ones(k)) < 1e-10


def test_dense_qp_solvers_vs_reference(cuda, golden):
    """tests/fast/test_BATCH.py:24-40,99-112,176-189 on the device closures."""
    import BATCH
    from algorithm_utils import get_solver_parts
    d = golden('batch.npz')
    Q, c, x_true = d['qp_Q'], d['qp_c'], d['qp_x_true']
    step, proj, ls, obj = get_solver_parts((Q, c), np.array([0]), float(d['qp_min_eig']))
    runs = {'gd': lambda: BATCH.solve(obj, proj, step, np.array([.5, .5])),
            'gdls': lambda: BATCH.solve(obj, proj, step, np.array([.5, .5]), ls),
            'bb': lambda: BATCH.solve_BB(obj, proj, ls, np.array([.5, .5])),
            'lbfgs': lambda: BATCH.solve_LBFGS(obj, proj, ls, np.array([.5, .5]))}
    for name, fn in runs.items():
        sol = fn()
        assert np.max(np.abs(sol['x'] - x_true)) < 1e-3, name       # the reference's check
        assert rel(sol['x'], d['qp_%s_x' % name]) < 1e-6, name
        assert sol['stop'][-10:] == str(d['qp_%s_stop' % name])[-10:], name
        assert abs(sol['iterations'] - int(d['qp_%s_it' % name])) <= 3, name
    sol = BATCH.solve_BB(obj, proj, ls, np.array([.5, .5]), f_min=float(d['qp_f_min']))
    assert sol['stop'][-10:] == ' < opt_tol'


def test_normalization_and_md_step(cuda, orc):
    import torch
    from algorithm_utils import normalization
    rs = np.random.RandomState(4)
    n = 5000
    starts = np.concatenate(([0], np.sort(rs.choice(np.arange(1, n), 300, replace=False))))
    ends = np.append(starts[1:], n)
    x = rs.rand(n)
    xd = torch.from_numpy(x.copy()).cuda()
    normalization(xd, starts, ends)
    ref = x.copy()
    for s, e in zip(starts, ends):
        ref[s:e] = ref[s:e] / np.sum(ref[s:e])
    assert rel(xd.cpu().numpy(), ref) < 1e-14
    # non-contiguous blocks: block by block
    xd = torch.from_numpy(x.copy()).cuda()
    normalization(xd, starts[::2], ends[::2])
    ref = x.copy()
    for s, e in zip(starts[::2], ends[::2]):
        ref[s:e] = ref[s:e] / np.sum(ref[s:e])
    assert rel(xd.cpu().numpy(), ref) < 1e-14


def test_fused_engine_larger_problem_matches_closure_loop(cuda, orc):
    """100k routes: the fused device rounds and the closure-by-closure loop
    both follow the oracle's restatement of BATCH.solve_BB over SciPy
    (oracle.batch_solve_bb / sparse_parts, BATCH.py:55-106,
    algorithm_utils.py:88-94,113-137) within 1e-6 relative at 25 iterations,
    with the same iteration count and objective trace (1e-8), and the fused engine is
    deterministic."""
    import BATCH
    from algorithm_utils import get_solver_parts
    from synthetic import make_shard, add_noise
    sh = make_shard(100_000, 5_000, 10_000, 16, seed=3)
    b = add_noise(sh['Ax'], 0.02, seed=3)
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1]))
    x0 = np.repeat(1.0 / sizes, sizes)
    step, proj, ls, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
    a = BATCH.solve_BB(obj, proj, ls, x0.copy(), max_iter=25)
    a2 = BATCH.solve_BB(obj, proj, ls, x0.copy(), max_iter=25)
    c = BATCH.solve_BB(obj, proj, ls, x0.copy(), max_iter=25, fused=False)
    assert np.array_equal(a['x'], a2['x'])
    assert a['iterations'] == c['iterations'] == 25
    assert rel(a['x'], c['x']) < 1e-6
    o_obj, o_proj, o_ls = orc.sparse_parts(sh['A'], b, starts)
    r = orc.batch_solve_bb(o_obj, o_proj, o_ls, x0.copy(), max_iter=25)
    assert r['iterations'] == 25 and r['stop'] == 'max_iter'
    for sol in (a, c):
        assert rel(sol['x'], r['x']) < 1e-6
        prog = np.array([q[1] for q in sol['progress']])
        assert prog.shape == r['progress'].shape
        assert np.max(np.abs(prog - r["progress"]) / np.abs(r["progress"])) < 1e-8


@pytest.mark.parametrize('with_ls', [False, True])
def test_batch_solve_sparse_vs_oracle(cuda, orc, with_ls):
    """BATCH.solve (projected gradient descent, BATCH.py:7-52) on a sparse
    100k-route problem (get_solver_parts(is_sparse=True): the device
    objective and projection, the decreasing step of algorithm_utils.py:97-100,
    with and without the backtracking line search) against the oracle's
    restatement over SciPy (oracle.batch_solve / sparse_parts): the same
    iteration count and stop, iterates within 1e-6, objective trace within
    1e-8."""
    import BATCH
    from algorithm_utils import get_solver_parts
    from synthetic import make_shard, add_noise
    sh = make_shard(100_000, 5_000, 10_000, 16, seed=4)
    b = add_noise(sh['Ax'], 0.02, seed=4)
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1]))
    x0 = np.repeat(1.0 / sizes, sizes)
    # (min_eig 1e7: steps t = 1 / (1e7 i + 1), small enough for the plain
    # projected descent to make progress on this matrix)
    step, proj, ls, obj = get_solver_parts((sh['A'], b), starts, 1e7, is_sparse=True)
    sol = BATCH.solve(obj, proj, step, x0.copy(), ls if with_ls else None, max_iter=25)
    o_obj, o_proj, o_ls = orc.sparse_parts(sh['A'], b, starts)
    r = orc.batch_solve(o_obj, o_proj, step, x0.copy(), o_ls if with_ls else None, max_iter=25)
    assert sol['iterations'] == r['iterations'] and sol['stop'] == r['stop'], (sol['stop'], r['stop'])
    assert rel(sol['x'], r['x']) < 1e-6
    prog = np.array([q[1] for q in sol['progress']])
    assert prog.shape == r['progress'].shape
    assert np.max(np.abs(prog - r['progress']) / np.abs(r['progress'])) < 1e-8
    assert r['progress'][-1] < r['progress'][0]          # the run made progress


LBFGS_RUNS = [(k, 50) for k in (2, 3, 6, 7, 10, 15, 40, 2000)] + [(30, 3)]


def _lbfgs_problem(golden, tag):
    d = golden('lbfgs.npz')
    A = sps.csr_matrix((d['%s_A_data' % tag], d['%s_A_indices' % tag], d['%s_A_indptr' % tag]),
                       shape=tuple(d['%s_A_shape' % tag]))
    return d, A, d['%s_b' % tag], d['%s_starts' % tag], d['%s_x_init' % tag]


@pytest.mark.parametrize('fused,panels', [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize('tag', ['s', 'c'])
def test_solve_lbfgs_vs_reference(cuda, golden, monkeypatch, tag, fused, panels):
    """BATCH.solve_LBFGS (python/BATCH.py:110-214) on the sparse x-space
    problems, against the reference's own runs (tests/golden/lbfgs.npz):
    the fused device rounds (LBFGS_helper's recursion in d's coefficients,
    csrc/xbb.hip) and the closure loop, BB steps for i <= 5, L-BFGS from 6,
    the queues' cap (corrections 3) -- iterates within 1e-6, the objective
    trace within 1e-6, the same exit (max_iter at the same iteration, or the
    revert's |f_old - f| < prog_tol at the same f)."""
    import BATCH
    from algorithm_utils import SparseLSQ, get_solver_parts
    monkeypatch.setattr(SparseLSQ, 'PANEL_MIN_NNZ', 0 if panels else 1 << 62)
    d, A, b, starts, x0 = _lbfgs_problem(golden, tag)
    step, proj, ls, obj = get_solver_parts((A, b), starts, 1.0, is_sparse=True)
    for k, corr in LBFGS_RUNS:
        key = '%s_lb%d' % (tag, k) + ('' if corr == 50 else '_c%d' % corr)
        sol = BATCH.solve_LBFGS(obj, proj, ls, x0.copy(), max_iter=k, corrections=corr,
                                fused=fused)
        ref_it = int(d[key + '_it'])
        ref_f = float(d[key + '_f'])
        if str(d[key + '_stop']) == 'max_iter':
            assert sol['iterations'] == ref_it and sol['stop'] == 'max_iter', (key, sol['stop'])
            assert rel(sol['x'], d[key + '_x']) < 1e-6, key
            prog = np.array([q[1] for q in sol['progress']])
            ref = d[key + '_prog']
            assert prog.shape == ref.shape, key
            assert np.max(np.abs(prog - ref) / np.maximum(np.abs(ref), 1e-3)) < 1e-6, key
        else:
            assert sol['stop'].endswith('< prog_tol'), (key, sol['stop'])
            assert abs(sol['f'] - ref_f) <= 1e-9 * max(abs(ref_f), 1.0), (key, sol['f'], ref_f)
            assert rel(sol['x'], d[key + '_x']) < 1e-5, key


def test_lbfgs_c3_size_vs_oracle(cuda, orc):
    """The fused L-BFGS rounds on the C3 matrix (1M routes / 50k blocks /
    100k links / 16M nnz, 2 % noise) against the oracle's restatement of
    BATCH.solve_LBFGS over SciPy (oracle.batch_solve_lbfgs): iterates within
    1e-6 and the objective trace within 1e-8 at 12 iterations (BB steps to 5,
    L-BFGS from 6)."""
    import BATCH
    from algorithm_utils import get_solver_parts
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02, seed=SEED)
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1]))
    x0 = np.repeat(1.0 / sizes, sizes)
    step, proj, ls, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
    a = BATCH.solve_LBFGS(obj, proj, ls, x0.copy(), max_iter=12)
    o_obj, o_proj, o_ls = orc.sparse_parts(sh['A'], b, starts)
    r = orc.batch_solve_lbfgs(o_obj, o_proj, o_ls, x0.copy(), max_iter=12)
    assert a['iterations'] == r['iterations'] == 12 and r['stop'] == 'max_iter'
    assert rel(a['x'], r['x']) < 1e-6
    prog = np.array([q[1] for q in a['progress']])
    assert prog.shape == r['progress'].shape
    assert np.max(np.abs(prog - r['progress']) / np.abs(r['progress'])) < 1e-8
