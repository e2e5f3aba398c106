#!/usr/bin/env python
"""Capture golden vectors from the REAL reference (megacell/block-simplex-least-squares).

Runs only in the build container, where /root/reference exists; the fixtures it
writes (tests/golden/*.npz) are data — inputs and expected outputs — and are
what travels.  Nothing here is imported by the product or by the GPU tests.

The reference is Python 2 + Cython + header-only C++.  To run it under this
image's Python 3.10 / NumPy 2 we make a scratch copy in /tmp and apply only
mechanical compatibility edits:
  1. lib2to3 fixers print/xrange/dict/zip/map/filter on the copy;
  2. np.int_t -> np.int64_t in the copy of c_extensions.pyx (Cython 3 dropped
     np.int_t), then `setup.py build_ext --inplace` (reference headers untouched);
  3. stub modules ipdb (set_trace) and config (ACCEPTED_LOG_LEVELS);
  4. np.float / np.int aliases; bsls_utils.generate_data block sizes cast to
     int (same RNG stream, NumPy 2 refuses float sizes).

Usage:  python tests/golden/make_golden.py   (takes ~1 minute)
"""
import os
import shutil
import subprocess
import sys

import numpy as np

REF = '/root/reference'
WORK = '/tmp/bsls_ref_golden'
OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 237423433  # the reference tests' seed (tests/fast/test_proj_simplex.py:19)


def prepare():
    if os.path.exists(WORK):
        shutil.rmtree(WORK)
    os.makedirs(WORK)
    shutil.copytree(os.path.join(REF, 'python'), os.path.join(WORK, 'python'))
    py = os.path.join(WORK, 'python')
    subprocess.check_call([sys.executable, '-m', 'lib2to3', '-w', '-n', '-f', 'print',
                           '-f', 'xrange', '-f', 'dict', '-f', 'zip', '-f', 'map',
                           '-f', 'filter', py], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)
    pyx = os.path.join(py, 'c_extensions', 'c_extensions.pyx')
    src = open(pyx).read().replace('np.int_t', 'np.int64_t')
    open(pyx, 'w').write(src)
    subprocess.check_call([sys.executable, 'setup.py', 'build_ext', '--inplace'],
                          cwd=os.path.join(py, 'c_extensions'),
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    open(os.path.join(py, 'ipdb.py'), 'w').write('def set_trace(*a, **k):\n    pass\n')
    open(os.path.join(py, 'config.py'), 'w').write(
        "ACCEPTED_LOG_LEVELS = ['CRITICAL','ERROR','WARNING','INFO','DEBUG','WARN']\n")
    bu = os.path.join(py, 'bsls_utils.py')
    s = open(bu).read()
    old = 'block_sizes = np.random.multinomial(n-m2,np.ones(m2)/m2) + np.ones(m2)\n'
    assert old in s
    s = s.replace(old, 'block_sizes = (np.random.multinomial(n-m2,np.ones(m2)/m2) '
                       '+ np.ones(m2)).astype(int)\n')
    open(bu, 'w').write(s)
    np.float = float
    np.int = int
    sys.path.insert(0, py)
    import c_extensions.c_extensions  # noqa: F401  (the .so name must win)


def rand_blocks(rs, n, nb, first=0, maxk=None):
    """Strictly increasing block starts in [first, n), nb of them."""
    if nb == 1:
        return np.array([first], dtype=np.int64)
    cut = np.sort(rs.choice(np.arange(first + 1, n), nb - 1, replace=False))
    starts = np.concatenate(([first], cut)).astype(np.int64)
    return starts


def y_family(rs, kind, n):
    if kind == 'unif':
        return rs.rand(n)
    if kind == 'gauss5':
        return 5.0 * rs.randn(n)
    if kind == 'ties':
        return np.round(rs.rand(n) * 4) / 4.0
    if kind == 'equal':
        return np.full(n, 0.3)
    if kind == 'tiny':
        return 1e-3 * rs.rand(n)
    if kind == 'big':
        return 1e3 * rs.randn(n)
    if kind == 'logtrend':   # tests/fast/test_isotonic_regression.py:30
        return rs.randint(-50, 50, size=(n,)) + 50. * np.log(1 + np.arange(n))
    if kind == 'decreasing':
        return np.sort(rs.randn(n))[::-1].copy()
    raise ValueError(kind)


def gen_projection_cases():
    from c_extensions.c_extensions import (proj_multi_simplex_c, proj_multi_ball_c,
                                           proj_simplex_c)
    rs = np.random.RandomState(SEED)
    out = {}
    cases = []
    # (n, nb, first, kind)
    for kind in ['unif', 'gauss5', 'ties', 'equal', 'tiny', 'big']:
        cases.append((3000, 100, 0, kind))     # mean 30
        cases.append((3000, 12, 0, kind))      # mean 250 (LDS path)
        cases.append((700, 650, 5, kind))      # many size-1/2 blocks, prefix kept
    cases.append((5000, 1, 0, 'unif'))         # one block of 5000
    cases.append((70000, 2, 0, 'gauss5'))      # blocks of ~35k (large path)
    for ci, (n, nb, first, kind) in enumerate(cases):
        y = y_family(rs, kind, n)
        b = rand_blocks(rs, n, nb, first)
        ys = y.copy(); proj_multi_simplex_c(ys, b)
        yb = y.copy(); proj_multi_ball_c(yb, b)
        out['c%d_y' % ci] = y
        out['c%d_blocks' % ci] = b
        out['c%d_simplex' % ci] = ys
        out['c%d_ball' % ci] = yb
    out['ncases'] = np.array(len(cases))
    # single-block API: start/end variants
    y = rs.rand(50)
    ys = y.copy(); proj_simplex_c(ys, 10, 40)
    out['single_y'], out['single_out'] = y, ys
    np.savez_compressed(os.path.join(OUT, 'proj_simplex.npz'), **out)


def gen_isotonic_cases():
    from c_extensions.c_extensions import (isotonic_regression_multi_c,
                                           isotonic_regression_multi_c_2,
                                           isotonic_regression_multi_c_3,
                                           isotonic_regression_c)
    rs = np.random.RandomState(SEED + 1)
    out = {}
    cases = []
    for kind in ['logtrend', 'gauss5', 'ties', 'decreasing', 'unif', 'equal']:
        cases.append((2000, 100, 0, kind))
        cases.append((2000, 8, 0, kind))
        cases.append((600, 550, 3, kind))
    cases.append((4000, 1, 0, 'decreasing'))   # worst case for PAVA+ passes
    cases.append((40000, 3, 0, 'gauss5'))
    for ci, (n, nb, first, kind) in enumerate(cases):
        y = y_family(rs, kind, n)
        b = rand_blocks(rs, n, nb, first)
        out['c%d_y' % ci] = y
        out['c%d_blocks' % ci] = b
        for tag, fn in [('v1', isotonic_regression_multi_c), ('v3', isotonic_regression_multi_c_3)]:
            for upd in (1, 0):
                yy = y.copy()
                w = np.ones(n, dtype=np.int32)        # int32: kernel writes land here
                fn(yy, b, w, upd)
                out['c%d_%s_u%d' % (ci, tag, upd)] = yy
                out['c%d_%s_u%d_w' % (ci, tag, upd)] = w
        yy = y.copy(); isotonic_regression_multi_c_2(yy, b)
        out['c%d_v2' % ci] = yy
    out['ncases'] = np.array(len(cases))
    # reference self-test KAT (isotonic_regression.h:169-194)
    y = np.array([4., 5., 1., 6., 8., 7.])
    isotonic_regression_c(y, 0, 6)
    out['kat_single'] = y
    np.savez_compressed(os.path.join(OUT, 'isotonic.npz'), **out)


def gen_xz_quad():
    from c_extensions.c_extensions import (x2z_c, z2x_c, quad_obj_c)
    rs = np.random.RandomState(SEED + 2)
    out = {}
    for ci, (n, nb) in enumerate([(500, 40), (300, 300), (1000, 1), (64, 10)]):
        b = rand_blocks(rs, n, nb, 0)
        x = rs.rand(n)
        sizes = np.diff(np.append(b, n))
        nz = int(np.sum(sizes - 1))
        z = np.zeros(nz)
        x2z_c(x, z, b)
        x2 = np.zeros(n)
        z2x_c(x2, z, b)
        out['c%d_x' % ci], out['c%d_blocks' % ci] = x, b
        out['c%d_z' % ci], out['c%d_xback' % ci] = z, x2
    out['nxz'] = np.array(4)
    for qi, n in enumerate([2, 5, 9, 33]):
        x = 2 * rs.rand(n) - 1
        Q = 2 * rs.rand(n, n) - 1
        c = 2 * rs.rand(n) - 1
        g = np.zeros(n)
        f = quad_obj_c(x, Q.flatten(), c, g)
        out['q%d_x' % qi], out['q%d_Q' % qi], out['q%d_c' % qi] = x, Q, c
        out['q%d_g' % qi], out['q%d_f' % qi] = g, np.array(f)
    out['nquad'] = np.array(4)
    np.savez_compressed(os.path.join(OUT, 'xz_quad.npz'), **out)


def sparse_problem(seed, n, p, m, per_col=16, noise=0.0):
    """Small instance of the synthetic recipe of SURVEY.md §8(d) (scaled
    incidence A, multinomial block sizes, Dirichlet splits)."""
    import scipy.sparse as sps
    rs = np.random.RandomState(seed)
    sizes = rs.multinomial(n - p, np.ones(p) / p) + 1
    f = np.maximum(np.floor(rs.rand(p) * 1000), 1.0)
    xs = np.concatenate([rs.dirichlet(np.ones(k)) for k in sizes])
    colscale = np.repeat(f, sizes)
    rows = np.concatenate([rs.choice(m, per_col, replace=False) for _ in range(n)])
    cols = np.repeat(np.arange(n), per_col)
    vals = colscale[cols]
    A = sps.csr_matrix((vals, (rows, cols)), shape=(m, n))
    A.sort_indices()
    b = A.dot(xs)
    if noise:
        b = b + rs.normal(scale=np.abs(b) * noise)
    return A, b, xs, sizes


def gen_solver_traces():
    import scipy.sparse as sps
    import BB
    import solvers
    import bsls_utils
    from bsls_utils import x2z, particular_x0, block_sizes_to_N, generate_data
    from c_extensions.c_extensions import isotonic_regression_multi_c
    import mirror_descent
    import main as refmain
    import argparse
    import random
    import numpy.linalg as la

    out = {}

    # --- generate_data pinning (bsls_utils.py:590-655), test seed
    np.random.seed(SEED)
    d = generate_data()
    for k in ('A', 'b', 'x_true', 'f', 'block_sizes'):
        out['gen_%s' % k] = np.asarray(d[k])
    np.random.seed(SEED)
    d = generate_data(n=300, m1=40, m2=12, A_sparse=0.3, alpha=0.5)
    for k in ('A', 'b', 'x_true', 'f', 'block_sizes'):
        out['gen2_%s' % k] = np.asarray(d[k])

    # --- end-to-end main.main on the tests/fast/test_main.py problems
    cwd = os.getcwd()
    os.chdir(WORK)
    for vi, kw in enumerate([{}, {'alpha': 0.5}, {'A_sparse': 0.05}]):
        random.seed(SEED); np.random.seed(SEED)
        generate_data(fname='test_main.mat', **kw)
        args = argparse.Namespace(noise=0, file='test_main.mat', log='WARN', init=False,
                                  eq='CP', method='BB')
        iters, times, states, output = refmain.main(args=args)
        out['main%d_iters' % vi] = np.array(iters)
        out['main%d_states' % vi] = np.array(states)
        out['main%d_err' % vi] = np.asarray(output['0.5norm(Ax-b)^2'])
        out['main%d_err0' % vi] = np.array(output['0.5norm(Ax_init-b)^2'])
        out['main%d_errstar' % vi] = np.array(output['0.5norm(Ax*-b)^2'])
        out['main%d_maxf' % vi] = np.asarray(output['max|f * (x-x_true)|'])
        out['main%d_pct' % vi] = np.asarray(output['percent flow allocated incorrectly'])
        # the CSR problem main.solve_in_z saw (after BSLSMatrices prep)
        from bsls_matrices import BSLSMatrices
        config = {'full': True, 'L': True, 'OD': True, 'CP': True, 'LP': True,
                  'eq': 'CP', 'init': False}
        bm = BSLSMatrices(fname='test_main.mat', **config)
        bm.degree_reduced_form()
        AA, bb, N, bsz, x_split, nz, scaling, rsort, x0 = bm.get_LS()
        AA = sps.csr_matrix(AA)
        out['main%d_A_data' % vi], out['main%d_A_indices' % vi] = AA.data, AA.indices
        out['main%d_A_indptr' % vi], out['main%d_A_shape' % vi] = AA.indptr, np.array(AA.shape)
        out['main%d_b' % vi], out['main%d_block_sizes' % vi] = bb, bsz
        out['main%d_x_split' % vi], out['main%d_scaling' % vi] = x_split, scaling
    os.chdir(cwd)

    # --- per-iteration BB trajectory (record_every=1) on sparse problems
    def bb_trace(A, b, sizes, iters, tag):
        x0 = particular_x0(sizes)
        N = block_sizes_to_N(sizes)
        z0 = x2z(x0, sizes)
        target = A.dot(x0) - b
        AT = A.T.tocsr(); NT = N.T.tocsr()
        f = lambda z: 0.5 * la.norm(A.dot(N.dot(z)) + target) ** 2
        nabla_f = lambda z: NT.dot(AT.dot(A.dot(N.dot(z)) + target))
        cum = np.concatenate(([0], np.cumsum(sizes - 1)))

        def proj(x):
            isotonic_regression_multi_c(x, cum[:-1])
            return np.maximum(np.minimum(x, 1.), 0.)
        rec = {}

        def log(i, state, dt):
            rec[i] = np.array(state)
            return 0.0
        opts = {'max_iter': iters, 'verbose': 0, 'opt_tol': 1e-30}
        BB.solve(z0, f, nabla_f, solvers.stopping, record_every=1, proj=proj, log=log,
                 options=opts)
        keep = sorted(rec)
        out['%s_iters' % tag] = np.array(keep)
        out['%s_states' % tag] = np.array([rec[i] for i in keep])
        out['%s_A_data' % tag], out['%s_A_indices' % tag] = A.data, A.indices
        out['%s_A_indptr' % tag], out['%s_A_shape' % tag] = A.indptr, np.array(A.shape)
        out['%s_b' % tag], out['%s_block_sizes' % tag] = b, np.asarray(sizes)

    A, b, xs, sizes = sparse_problem(SEED, 3000, 150, 300, per_col=16, noise=0.02)
    bb_trace(A, b, sizes, 60, 'bbs')
    A, b, xs, sizes = sparse_problem(SEED + 5, 1200, 40, 150, per_col=8, noise=0.0)
    bb_trace(A, b, sizes, 60, 'bbc')

    # --- DORE through GradientDescent (gradient_descent.py:55-67)
    from gradient_descent import GradientDescent
    A, b, xs, sizes = sparse_problem(SEED + 7, 800, 40, 100, per_col=8, noise=0.01)
    x0 = particular_x0(sizes); N = block_sizes_to_N(sizes)
    z0 = x2z(x0, sizes); target = A.dot(x0) - b
    cum = np.concatenate(([0], np.cumsum(sizes - 1)))

    def proj(x):
        isotonic_regression_multi_c(x, cum[:-1])
        return np.maximum(np.minimum(x, 1.), 0.)
    opts = {'max_iter': 300, 'verbose': 0, 'opt_tol': 1e-30}
    gd = GradientDescent(z0=z0, f=None, nabla_f=None, proj=proj, method='DORE',
                         options=opts, A=A, N=N, target=target)
    iters, times, states = gd.run()
    out['dore_iters'], out['dore_states'] = np.array(iters), np.array(states)
    out['dore_lsv'] = np.array(bsls_utils.lsv_operator(A, N))
    out['dore_A_data'], out['dore_A_indices'] = A.data, A.indices
    out['dore_A_indptr'], out['dore_A_shape'] = A.indptr, np.array(A.shape)
    out['dore_b'], out['dore_block_sizes'] = b, sizes

    # --- mirror descent (mirror_descent.py:7-53); equal block sizes because the
    #     reference builds a ragged array at :10-11 that NumPy >= 1.24 refuses
    eq = np.full(50, 20)
    A2, _, _, _ = sparse_problem(SEED + 9, 1000, 50, 120, per_col=8, noise=0.0)
    A2.data[:] = 1.0
    rs = np.random.RandomState(SEED + 9)
    xs2 = np.concatenate([rs.dirichlet(np.ones(k)) for k in eq])
    b2 = A2.dot(xs2)
    for it in (1, 5, 40):
        xm = mirror_descent.least_squares(A2, b2, list(eq), iters=it, tolerance=0.0)
        out['md_x_%d' % it] = xm
    out['md_A_data'], out['md_A_indices'] = A2.data, A2.indices
    out['md_A_indptr'], out['md_A_shape'] = A2.indptr, np.array(A2.shape)
    out['md_b'], out['md_blocks'] = b2, eq

    np.savez_compressed(os.path.join(OUT, 'solvers.npz'), **out)


def gen_batch_traces():
    """x-space batch solvers (python/BATCH.py) over get_solver_parts
    (python/algorithm_utils.py:182-271): sparse least squares with the block
    simplex / l1-ball projection, and the dense 2-D QP of test_BATCH.py."""
    from algorithm_utils import get_solver_parts
    import BATCH as batch
    from bsls_utils import generate_small_qp
    out = {}
    cases = [('s', SEED + 11, 3000, 150, 300, 16, 0.02, False),
             ('c', SEED + 12, 1500, 60, 200, 8, 0.0, False),
             ('l', SEED + 13, 2000, 100, 250, 8, 0.05, True)]
    for tag, seed, n, p, m, pc, noise, lasso in cases:
        A, b, xs, sizes = sparse_problem(seed, n, p, m, per_col=pc, noise=noise)
        starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
        x_init = np.repeat(1.0 / sizes, sizes)
        if lasso:
            x_init = 0.5 * x_init
        step_size, proj, line_search, obj = get_solver_parts((A, b), starts, 1.0,
                                                            is_sparse=True, lasso=lasso)
        for k in (2, 3, 6, 15, 40, 2000):
            sol = batch.solve_BB(obj, proj, line_search, x_init.copy(), max_iter=k)
            out['%s_bb%d_x' % (tag, k)] = sol['x']
            out['%s_bb%d_f' % (tag, k)] = np.array(sol['f'])
            out['%s_bb%d_it' % (tag, k)] = np.array(sol['iterations'])
            out['%s_bb%d_stop' % (tag, k)] = np.array(sol['stop'])
            out['%s_bb%d_prog' % (tag, k)] = np.array([q[1] for q in sol['progress']])
        if not lasso:
            # mirror descent over the same parts (BATCH.py:217-250); min_eig
            # sized so that t g stays O(1) (A's entries are the flows, ~500)
            md_step = get_solver_parts((A, b), starts, 1e8, is_sparse=True)[0]
            for k in (2, 10, 50):
                sol = batch.solve_MD(obj, starts, md_step, x_init.copy(), max_iter=k)
                out['%s_md%d_x' % (tag, k)] = sol['x']
                out['%s_md%d_prog' % (tag, k)] = np.array([q[1] for q in sol['progress']])
        out['%s_A_data' % tag], out['%s_A_indices' % tag] = A.data, A.indices
        out['%s_A_indptr' % tag], out['%s_A_shape' % tag] = A.indptr, np.array(A.shape)
        out['%s_b' % tag], out['%s_starts' % tag] = b, starts
        out['%s_x_init' % tag] = x_init
    # dense 2-D QP of tests/fast/test_BATCH.py:24-40 (seeded like its setUp)
    np.random.seed(SEED)
    Q, c, x_true, f_min, min_eig = generate_small_qp()
    step_size, proj, line_search, obj = get_solver_parts((Q, c), np.array([0]), min_eig)
    for name, fn in (('gd', lambda: batch.solve(obj, proj, step_size, np.array([.5, .5]))),
                     ('gdls', lambda: batch.solve(obj, proj, step_size, np.array([.5, .5]),
                                                  line_search)),
                     ('bb', lambda: batch.solve_BB(obj, proj, line_search, np.array([.5, .5]))),
                     ('lbfgs', lambda: batch.solve_LBFGS(obj, proj, line_search,
                                                        np.array([.5, .5])))):
        sol = fn()
        out['qp_%s_x' % name] = sol['x']
        out['qp_%s_it' % name] = np.array(sol['iterations'])
        out['qp_%s_stop' % name] = np.array(sol['stop'])
    out['qp_Q'], out['qp_c'], out['qp_x_true'] = Q, c, x_true
    out['qp_f_min'], out['qp_min_eig'] = np.array(f_min), np.array(min_eig)
    np.savez_compressed(os.path.join(OUT, 'batch.npz'), **out)


def gen_lbfgs_traces():
    """BATCH.solve_LBFGS (python/BATCH.py:110-214) on the sparse x-space
    problems of gen_batch_traces ('s': 3000 routes / 150 blocks, 2 % noise;
    'c': 1500 / 60, exact data) with the block simplex projection, stopped at
    several max_iter (iterations 2-5 take the BB step, LBFGS_helper from 6)
    and run to its own stop; also corrections = 3 (the queues cap)."""
    import contextlib
    import io
    from algorithm_utils import get_solver_parts
    import BATCH as batch
    out = {}
    cases = [('s', SEED + 11, 3000, 150, 300, 16, 0.02),
             ('c', SEED + 12, 1500, 60, 200, 8, 0.0)]
    for tag, seed, n, p, m, pc, noise in cases:
        A, b, xs, sizes = sparse_problem(seed, n, p, m, per_col=pc, noise=noise)
        starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
        x_init = np.repeat(1.0 / sizes, sizes)
        step_size, proj, line_search, obj = get_solver_parts((A, b), starts, 1.0,
                                                            is_sparse=True)
        runs = [(k, 50) for k in (2, 3, 6, 7, 10, 15, 40, 2000)] + [(30, 3)]
        for k, corr in runs:
            with contextlib.redirect_stdout(io.StringIO()):
                sol = batch.solve_LBFGS(obj, proj, line_search, x_init.copy(), max_iter=k,
                                        corrections=corr)
            key = '%s_lb%d' % (tag, k) + ('' if corr == 50 else '_c%d' % corr)
            out[key + '_x'] = sol['x']
            out[key + '_f'] = np.array(sol['f'])
            out[key + '_it'] = np.array(sol['iterations'])
            out[key + '_stop'] = np.array(sol['stop'])
            out[key + '_prog'] = np.array([q[1] for q in sol['progress']])
        out['%s_A_data' % tag], out['%s_A_indices' % tag] = A.data, A.indices
        out['%s_A_indptr' % tag], out['%s_A_shape' % tag] = A.indptr, np.array(A.shape)
        out['%s_b' % tag], out['%s_starts' % tag] = b, starts
        out['%s_x_init' % tag] = x_init
    # LBFGS.solve (python/LBFGS.py:56-123) through GradientDescent('LBFGS')'s
    # start (z0 + 1, gradient_descent.py:49) on a well-conditioned z-space
    # problem (2000 links for 1000 routes: a 1e-15 gradient perturbation stays
    # below 1e-12 over 60 iterations, where the plugins.npz problem amplifies
    # it to 4e-8 by iteration 6), every iterate (record_every = 1)
    import numpy.linalg as la
    import LBFGS
    import solvers
    from bsls_utils import x2z, particular_x0, block_sizes_to_N
    from c_extensions.c_extensions import isotonic_regression_multi_c
    A, b, xs, sizes = sparse_problem(SEED + 33, 1000, 50, 2000, per_col=16, noise=0.01)
    x0 = particular_x0(sizes)
    N = block_sizes_to_N(sizes)
    z0 = x2z(x0, sizes)
    target = A.dot(x0) - b
    AT = A.T.tocsr(); NT = N.T.tocsr()
    f = lambda z: 0.5 * la.norm(A.dot(N.dot(z)) + target) ** 2
    nabla_f = lambda z: NT.dot(AT.dot(A.dot(N.dot(z)) + target))
    cum = np.concatenate(([0], np.cumsum(sizes - 1)))

    def proj(x):
        isotonic_regression_multi_c(x, cum[:-1])
        return np.maximum(np.minimum(x, 1.), 0.)
    rec = {}

    def log(i, state, dt):
        rec[i] = np.array(state)
        return 0.0
    with contextlib.redirect_stdout(io.StringIO()):
        LBFGS.solve(z0 + 1, f, nabla_f, solvers.stopping, record_every=1, proj=proj, log=log,
                    options={'max_iter': 60, 'verbose': 0, 'opt_tol': 1e-30})
    keep = sorted(rec)
    out['gd_iters'] = np.array(keep)
    out['gd_states'] = np.array([rec[i] for i in keep])
    out['gd_A_data'], out['gd_A_indices'] = A.data, A.indices
    out['gd_A_indptr'], out['gd_A_shape'] = A.indptr, np.array(A.shape)
    out['gd_b'], out['gd_block_sizes'] = b, np.asarray(sizes)
    np.savez_compressed(os.path.join(OUT, 'lbfgs.npz'), **out)


def gen_plugin_traces():
    """GradientDescent dispatch (python/gradient_descent.py:47-69) over the
    z-space closures of main.solve_in_z (python/main.py:47-65): every exit of
    solvers.stopping reachable from BB.solve (python/solvers.py:40-63, BB.py:22)
    with its iteration and message, and the LBFGS method (python/LBFGS.py)."""
    import contextlib
    import io
    import logging
    import numpy.linalg as la
    import BB
    import LBFGS
    from bsls_utils import x2z, particular_x0, block_sizes_to_N
    from c_extensions.c_extensions import isotonic_regression_multi_c
    from gradient_descent import GradientDescent

    def closures(A, b, sizes):
        x0 = particular_x0(sizes)
        N = block_sizes_to_N(sizes)
        z0 = x2z(x0, sizes)
        target = A.dot(x0) - b
        AT = A.T.tocsr(); NT = N.T.tocsr()
        f = lambda z: 0.5 * la.norm(A.dot(N.dot(z)) + target) ** 2
        nabla_f = lambda z: NT.dot(AT.dot(A.dot(N.dot(z)) + target))
        cum = np.concatenate(([0], np.cumsum(sizes - 1)))

        def proj(x):
            isotonic_regression_multi_c(x, cum[:-1])
            return np.maximum(np.minimum(x, 1.), 0.)
        return z0, f, nabla_f, proj

    class Grab(logging.Handler):
        def __init__(self):
            logging.Handler.__init__(self, logging.WARNING)
            self.msgs = []

        def emit(self, rec):
            self.msgs.append(rec.getMessage())

    def run(tag, A, b, sizes, method, options):
        z0, f, nabla_f, proj = closures(A, b, sizes)
        grab = Grab()
        logging.getLogger().addHandler(grab)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            gd = GradientDescent(z0=z0, f=f, nabla_f=nabla_f, proj=proj, method=method,
                                 options=options)
            iters, times, states = gd.run()
        logging.getLogger().removeHandler(grab)
        msgs = grab.msgs + [ln for ln in buf.getvalue().splitlines() if 'Exiting' in ln]
        out['%s_iters' % tag] = np.array(iters)
        out['%s_states' % tag] = np.array(states)
        out['%s_exit' % tag] = np.array(msgs[-1] if msgs else 'max_iter')
        out['%s_A_data' % tag], out['%s_A_indices' % tag] = A.data, A.indices
        out['%s_A_indptr' % tag], out['%s_A_shape' % tag] = A.indptr, np.array(A.shape)
        out['%s_b' % tag], out['%s_block_sizes' % tag] = b, np.asarray(sizes)

    out = {}
    A, b, xs, sizes = sparse_problem(SEED + 5, 1200, 40, 150, per_col=8, noise=0.0)
    # ||g||^2 <= opt_tol (1 + |f|) with a realistic tolerance
    run('grad8', A, b, sizes, 'BB', {'max_iter': 20000, 'verbose': 0, 'opt_tol': 1e-8})
    # no opt_tol in options: stopping's TOLER = 1e-6 default
    run('noopt', A, b, sizes, 'BB', {'max_iter': 20000, 'verbose': 0})
    # max_iter
    run('maxit', A, b, sizes, 'BB', {'max_iter': 777, 'verbose': 0, 'opt_tol': 1e-30})
    # BB.py:22 builtin sum(delta_g) == 0: a target pushing every block to a vertex,
    # where the projection returns the same z and the gradient repeats exactly
    A2, _, _, sizes2 = sparse_problem(SEED + 21, 600, 40, 100, per_col=8, noise=0.0)
    bneg = -A2.dot(np.ones(A2.shape[1])) * 1000.0
    run('vertex', A2, bneg, sizes2, 'BB', {'max_iter': 2000, 'verbose': 0, 'opt_tol': 1e-30})
    # LBFGS through GradientDescent (starts at z0 + 1, gradient_descent.py:49)
    A3, b3, _, sizes3 = sparse_problem(SEED + 23, 600, 30, 80, per_col=8, noise=0.01)
    # (5 iterations: LBFGS on this problem amplifies a 1e-15 gradient perturbation
    #  to 4e-8 by iteration 6 and 1e-3 by 25 -- measured with the CPU restatement)
    run('lbfgs', A3, b3, sizes3, 'LBFGS', {'max_iter': 5, 'verbose': 0, 'opt_tol': 1e-30})
    # and its per-iteration trajectory (record_every=1)
    z0, f, nabla_f, proj = closures(A3, b3, sizes3)
    rec = {}

    def log(i, state, dt):
        rec[i] = np.array(state)
        return 0.0
    with contextlib.redirect_stdout(io.StringIO()):
        LBFGS.solve(z0 + 1, f, nabla_f, __import__('solvers').stopping, record_every=1,
                    proj=proj, log=log, options={'max_iter': 25, 'verbose': 0, 'opt_tol': 1e-30})
    keep = sorted(rec)
    out['lbfgs_trace_iters'] = np.array(keep)
    out['lbfgs_trace_states'] = np.array([rec[i] for i in keep])
    np.savez_compressed(os.path.join(OUT, 'plugins.npz'), **out)


def main():
    prepare()
    if len(sys.argv) > 1 and sys.argv[1] == 'batch':
        gen_batch_traces()
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'plugins':
        gen_plugin_traces()
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'lbfgs':
        gen_lbfgs_traces()
        return
    gen_projection_cases()
    gen_isotonic_cases()
    gen_xz_quad()
    gen_solver_traces()
    gen_batch_traces()
    gen_lbfgs_traces()
    gen_plugin_traces()
    for f in sorted(os.listdir(OUT)):
        if f.endswith('.npz'):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == '__main__':
    main()
