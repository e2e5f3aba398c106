"""The solver plugin surface end to end on the device, against runs of the
reference itself (tests/golden/make_golden.py):

* main.main(args) on the three tests/fast/test_main.py problems -- .mat file
  -> BSLSMatrices -> solve_in_z -> GradientDescent('BB') -> LS_postprocess
  (python/main.py:146-176, 41-79, 81-136); acceptance as
  tests/fast/test_main.py:31-47 (0.5||Ax-b||^2 < 1e-16) plus the output dict;
* every exit of solvers.stopping reachable from BB.solve (python/solvers.py:
  40-63, BB.py:22): same exit iteration and same reason as the reference,
  including the opt_tol-absent default TOLER = 1e-6;
* GradientDescent('DORE') (python/DORE.py:6-90, gradient_descent.py:55-67)
  and its largest singular value (bsls_utils.py:334-369);
* GradientDescent('LBFGS') (python/LBFGS.py:56-123, gradient_descent.py:48-52).

Tolerances: iterates 1e-6 relative (north star); the singular value 1e-12.
The device sums in a different order than NumPy/SciPy, so iterates agree to
rounding, not bit for bit.
"""
import argparse
import os

import numpy as np
import pytest
import scipy.sparse as sps

pytestmark = pytest.mark.gpu

SEED = 237423433


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _csr(G, tag):
    return sps.csr_matrix((G['%s_A_data' % tag], G['%s_A_indices' % tag],
                           G['%s_A_indptr' % tag]), shape=tuple(G['%s_A_shape' % tag]))


def _gd_run(G, tag, method, options):
    import _native
    from bsls_utils import particular_x0, x2z
    from device import BBEngine
    from gradient_descent import GradientDescent
    A, b, sizes = _csr(G, tag), G['%s_b' % tag], G['%s_block_sizes' % tag]
    eng = BBEngine(A, b, sizes, options=options)
    z0 = x2z(particular_x0(sizes), sizes)
    gd = GradientDescent(z0=z0, method=method, options=dict(options), engine=eng)
    iters, times, states = gd.run()
    return eng, gd, iters, states


@pytest.mark.parametrize('det', [False, True])
@pytest.mark.parametrize('vi', [0, 1, 2])
def test_main_end_to_end(cuda, golden, tmp_path, vi, det):
    import bsls_utils
    import main
    G = golden('solvers.npz')
    kw = [{}, {'alpha': 0.5}, {'A_sparse': 0.05}][vi]
    np.random.seed(SEED)
    fname = os.path.join(str(tmp_path), 'test_main.mat')
    bsls_utils.generate_data(fname=fname, **kw)
    args = argparse.Namespace(noise=0, file=fname, log='WARN', init=False, eq='CP',
                              method='BB', deterministic=det)
    iters, times, states, output = main.main(args=args)
    if det:
        # the fixed-order engine (main.py --deterministic): a second run repeats
        # the first bit for bit, exit iteration included
        iters2, _, states2, _ = main.main(args=args)
        assert list(iters2) == list(iters)
        assert all(np.array_equal(a, b2) for a, b2 in zip(states, states2))
    err = np.asarray(output['0.5norm(Ax-b)^2'])
    # tests/fast/test_main.py:31-47
    assert err[-1] < 1e-16, err
    ref_iters = list(G['main%d_iters' % vi])
    # every periodic log point of the reference run is hit, with the same state
    assert list(iters[:-1]) == ref_iters[:-1]
    for k in range(len(ref_iters) - 1):
        assert rel(states[k], G['main%d_states' % vi][k]) < 1e-6, k
    # the LS_postprocess metrics that do not depend on where the run ends
    assert rel(output['0.5norm(Ax_init-b)^2'], G['main%d_err0' % vi]) < 1e-12
    assert abs(output['0.5norm(Ax*-b)^2'] - G['main%d_errstar' % vi]) < 1e-20
    assert rel(err[:-1], G['main%d_err' % vi][:-1]) < 1e-6
    assert rel(output['max|f * (x-x_true)|'][:-1], G['main%d_maxf' % vi][:-1]) < 1e-6
    assert rel(output['percent flow allocated incorrectly'][:-1],
               G['main%d_pct' % vi][:-1]) < 1e-6
    # the run ends at an exact-zero sum(delta_g) (BB.py:22) or at ||g||^2 <= 1e-30:
    # both depend on the last bits of a converged trajectory (the device sums
    # in another order than NumPy), so the final iteration is pinned to a band
    # around the reference's and the final state to the solution (both runs
    # reach 0.5||Ax-b||^2 < 1e-16).  Measured on MI355X (tools/exit_iters.py,
    # round 3): reference 454 / 569 / 745; fixed-order engine 443 / 572 / 774
    # on every run (so pinned exactly, a regression check of its order); the
    # default engine 443-445 / 552-570 / 773-785
    DET_EXIT = [443, 572, 774]
    if det:
        assert iters[-1] == DET_EXIT[vi], (iters[-1], DET_EXIT[vi])
    assert abs(iters[-1] - ref_iters[-1]) <= max(10, ref_iters[-1] // 16), (iters, ref_iters)
    assert G['main%d_err' % vi][-1] < 1e-16


@pytest.mark.parametrize('tag,reason', [('grad8', 'STOP_GRAD'), ('noopt', 'STOP_GRAD'),
                                        ('maxit', 'STOP_MAXITER'),
                                        ('vertex', 'STOP_NOCHANGE')])
def test_stopping_exits_match_reference(cuda, golden, tag, reason):
    """Same exit, same iteration, same logged states as the reference's
    GradientDescent('BB') run (record_every = 500, BB.py:39-44)."""
    import _native
    G = golden('plugins.npz')
    opts = {'max_iter': 20000, 'verbose': 0}
    if tag == 'grad8':
        opts['opt_tol'] = 1e-8
    elif tag == 'maxit':
        opts.update(max_iter=777, opt_tol=1e-30)
    elif tag == 'vertex':
        opts.update(max_iter=2000, opt_tol=1e-30)
    # noopt: no 'opt_tol' key -> solvers.stopping's TOLER = 1e-6
    eng, gd, iters, states = _gd_run(G, tag, 'BB', opts)
    want = getattr(_native, reason)
    assert eng.stop_reason == want, (eng.stop_reason, want)
    assert _native.STOP_TEXT[eng.stop_reason] == str(G['%s_exit' % tag])
    assert list(iters) == list(G['%s_iters' % tag])
    for k, s in enumerate(states):
        assert rel(s, G['%s_states' % tag][k]) < 1e-6, (k, iters[k])


def test_dore_vs_reference(cuda, golden):
    G = golden('solvers.npz')
    opts = {'max_iter': 300, 'verbose': 0, 'opt_tol': 1e-30}
    eng, gd, iters, states = _gd_run(G, 'dore', 'DORE', opts)
    assert abs(gd.lsv - float(G['dore_lsv'])) <= 1e-12 * float(G['dore_lsv'])
    assert list(iters) == list(G['dore_iters'])
    for k, s in enumerate(states):
        assert rel(s, G['dore_states'][k]) < 1e-6, (k, iters[k])


@pytest.mark.parametrize('eps,record_every,max_iter', [(-1.0, 1, 40), (1e30, 1, 40),
                                                      (-1.0, 7, 40), ('mid', 7, 40),
                                                      (-1.0, 1, 0)])
def test_dore_device_loop_vs_closures(cuda, eps, record_every, max_iter):
    """DORE.solve_engine (every step and branch on the device, what
    GradientDescent('DORE') runs) against DORE.solve over the engine's
    closures (host branch decisions) on a 60k-route problem: every logged
    iterate within 1e-8 (the dot products round in different orders), the
    extrapolated path taken, and the norm-change break (eps = 1e30: stop at
    iteration 1 with the iterate of iteration 0) at the same iteration.
    record_every = 7 runs solve_engine's chunking (up to 25 iterations
    enqueued between reads of the stop flag, log points at multiples of 7);
    eps = 'mid' sets the threshold between two iterations' norm changes so the
    break falls inside a chunk; max_iter = 0 logs iteration 0 with x0 twice,
    as the reference does."""
    import torch
    import DORE
    from device import BBEngine
    from bsls_utils import lsv_operator
    from synthetic import make_shard, add_noise
    sh = make_shard(60000, 3000, 8000, per_col=16, seed=3)
    b = add_noise(sh['Ax'], 0.02, seed=3)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], AT=sh['AT'])
    scale = 0.99 / lsv_operator(eng, None)
    tgt = eng.target * scale
    z0 = torch.zeros(eng.nz, dtype=torch.float64, device='cuda')

    def run(fused, eps_, every):
        opts = {'max_iter': max_iter, 'opt_tol': eps_}
        rec = []

        def log(i, st, dt):
            rec.append((i, st.detach().cpu().numpy().copy()))
            return 0.0
        if fused:
            DORE.solve_engine(eng, z0, scale, tgt, record_every=every, log=log, options=opts)
        else:
            DORE.solve(z0, lambda z: eng.apply_A(z, alpha=scale),
                       lambda r: eng.apply_AT(r, alpha=scale), tgt, record_every=every,
                       proj=eng.proj, log=log, options=opts)
        return rec
    brk = None
    if eps == 'mid':
        # norm_change of iteration k = ||x_k - x_{k-1}||^2, x_k = the state logged
        # after iteration k - 1 (entry k of a record_every = 1 run, entry 0 = x0);
        # pick the last k >= 9 that is not the first iteration of a chunk
        # (chunks [1, 8), [8, 15), [15, 22), ... with record_every = 7) where it
        # drops below every earlier one, and put eps between the two
        st = [s for _, s in run(False, -1.0, 1)][:-1]      # (the final log repeats the last)
        nc = [float(np.sum((st[k] - st[k - 1]) ** 2)) for k in range(1, len(st))]
        for k in range(min(len(nc), max_iter - 1), 8, -1):
            lo = min(nc[:k - 1])
            if (k - 1) % 7 and nc[k - 1] < 0.99 * lo:
                brk, eps = k, float(np.sqrt(nc[k - 1] * lo))
                break
        assert brk is not None, nc
    ref, got = run(False, eps, record_every), run(True, eps, record_every)
    assert [i for i, _ in got] == [i for i, _ in ref]
    for (i, a), (_, bb) in zip(got, ref):
        assert rel(a, bb) < 1e-8, i
    if max_iter == 0:
        assert [i for i, _ in got] == [0, 0]
    elif brk is not None:
        assert got[-1][0] == brk
    elif eps < 0:
        assert eng.dore_scalars[3] != 0.0          # a2: the extrapolated path ran
        assert got[-1][0] == max_iter - 1
    else:
        assert got[-1][0] == 1


def test_lbfgs_vs_reference(cuda, golden):
    """GradientDescent('LBFGS') over the engine's device closures, 5 iterations
    (the fixture's run): LBFGS on this problem is ill-conditioned in the
    rounding -- the CPU restatement with a 1e-15 relative perturbation of the
    gradient drifts 4e-8 by iteration 6 and 1e-3 by 25 -- so the whole-run
    comparison stops where a 1e-6 contract is meaningful; every later
    reference iterate is checked through the closures below."""
    G = golden('plugins.npz')
    opts = {'max_iter': 5, 'verbose': 0, 'opt_tol': 1e-30}
    eng, gd, iters, states = _gd_run(G, 'lbfgs', 'LBFGS', opts)
    assert list(iters) == list(G['lbfgs_iters'])
    for k, s in enumerate(states):
        assert rel(s, G['lbfgs_states'][k]) < 1e-6, (k, iters[k])


def test_lbfgs_closures_on_reference_trajectory(cuda, golden, orc):
    """LBFGS.solve's inputs, iterate by iterate: the device closures f /
    nabla_f / proj (main.py:53-65) evaluated at every iterate of the
    reference's 25-iteration trajectory agree with the CPU restatement
    (f, nabla_f to 1e-12 relative, proj bit for bit); and LBFGS.solve on the
    device follows the trajectory through iteration 5."""
    import torch
    import LBFGS
    import solvers
    from device import BBEngine
    G = golden('plugins.npz')
    A, b, sizes = _csr(G, 'lbfgs'), G['lbfgs_b'], G['lbfgs_block_sizes']
    eng = BBEngine(A, b, sizes)
    P = orc.solve_in_z_parts(A, b, sizes)
    for z in G['lbfgs_trace_states']:
        zd = torch.from_numpy(z.copy()).cuda()
        fr = P['f'](z)
        assert abs(eng.f(zd) - fr) <= 1e-12 * max(1.0, abs(fr))
        assert rel(eng.nabla_f(zd).cpu().numpy(), P['nabla_f'](z)) < 1e-12
        w = z - 0.3 * P['nabla_f'](z) / max(1.0, np.abs(P['nabla_f'](z)).max())
        got = eng.proj(torch.from_numpy(w.copy()).cuda()).cpu().numpy()
        assert np.array_equal(got.view(np.int64), P['proj'](w.copy()).view(np.int64))
    rec = {}

    def log(i, s, dt):
        rec[i] = s.detach().cpu().numpy().copy() if hasattr(s, 'detach') else np.array(s)
        return 0.0
    z0 = torch.ones(eng.nz, dtype=torch.float64, device='cuda')   # z0 + 1, z0 = 0
    LBFGS.solve(z0, eng.f, eng.nabla_f, solvers.stopping, record_every=1, proj=eng.proj,
                log=log, options={'max_iter': 5, 'verbose': 0, 'opt_tol': 1e-30})
    assert sorted(rec) == list(range(6))
    for i in range(6):
        assert rel(rec[i], G['lbfgs_trace_states'][i]) < 1e-6, i


def test_lbfgs_60_iterations_vs_reference(cuda, golden):
    """GradientDescent('LBFGS') on the device (engine closures, the history
    ring of csrc/lbfgs.hip) over the 60-iteration fixture of a
    well-conditioned problem (tests/golden/lbfgs.npz gd_*, where a 1e-15
    perturbation stays below 1e-12): every iterate within 1e-6 of the
    reference's run."""
    import torch
    import LBFGS
    import solvers
    from device import BBEngine
    G = golden('lbfgs.npz')
    eng = BBEngine(_csr(G, 'gd'), G['gd_b'], G['gd_block_sizes'])
    rec = {}

    def log(i, s, dt):
        rec[i] = s.detach().cpu().numpy().copy()
        return 0.0
    z0 = torch.ones(eng.nz, dtype=torch.float64, device='cuda')
    LBFGS.solve(z0, eng.f, eng.nabla_f, solvers.stopping, record_every=1, proj=eng.proj,
                log=log, options={'max_iter': 60, 'verbose': 0, 'opt_tol': 1e-30})
    assert sorted(rec) == list(G['gd_iters'])
    for k, it in enumerate(G['gd_iters']):
        assert rel(rec[int(it)], G['gd_states'][k]) < 1e-6, it
    # and through the dispatcher (logs 0 and the end)
    opts = {'max_iter': 60, 'verbose': 0, 'opt_tol': 1e-30}
    eng2, gd, iters, states = _gd_run(G, 'gd', 'LBFGS', opts)
    assert list(iters) == [0, 60]
    assert rel(states[-1], G['gd_states'][-1]) < 1e-6


@pytest.mark.parametrize('problem,max_iter', [('synthetic', 2), ('synthetic', 4),
                                              ('gd', 60)])
def test_lbfgs_device_line_search_vs_closures(cuda, monkeypatch, golden, problem, max_iter):
    """LBFGS.solve with the weak Wolfe line search on the device
    (device.LineSearch: gated trials, the state read once per chunk of 4)
    against the same solve with the search's decisions on the host over the
    engine's closures (BSLS_LBFGS_LS=host), on the fixed-order engine: every
    logged iterate within 1e-8 (the searches' dot products round in other
    orders), the same iterations logged -- a 60k-route problem for a few
    iterations (L-BFGS there amplifies a 1e-16 difference to ~1e-6 within ~8
    iterations) and the 60-iteration well-conditioned fixture
    (tests/golden/lbfgs.npz gd_*)."""
    import torch
    import LBFGS
    import solvers
    from device import BBEngine
    from synthetic import make_shard, add_noise
    if problem == 'gd':
        G = golden('lbfgs.npz')
        eng = BBEngine(_csr(G, 'gd'), G['gd_b'], G['gd_block_sizes'], deterministic=True)
    else:
        sh = make_shard(60000, 3000, 8000, per_col=16, seed=3)
        b = add_noise(sh['Ax'], 0.02, seed=3)
        eng = BBEngine(sh['A'], b, sh['block_sizes'], AT=sh['AT'], deterministic=True)
    opts = {'max_iter': max_iter, 'verbose': 0, 'opt_tol': 1e-30}

    def run(mode):
        monkeypatch.setenv('BSLS_LBFGS_LS', mode)
        rec = {}

        def log(i, s, dt):
            rec[i] = s.detach().cpu().numpy().copy()
            return 0.0
        z0 = torch.ones(eng.nz, dtype=torch.float64, device='cuda')
        LBFGS.solve(z0, eng.f, eng.nabla_f, solvers.stopping, record_every=1, proj=eng.proj,
                    log=log, options=dict(opts))
        return rec
    dev = run('device')
    host = run('host')
    assert sorted(dev) == sorted(host) == list(range(max_iter + 1))
    for i in dev:
        assert rel(dev[i], host[i]) < 1e-8, (i, rel(dev[i], host[i]))
    if max_iter >= 2:
        ls = eng.line_search()
        # the last search ran on the device and evaluated at least one trial
        st = ls.st.cpu().numpy()
        assert st[7] >= 1 and st[3] != 0


def test_lbfgs_line_search_kernels_vs_reference_ls(cuda, orc):
    """One device search against the reference's weak_wolfe_ls (the oracle's
    restatement, LBFGS.py:9-53) from the same point and direction, on
    directions that force the three exits' paths: a descent direction (accept,
    maybe after bisection), a scaled-up one (Armijo failures first), a
    scaled-down one (curvature failures: doubling).  Same t, same exit."""
    import torch
    import _native
    from device import BBEngine
    from synthetic import make_shard, add_noise
    sh = make_shard(20000, 1000, 3000, per_col=8, seed=5)
    b = add_noise(sh['Ax'], 0.02, seed=5)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], AT=sh['AT'])
    P = orc.solve_in_z_parts(sh['A'], b, sh['block_sizes'])
    rs = np.random.RandomState(7)
    x = P['proj'](rs.rand(eng.nz))
    gx = P['nabla_f'](x)
    ls = eng.line_search()
    seen = set()
    for scale in (1e-3, 1e-1, 1.0, 10.0, 1e-5):
        d = -scale * gx / max(1.0, np.abs(gx).max()) + 1e-3 * scale * rs.randn(eng.nz)
        t_ref = orc.weak_wolfe_ls(x, d, P['f'], P['nabla_f'], proj=P['proj'])
        xd = torch.from_numpy(x.copy()).cuda()
        dd = torch.from_numpy(d.copy()).cuda()
        gd = eng.nabla_f(xd)
        fx = torch.tensor([eng.f(xd)], dtype=torch.float64, device='cuda')
        yo, so = torch.full_like(dd, np.nan), torch.full_like(dd, np.nan)
        t, why, ntr, dn = ls.search(xd, dd, gd, fx, y_out=yo, s_out=so)
        assert abs(t - t_ref) <= 1e-12 * max(1.0, abs(t_ref)), (scale, t, t_ref)
        seen.add((why, ntr > 1))
        if why == _native.LS_ACCEPTED:
            # bsls_lbfgs_ls_finish: y = g(x_next) - gx, s = t d, y.s, g.g, f(x_next)
            f_last, ys, gg = ls.last
            xn, gn, fn = ls.take()
            want = P['proj'](x + t_ref * d)
            g_want = P['nabla_f'](want)
            assert rel(xn.cpu().numpy(), want) < 1e-12
            assert rel(gn.cpu().numpy(), g_want) < 1e-10
            assert abs(float(fn) - P['f'](want)) <= 1e-10 * max(1.0, abs(P['f'](want)))
            assert float(fn) == f_last
            y_want, s_want = gn.cpu().numpy() - gd.cpu().numpy(), t * d
            assert np.array_equal(yo.cpu().numpy(), y_want)
            assert np.array_equal(so.cpu().numpy(), s_want)
            assert abs(ys - y_want.dot(s_want)) <= 1e-12 * max(1e-300, np.abs(y_want * s_want).sum())
            gg_want = float(gn.cpu().numpy().dot(gn.cpu().numpy()))
            assert abs(gg - gg_want) <= 1e-13 * gg_want
        else:
            assert ls.last is None
    assert any(w == _native.LS_ACCEPTED for w, _ in seen)


@pytest.mark.parametrize('m,pushes', [(1, 3), (5, 3), (5, 12), (50, 70), (64, 66), (70, 75), (100, 103)])
def test_lbfgs_device_history_direction(cuda, m, pushes):
    """_DeviceHistory.direction / push (csrc/lbfgs.hip: multi-dot, one-wave
    recursion on the Gram matrices, combine) against the reference's vector
    recursion (python/LBFGS.py:60-71) over the same lists, before and after
    the ring wraps: 1e-11 relative."""
    import torch
    import LBFGS
    rs = np.random.RandomState(m * 100 + pushes)
    n = 3001
    Y, S, rho = [np.zeros(n)] * m, [np.zeros(n)] * m, [0.0] * m
    x = torch.zeros(n, dtype=torch.float64, device='cuda')
    H = LBFGS._DeviceHistory(x, m)

    def ref_dir(g, yn, sn):
        q = g
        alpha = [0.0] * m
        for k in range(m - 1, -1, -1):
            alpha[k] = rho[k] * S[k].dot(q)
            q = q - alpha[k] * Y[k]
        r = (yn.dot(sn) / yn.dot(yn)) * q
        for k in range(m):
            beta = rho[k] * Y[k].dot(r)
            r = r + S[k] * (alpha[k] - beta)
        return -r
    T = lambda v: torch.from_numpy(v.copy()).cuda()
    for p in range(pushes):
        g, sn = rs.randn(n), rs.randn(n)
        yn = sn * (1 + rs.rand(n)) + 0.1 * rs.randn(n)      # y.s > 0, as on a convex f
        rn = 1.0 / yn.dot(sn)
        d = H.direction(T(g), T(yn), T(sn)).cpu().numpy()
        want = ref_dir(g, yn, sn)
        assert rel(d, want) < 1e-11, p
        H.push(rn)
        Y, S, rho = Y[1:] + [yn], S[1:] + [sn], rho[1:] + [rn]
    assert H.head == pushes % m


def test_multi_dot_and_axpy(cuda):
    """bsls_multi_dot / bsls_multi_axpy against NumPy (J = 1..4, K across
    column chunks, ragged n), 1e-13 relative; deterministic (two runs bit
    for bit)."""
    import torch
    import _native
    L = _native.lib()
    rs = np.random.RandomState(5)
    n = 70_001
    V = torch.from_numpy(rs.randn(40, n)).cuda()
    ptrs = lambda rows: torch.tensor([V[i].data_ptr() for i in rows], dtype=torch.int64).cuda()
    st = _native.stream_handle()
    Vh = V.cpu().numpy()
    for J, K in [(1, 1), (2, 17), (3, 33), (4, 16)]:
        rows, cols = list(range(J)), list(range(40 - K, 40))
        out = torch.empty(J * K, dtype=torch.float64, device='cuda')
        wb = L.bsls_multi_dot_workspace_size(J, K)
        w = torch.empty((wb + 7) // 8, dtype=torch.float64, device='cuda')
        R, C = ptrs(rows), ptrs(cols)
        outs = []
        for _ in range(2):
            _native.check(L.bsls_multi_dot(_native.ptr(R), J, _native.ptr(C), K, n,
                                           _native.ptr(out), _native.ptr(w), wb, st))
            outs.append(out.cpu().numpy().copy())
        want = (Vh[rows] @ Vh[cols].T).reshape(-1)
        assert rel(outs[0], want) < 1e-13
        assert np.array_equal(outs[0], outs[1])
    coef = torch.from_numpy(rs.randn(25)).cuda()
    out = torch.empty(n, dtype=torch.float64, device='cuda')
    _native.check(L.bsls_multi_axpy(_native.ptr(ptrs(range(25))), 25, _native.ptr(coef), n,
                                    _native.ptr(out), st))
    assert rel(out.cpu().numpy(), coef.cpu().numpy() @ Vh[:25]) < 1e-13
