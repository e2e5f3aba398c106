#!/usr/bin/env python
"""Benchmark: BB solver iterations/sec (1M-route block-LSQ) + proj_simplex HBM
GB/s on MI355X.  One JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C3|C5]

A step = one full projected-BB iteration (python/BB.py:17-41 semantics, fused
K2 -> K3 -> K1 on the device) over the whole problem, inputs resident in HBM.

Headline (BASELINE.json's metric and configs[2]): C3, 1M routes / 50k blocks /
100k links / 16M nnz.  At N = 1 `value` is C3's iterations/s on one GPU.  At
N > 1 every rank holds one C3-sized column shard (synthetic.make_shard with the
rank in its seed; rank 0's shard IS the C3 problem) of one N x 1M-route problem
over the same 100k links: weak scaling, per-GPU work fixed, one RCCL all-reduce
of the residual (800 KB) and of the four BB sums per iteration
(distributed.ShardedBB), `value` = N x iterations/s = 1M-route iterations/s of
the whole job.  The north star's strong-scaling problem (BASELINE configs[4],
C5: 10M routes / 500k blocks / 1M links, ONE problem column-sharded over the N
ranks) is timed beside it at every N as "c5".  At N = 1 the line also carries
the C2 projection, the standalone PAVA, the x-space / mirror-descent / DORE /
L-BFGS legs and the CPU baselines (C3).

Early exits are disabled for timing: exactly K iterations run.
"""
import argparse
import json
import os
import sys
import time

# the 1-thread CPU baseline leg runs like the reference (single-threaded BLAS);
# the box presets OPENBLAS_NUM_THREADS / OMP_NUM_THREADS to its CPU share
HOST_THREADS = int(os.environ.get('OMP_NUM_THREADS') or os.cpu_count() or 1)
os.environ['OPENBLAS_NUM_THREADS'] = '1'
ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

# BASELINE.json's metric text, verbatim; `value` is its 1M-route (C3) rate
METRIC = 'BB solver iterations/sec (1M-route block-LSQ) + proj_simplex HBM GB/s'
ROUND = 'r06'
HBM_PEAK = 8.0e12   # MI355X_MICROARCH.md chip table (spec)


def kernel_bytes(m, n, nz, p, nnz_a, nnz_at):
    """Algorithmic HBM bytes per launch, general fp64 CSR (SURVEY.md §8(d)'s
    accounting split by kernel): 12 B per entry, 4-B row
    pointers, each vector touched once."""
    return {
        'K1_spmv_A': 12 * nnz_a + 4 * (m + 1) + 8 * n + 16 * m,
        'K2_spmvT_Nt_dots': 12 * nnz_at + 4 * (n + 1) + 8 * m + 32 * nz,
        'K3_pava_clip_z2x': 24 * nz + 8 * n + 4 * p,
    }


def format_bytes(eng):
    """Bytes the kernels actually stream with the engine's images (the
    compressed figure SURVEY.md §8(d) asks to state beside the general one):
    the image, the vectors once, and the group partials (written + read)."""
    m, n, nz = eng.m, eng.n, eng.nz
    scale = 8 * n if eng.scaled else 0
    if eng.A_pan is not None:
        k1 = eng.A_pan.bytes() + 8 * n + 16 * m + 8 * m * (eng.A_pan.img['ngroups'] - 1) * 2
    else:
        g = eng.A_til.img['ngroups']
        k1 = eng.A_til.bytes() + 8 * n + 16 * m + (8 * m * g * 2 if g > 1 else 0)
    if eng.AT_pan is not None:
        k2 = eng.AT_pan.bytes() + 8 * m + 4 * n + 24 * nz + scale
    else:
        ti = eng.AT_til.img
        wp = 8 * ti['ngroups'] * ti['nrb'] * (ti['H'] + 1) * 2 if ti['ngroups'] > 1 else 0
        k2 = eng.AT_til.bytes() + 8 * m + 4 * n + 24 * nz + scale + wp
    return {'K1_spmv_A': k1, 'K2_spmvT_Nt_dots': k2,
            'K3_pava_clip_z2x': 32 * nz + 8 * n + 4 * eng.layout.p + scale}


def survey_iter_bytes(m, n, nz, nnz):
    """B_iter = 24 nnz + 4 (m+n+2) + 8 (3m + n + 5 n_z)."""
    return 24 * nnz + 4 * (m + n + 2) + 8 * (3 * m + n + 5 * nz)


def cpu_baseline_bb(A, b, sizes, budget_s=12.0):
    """The oracle's restatement of BB.solve over main.solve_in_z's closures
    (SciPy csr_matvec + the C PAVA restatement), 1 thread, bounded sample."""
    from oracle import oracle as orc
    P = orc.solve_in_z_parts(A, b, sizes)
    z = P['z0']
    z_prev = z + 1
    g_prev = P['nabla_f'](z_prev)
    t0 = time.perf_counter()
    it = 0
    while True:
        g = P['nabla_f'](z)
        dg = g - g_prev
        _ = sum(dg)                      # BB.py:22 (22 % of the reference's time)
        dx = z - z_prev
        t = dx.dot(dg) / dg.dot(dg)
        z_prev, z = z, P['proj'](z - t * g)
        g_prev = g
        _fx = P['f'](z)
        _ = orc.stopping(g, _fx, it + 1, t, delta_g=dg, options={'max_iter': 10 ** 9,
                                                                   'opt_tol': 1e-30})
        it += 1
        el = time.perf_counter() - t0
        if el >= budget_s or it >= 200:
            return it / el, it, el


def cpu_baseline_bb_omp(A, b, sizes, threads, budget_s=10.0):
    """The z-space BB loop in C + OpenMP (oracle/bsls_cpu_bb.c: the reference's
    work per iteration, rows / blocks over `threads` threads): calibrated on 3
    iterations, then a fixed count of about `budget_s` seconds."""
    from oracle import oracle as orc
    AT = sps_csr(A).T.tocsr()
    t0 = time.perf_counter()
    orc.cpu_bb_run(A, b, sizes, 3, threads=threads, AT=AT)
    per = (time.perf_counter() - t0) / 3
    iters = int(max(5, min(400, budget_s / max(per, 1e-6))))
    t0 = time.perf_counter()
    orc.cpu_bb_run(A, b, sizes, iters, threads=threads, AT=AT)
    el = time.perf_counter() - t0
    return iters / el, iters, el


def sps_csr(A):
    import scipy.sparse as sps
    return sps.csr_matrix(A)


def bench_stored_values(sh, b, steps, warmup, codec=None):
    """The C3 BB loop on the general images (values stored: what a matrix that
    is not a scaled incidence runs) -- BBEngine(general=True).  The values
    travel in the narrowest type that holds every one of them exactly (the C3
    flows are integers < 1000: _Float16, 2 B per entry; BSLS_TILE_VAL16);
    codec='f64' forces the 8-B doubles, what arbitrary real values need."""
    import torch
    from device import BBEngine
    old = os.environ.get('BSLS_VAL_CODEC')
    if codec:
        os.environ['BSLS_VAL_CODEC'] = codec
    try:
        eng = BBEngine(sh['A'], b, sh['block_sizes'],
                       options={'max_iter': 10 ** 12, 'opt_tol': 1e-30},
                       early_exit=False, AT=sh['AT'], general=True)
    finally:
        if old is None:
            os.environ.pop('BSLS_VAL_CODEC', None)
        else:
            os.environ['BSLS_VAL_CODEC'] = old
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    eng.prologue()
    el = float(np.median(time_run(eng.iterate, steps, warmup, None, windows=5)))
    m, n, nz, p, nnz = eng.m, eng.n, eng.nz, eng.layout.p, sh['A'].nnz
    ib = survey_iter_bytes(m, n, nz, nnz)
    its = steps / el
    return {'value': its, 'unit': 'BB iterations/s (C3, values stored)',
            'ms_per_step': el / steps * 1e3, 'formats': {'K1': eng.fmt_A, 'K2': eng.fmt_AT},
            'value_codec': getattr(eng.A_til, 'val_codec', 'f64') if eng.A_til else 'f64',
            'iteration_roofline': {'survey_bytes_per_iter': ib, 'achieved_GB_s': ib * its / 1e9,
                                   'frac': ib * its / HBM_PEAK}}


def bench_proj(reps=30, batch=16, fast=False):
    """C2 proj_multi_simplex (100k blocks x mean 32, 3.2M fp64) on the device,
    every launch on fresh input: the sort-free path (bsls_proj_multi_simplex_fast:
    Michelot's threshold passes, one lane per block, the north star's 1e-12
    contract) or, fast=False, the bit-identical sorting path.  avg_us: `batch` launches back to back on `batch` distinct copies of
    the input between two events on the launch stream (the stream held by a
    spin kernel while the host enqueues) -- the kernel time rocprofv3 reports,
    HBM-fed, dispatch gaps amortised; isolated_*: one launch per event pair
    (adds the launch latency)."""
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import proj_input
    L = _native.lib()
    name = 'bsls_proj_multi_simplex_fast' if fast else 'bsls_proj_multi_simplex'
    fn = getattr(L, name)
    y_h, starts_h = proj_input()
    n, p = y_h.shape[0], starts_h.shape[0]
    mb = int(np.max(np.diff(np.append(starts_h, n))))
    y0 = torch.from_numpy(y_h).cuda()
    st = torch.from_numpy(starts_h).cuda()
    ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')

    def proj(t):
        check(fn(ptr(t), ptr(st), p, n, mb, ptr(ws), ws.numel(), stream_handle()), name)
    ys = [y0.clone() for _ in range(batch)]
    for t in ys[:3]:
        proj(t)
    avg = []
    for _ in range(5):
        for t in ys:
            t.copy_(y0)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e8))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in ys:
            proj(t)
        e1.record()
        torch.cuda.synchronize()
        avg.append(e0.elapsed_time(e1) / batch)
    us = sorted(avg)[2] * 1e3
    # the size's practical floor: torch's in-place scale of the same y (16 n
    # bytes, vectorised, no block structure) timed the same way
    fl = []
    for _ in range(5):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e8))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in ys:
            t.mul_(1.0000001)
        e1.record()
        torch.cuda.synchronize()
        fl.append(e0.elapsed_time(e1) / batch)
    floor_us = sorted(fl)[2] * 1e3
    y = ys[0]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    torch.cuda._sleep(int(2e8))
    for k in range(reps):
        y.copy_(y0)
        evs[k][0].record()
        proj(y)
        evs[k][1].record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    med = ms[len(ms) // 2]
    byt = 16 * n + 4 * (p + 1)
    del ys
    # CPU baseline for the same call: the oracle (1 thread), and the check
    from oracle import oracle as orc
    yc = y_h.copy()
    t0 = time.perf_counter()
    orc.proj_multi_simplex_c(yc, starts_h)
    cpu_s = time.perf_counter() - t0
    out = y.cpu().numpy()
    rel = float(np.max(np.abs(out - yc) / np.maximum(1.0, np.abs(yc))))
    return {'entry': name, 'n': n, 'blocks': p, 'avg_us': us, 'GB_s': byt / (us * 1e-6) / 1e9,
            'alg_bytes': byt, 'frac_hbm_peak': byt / (us * 1e-6) / HBM_PEAK,
            'rocprof_kernels': [('proj_pipe' if fast else 'proj_lds_kernel<false, 2, false>')],
            'isolated_median_us': med * 1e3, 'isolated_min_us': ms[0] * 1e3,
            'same_size_scale_floor_us': floor_us,
            'frac_of_floor': floor_us / us,
            'cpu_oracle_ms_1thread': cpu_s * 1e3,
            'max_rel_diff_vs_oracle': rel, 'within_1e-12': rel <= 1e-12,
            'bit_exact_vs_oracle': bool(np.array_equal(yc.view(np.int64), out.view(np.int64)))}


def bench_xspace(sh, b, rounds=40, reps=5, k1=None):
    """x-space BB (BATCH.solve_BB over get_solver_parts(is_sparse=True),
    SURVEY.md §8 rows a14/f2) on the same C3 matrix with the block simplex
    projection: device rounds (csrc/xbb.hip) over the panel operator
    (csrc/lsq.hip).  A run converges (revert of a too-small step) after ~50
    rounds, so each rep restarts from x0 and runs `rounds` rounds with
    prog_tol < 0.  Reports rounds/s (a round = one BB step or one backtracking
    step, each a full objective evaluation) and accepted iterations/s."""
    import torch
    from algorithm_utils import get_solver_parts
    from device import XBBEngine
    import _native
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    x0 = np.repeat(1.0 / sizes, sizes)
    saved = os.environ.get('BSLS_LSQ_K1')
    if k1:
        os.environ['BSLS_LSQ_K1'] = k1      # DeviceLSQ reads it when it is built
    try:
        _, proj, _, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
    finally:
        if saved is None:
            os.environ.pop('BSLS_LSQ_K1', None)
        else:
            os.environ['BSLS_LSQ_K1'] = saved
    eng = XBBEngine(obj, proj)
    x0d = torch.from_numpy(x0).cuda()
    eng.start(x0d, max_iter=10 ** 12, prog_tol=-1.0, hist_cap=1)
    eng.rounds(rounds)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    its = bts = 0
    ok = True
    for k in range(reps):
        eng.start(x0d, max_iter=10 ** 12, prog_tol=-1.0, hist_cap=1)
        ev[2 * k].record()
        eng.rounds(rounds)
        ev[2 * k + 1].record()
        s = eng.scalars()
        its += int(s[_native.XS_ITER])
        bts += int(s[_native.XS_BACKTRACKS])
        ok = ok and bool(np.isfinite(s[_native.XS_F]))
    torch.cuda.synchronize()
    ms = sum(ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(reps))
    A = sh['A']
    m, n, nnz, p = A.shape[0], A.shape[1], A.nnz, len(sizes)
    # SURVEY 8(d)-style general-CSR bytes of a round (csrc/xbb.hip): residual
    # 12 nnz + 4 (m+1) + 8 n + 16 m, gradient 12 nnz + 4 (n+1) + 8 m + 8 n, the
    # finish's four vectors 32 n; a STEP round adds the step (x_new, g_new in,
    # x, g, x_new out: 40 n) and the projection 16 n + 4 (p+1), a BACKTRACK
    # round its blend (24 n)
    nr = rounds * reps
    common = 24 * nnz + 4 * (m + n + 2) + 24 * m + 16 * n + 32 * n
    byt = nr * common + (nr - bts) * (40 * n + 16 * n + 4 * (p + 1)) + bts * 24 * n
    opname = 'csr' if obj.lsq is None else {
        'tiles': 'tiles residual + panels gradient',
        'tiles_fixed': 'fixed-point tiles residual + panels gradient'}.get(obj.lsq.k1, 'panels')
    return {'operator': opname,
            'rounds': nr, 'us_per_round': ms * 1e3 / nr,
            'rounds_per_s': nr / (ms * 1e-3), 'iterations_per_s': its / (ms * 1e-3),
            'backtracks': bts, 'finite': ok,
            'roofline': {'bound': 'hbm', 'alg_bytes_per_round': byt / nr,
                         'achieved': byt / (ms * 1e-3) / 1e9, 'peak': HBM_PEAK / 1e9,
                         'unit': 'GB/s', 'frac': byt / (ms * 1e-3) / HBM_PEAK}}


def bench_lbfgs(sh, b, rounds=16, reps=10, corrections=50):
    """BATCH.solve_LBFGS (python/BATCH.py:110-214) on the C3
    matrix with the block simplex projection: the fused device rounds of
    device.XBBEngine(lbfgs=50) -- BB steps to iteration 5, LBFGS_helper's
    two-loop recursion from 6 (csrc/xbb.hip xlb_step / xlb_dir: four dot
    products and one combine pass per direction) -- each rep restarting from
    x0 with prog_tol < 0 (no early stop), `rounds` short of where the run
    converges (a revert makes delta_x = 0 and rho = 1/0, which the reference's
    own prog_tol test stops on).  Reports us per round (one step or
    one backtracking step, each a full objective) and per accepted iteration."""
    import torch
    from algorithm_utils import get_solver_parts
    from device import XBBEngine
    import _native
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    x0 = np.repeat(1.0 / sizes, sizes)
    _, proj, _, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
    eng = XBBEngine(obj, proj, lbfgs=corrections)
    x0d = torch.from_numpy(x0).cuda()
    eng.start(x0d, max_iter=10 ** 12, prog_tol=-1.0, hist_cap=1)
    eng.rounds(rounds)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    its = bts = 0
    ok = True
    for k in range(reps):
        eng.start(x0d, max_iter=10 ** 12, prog_tol=-1.0, hist_cap=1)
        ev[2 * k].record()
        eng.rounds(rounds)
        ev[2 * k + 1].record()
        s = eng.scalars()
        its += int(s[_native.XS_ITER]) - 1
        bts += int(s[_native.XS_BACKTRACKS])
        ok = ok and bool(np.isfinite(s[_native.XS_F]))
    torch.cuda.synchronize()
    ms = sum(ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(reps))
    nr = rounds * reps
    return {'operator': 'panels' if obj.lsq is not None else 'csr', 'corrections': corrections,
            'rounds': nr, 'us_per_round': ms * 1e3 / nr,
            'iterations': its, 'us_per_iter': ms * 1e3 / max(its, 1),
            'iterations_per_s': its / (ms * 1e-3), 'backtracks': bts, 'finite': ok}


def bench_gd_lbfgs(sh, b, iters=20, reps=20, m=50):
    """LBFGS.solve (python/LBFGS.py:56-123) through GradientDescent('LBFGS') on
    the C3 z-space problem over the BBEngine closures: wall time per
    iteration (the weak Wolfe line search decided on the device,
    device.LineSearch; its first iteration's search on the host, as
    LBFGS.solve does before x is a projected point), and the device direction alone (csrc/lbfgs.hip: multi-dot
    of {g, y_new, s_new} against the 2m + 2 history columns, one-wave
    recursion, combine over 2m + 1 vectors, the push) on a full ring of m
    pairs, timed with HIP events on the stream it runs on.  Algorithmic
    bytes per direction + push: (3 + 2m + 2) n reads (multi-dot, each vector
    once) + (2m + 1) n reads + n writes (combine) + 3 n copies in (6 n) + the
    pair's copy into its slot (4 n), 8 B each."""
    import torch
    import LBFGS
    from device import BBEngine
    from gradient_descent import GradientDescent
    opts = {'max_iter': iters, 'verbose': 0, 'opt_tol': 1e-30}
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options=opts, AT=sh['AT'])
    # z0 resident on the device, like every other input of a timed region (a
    # numpy z0 costs GradientDescent a 7.6-MB pageable upload, ~26 ms here)
    z0d = torch.zeros(eng.nz, dtype=torch.float64, device='cuda')
    gd = GradientDescent(z0=z0d, method='LBFGS', options=dict(opts), engine=eng)
    gd.run()                                    # warm (allocations, first launches)
    torch.cuda.synchronize()

    def timed(k):
        o = dict(opts, max_iter=k)
        gd = GradientDescent(z0=z0d, method='LBFGS', options=o, engine=eng)
        t0 = time.perf_counter()
        it, _, _ = gd.run()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, int(it[-1])
    wall, n1 = timed(iters)
    # the marginal cost of an iteration: a run twice as long, minus this one
    # (the first iteration's line search runs on the host over the closures --
    # LBFGS.solve's x0 is not a projected point -- and weighs on a short run)
    wall2, n2 = timed(2 * iters)
    iters_ = [n1]
    n = eng.nz
    rs = np.random.RandomState(1)
    H = LBFGS._DeviceHistory(torch.zeros(n, dtype=torch.float64, device='cuda'), m)
    vec = lambda: torch.from_numpy(rs.randn(n)).cuda()
    g, yn, sn = vec(), vec(), vec()
    for _ in range(m):                          # a full ring
        H.direction(g, yn, sn)
        H.push(1.0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        d = H.direction(g, yn, sn)
        H.push(1.0)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    byts = 8 * n * ((3 + 2 * m + 2) + (2 * m + 2) + 6 + 4)
    del H, d
    torch.cuda.empty_cache()
    return {'n': n, 'corrections': m, 'iterations': int(iters_[-1]),
            'ms_per_iteration': wall * 1e3 / max(int(iters_[-1]), 1),
            'ms_per_iteration_marginal': ((wall2 - wall) * 1e3 / (n2 - n1)) if n2 > n1 else None,
            'iterations_long_run': n2,
            'direction': {'us': us, 'alg_bytes': byts, 'achieved_GB_s': byts / us * 1e-3,
                          'peak_GB_s': HBM_PEAK / 1e9, 'frac': byts / us * 1e-3 / (HBM_PEAK / 1e9),
                          'note': 'direction + push per iteration (multi-dot, coef, combine, '
                                  'copies), HIP events, full ring of m pairs'}}


def bench_c1():
    """BASELINE configs[0]: main.py --method BB --device cpu on the
    tests/fast/test_main.py problem (bsls_utils.generate_data() defaults, the
    reference tests' seed): the host path of the drop-in (SciPy closures + the
    host c_extensions library, include/bsls_cpu.h), end to end from the .mat
    file through LS_postprocess.  Plumbing, not a GPU number."""
    import argparse
    import tempfile
    import bsls_utils
    import main as bmain
    np.random.seed(237423433)
    with tempfile.TemporaryDirectory() as d:
        fname = os.path.join(d, 'test_main.mat')
        bsls_utils.generate_data(fname=fname)
        args = argparse.Namespace(noise=0, file=fname, log='WARN', init=False, eq='CP',
                                  method='BB', device='cpu')
        t0 = time.perf_counter()
        iters, times, states, output = bmain.main(args=args)
        el = time.perf_counter() - t0
    err = np.asarray(output['0.5norm(Ax-b)^2'])
    return {'device': 'cpu', 'iterations': int(iters[-1]), 'seconds': el,
            'final_0.5norm(Ax-b)^2': float(err[-1]), 'converged_below_1e-16': bool(err[-1] < 1e-16)}


def bench_dore(sh, b, iters=30):
    """DORE (python/DORE.py:6-90 through gradient_descent.py:55-67's setup) on
    the C3 problem, the loop gradient_descent runs: DORE.solve_engine, every
    step and branch on the device (bsls_dore_iterate: linop / linop_T on the
    engine's K1 / K2 images with A and the target scaled by 0.99 / lsv -- lsv
    from ARPACK over the same operators, not timed -- proj = PAVA v1 + clip
    by K3).  `iters` iterations after 3 untimed ones, eps < 0 so the
    norm-change exit never fires.  Roofline: the algorithmic bytes of the
    kernels an iteration launches (2 K1 general-CSR passes -- the reference's
    third, linop(x) of the last x_select, is the Ax the previous iteration
    formed -- 1 K2, 2 projections at 16 n_z + 4 (p+1) each) over the wall
    time; the
    host-decided closure loop (DORE.solve) is timed beside it."""
    import torch
    import DORE
    from device import BBEngine
    from bsls_utils import lsv_operator
    eng = BBEngine(sh['A'], b, sh['block_sizes'], AT=sh['AT'])
    lsv = lsv_operator(eng, None)
    scale = 0.99 / lsv
    z0 = torch.zeros(eng.nz, dtype=torch.float64, device='cuda')
    tgt = eng.target * scale
    log = lambda i, s, d: 0.0
    DORE.solve_engine(eng, z0, scale, tgt, log=log, options={'max_iter': 3, 'opt_tol': -1.0})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x = DORE.solve_engine(eng, z0, scale, tgt, log=log, record_every=10 ** 9,
                          options={'max_iter': iters, 'opt_tol': -1.0})
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    taken = bool(eng.dore_scalars[3] != 0.0)
    # the closure loop (host branch decisions), for comparison
    t1 = time.perf_counter()
    DORE.solve(z0, lambda z: eng.apply_A(z, alpha=scale), lambda r: eng.apply_AT(r, alpha=scale),
               tgt, proj=eng.proj, log=log, options={'max_iter': 10, 'opt_tol': -1.0})
    torch.cuda.synchronize()
    host_us = (time.perf_counter() - t1) * 1e6 / 10
    # linop(x) at the top of an iteration reuses the last x_select's Ax from
    # iteration 1 on (csrc/bb.hip dore_top): 2 K1 per iteration + 1
    calls = {'A': 2 * iters + 1, 'AT': iters, 'proj': 2 * iters}
    m, n, nz, p, nnz = eng.m, eng.n, eng.nz, eng.layout.p, sh['A'].nnz
    kb = kernel_bytes(m, n, nz, p, nnz, nnz)
    byt = (calls['A'] * kb['K1_spmv_A'] + calls['AT'] * kb['K2_spmvT_Nt_dots']
           + calls['proj'] * (16 * nz + 4 * (p + 1)))
    return {'operator': 'K1/K2 images (%s, %s)' % (eng.fmt_A, eng.fmt_AT), 'lsv': float(lsv),
            'loop': 'device (DORE.solve_engine)', 'extrapolation_taken': taken,
            'iterations': iters, 'us_per_iter': el * 1e6 / iters, 'iterations_per_s': iters / el,
            'host_decided_loop_us_per_iter': host_us, 'launches': dict(calls),
            'roofline': {'bound': 'hbm', 'alg_bytes': byt, 'achieved': byt / el / 1e9,
                         'peak': HBM_PEAK / 1e9, 'unit': 'GB/s', 'frac': byt / el / HBM_PEAK},
            'finite': bool(torch.isfinite(x).all())}


def bench_md(sh, b, iters=30):
    """Mirror descent (mirror_descent.least_squares, SURVEY.md §8 row a12;
    BASELINE config C4) on the same C3 problem: r = A x - b and A' r on the
    panel operator, the exp / block-normalise / ||dx||_inf step with the
    device-side stopping test (tolerance < 0: never stops), `iters` iterations
    between two events, inputs resident.  A and b scaled by 1/100: the step
    t_k = sqrt(2 ln k_b)/(sqrt(k) Lf) scales as 1/s and g as s^2, so on the
    unscaled problem exp(-t g) overflows in the first iteration (in the
    reference as here: NaN); the cost per iteration does not depend on s."""
    import torch
    from mirror_descent import MirrorDescent
    md = MirrorDescent(sh['A'] * 0.01, b * 0.01, sh['block_sizes'])
    md.start()
    md.iterate(1, 5, -1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    md.iterate(6, iters, -1.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    x = md.x.cpu().numpy()
    A = sh['A']
    m, n, nnz, p = A.shape[0], A.shape[1], A.nnz, len(sh['block_sizes'])
    # general-CSR bytes per iteration: residual 12 nnz + 4 (m+1) + 8 n + 16 m,
    # gradient 12 nnz + 4 (n+1) + 8 m + 8 n, the update (x, g in, x out) 24 n +
    # 4 (p+1)
    byt = 24 * nnz + 4 * (m + n + 2) + 24 * m + 16 * n + 24 * n + 4 * (p + 1)
    us = ms * 1e3 / iters
    op = ('residual %s, gradient %s' % (md.lsq.k1, md.lsq.k2)) if md.lsq is not None else 'csr'
    return {'operator': op, 'scale': 0.01,
            'iterations': iters,
            'us_per_iter': us, 'iterations_per_s': iters / (ms * 1e-3),
            'finite': bool(np.all(np.isfinite(x))),
            'roofline': {'bound': 'hbm', 'alg_bytes_per_iter': byt,
                         'achieved': byt / (us * 1e-6) / 1e9, 'peak': HBM_PEAK / 1e9,
                         'unit': 'GB/s', 'frac': byt / (us * 1e-6) / HBM_PEAK}}


def bench_iso(reps=3, batch=16):
    """Standalone PAVA (variant 1 -- the isotonic_regression path of main.py's
    proj, isotonic_regression.h:85-92) on the C3/C4 z layout: 950k entries in
    50k blocks, inputs like K3's (z - t g); `batch` calls back to back on
    distinct copies between two events.  The call is the planned one
    (bsls_isotonic_packs over the layout's pack plan, made once and cached the
    way c_extensions and BBEngine.proj cache it); `unplanned_avg_us` is
    bsls_isotonic_multi, which plans on the device every call.  Bytes 16 n +
    4 (p+1)."""
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import make_shard, CONFIGS, SEED
    L = _native.lib()
    c = CONFIGS['C3']
    rs = np.random.RandomState(SEED)
    sizes = rs.multinomial(c['n'] - c['p'], np.ones(c['p']) / c['p']) + 1
    zs = np.concatenate(([0], np.cumsum(sizes - 1)[:-1])).astype(np.int64)
    nz = int((sizes - 1).sum())
    y0 = torch.from_numpy(rs.rand(nz) - 0.3 * rs.randn(nz)).cuda()
    st = torch.from_numpy(zs).cuda()
    mb = int(np.max(sizes))
    ws = torch.zeros(L.bsls_isotonic_workspace_size(nz), dtype=torch.uint8, device='cuda')
    status = torch.zeros(4, dtype=torch.int32, device='cuda')
    ys = [y0.clone() for _ in range(batch)]

    from device import iso_plan
    plan = iso_plan(zs, nz)

    def iso_unplanned(t):
        check(L.bsls_isotonic_multi(1, ptr(t), ptr(st), zs.size, nz, None, 1, mb, ptr(ws),
                                    ws.numel(), ptr(status), stream_handle()), 'iso')

    def timed(fn):
        for t in ys[:2]:
            fn(t)
        out = []
        for _ in range(reps):
            for t in ys:
                t.copy_(y0)
            torch.cuda.synchronize()
            torch.cuda._sleep(int(2e8))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for t in ys:
                fn(t)
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / batch * 1e3)
        return sorted(out)[len(out) // 2]
    floor_us = timed(lambda t: t.mul_(1.0000001))   # the size's practical floor (as bench_proj)
    us_un = timed(iso_unplanned)
    us = timed(plan.apply)
    from oracle import oracle as orc
    yc = y0.cpu().numpy().copy()
    t0 = time.perf_counter()
    orc.isotonic_regression_multi_c(yc, zs)
    cpu_s = time.perf_counter() - t0
    ok = bool(np.array_equal(yc.view(np.int64), ys[0].cpu().numpy().view(np.int64)))
    byt = 16 * nz + 4 * (zs.size + 1)
    return {'n': nz, 'blocks': int(zs.size), 'packs': plan.npacks, 'avg_us': us,
            'alg_bytes': byt, 'GB_s': byt / (us * 1e-6) / 1e9,
            'frac_hbm_peak': byt / (us * 1e-6) / HBM_PEAK, 'unplanned_avg_us': us_un,
            'same_size_scale_floor_us': floor_us, 'frac_of_floor': floor_us / us,
            'rocprof_kernels': ['iso_packs_kernel'],
            'cpu_oracle_ms_1thread': cpu_s * 1e3, 'bit_exact_vs_oracle': ok}


def log(msg):
    """Progress on stderr (the GPU box kills a command silent for 3 minutes)."""
    print('[bench %.1fs] %s' % (time.perf_counter() - T0, msg), file=sys.stderr, flush=True)


T0 = time.perf_counter()


def build_problem(name, world, rank, dist, shard_of=None):
    """The rank's column shard of workload `name` and the full b (SURVEY §8(d)
    recipe, 2 % multiplicative noise so the exact-zero exit never fires).
    C5: rank's share of the one 10M-route problem (strong scaling).  C3: one
    C3-sized shard per rank, seeded by the rank (rank 0's is the C3 problem
    itself), all over the same 100k links (weak scaling).  shard_of
    (rehearsal on one GPU): rank 0's C5 shard of that many ranks, b its own
    A x (the timing does not depend on b)."""
    import torch
    from synthetic import make_partitioned, make_shard, add_noise, CONFIGS, SEED
    c = CONFIGS[name]
    if name == 'C5':
        sh = make_partitioned(c['n'], c['p'], c['m'], c['per_col'], rank=rank,
                              world=shard_of or world)
    else:
        sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED, rank=rank)
        sh['colv'] = None
        sh['n_total'], sh['p_total'] = world * c['n'], world * c['p']
    Ax = torch.from_numpy(sh['Ax']).cuda()
    if dist:
        dist.all_reduce(Ax)
    b = add_noise(Ax.cpu().numpy(), 0.02, seed=SEED)
    return sh, b


def build_engine(sh, b, world, dist, parts, sharded=False, slices=None, model=None,
                 force_comm=False):
    """(engine, run(first, count)) for one rank: the fused single-GPU loop, or
    the column-sharded stages with the RCCL all-reduces (distributed.ShardedBB;
    `sharded` forces them at world 1 -- the per-rank host and launch path of
    an N-GPU run, rehearsed on one GPU).  parts > 1: the exchange pipelined
    behind both walks (link parts, bsls_bb_shard_iterate_parts).  model
    (us_per_mb, fixed_us), rehearsal only: every exchange a spin of that cost
    on its stream instead of the skipped one-rank collectives
    (distributed.ModelComm) -- how much of such an exchange the schedule hides.
    force_comm: an RCCL communicator that runs its collectives at world 1 too
    (bsls_comm_force_collectives: the one-rank self-check of the transport)."""
    import torch
    from device import BBEngine
    opts = {'max_iter': 10 ** 12, 'opt_tol': 1e-30}
    if world == 1 and not sharded:
        eng = BBEngine(sh['A'], b, sh['block_sizes'], options=opts, early_exit=False,
                       AT=sh['AT'], colv=sh.get('colv'))
        eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
        eng.prologue()
        return eng, eng.iterate
    from distributed import ShardedBB, torch_all_reduce, torch_all_reduce_async
    eng = BBEngine(sh['A'], None, sh['block_sizes'], options=opts, early_exit=False,
                   AT=sh['AT'], colv=sh.get('colv'),
                   target=torch.zeros(sh['m'], dtype=torch.float64),
                   link_parts=parts if parts > 1 else None)
    # target = sum_g A_g x0_g - b (main.py:48 over the shards)
    eng.x.copy_(eng.colv * eng.x0 if eng.scaled else eng.x0)
    eng.stage(1, 0)
    dist.all_reduce(eng.r)
    eng.target.copy_(eng.r - torch.from_numpy(b).cuda())
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    # the schedule enqueued from C++ with RCCL in the loop (BSLS_SHARD_NATIVE=0:
    # the Python loop over torch.distributed, for A/B)
    comm = None
    if model is not None and world == 1:
        from distributed import ModelComm
        comm = ModelComm(slices or 1, 0, fixed_us=model[1], us_per_mb=model[0])
    elif os.environ.get('BSLS_SHARD_NATIVE', '1') != '0' and dist.get_backend() == 'nccl':
        from distributed import RcclComm
        comm = RcclComm(force=force_comm)
    elif os.environ.get('BSLS_SHARD_NATIVE', '1') != '0' and world > 1:
        # another backend (the gloo rehearsal of N ranks on one GPU): the same
        # native loop, its all-reduces through torch.distributed callbacks
        from distributed import CallbackComm
        comm = CallbackComm(torch_all_reduce(), rank=dist.get_rank(), world=world, engine=eng)
    drv = ShardedBB(eng, torch_all_reduce(), parts=parts,
                    all_reduce_async=torch_all_reduce_async(),
                    rank=dist.get_rank(), native=comm, slices=slices)
    drv.prologue()
    eng._comm = comm            # kept alive with the engine
    return eng, drv.iterate


def time_run(run, steps, warmup, dist, windows=1):
    """W untimed iterations, then `windows` windows of exactly K iterations,
    each between barrier + synchronize on both sides, max over ranks per
    window.  Returns the per-window seconds (the headline takes the median:
    a 20-step window of C3 is ~1.7 ms of device time, so one window alone is
    at the mercy of a single clock or launch hiccup)."""
    import torch
    run(1, warmup)
    torch.cuda.synchronize()
    els = []
    first = 1 + warmup
    for _ in range(max(1, windows)):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(first, steps)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device='cuda')
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        els.append(el)
        first += steps
    return els


def kernel_table(eng, it0, reps, world, m, n, nz, p, nnz):
    """Per-kernel HIP-event timing on the stream the kernels run on: each stage
    launched `reps` times back to back between two events (the stages are
    idempotent for a fixed iteration index), the stream held by a spin kernel
    while the host enqueues, so no host gap sits inside an interval."""
    import torch
    kb = kernel_bytes(m, n, nz, p, nnz, nnz)
    fb = format_bytes(eng)
    k1 = 7 if world == 1 else 1          # sharded: the partial residual (stage 1)
    kern = {}
    for stg, nm in ((3, 'K2_spmvT_Nt_dots'), (k1, 'K1_spmv_A'), (4, 'K3_pava_clip_z2x')):
        torch.cuda._sleep(int(2e8))
        if stg == 4 and world == 1:
            # K3 keeps each pack's PAVA partition from its last call (the warm
            # start): relaunched on one state every partition holds, so it is
            # timed inside real iterations instead -- `reps` whole iterations
            # (K2, K3, K1) back to back between two events, less the K2 and K1
            # times measured above
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for k in range(reps):
                eng.stage(3, it0 + k)
                eng.stage(4, it0 + k)
                eng.stage(7, it0 + k)
            ev[1].record()
            torch.cuda.synchronize()
            us = (ev[0].elapsed_time(ev[1]) * 1e3 / reps - kern['K2_spmvT_Nt_dots']['avg_us']
                  - kern['K1_spmv_A']['avg_us'])
        else:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(reps):
                eng.stage(stg, it0)
            ev[1].record()
            torch.cuda.synchronize()
            us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
        kern[nm] = {'avg_us': us, 'alg_bytes': kb[nm], 'GB_s': kb[nm] / (us * 1e-6) / 1e9,
                    'frac': kb[nm] / (us * 1e-6) / HBM_PEAK, 'format_bytes': fb[nm],
                    'format_GB_s': fb[nm] / (us * 1e-6) / 1e9,
                    'format_frac': fb[nm] / (us * 1e-6) / HBM_PEAK,
                    'rocprof_kernels': rocprof_names(eng, nm, world)}
        if stg == 4 and world == 1:
            kern[nm]['timing'] = ('inside real iterations (the warm start sees the loop\'s '
                                  'inputs): whole iterations back to back, less the K2 and K1 '
                                  'times')
    kern['formats'] = {'K1': eng.fmt_A, 'K2': eng.fmt_AT}
    return kern


def rocprof_names(eng, nm, world):
    """The kernel names (rocprofv3 'Kernel_Name' prefixes) one stage launch of
    `nm` runs: the rows of profiles/*_kernel_stats.csv its avg_us is the sum
    of."""
    if nm == 'K3_pava_clip_z2x':
        return ['bb_k3']
    if nm == 'K2_spmvT_Nt_dots':
        return ['bb_k2t' if eng.AT_til is not None else 'bb_k2']
    if eng.A_til is not None:
        return ['bb_k1t'] + (['bb_k1_sum'] if eng.A_til.img['ngroups'] > 1 else [])
    return ['bb_k1']


def roofline_of(kern, traffic_file=None, config=None):
    """The dominant kernel's roofline; traffic = its HBM bytes per launch from
    the rocprofv3 PMC passes of the same build (tools/traffic.py, keyed by
    workload), None when absent."""
    names = [k for k in kern if k != 'formats']
    dom = max(names, key=lambda k: kern[k]['avg_us'])
    per = {}
    if traffic_file and os.path.exists(traffic_file):
        try:
            per = json.load(open(traffic_file)).get(config, {})
        except Exception:
            per = {}
    # physical rate next to the algorithmic one: the PMC bytes of each kernel
    # over this run's average launch time (the bytes the images, gathers and
    # partials really move, C5 images beyond the Infinity Cache)
    for k in names:
        tb = per.get(k, {}).get('hbm_bytes_per_launch')
        if tb:
            kern[k]['pmc_bytes'] = tb
            kern[k]['pmc_GB_s'] = tb / (kern[k]['avg_us'] * 1e-6) / 1e9
    traffic = per.get(dom, {}).get('hbm_bytes_per_launch')
    return {'bound': 'hbm', 'kernel': dom, 'rocprof_kernels': kern[dom].get('rocprof_kernels'),
            'avg_us': kern[dom]['avg_us'], 'alg_bytes': kern[dom]['alg_bytes'],
            'achieved': kern[dom]['GB_s'],
            'peak': HBM_PEAK / 1e9, 'unit': 'GB/s', 'frac': kern[dom]['frac'],
            'format_bytes': kern[dom]['format_bytes'], 'format_frac': kern[dom]['format_frac'],
            'traffic': traffic, 'traffic_source': traffic_file and os.path.basename(traffic_file),
            'physical_GB_s': kern[dom].get('pmc_GB_s'),
            'physical_frac': (kern[dom]['pmc_GB_s'] * 1e9 / HBM_PEAK
                              if kern[dom].get('pmc_GB_s') else None),
            'note': 'frac = SURVEY 8(d) general-CSR bytes / avg_us / 8 TB/s; format_frac = '
                    'the bytes the compressed images stream; physical_frac = PMC '
                    'FETCH+WRITE bytes (traffic) / avg_us'}


def host_info(threads):
    import platform
    model = platform.processor()
    try:
        for ln in open('/proc/cpuinfo'):
            if ln.startswith('model name'):
                model = ln.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return {'nproc': os.cpu_count(), 'cpu_model': model, 'threads_used': threads,
            'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS'),
            'OPENBLAS_NUM_THREADS': os.environ.get('OPENBLAS_NUM_THREADS')}


LEGS = ('main', 'c5', 'c3sv', 'proj', 'iso', 'xspace', 'md', 'dore', 'lbfgs', 'gdlbfgs', 'c1',
        'cpu', 'rccl1')


def traffic_file():
    """The newest PMC traffic summary of the default build under profiles/
    (tools/traffic.py: traffic_rNN.json; suffixed files such as
    traffic_r05_sydr.json profile an opt-in variant and are not the line's)."""
    import glob
    import re
    fs = sorted(f for f in glob.glob(os.path.join(ROOT, 'profiles', 'traffic_r*.json'))
                if re.fullmatch(r'traffic_r\d+\.json', os.path.basename(f)))
    return fs[-1] if fs else None


# The N > 1 self-check's problem: one column-sharded BB
# problem, the same for every world size (synthetic.make_partitioned), large
# enough that every rank's shard takes the C5 shards' kernels (dealt tiles, an
# atomic K1 of several column groups, the int64 fixed-point r) and small
# enough for the oracle to replay 20 iterations on rank 0 in a few seconds.
SELFCHECK = dict(n=1_600_000, p=80_000, m=160_000, per_col=16, iters=20, tol=1e-6)


def gather_z(z, dist, world):
    """Every rank's z slice, concatenated in rank order on every rank (a
    padded all_gather: the slices differ in length).  Tensors travel on the
    GPU under nccl, on the host under gloo."""
    import torch
    dev = z.device if dist.get_backend() == 'nccl' else torch.device('cpu')
    z = z.to(dev)
    n = torch.tensor([z.numel()], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    pad = torch.zeros(max(ns), dtype=torch.float64, device=dev)
    pad[:z.numel()] = z
    parts = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return np.concatenate([p[:k].cpu().numpy() for p, k in zip(parts, ns)])


def selfcheck_verdict(got, ref, tol):
    """max over elements of |got - ref| / max(1, |ref|) (the iterate contract of
    the north star, 1e-6) and whether it holds; a length mismatch fails."""
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    if got.shape != ref.shape:
        return float('inf'), False
    err = float(np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref)))) if ref.size else 0.0
    return err, bool(np.isfinite(err) and err <= tol)


def selfcheck_sharded(world, rank, dist, parts=1, problem=None, force=False):
    """Before any timing at N > 1: a column-sharded BB problem through the
    shipped transport -- RcclComm + bsls_bb_shard_iterate under nccl (the
    five-sum and the int64 fixed-point r all-reduces of every iteration), the
    callback transport under gloo -- for SELFCHECK['iters'] iterations; the
    ranks' z slices gathered and compared on rank 0 with the oracle's
    trajectory of the whole problem (python/BB.py:7-45 over main.py:53-65).
    The oracle is the check leg only, outside every timed region.  Returns the
    line's fields on every rank (the verdict broadcast from rank 0).  force
    (N = 1, leg rccl1): the sharded driver on one nccl rank with its RCCL
    collectives forced on (a one-rank sum is the identity), so the N = 1 line
    shows the transport's calls executing against the oracle as well."""
    import torch
    from synthetic import make_partitioned, add_noise, SEED
    c = dict(SELFCHECK, **(problem or {}))
    t0 = time.perf_counter()
    with _StdoutToStderr():
        sh = make_partitioned(c['n'], c['p'], c['m'], c['per_col'], rank=rank, world=world)
        Ax = torch.from_numpy(sh['Ax']).cuda()
        dist.all_reduce(Ax)
        b = add_noise(Ax.cpu().numpy(), 0.02, seed=SEED)
        eng, run = build_engine(sh, b, world, dist, parts, sharded=force, force_comm=force)
    comm = getattr(eng, '_comm', None)
    run(1, c['iters'])
    torch.cuda.synchronize()
    z = gather_z(eng.current_z(c['iters'] & 1), dist, world)
    sc = eng.scalars()
    info = {'transport': type(comm).__name__ if comm is not None else 'torch.distributed',
            'rccl_ranks': comm.count() if hasattr(comm, 'count') else None,
            'r_fixed_point': bool(float(eng.P.r_fx) > 0),
            'k1_groups': int(eng.A_til.img['ngroups']) if eng.A_til is not None else None,
            'formats': [eng.fmt_A, eng.fmt_AT], 'collectives_forced': bool(force)}
    if comm is not None:
        comm.close()
    del eng, run
    torch.cuda.empty_cache()
    v = torch.zeros(2, dtype=torch.float64)
    if rank == 0:
        from oracle import oracle as orc
        full = make_partitioned(c['n'], c['p'], c['m'], c['per_col'])
        ref = orc.bb_trace(full['A'], b, full['block_sizes'], c['iters'],
                           record_every=c['iters'])[c['iters']]
        err, ok = selfcheck_verdict(z, ref, c['tol'])
        v[0], v[1] = err, 1.0 if ok else 0.0
    v = v.cuda() if dist.get_backend() == 'nccl' else v
    dist.broadcast(v, src=0)
    # one verdict on every rank: rank 0's comparison, and a rank whose RCCL
    # communicator counts other than the job's ranks fails it for all
    mine = 1.0 if (info['rccl_ranks'] is None or info['rccl_ranks'] == world) else 0.0
    flag = torch.tensor([mine * float(v[1].item())], dtype=torch.float64, device=v.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    err, ok = float(v[0].item()), bool(flag.item() == 1.0)
    res = dict(info, err=err, ok=ok, tol=c['tol'], iters=c['iters'], finite=bool(np.isfinite(sc[4])),
               problem='%d routes / %d blocks / %d links / %d nnz, column-sharded over %d ranks '
                       '(synthetic.make_partitioned), 2 %% noise' % (c['n'], c['p'], c['m'],
                                                                     c['per_col'] * c['n'], world),
               seconds=time.perf_counter() - t0)
    log('self-check: %s, %s ranks, fixed-point r %s, max elem err %.3e vs the oracle at '
        'iteration %d -> %s' % (res['transport'], res['rccl_ranks'], res['r_fixed_point'], err,
                                c['iters'], 'ok' if ok else 'MISMATCH'))
    return res


class _StdoutToStderr:
    """fd 1 -> fd 2 for a block: RCCL prints its version banner on stdout
    when it initialises, and bench.py's stdout must be the one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--workload', default='C3', choices=['C3', 'C5'])
    ap.add_argument('--parts', type=int, default=1,
                    help='row parts of the pipelined residual all-reduce (N > 1)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-extras', action='store_true', help='only the headline workload')
    ap.add_argument('--legs', default='all',
                    help='comma list of %s (N = 1; default all): one rocprofv3 run per leg '
                         'keeps each workload\'s kernel rows apart' % ','.join(LEGS))
    ap.add_argument('--profile-iters', type=int, default=20)
    ap.add_argument('--model-exchange', default=None,
                    help='US_PER_MB[,FIXED_US]: with --rehearse-shard, model every exchange '
                         'as a spin of that cost on its stream (timing only)')
    ap.add_argument('--windows', type=int, default=10,
                    help='timed windows of --steps iterations each; the line reports the '
                         'median window and the spread')
    ap.add_argument('--rehearse-shard', type=int, default=0,
                    help='one GPU, one process: time rank 0 of an N-way C5 partition through '
                         'the sharded (RCCL) driver -- per-rank cost without the fabric')
    ap.add_argument('--rehearse-workload', default='C5', choices=['C3', 'C5'],
                    help='the rehearsed partition: C5 (rank 0 of N), or C3 (rank 0\'s C3-sized '
                         'shard of the weak-scaled N-GPU headline; the rank count does not '
                         'change its shard)')
    args = ap.parse_args()
    legs = set(LEGS) if args.legs == 'all' else set(args.legs.split(','))
    if legs - set(LEGS):
        raise SystemExit('unknown legs %s' % sorted(legs - set(LEGS)))
    if args.no_extras:
        legs = {'main'}
    if args.no_cpu_baseline:
        legs.discard('cpu')

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    if args.rehearse_shard:
        legs, args.workload = {'main'}, args.rehearse_workload
    elif world > 1:
        legs &= {'main', 'c5'}
    # (modulo: the gloo rehearsal puts several ranks on one GPU)
    local = local % max(1, torch.cuda.device_count())
    if torch.cuda.device_count():
        torch.cuda.set_device(local)
    # (no device: only the CPU tests of the line's contract get here, with
    # the legs replaced; every leg itself needs the HIP library and a GPU)
    dist = None
    if world > 1 or args.rehearse_shard:
        import torch.distributed as dist
        if world == 1:
            for k, v in (('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29533'), ('RANK', '0'),
                         ('WORLD_SIZE', '1')):
                os.environ.setdefault(k, v)
        backend = os.environ.get('BSLS_DIST_BACKEND', 'nccl')
        with _StdoutToStderr():
            if backend == 'nccl':
                dist.init_process_group('nccl', device_id=torch.device('cuda', local))
            else:
                dist.init_process_group(backend)

    tfile = traffic_file()
    out = {} if rank == 0 else None
    wl = args.workload
    if world > 1 and not args.rehearse_shard:
        # parity before rate: the shipped transport against the oracle, before
        # anything is timed; a mismatch ends the job non-zero on every rank
        sc = selfcheck_sharded(world, rank, dist, parts=args.parts)
        if rank == 0:
            out.update({'selfcheck': sc, 'selfcheck_err': sc['err'],
                        'rccl_ranks': sc['rccl_ranks']})
        if not sc['ok']:
            if rank == 0:
                out.update({'metric': METRIC, 'value': None, 'n_gpus': world,
                            'error': 'N > 1 self-check failed: the sharded iterate differs from '
                                     'the oracle (max elem err %.3e > %.0e) or the communicator '
                                     'spans another rank count' % (sc['err'], sc['tol'])})
                print(json.dumps(out), flush=True)
            dist.destroy_process_group()
            sys.exit(3)
    if 'main' in legs:
        res = bench_workload(wl, args, world, rank, dist, tfile, args.steps,
                             shard_of=args.rehearse_shard or None)
        if rank == 0:
            out.update({'metric': METRIC, 'n_gpus': world, 'steps': args.steps,
                        'warmup': args.warmup, 'higher_is_better': True,
                        'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic'})
            out.update(res)
    # the north star's strong-scaling problem beside the headline, at every N
    if 'c5' in legs and wl != 'C5':
        res = bench_workload('C5', args, world, rank, dist, tfile, max(args.steps, 100))
        if rank == 0:
            out['c5'] = res
    # --- N = 1 legs: the other paths -------------------------------------------------
    if world == 1 and not args.rehearse_shard and legs - {'main', 'c5'}:
        extras(args, legs, out, tfile)
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def bench_workload(wl, args, world, rank, dist, tfile, steps, shard_of=None):
    """Build workload `wl` on this rank, time `steps` iterations after the
    warmup (max over ranks), and on rank 0 return the line's fields: value
    (whole-job rate in the workload's unit), kernels (HIP-event table of the
    rank-0 stages) and their roofline."""
    import torch
    # (the first collectives and the driver's communicator initialise RCCL:
    # its banner goes to stderr)
    with _StdoutToStderr():
        sh, b = build_problem(wl, world, rank, dist, shard_of=shard_of)
        log('%s shard %d/%d: %d routes, %d blocks, %d links, %d nnz'
            % (wl, rank, world, sh['n'], sh['p'], sh['m'],
               sh['nnz'] if 'nnz' in sh else sh['A'].nnz))
        model = None
        if shard_of and args.model_exchange:
            v = [float(a) for a in args.model_exchange.split(',')]
            model = (v[0], v[1] if len(v) > 1 else 0.0)
        eng, run = build_engine(sh, b, world, dist, args.parts, sharded=bool(shard_of),
                                slices=shard_of, model=model)
    log('engine up (K1 %s, K2 %s)' % (eng.fmt_A, eng.fmt_AT))
    els = time_run(run, steps, args.warmup, dist, windows=args.windows)
    el = float(np.median(els))
    it_s = steps / el
    sc = eng.scalars()
    finite = bool(np.isfinite(sc[4]))
    log('%s: %d iterations in %.3f s: %.1f it/s (f %.6e, stop flag %g, iteration %g)'
        % (wl, steps, el, it_s, sc[4], sc[0], sc[1]))
    m, n_g, nz_g, p_g, nnz_g = eng.m, eng.n, eng.nz, eng.layout.p, sh['A'].nnz
    kern = {}
    if args.profile_iters > 0 and rank == 0:
        kern = kernel_table(eng, 1 + args.warmup + steps * len(els), args.profile_iters,
                            world if not shard_of else 2, m, n_g, nz_g, p_g, nnz_g)
        log('kernel table done')
    if dist:
        dist.barrier()
    res = None
    if rank == 0:
        n_tot, p_tot = sh['n_total'], sh['p_total']
        nnz_tot = 16 * n_tot
        # the PMC traffic and kernel-trace key: the one-GPU workload, or the
        # shard ('C5_x8': rank 0 of 8); a shard nobody profiled gets traffic
        # null rather than the one-GPU kernels' bytes
        key = ('%s_x%d' % (wl, shard_of or world)) if (shard_of or world > 1) else wl
        weak = wl == 'C3'
        # weak: the job is world C3-sized shards; its unit is the 1M-route
        # iteration, so the rate is world x iterations/s of the whole problem
        value = it_s * world if weak else it_s
        ib = survey_iter_bytes(m, n_tot, n_tot - p_tot, nnz_tot)
        res = {
            'value': value,
            'unit': ('1M-route BB iterations/s of the whole job (%d x C3: %d routes / %d '
                     'blocks / %d links)' % (world, n_tot, p_tot, m)) if weak else
                    ('BB iterations/s of the whole job (%s: %d routes / %d blocks / %d links)'
                     % (wl, n_tot, p_tot, m)),
            'iterations_per_s': it_s, 'steps': steps,
            'ms_per_step': el / steps * 1e3,
            'windows': {'count': len(els), 'steps_each': steps,
                        'ms_per_step': {'median': el / steps * 1e3,
                                        'min': min(els) / steps * 1e3,
                                        'max': max(els) / steps * 1e3},
                        'iterations_per_s': {'median': it_s, 'min': steps / max(els),
                                             'max': steps / min(els)},
                        'note': 'value = the median window; every window K iterations '
                                'between barrier + synchronize, max over ranks'},
            'scaling': 'weak' if weak else 'strong',
            'config': {'workload': ('C3 (BASELINE configs[2]): BB (z-space, PAVA projection) on '
                                    '%d x (1M routes / 50k blocks / 16M nnz), %d links, one '
                                    'C3 column shard per GPU' % (world, m)) if weak else
                                   ('%s: BB (z-space, PAVA projection) on %d routes / %d blocks '
                                    '/ %d links / %d nnz, column-sharded over %d GPU(s)'
                                    % (wl, n_tot, p_tot, m, nnz_tot, world)),
                       'routes': n_tot, 'blocks': p_tot, 'links': m, 'nnz': nnz_tot,
                       'routes_rank0': n_g, 'nnz_rank0': nnz_g,
                       'parallelism': 'column-shard x%d' % world,
                       'residual_allreduce_parts': args.parts if world > 1 else None},
            'roofline': roofline_of(kern, tfile, key) if kern else None,
            'iteration_roofline': {'survey_bytes_per_iter': ib,
                                   'achieved_GB_s': ib * it_s / 1e9,
                                   'frac': ib * it_s / HBM_PEAK,
                                   'note': 'whole job over all GPUs; peak is one GPU'},
            'kernels': kern, 'finite': finite,
            'profiles': 'profiles/%s_%s_kernel_stats.csv' % (ROUND, key),
        }
        if shard_of:
            res['config']['rehearsal'] = ('rank 0 of a %d-way C5 partition on one GPU through '
                                          'the sharded driver: every kernel of its iteration '
                                          '(||r||^2 over its 1/%d slice), the collectives of a '
                                          'one-rank communicator skipped -- per-rank compute, '
                                          'no fabric' % (shard_of, shard_of))
            if args.model_exchange:
                res['config']['rehearsal'] += (
                    '; every exchange modelled as a spin of %s (us per MB[, fixed us]) on its '
                    'stream, %d link part(s)' % (args.model_exchange, args.parts))
            res['config']['link_parts'] = args.parts
    if getattr(eng, '_comm', None) is not None:
        torch.cuda.synchronize()
        eng._comm.close()
    del eng, run
    torch.cuda.empty_cache()
    return res


def extras(args, legs, out, tfile):
    import torch
    steps3 = max(args.steps, 50)
    sh3 = b3 = None
    if legs & {'c3sv', 'xspace', 'md', 'dore', 'lbfgs', 'gdlbfgs', 'cpu'}:
        sh3, b3 = build_problem('C3', 1, 0, None)
    if 'c3sv' in legs:
        out['c3_stored_values'] = bench_stored_values(sh3, b3, steps3, args.warmup)
        torch.cuda.empty_cache()
        out['c3_stored_values_f64'] = bench_stored_values(sh3, b3, steps3, args.warmup, 'f64')
        torch.cuda.empty_cache()
    if 'proj' in legs:
        # the product default (bit-identical sorting kernels) and the sort-free
        # entry (1e-12 contract) beside it
        out['proj_simplex'] = bench_proj(fast=False)
        out['proj_simplex_fast'] = bench_proj(fast=True)
        log('C2 projection done')
    if 'iso' in legs:
        out['isotonic'] = bench_iso()
    if 'xspace' in legs:
        # the default operator: the dealt tile residual with two-word
        # fixed-point row sums (bit-repeatable, as the reference's revert exit
        # needs); beside it the fixed-order panels (the round-3 default) and
        # the float-atomic tiles (opt-in, not bit-repeatable)
        out['xspace_bb'] = bench_xspace(sh3, b3)
        out['xspace_bb_panels'] = bench_xspace(sh3, b3, k1='panels')
        out['xspace_bb_tiles'] = bench_xspace(sh3, b3, k1='tiles')
        torch.cuda.empty_cache()
    if 'md' in legs:
        out['mirror_descent'] = bench_md(sh3, b3)
    if 'dore' in legs:
        out['dore'] = bench_dore(sh3, b3)
    if 'lbfgs' in legs:
        out['lbfgs'] = bench_lbfgs(sh3, b3)
    if 'gdlbfgs' in legs:
        out['lbfgs_solve'] = bench_gd_lbfgs(sh3, b3)
        torch.cuda.empty_cache()
    if 'c1' in legs:
        out['c1_cpu_path'] = bench_c1()
    log('extras done')
    if 'cpu' in legs:
        cps, cit, cel = cpu_baseline_bb(sh3['A'], b3, sh3['block_sizes'])
        aps, ait, ael = cpu_baseline_bb_omp(sh3['A'], b3, sh3['block_sizes'], HOST_THREADS)
        out['cpu_baseline'] = {
            'value': cps, 'unit': 'BB it/s (C3)', 'cores': 1, 'kind': 'port',
            'sample': '%d BB iterations (%.1f s) of the C3 problem: oracle restatement of '
                      'BB.py over SciPy csr_matvec + C PAVA' % (cit, cel),
            'host': host_info(1),
            'all_cores': {'value': aps, 'unit': 'BB it/s (C3)', 'cores': HOST_THREADS,
                          'kind': 'port',
                          'sample': '%d BB iterations (%.1f s) of the C3 problem: the BB '
                                    'loop in C + OpenMP (oracle/bsls_cpu_bb.c)' % (ait, ael),
                          'host': host_info(HOST_THREADS)}}
        log('CPU baseline done')
    if 'rccl1' in legs:
        # (an extra of the N = 1 line: a failure here is reported in the line,
        # it does not take the measured legs with it)
        try:
            out['rccl_forced_selfcheck'] = rccl_forced_selfcheck()
        except Exception as exc:
            out['rccl_forced_selfcheck'] = {'ok': False, 'error': repr(exc)[:400]}
        log('RCCL one-rank self-check done')


def rccl_forced_selfcheck():
    """The N > 1 self-check's problem through RcclComm + bsls_bb_shard_iterate
    on a one-rank nccl group with the collectives forced on (every
    ncclAllReduce of the shipped loop runs: the five-sum in doubles, the r
    exchange in int64 words), z against the oracle -- the RCCL transport
    exercised on the one-GPU box, outside every timed region."""
    import torch
    import torch.distributed as dist
    for k, v in (('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29547')):
        os.environ.setdefault(k, v)
    with _StdoutToStderr():
        dist.init_process_group('nccl', rank=0, world_size=1,
                                device_id=torch.device('cuda', torch.cuda.current_device()))
    try:
        res = selfcheck_sharded(1, 0, dist, force=True)
    finally:
        dist.destroy_process_group()
    return res


if __name__ == '__main__':
    main()
