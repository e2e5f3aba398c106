#!/usr/bin/env python
"""Benchmark: BB solver iterations/sec on the 1M-route block-LSQ problem (C3) +
proj_simplex HBM GB/s (C2), on MI355X.  One JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step = one full projected-BB iteration (python/BB.py:17-41 semantics, fused
K2 -> K3 -> K1 on the device) over the whole problem, inputs resident in HBM.
N = 1: config C3 (1M routes, 50k blocks, 100k links, 16M nnz, fp64).
N > 1 (torchrun, one rank per GPU): weak scaling -- every rank owns a C3-sized
column shard (1M routes, 50k blocks, 16M nnz) of an N x 1M-route problem on
the same 100k-link network (m stays 100k: more routes over one network, so
every rank's shard has exactly the C3 shape); per iteration one RCCL
all-reduce of the residual r (8 m = 800 kB) and one of the four BB sums.
value = N x (iterations/s of the whole job), i.e. 1M-route-equivalent BB
iterations per second.  BSLS_DIST_BACKEND=gloo rehearses the N > 1 path with
several ranks on one GPU (RCCL refuses two ranks on one device).

Early exits are disabled for timing: exactly K iterations run.
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault('OPENBLAS_NUM_THREADS', '1')   # CPU baseline = 1 thread, like the reference
ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = 'BB solver iterations/sec (1M-route block-LSQ) + proj_simplex HBM GB/s'
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
    """Bytes the kernels actually stream with the panel images (the compressed
    figure SURVEY.md §8(d) asks to state beside the general one)."""
    m, n, nz = eng.m, eng.n, eng.nz
    scale = 8 * n if eng.scaled else 0
    return {
        'K1_spmv_A': eng.A_pan.bytes() + 8 * n + 16 * m + 8 * m * (eng.A_pan.img['ngroups'] - 1) * 2,
        'K2_spmvT_Nt_dots': eng.AT_pan.bytes() + 8 * m + 4 * n + 32 * nz + scale,
        'K3_pava_clip_z2x': 24 * nz + 8 * n + 4 * eng.layout.p + scale,
    }


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


def bench_proj(reps=30, batch=16):
    """C2 proj_multi_simplex (100k blocks x mean 32, 3.2M fp64) on the device,
    every launch on fresh input.  avg_us: `batch` launches back to back on
    `batch` distinct copies of the input between two events on the launch
    stream (the stream held by a spin kernel while the host enqueues) -- the
    kernel time rocprofv3 reports, dispatch gaps amortised; isolated_*: one
    launch per event pair (adds the launch latency)."""
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import proj_input
    L = _native.lib()
    y_h, starts_h = proj_input()
    n, p = y_h.shape[0], starts_h.shape[0]
    mb = int(np.max(np.diff(np.append(starts_h, n))))
    y0 = torch.from_numpy(y_h).cuda()
    st = torch.from_numpy(starts_h).cuda()
    ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')

    def proj(t):
        check(L.bsls_proj_multi_simplex(ptr(t), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                        stream_handle()), 'proj')
    ys = [y0.clone() for _ in range(batch)]
    for t in ys[:3]:
        proj(t)
    avg = []
    for _ in range(3):
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
    us = sorted(avg)[1] * 1e3
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
    # CPU baseline for the same call: the oracle (1 thread)
    from oracle import oracle as orc
    yc = y_h.copy()
    t0 = time.perf_counter()
    orc.proj_multi_simplex_c(yc, starts_h)
    cpu_s = time.perf_counter() - t0
    ok = bool(np.array_equal(yc.view(np.int64), y.cpu().numpy().view(np.int64)))
    return {'n': n, 'blocks': p, 'avg_us': us, 'GB_s': byt / (us * 1e-6) / 1e9,
            'alg_bytes': byt, 'frac_hbm_peak': byt / (us * 1e-6) / HBM_PEAK,
            'isolated_median_us': med * 1e3, 'isolated_min_us': ms[0] * 1e3,
            'cpu_oracle_ms_1thread': cpu_s * 1e3, 'bit_exact_vs_oracle': ok}


def bench_xspace(sh, b, rounds=40, reps=5):
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
    _, proj, _, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
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
    return {'operator': 'panels' if obj.lsq is not None else 'csr',
            'rounds': rounds * reps, 'us_per_round': ms * 1e3 / (rounds * reps),
            'rounds_per_s': rounds * reps / (ms * 1e-3), 'iterations_per_s': its / (ms * 1e-3),
            'backtracks': bts, 'finite': ok}


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
    return {'operator': 'panels' if md.lsq is not None else 'csr', 'scale': 0.01,
            'iterations': iters,
            'us_per_iter': ms * 1e3 / iters, 'iterations_per_s': iters / (ms * 1e-3),
            'finite': bool(np.all(np.isfinite(x)))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--profile-iters', type=int, default=50)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    # (modulo: the gloo rehearsal puts several ranks on one GPU)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get('BSLS_DIST_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)

    from synthetic import make_shard, add_noise, SEED
    from device import BBEngine, DeviceCSR
    n_g, p_g, m_per, per_col = 1_000_000, 50_000, 100_000, 16
    m = m_per   # weak scaling over routes: the network (rows) is shared, see the docstring
    sh = make_shard(n_g, p_g, m, per_col, seed=SEED, rank=rank)
    Ax = torch.from_numpy(sh['Ax']).cuda()
    if dist:
        dist.all_reduce(Ax)
    b = add_noise(Ax.cpu().numpy(), 0.02, seed=SEED)
    opts = {'max_iter': 10 ** 12, 'opt_tol': 1e-30}
    if dist:
        from distributed import ShardedBB, torch_all_reduce
        A_dev = DeviceCSR(sh['A'])
        x0 = torch.zeros(n_g, dtype=torch.float64, device='cuda')
        x0[torch.from_numpy(np.cumsum(sh['block_sizes']) - 1).cuda()] = 1.0
        part = A_dev.matvec(x0)
        dist.all_reduce(part)
        target = part - torch.from_numpy(b).cuda()
        eng = BBEngine(sh['A'], None, sh['block_sizes'], options=opts, early_exit=False,
                       A_dev=A_dev, AT=sh['AT'], target=target)
        eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
        drv = ShardedBB(eng, torch_all_reduce())
        drv.prologue()
        run = drv.iterate
    else:
        eng = BBEngine(sh['A'], b, sh['block_sizes'], options=opts, early_exit=False,
                       AT=sh['AT'])
        eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
        eng.prologue()
        run = eng.iterate
    nnz = sh['A'].nnz
    run(1, args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(1 + args.warmup, args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    it_s = args.steps / el
    value = it_s * world
    s = eng.scalars()
    finite = bool(np.isfinite(s[4]))

    out = None
    if rank == 0:
        kb = kernel_bytes(m, n_g, eng.nz, p_g, nnz, sh['AT'].nnz)
        fb = format_bytes(eng)
        kern = {}
        if world == 1 and args.profile_iters > 0:
            # per-kernel HIP-event timing on the stream the kernels run on:
            # each stage launched profile_iters times back to back between two
            # events (the stages are idempotent for a fixed iteration index:
            # same inputs, same outputs, tickets self-resetting), after the
            # timed run.  The stream is held by a spin kernel while the host
            # enqueues, so no host gap sits inside an interval; what remains
            # beyond rocprofv3's kernel time is the dispatch gap, amortised.
            names = [(3, 'K2_spmvT_Nt_dots'), (4, 'K3_pava_clip_z2x'), (7, 'K1_spmv_A')]
            acc = {nm: [] for _, nm in names}
            it0 = 1 + args.warmup + args.steps
            for stg, nm in names:
                torch.cuda._sleep(int(2e8))
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(args.profile_iters):
                    eng.stage(stg, it0)
                ev[1].record()
                torch.cuda.synchronize()
                acc[nm].append(ev[0].elapsed_time(ev[1]) * 1e3 / args.profile_iters)
            for nm, v in acc.items():
                us = float(np.mean(v))
                kern[nm] = {'avg_us': us, 'alg_bytes': kb[nm],
                            'GB_s': kb[nm] / (us * 1e-6) / 1e9,
                            'frac': kb[nm] / (us * 1e-6) / HBM_PEAK,
                            'format_bytes': fb[nm],
                            'format_GB_s': fb[nm] / (us * 1e-6) / 1e9}
        dom = max(kern, key=lambda k: kern[k]['avg_us']) if kern else None
        traffic = None
        tfile = os.path.join(ROOT, 'profiles', 'traffic_r01.json')
        if dom and os.path.exists(tfile):
            try:
                traffic = json.load(open(tfile)).get(dom, {}).get('hbm_bytes_per_launch')
            except Exception:
                traffic = None
        roof = None
        if dom:
            roof = {'bound': 'hbm', 'kernel': dom,
                    'achieved': kern[dom]['GB_s'], 'peak': HBM_PEAK / 1e9, 'unit': 'GB/s',
                    'frac': kern[dom]['frac'], 'traffic': traffic}
        ib = survey_iter_bytes(m, n_g * world, eng.nz * world, nnz * world)
        proj = bench_proj() if world == 1 else None
        xspace = bench_xspace(sh, b) if world == 1 else None
        mdr = bench_md(sh, b) if world == 1 else None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cps, cit, cel = cpu_baseline_bb(sh['A'], b, sh['block_sizes'])
            cpu = {'value': cps, 'unit': 'BB it/s', 'cores': 1, 'kind': 'port',
                   'sample': '%d BB iterations (%.1f s) of the same C3 problem: oracle '
                             'restatement of BB.py over SciPy csr_matvec + C PAVA, '
                             'OPENBLAS_NUM_THREADS=1' % (cit, cel)}
        out = {
            'metric': METRIC, 'value': value,
            'unit': 'BB iterations/s (1M-route problem; N x 1M routes at N GPUs)',
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': el / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'workload': 'C3: BB (z-space, PAVA projection) on 1M routes / 50k '
                                   'blocks / %d links / %d nnz per GPU' % (m, nnz),
                       'routes_per_gpu': n_g, 'blocks_per_gpu': p_g, 'links': m,
                       'nnz_per_gpu': nnz, 'parallelism': 'column-shard x%d' % world},
            'roofline': roof,
            'iteration_roofline': {'survey_bytes_per_iter': ib,
                                   'achieved_GB_s': ib * it_s / 1e9,
                                   'frac': ib * it_s / HBM_PEAK},
            'kernels': kern, 'proj_simplex': proj, 'xspace_bb': xspace, 'mirror_descent': mdr,
            'cpu_baseline': cpu,
            'finite': finite,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
