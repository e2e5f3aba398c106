"""The reference's stress shapes on the device vs the CPU oracle (GPU box):
python/experiments/test_stress_proj_simplex.py:24-44 (single U[0,1) blocks of
1e3..1e6; 1e6 elements in 10..1e4 random blocks) and
python/experiments/PAVA_worst_case.py:12-40 (PAVA on the log-trend data of
1e1..1e6 and on its worst case, arange with y[-1] = -1e12, up to 1e5; here
variant 1, main.py's).  Every device result is checked bit for bit against
the oracle.  python tools/stress_time.py [--max 1000000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def dev_time(fn, y, reps=3):
    import torch
    best = None
    out = None
    for _ in range(reps):
        yd = torch.from_numpy(y.copy()).cuda()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(yd)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
        out = yd
    return best, out.cpu().numpy()


def cpu_time(fn, y):
    yc = y.copy()
    t0 = time.perf_counter()
    fn(yc)
    return time.perf_counter() - t0, yc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--max', type=int, default=1_000_000)
    ap.add_argument('--what', default='proj,multi,pava,worst')
    ap.add_argument('--worst-max', type=int, default=10000)
    args = ap.parse_args()
    import torch
    from c_extensions import c_extensions as cx
    from oracle import oracle as orc
    SEED = 237423433
    res = []

    def rec(kind, size, fn_dev, fn_cpu, y):
        gt, gy = dev_time(fn_dev, y)
        ct, cy = cpu_time(fn_cpu, y)
        ok = bool(np.array_equal(gy.view(np.int64), cy.view(np.int64)))
        r = {'kind': kind, 'size': size, 'gpu_ms': gt * 1e3, 'cpu_oracle_ms': ct * 1e3,
             'bit_exact': ok}
        res.append(r)
        print(json.dumps(r), flush=True)

    what = args.what.split(',')
    if 'proj' in what:
        np.random.seed(SEED)
        for n in (1000, 10000, 100000, 1000000):
            if n > args.max:
                break
            y = np.random.rand(n)
            rec('proj_single', n, lambda t: cx.proj_simplex_c(t, 0, t.shape[0]),
                lambda a: orc.proj_simplex_c(a, 0, a.shape[0]), y)
    if 'multi' in what:
        np.random.seed(SEED)
        for nb in (10, 100, 1000, 10000):
            y = np.random.rand(args.max)
            blocks = np.sort(np.random.choice(args.max, nb, replace=False)).astype(np.int64)
            bd = torch.from_numpy(blocks).cuda()
            rec('proj_multi_%d' % nb, args.max, lambda t: cx.proj_multi_simplex_c(t, bd),
                lambda a: orc.proj_multi_simplex_c(a, blocks), y)
    if 'pava' in what:
        rs = np.random.RandomState(0)
        for n in (10, 100, 1000, 10000, 100000, 1000000):
            if n > args.max:
                break
            y = rs.randint(-50, 50, size=(n,)) + 50. * np.log(1 + np.arange(n))
            rec('pava_log', n, lambda t: cx.isotonic_regression_c(t, 0, t.shape[0]),
                lambda a: orc.isotonic_regression_c(a, 0, a.shape[0]), y)
    if 'worst' in what:
        for n in (10, 100, 1000, 10000):
            if n > args.worst_max:
                break
            y = np.arange(n).astype(float)
            y[-1] = -1e12
            rec('pava_worst', n, lambda t: cx.isotonic_regression_c(t, 0, t.shape[0]),
                lambda a: orc.isotonic_regression_c(a, 0, a.shape[0]), y)
    print(json.dumps({'results': res}))


if __name__ == '__main__':
    main()
