"""Does a HIP graph shorten the fused BB iteration?  Captures `k` iterations
of bsls_bb_iterate (an even count, so the z/g ping-pong parity is the same
after every replay) with torch.cuda.CUDAGraph and replays them, against the
same iterations enqueued eagerly.  Timing probe only (the captured iteration
numbers repeat, so scal[ITER] is not meaningful).  python tools/graph_probe.py"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', default='C3')
    ap.add_argument('--k', type=int, default=10)
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch
    from synthetic import make_shard, make_partitioned, add_noise, CONFIGS, SEED
    from device import BBEngine
    c = CONFIGS[args.shape]
    if args.shape == 'C5':
        sh = make_partitioned(c['n'], c['p'], c['m'], c['per_col'], rank=0, world=1)
    else:
        sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 10 ** 12, 'opt_tol': 1e-30},
                   early_exit=False, AT=sh['AT'], colv=sh.get('colv'))
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    eng.prologue()
    eng.iterate(1, 20)
    torch.cuda.synchronize()
    k = args.k
    t0 = time.perf_counter()
    for r in range(args.reps):
        eng.iterate(21 + k * r, k)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / (args.reps * k)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        eng.iterate(21, k)          # warm the stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            eng.iterate(21, k)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(args.reps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / (args.reps * k)
    print('%s: eager %.2f us / iteration, graph %.2f us / iteration, f finite %s'
          % (args.shape, eager * 1e6, graph * 1e6, bool(np.isfinite(eng.scalars()[4]))))


if __name__ == '__main__':
    main()
