#!/usr/bin/env python
"""Per-rank compute of the weak-scaling bench, emulated on ONE GPU.

bench.py --gpus W gives every rank a 1M-route column shard of a W x 1M-route
problem whose m = W x 100k rows are shared.  The rank's kernels then see a
longer residual (K2 stages r in LDS chunks; K1 writes m partial rows).  This
tool builds rank 0's shard for each W, runs the fused single-GPU iteration on
it and times each stage with HIP events, so the compute side of the N-GPU
iteration can be measured without N GPUs (the all-reduces are not included).

    python tools/shard_scaling.py --worlds 1 2 4 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def time_stage(eng, stg, it, reps):
    torch.cuda._sleep(int(1e8))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        eng.stage(stg, it)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--worlds', type=int, nargs='+', default=[1, 2, 4, 8])
    ap.add_argument('--iters', type=int, default=100)
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--c5', action='store_true',
                    help='rank 0 of C5 (10M routes, 500k blocks, m = 1M) split W ways '
                         '(strong scaling) instead of the weak-scaling shard')
    ap.add_argument('--fixed-m', action='store_true',
                    help='weak scaling with m fixed at 100k (bench.py N > 1 shape)')
    args = ap.parse_args()
    from synthetic import make_shard, add_noise, SEED
    from device import BBEngine
    out = []
    for W in args.worlds:
        t0 = time.time()
        if args.c5:
            sh = make_shard(10_000_000 // W, 500_000 // W, 1_000_000, 16, seed=SEED, rank=0)
        else:
            sh = make_shard(1_000_000, 50_000, 100_000 * (1 if args.fixed_m else W), 16,
                            seed=SEED, rank=0)
        b = add_noise(sh['Ax'], 0.02)
        eng = BBEngine(sh['A'], b, sh['block_sizes'],
                       options={'max_iter': 10 ** 12, 'opt_tol': 1e-30},
                       early_exit=False, AT=sh['AT'])
        eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
        eng.prologue()
        eng.iterate(1, 10)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        eng.iterate(11, args.iters)
        ev[1].record()
        torch.cuda.synchronize()
        us_it = ev[0].elapsed_time(ev[1]) * 1e3 / args.iters
        it0 = 11 + args.iters
        st = {nm: time_stage(eng, k, it0, args.reps)
              for k, nm in ((3, 'K2'), (4, 'K3'), (7, 'K1'))}
        rec = {'world': W, 'm': eng.m, 'n': eng.n, 'nnz': int(sh['A'].nnz), 'us_per_iter': us_it, 'stages_us': st,
               'K1_chunks': int(eng.A_pan.img['nchunks']),
               'K2_chunks': int(eng.AT_pan.img['nchunks']),
               'setup_s': time.time() - t0}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del eng
        torch.cuda.empty_cache()
    return out


if __name__ == '__main__':
    main()
