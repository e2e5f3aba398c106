"""Per-stage timing of the fused BB engine on C3 (GPU box), as bench.py does
it: each stage launched `--reps` times back to back between two events on
the engine's stream (held by a spin kernel while enqueuing); then `--iters`
full iterations.  python tools/stage_time.py"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--shape', type=str, default='C3',
                    help="C3, C5, or 'n,p,m' (e.g. a C5 shard: 1250000,62500,1000000)")
    ap.add_argument('--world', type=int, default=1, help='C5: time rank --rank of this many shards')
    ap.add_argument('--rank', type=int, default=0)
    ap.add_argument('--fmt', type=str, default=None, help='panels / tiles (default: auto)')
    args = ap.parse_args()
    import numpy as np
    import torch
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    from device import BBEngine
    if args.shape in CONFIGS:
        c = CONFIGS[args.shape]
    else:
        n, p, m = (int(v) for v in args.shape.split(','))
        c = dict(n=n, p=p, m=m, per_col=16)
    t0 = time.perf_counter()
    if args.shape == 'C5':
        from synthetic import make_partitioned
        sh = make_partitioned(c['n'], c['p'], c['m'], c['per_col'], rank=args.rank,
                              world=args.world)
        c = dict(c, n=sh['n'], p=sh['p'])
    else:
        sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    print('shape n %d p %d m %d nnz %d: generated in %.1f s' % (c['n'], c['p'], c['m'],
                                                                 sh['A'].nnz, time.perf_counter() - t0),
          flush=True)
    b = add_noise(sh['Ax'], 0.02)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 10 ** 12, 'opt_tol': 1e-30},
                   early_exit=False, AT=sh['AT'], colv=sh.get('colv'), fmt=args.fmt)
    print('formats: K1 %s, K2 %s' % (eng.fmt_A, eng.fmt_AT), flush=True)
    for nm, t in (('K1', eng.A_til), ('K2', eng.AT_til)):
        if t is not None:
            i = t.img
            print('  %s tiles: H %d groups %d order %d row blocks %d, %.0f MB stream'
                  % (nm, i['H'], i['ngroups'], i['order'], i['nrb'], t.bytes() / 1e6), flush=True)
    print('engine built in %.1f s' % (time.perf_counter() - t0), flush=True)
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    eng.prologue()
    eng.iterate(1, 20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(21, args.iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print('iteration: %.2f us  (%.0f it/s)  f finite %s' % (el / args.iters * 1e6, args.iters / el,
                                                         bool(np.isfinite(eng.scalars()[4]))))
    it0 = 21 + args.iters
    for stg, nm in ((3, 'K2'), (4, 'K3'), (7, 'K1')):
        torch.cuda._sleep(int(2e8))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(args.reps):
            eng.stage(stg, it0)
        ev[1].record()
        torch.cuda.synchronize()
        print('%s: %.2f us' % (nm, ev[0].elapsed_time(ev[1]) * 1e3 / args.reps), flush=True)


if __name__ == '__main__':
    main()
