#!/usr/bin/env python
"""Kernel-level profiling driver: build the C3 problem once, run the fused BB
kernels `--iters` times (stages 3, 4, 7 = K2, K3, K1) and optionally the C2
projection, so rocprofv3 --kernel-trace / --pmc passes see only these kernels.
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -- python3 tools/kprof.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--proj', type=int, default=20)
    ap.add_argument('--config', default='C3')
    ap.add_argument('--iso', type=int, default=0,
                    help='planned standalone PAVA calls on the C3/C4 z layout')
    args = ap.parse_args()
    from synthetic import make_shard, add_noise, proj_input, CONFIGS, SEED
    from device import BBEngine
    import _native
    from _native import ptr, stream_handle, check
    c = CONFIGS[args.config]
    if args.config == 'C5':
        from synthetic import make_partitioned
        sh = make_partitioned(c['n'], c['p'], c['m'], c['per_col'], rank=0, world=1)
    else:
        sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 10 ** 9, 'opt_tol': 1e-30},
                   early_exit=False, AT=sh['AT'], colv=sh.get('colv'))
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    eng.prologue()
    eng.iterate(1, 5)
    for it in range(6, 6 + args.iters):
        for stg in (3, 4, 7):
            eng.stage(stg, it)
    torch.cuda.synchronize()
    if args.proj:
        L = _native.lib()
        y_h, st_h = proj_input()
        n, p = y_h.shape[0], st_h.shape[0]
        mb = int(np.max(np.diff(np.append(st_h, n))))
        y0 = torch.from_numpy(y_h).cuda()
        y = y0.clone()
        st = torch.from_numpy(st_h).cuda()
        ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')
        for _ in range(args.proj):
            y.copy_(y0)
            check(L.bsls_proj_multi_simplex(ptr(y), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                            stream_handle()), 'proj')
        for _ in range(args.proj):   # the sort-free form (proj_simplex_fast)
            y.copy_(y0)
            check(L.bsls_proj_multi_simplex_fast(ptr(y), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                                 stream_handle()), 'proj fast')
        torch.cuda.synchronize()
    if args.iso:
        from device import iso_plan
        c3 = CONFIGS['C3']
        rs = np.random.RandomState(SEED)
        sizes = rs.multinomial(c3['n'] - c3['p'], np.ones(c3['p']) / c3['p']) + 1
        zs = np.concatenate(([0], np.cumsum(sizes - 1)[:-1])).astype(np.int64)
        nz = int((sizes - 1).sum())
        y0 = torch.from_numpy(rs.rand(nz) - 0.3 * rs.randn(nz)).cuda()
        y = y0.clone()
        plan = iso_plan(zs, nz)
        for _ in range(args.iso):
            y.copy_(y0)
            plan.apply(y)
        torch.cuda.synchronize()
    print('kprof done', eng.scalars()[:5])


if __name__ == '__main__':
    main()
