#!/usr/bin/env python
"""Trace the fused x-space BB engine (csrc/xbb.hip) round by round on the C3
problem: mode, iteration, f, t, backtracks -- to see where a long run
(prog_tol < 0, no early stop) leaves the finite range, and time rounds on the
CSR and panel operators."""
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
    ap.add_argument('--rounds', type=int, default=80)
    ap.add_argument('--panels', type=int, default=1)
    args = ap.parse_args()
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    from algorithm_utils import get_solver_parts, SparseLSQ
    from device import XBBEngine
    import _native
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02)
    sizes = sh['block_sizes']
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    x0 = np.repeat(1.0 / sizes, sizes)
    SparseLSQ.PANEL_MIN_NNZ = 0 if args.panels else 1 << 62
    _, proj, _, obj = get_solver_parts((sh['A'], b), starts, 1.0, is_sparse=True)
    eng = XBBEngine(obj, proj)
    eng.start(x0, max_iter=10 ** 12, prog_tol=-1.0, hist_cap=1)
    names = ['MODE', 'ITER', 'F', 'FOLD', 'T', 'TT', 'REVERT', 'GD', 'DXDG', 'DGDG', 'STEPINF',
             'SQ', 'STOP', 'ROUNDS', 'BACKTRACKS']
    for k in range(args.rounds):
        eng.rounds(1)
        s = eng.scalars()
        print(k, ' '.join('%s=%.6g' % (nm, s[i]) for i, nm in enumerate(names)), flush=True)
        if not np.isfinite(s[_native.XS_F]):
            break
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.rounds(50)
    ev[1].record()
    torch.cuda.synchronize()
    print('us/round (50 rounds):', ev[0].elapsed_time(ev[1]) * 1e3 / 50, flush=True)


if __name__ == '__main__':
    main()
