#!/usr/bin/env python
"""Exit iteration of main.main (python/main.py) on the three tests/fast
test_main.py problems: the reference's (tests/golden/solvers.npz), the default
engine's and the fixed-order engine's (--deterministic), twice each -- to size
the band tests/test_gpu_plugins.py::test_main_end_to_end pins."""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'block-simplex-least-squares_amd')]

import numpy as np  # noqa: E402

SEED = 237423433


def main():
    import bsls_utils
    import main as bmain
    G = np.load(os.path.join(ROOT, 'tests', 'golden', 'solvers.npz'))
    for vi, kw in enumerate([{}, {'alpha': 0.5}, {'A_sparse': 0.05}]):
        row = {'ref': int(G['main%d_iters' % vi][-1])}
        for det in (False, True):
            for rep in range(2):
                np.random.seed(SEED)
                with tempfile.TemporaryDirectory() as d:
                    fname = os.path.join(d, 'test_main.mat')
                    bsls_utils.generate_data(fname=fname, **kw)
                    args = argparse.Namespace(noise=0, file=fname, log='WARN', init=False,
                                              eq='CP', method='BB', deterministic=det)
                    iters, _, _, out = bmain.main(args=args)
                row['%s%d' % ('det' if det else 'dealt', rep)] = int(iters[-1])
        print(vi, row, flush=True)


if __name__ == '__main__':
    main()
