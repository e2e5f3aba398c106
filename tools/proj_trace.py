"""Driver for tools/proj_trace.hip on the C2 input (GPU box): per-wave phase
times and how the waves' phases overlap.  python tools/proj_trace.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    from synthetic import proj_input
    lib = ctypes.CDLL(os.path.join(ROOT, 'build', 'libproj_trace.so'))
    lib.proj_trace.restype = ctypes.c_float
    lib.proj_trace.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 2 + [ctypes.c_void_p]
    y_h, st_h = proj_input(kind=os.environ.get('PROJ_KIND', 'unif'))
    y0 = torch.from_numpy(y_h).cuda()
    y = y0.clone()
    st = torch.from_numpy(st_h).cuda()
    nw = (len(st_h) + 63) // 64
    tr = torch.zeros(nw * 8, dtype=torch.int64, device='cuda')
    us = lib.proj_trace(y.data_ptr(), y0.data_ptr(), st.data_ptr(), len(st_h), len(y_h), tr.data_ptr())
    t = tr.cpu().numpy().reshape(nw, 8)
    T = t[:, :5].astype(np.float64) * 0.01     # 100 MHz ticks -> us
    T -= T[:, 0].min()
    print('event time %.1f us, waves %d' % (us, nw))
    ph = np.diff(T, axis=1)
    for i, nm in enumerate(['stage-in', 'compute', 'store-issue', 'store-drain']):
        q = np.percentile(ph[:, i], [5, 50, 95, 100])
        print('  %-12s p5 %6.2f  p50 %6.2f  p95 %6.2f  max %6.2f us' % (nm, *q))
    for i, nm in enumerate(['start', 'staged', 'computed', 'stored', 'drained']):
        q = np.percentile(T[:, i], [0, 5, 50, 95, 100])
        print('  %-9s at  min %6.2f p5 %6.2f p50 %6.2f p95 %6.2f max %6.2f us' % (nm, *q))
    hw = t[:, 5]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    xcc = t[:, 6] & 0xF
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    _, cnt = np.unique(key, return_counts=True)
    print('  CUs used %d, waves per CU: %s' % (cnt.size, np.bincount(cnt)))
    key2 = key * 4 + simd
    _, c2 = np.unique(key2, return_counts=True)
    print('  waves per SIMD: %s' % np.bincount(c2))
    # concurrency profile: how many waves are in each phase over time
    grid = np.linspace(0, T[:, 4].max(), 25)
    print('  time   staging computing storing')
    for g in grid:
        a = np.sum((T[:, 0] <= g) & (T[:, 1] > g))
        b = np.sum((T[:, 1] <= g) & (T[:, 2] > g))
        c = np.sum((T[:, 2] <= g) & (T[:, 4] > g))
        print('  %6.2f %6d %6d %6d' % (g, a, b, c))


if __name__ == '__main__':
    main()
