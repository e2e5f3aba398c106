"""Driver for tools/panel_ubench.hip: K2-loop variants on the C3 A' panel image.
Usage (GPU box): python tools/panel_ubench.py"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    import torch
    import device
    import _native
    from synthetic import make_shard
    sh = make_shard(1_000_000, 50_000, 100_000, per_col=16, seed=1)
    AT = sh['AT']
    colv = device.scaled_incidence_scale(sh['A'])
    lib = ctypes.CDLL(os.path.join(ROOT, 'build', 'libpanel_ubench.so'))
    lib.panel_ubench.restype = ctypes.c_float
    lib.panel_ubench.argtypes = [ctypes.c_int, ctypes.POINTER(_native.Panels), ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    r = torch.from_numpy(np.random.RandomState(0).randn(AT.shape[1])).cuda()
    cv = torch.from_numpy(colv).cuda()
    out = torch.zeros(AT.shape[0], dtype=torch.float64, device='cuda')
    want = AT.dot(r.cpu().numpy())
    prow = device.panel_rows(AT.shape[0], 256)
    for dma in (True,):
        pan = device.DevicePanels(AT, prow, True, 1, values=False)
        img = pan.img
        print('prow %d panels %d chunks %d tab_cap %d' % (
            prow, img['npanels'], img['nchunks'], img['tab_cap']))
        for v, nm in enumerate(['full', 'stage only']):
            out.zero_()
            us = lib.panel_ubench(v, ctypes.byref(pan.struct), r.data_ptr(), cv.data_ptr(),
                                  out.data_ptr(), args.reps)
            print('  %-12s %8.1f us' % (nm, us))
            if v == 0:
                o = out.cpu().numpy()
                bad = np.flatnonzero(o != want)
                print('     bit-exact vs SciPy:', bad.size == 0, 'mismatches', bad.size,
                      'first', bad[:5], 'max rel', float(np.max(np.abs(o - want) / (np.abs(want) + 1e-300))))
        T = torch.zeros(4096 * 64 + 4096 * 16 * 16, dtype=torch.int64, device='cuda')
        lib.panel_trace.restype = ctypes.c_int
        lib.panel_trace.argtypes = [ctypes.POINTER(_native.Panels), ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        grid = lib.panel_trace(ctypes.byref(pan.struct), r.data_ptr(), cv.data_ptr(),
                               out.data_ptr(), T.data_ptr())
        TT = T.cpu().numpy()
        t = TT[:4096 * 64].reshape(-1, 64)[:grid]
        u = TT[4096 * 64:].reshape(4096, 16, 16)[:grid]
        nch = img['nchunks']
        base = t[:, 0].min()
        us = lambda v: (v - base) / 100.0          # wall_clock64: 100 MHz
        print('  trace (us from first WG start; median over %d WGs):' % grid)
        print('    start %.2f  prologue loads issued %.2f' % (np.median(us(t[:, 0])), np.median(us(t[:, 1]))))
        for c in range(nch):
            a, b_, w = t[:, 2 + 3 * c], t[:, 3 + 3 * c], t[:, 4 + 3 * c]
            print('    chunk %d: barrierA %.2f  staged(barrierB) %.2f  walked %.2f   [stage %.2f walk %.2f]' % (
                c, np.median(us(a)), np.median(us(b_)), np.median(us(w)),
                np.median((b_ - a) / 100.0), np.median((w - b_) / 100.0)))
        print('    end %.2f   (max end %.2f)' % (np.median(us(t[:, 63])), us(t[:, 63]).max()))
        for c in range(min(nch, 5)):
            wt = u[:, :, 2 * c] / 100.0
            deep = u[:, :, 2 * c + 1] != 0
            print('    chunk %d walk us per wave: median %.2f  p90 %.2f  max-per-WG median %.2f | deep waves %.0f%%: median %.2f, shallow median %.2f' % (
                c, np.median(wt), np.percentile(wt, 90), np.median(wt.max(axis=1)), 100 * deep.mean(),
                np.median(wt[deep]) if deep.any() else 0, np.median(wt[~deep])))
        lib.panel_ko.restype = ctypes.c_float
        lib.panel_ko.argtypes = lib.panel_ubench.argtypes
        names = {1: 'no gathers', 2: 'no entry loads', 4: 'no count loads', 8: 'no staging'}
        for ko in (0, 1, 2, 3, 4, 7, 8, 9, 10, 11, 15):
            us = lib.panel_ko(ko, ctypes.byref(pan.struct), r.data_ptr(), cv.data_ptr(),
                              out.data_ptr(), args.reps)
            print('  KO %2d %-40s %8.1f us' % (ko, ', '.join(v for b, v in names.items() if ko & b)
                                              or 'copy of full', us))


if __name__ == '__main__':
    main()
