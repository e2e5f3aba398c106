"""Driver for tools/proj_ubench.hip on the C2 input (GPU box):
python tools/proj_ubench.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    from synthetic import proj_input
    lib = ctypes.CDLL(os.path.join(ROOT, 'build', 'libproj_ubench.so'))
    lib.proj_ubench.restype = ctypes.c_float
    lib.proj_ubench.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int64, ctypes.c_int]
    names = ['full', 'no sort', 'no lambda', 'LDS stage only', 'regs in/out only',
             'full, unpredicated LDS loads', 'transposed LDS', 'transposed + early-stop lambda',
             'T batched staging + early stop', 'T batched + early stop (Mx bound)',
             'T batched staging only', '2-instr CE', '+ pruned flip network',
             '+ early-stop lambda', '+ early-stop lambda v2', 'product kernel']
    lib.proj_ubench_once.argtypes = lib.proj_ubench.argtypes[:-1]
    ref = None
    kinds = ('unif',) if os.environ.get('PROJ_UB_VARIANTS') else ('unif', 'normal')
    for kind in kinds:
        y_h, st_h = proj_input(kind=kind)
        st = torch.from_numpy(st_h).cuda()
        print(kind)
        sel = os.environ.get('PROJ_UB_VARIANTS')
        for v, nm in enumerate(names):
            if sel and str(v) not in sel.split(','):
                continue
            y = torch.from_numpy(y_h).cuda()
            lib.proj_ubench_once(v, y.data_ptr(), st.data_ptr(), len(st_h), len(y_h))
            out = y.cpu().numpy()
            if v == 0:
                ref = out
            same = np.array_equal(out.view(np.int64), ref.view(np.int64))
            us = lib.proj_ubench(v, y.data_ptr(), st.data_ptr(), len(st_h), len(y_h), 20)
            print('  V%d %-32s %8.1f us  same-as-V0 %s' % (v, nm, us, same))


if __name__ == '__main__':
    main()
