"""Driver for tools/proj_ko.hip (GPU box): python tools/proj_ko.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    from synthetic import proj_input
    lib = ctypes.CDLL(os.path.join(ROOT, 'build', 'libproj_ko.so'))
    lib.proj_ko.restype = ctypes.c_float
    lib.proj_ko.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 2
    names = {0: 'full', 1: 'no network', 2: 'no chain', 3: 'no network, no chain',
             4: 'no fallback sort', 7: 'no network/chain/fallback', 8: 'conflict-free LDS idx',
             12: 'conflict-free + no fallback', 16: 'no output pass',
             23: 'only load loop', 32: 'no HBM staging', 36: 'no staging, no fallback',
             55: 'no staging, only load loop', 64: 'x4 plain stores', 128: 'x4 sc1 stores',
             87: 'x4 plain, only load loop', 151: 'x4 sc1, only load loop',
             384: 'x4 sc1 + nt loads', 407: 'x4 sc1 + nt, only load loop',
             512: 'empty (metadata only)', 2048: 'empty kernel (1563 WGs)', 4096: 'empty 1 WG (20KB LDS)', 8192: 'empty 391 WGs x256 (80KB)',
             12288: 'empty 1563 WGs no LDS', 16384: 'empty 1563 WGs 20KB', 1536: 'streaming copy x4 sc1'}
    for kind in ('unif',):
        y_h, st_h = proj_input(kind=kind)
        y0 = torch.from_numpy(y_h).cuda()
        y = y0.clone()
        st = torch.from_numpy(st_h).cuda()
        print(kind, flush=True)
        for v, nm in names.items():
            us = lib.proj_ko(v, y.data_ptr(), y0.data_ptr(), st.data_ptr(), len(st_h), len(y_h))
            print('  KO%-3d %-30s %7.1f us' % (v, nm, us), flush=True)


if __name__ == '__main__':
    main()
