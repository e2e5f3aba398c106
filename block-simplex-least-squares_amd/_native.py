"""Loader for the gfx950 C-ABI library lib/libbsls_hip.so (include/bsls_hip.h).

There is deliberately no CPU fallback: every compute entry point of this
package goes through this library on a HIP device, and `lib()` raises if the
library is missing or no device is present.  (Loading the .so itself works
without a GPU, which is what the CPU test-suite checks.)
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# BSLS_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get('BSLS_LIB') or os.path.join(HERE, 'lib', 'libbsls_hip.so')
CSRC = os.path.join(HERE, 'csrc')
HEADER = os.path.join(os.path.dirname(HERE), 'include', 'bsls_hip.h')

BSLS_OK = 0
BSLS_E_ARG = -1
BSLS_E_WORKSPACE = -2
BSLS_E_COMM = -100

# scal[] slots and stop reasons (include/bsls_hip.h)
S_STOP, S_ITER, S_ZBUF, S_T, S_FX, S_SUMDG, S_DZDG, S_DGDG, S_GG, S_RR, S_WARN = range(11)
S_DD = 15
S_PSUMDG = 11    # .. 14: stage 10's copy of iteration i - 1's four sums
S_COUNT = 16
STOP_NOCHANGE, STOP_MAXITER, STOP_GRAD, STOP_DG = 1, 2, 3, 4
STOP_TEXT = {STOP_NOCHANGE: 'Exiting... no change in gradient',
             STOP_MAXITER: 'max_iter',
             STOP_GRAD: 'Exiting... norm(grad) too small',
             STOP_DG: 'Exiting... no change in gradient'}

_vp = ctypes.c_void_p
# bsls_all_reduce_fn (include/bsls_hip.h): (d_buf, count, stream, user) -> 0 / error
ALL_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                 ctypes.c_void_p)
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_dbl = ctypes.c_double
_sz = ctypes.c_size_t
_int = ctypes.c_int


PANEL_CHUNK = 20224      # BSLS_PANEL_CHUNK
PANEL_ROWS = 255         # BSLS_PANEL_ROWS
PANEL_WAVES = 16         # BSLS_PANEL_WAVES


class Panels(ctypes.Structure):
    """Mirror of struct bsls_panels (include/bsls_hip.h)."""
    _fields_ = [('rows', _i64), ('cols', _i64), ('prow', _i64), ('halo', _i64),
                ('npanels', _i64), ('nchunks', _i64), ('ngroups', _i64), ('tab_cap', _i64),
                ('chunk_col', _vp), ('group_chunk', _vp), ('ent_off', _vp), ('cnt_off', _vp),
                ('seg_info', _vp), ('cnt', _vp), ('ent', _vp), ('val', _vp)]


TILE_THREADS = 1024       # BSLS_TILE_THREADS
TILE_MAXSLOTS = 20        # BSLS_TILE_MAXSLOTS
TILE_LDS_BYTES = 163840 - 512   # dynamic LDS a tile kernel may take (bb.hip PANEL_LDS_MAX)
TILE_NT = 0x100                  # bsls_tiles.layout flag BSLS_TILE_NT
TILE_VAL32, TILE_VAL16 = 0x200, 0x400   # BSLS_TILE_VAL32 / VAL16


class Tiles(ctypes.Structure):
    """Mirror of struct bsls_tiles (include/bsls_hip.h)."""
    _fields_ = [('rows', _i64), ('cols', _i64), ('H', _i64), ('halo', _i64), ('nrb', _i64),
                ('ngroups', _i64), ('order', _i64), ('nquads', _i64), ('group_col', _vp),
                ('wave_off', _vp), ('ent', _vp), ('val', _vp), ('layout', _i64),
                ('base', _vp)]


class BBProblem(ctypes.Structure):
    """Mirror of struct bsls_bb_problem (include/bsls_hip.h)."""
    _fields_ = [('m', _i64), ('n', _i64), ('nz', _i64), ('nblocks', _i64),
                ('A', Panels), ('AT', Panels), ('colv', _vp), ('rpart', _vp),
                ('target', _vp), ('xstarts', _vp), ('zstarts', _vp), ('xz', _vp),
                ('pk_z0', _vp), ('pk_b0', _vp), ('pk_mask', _vp), ('pk_len', _vp),
                ('npacks', _i64),
                ('z', _vp * 2), ('g', _vp * 2), ('x', _vp), ('r', _vp), ('scal', _vp),
                ('work', _vp),
                ('max_zblock', _i64), ('max_iter', _i64), ('opt_tol', _dbl),
                ('early_exit', _i32), ('shard_role', _i32),
                ('At', Tiles), ('ATt', Tiles), ('wpart', _vp), ('work_bytes', _sz),
                ('long_packs', _vp), ('nlong', _i64), ('long_off', _vp), ('long_scratch', _vp),
                ('colv_n', _vp), ('colv_codec', _i64), ('rr_lo', _i64), ('rr_hi', _i64),
                ('pava_warm', _i64), ('k1_atomic', _i64), ('k3_merge', _i64), ('r_fx', _dbl),
                ('sy_dr', _i64)]


class DoreState(ctypes.Structure):
    """Mirror of struct bsls_dore_state (include/bsls_hip.h)."""
    _fields_ = [('X', _vp * 3), ('X1', _vp), ('D', _vp), ('X2', _vp), ('AX', _vp * 3),
                ('AX2', _vp), ('err', _vp), ('b', _vp), ('S', _vp), ('S2', _vp), ('dsc', _vp),
                ('part', _vp), ('tickets', _vp), ('scale', _dbl), ('eps', _dbl)]


DORE_NC, DORE_EE, DORE_A1, DORE_A2, DORE_SEL, DORE_STOPIT = range(6)
DORE_COUNT = 16


class LsState(ctypes.Structure):
    """Mirror of bsls_ls_state (include/bsls_hip.h): LBFGS.solve's line search."""
    _fields_ = [('x', _vp), ('d', _vp), ('gx', _vp), ('pt', _vp), ('gpt', _vp), ('zero', _vp),
                ('fx', _vp), ('st', _vp), ('S1', _vp), ('S2', _vp), ('part', _vp),
                ('tickets', _vp), ('c1', _dbl), ('c2', _dbl)]


(LS_T, LS_LO, LS_HI, LS_STOP, LS_SLOPE, LS_FX, LS_DNORM, LS_NTRIAL, LS_TLAST, LS_FT, LS_DGT,
 LS_YS, LS_GG, LS_DONE) = range(14)
LS_COUNT = 16
LS_ACCEPTED, LS_BRACKET, LS_SMALL = 1, 2, 3


class CSR(ctypes.Structure):
    """Mirror of struct bsls_csr (include/bsls_hip.h)."""
    _fields_ = [('rows', _i64), ('indptr', _vp), ('indices', _vp), ('data', _vp),
                ('tiles', _vp), ('ntiles', _i64), ('group', _i64)]


class LsqOp(ctypes.Structure):
    """Mirror of struct bsls_lsq_op (include/bsls_hip.h)."""
    _fields_ = [('m', _i64), ('n', _i64), ('A', Panels), ('AT', Panels), ('colv', _vp),
                ('rpart', _vp), ('xs', _vp), ('work', _vp), ('work_bytes', _sz),
                ('At', Tiles), ('ATt', Tiles), ('fixed', _i64), ('fx_amax', _dbl), ('x_bound', _dbl)]


class XBBProblem(ctypes.Structure):
    """Mirror of struct bsls_xbb_problem (include/bsls_hip.h)."""
    _fields_ = [('m', _i64), ('n', _i64), ('nblocks', _i64), ('max_block', _i64),
                ('ball', _i64), ('A', CSR), ('AT', CSR), ('neg_b', _vp), ('starts', _vp),
                ('x', _vp), ('g', _vp), ('xn', _vp), ('gn', _vp), ('r', _vp), ('scal', _vp),
                ('hist', _vp), ('hist_cap', _i64), ('proj_work', _vp), ('proj_work_bytes', _sz),
                ('work', _vp), ('work_bytes', _sz), ('max_iter', _i64), ('opt_tol', _dbl),
                ('prog_tol', _dbl), ('f_min', _dbl), ('has_fmin', _i64),
                ('lsq', ctypes.POINTER(LsqOp)), ('lbfgs', _i64), ('s', _vp), ('y', _vp),
                ('lb', _vp)]


# x-space engine scal[] slots / modes / stop reasons (include/bsls_hip.h)
(XS_MODE, XS_ITER, XS_F, XS_FOLD, XS_T, XS_TT, XS_REVERT, XS_GD, XS_DXDG, XS_DGDG, XS_STEPINF,
 XS_SQ, XS_STOP, XS_ROUNDS, XS_BACKTRACKS) = range(15)
XS_COUNT = 16
XM_INIT, XM_STEP, XM_BACKTRACK, XM_STOPPED = range(4)
XSTOP_MAXITER, XSTOP_OPT, XSTOP_PROG = 1, 2, 3


_SIGS = {
    'bsls_proj_workspace_size': (_sz, [_i64, _i64, _i64]),
    'bsls_proj_multi_simplex': (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _sz, _vp]),
    'bsls_proj_multi_ball': (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _sz, _vp]),
    'bsls_proj_multi_simplex_fast': (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _sz, _vp]),
    'bsls_proj_multi_ball_fast': (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _sz, _vp]),
    'bsls_isotonic_workspace_size': (_sz, [_i64]),
    'bsls_isotonic_multi': (_int, [_int, _vp, _vp, _i64, _i64, _vp, _int, _i64, _vp, _sz, _vp,
                                   _vp]),
    'bsls_isotonic_pack_plan': (_i64, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64]),
    'bsls_isotonic_packs': (_int, [_vp, _vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _sz, _vp]),
    'bsls_x2z': (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    'bsls_z2x': (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    'bsls_n_apply': (_int, [_vp, _vp, _vp, _i64, _i64, _int, _vp]),
    'bsls_nt_apply': (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    'bsls_lsq_workspace_size': (_sz, [_i64, _i64]),
    'bsls_lsq_residual': (_int, [ctypes.POINTER(LsqOp), _vp, _vp, _vp, _vp, _vp]),
    'bsls_lsq_gradient': (_int, [ctypes.POINTER(LsqOp), _vp, _vp, _vp]),
    'bsls_xbb_workspace_size': (_sz, [_i64, _i64, _i64, _i64]),
    'bsls_xbb_lbfgs_size': (_sz, [_i64]),
    'bsls_xbb_init': (_int, [ctypes.POINTER(XBBProblem), _vp]),
    'bsls_xbb_rounds': (_int, [ctypes.POINTER(XBBProblem), _i64, _vp]),
    'bsls_md_step': (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _dbl, _vp]),
    'bsls_multi_dot_workspace_size': (_sz, [_i64, _i64]),
    'bsls_multi_dot': (_int, [_vp, _int, _vp, _int, _i64, _vp, _vp, _sz, _vp]),
    'bsls_multi_axpy': (_int, [_vp, _int, _vp, _i64, _vp, _vp]),
    'bsls_lbfgs_state_size': (_sz, [_i64]),
    'bsls_lbfgs_coef': (_int, [_i64, _i64, _vp, _vp, _vp]),
    'bsls_lbfgs_push': (_int, [_i64, _i64, _dbl, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    'bsls_quad_obj': (_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    'bsls_line_search': (_int, [_vp, _dbl, _vp, _vp, _dbl, _vp, _vp, _vp, _i64, _vp, _vp]),
    'bsls_csr_plan_tiles': (_i64, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64]),
    'bsls_spmv_workspace_size': (_sz, [_i64]),
    'bsls_csr_spmv': (_int, [_i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _dbl, _vp, _vp, _int, _vp,
                             _sz, _vp]),
    'bsls_bb_workspace_size': (_sz, [_i64, _i64, _i64]),
    'bsls_bb_dz_offset': (_sz, [_i64, _i64, _i64]),
    'bsls_bb_long_scratch_size': (_sz, [_i64]),
    'bsls_bb_prologue': (_int, [ctypes.POINTER(BBProblem), _vp]),
    'bsls_bb_iterate': (_int, [ctypes.POINTER(BBProblem), _i64, _i64, _vp]),
    'bsls_dore_work_size': (_sz, [_i64, _i64]),
    'bsls_ticket_bytes': (_sz, []),
    'bsls_dore_iterate': (_int, [ctypes.POINTER(BBProblem), ctypes.POINTER(DoreState), _i64,
                                 _i64, _vp]),
    'bsls_bb_stage': (_int, [ctypes.POINTER(BBProblem), _int, _i64, _vp]),
    'bsls_lbfgs_ls_work_size': (_sz, [_i64]),
    'bsls_lbfgs_ls_begin': (_int, [ctypes.POINTER(BBProblem), ctypes.POINTER(LsState), _vp]),
    'bsls_lbfgs_ls_trials': (_int, [ctypes.POINTER(BBProblem), ctypes.POINTER(LsState), _i64,
                                    _vp]),
    'bsls_lbfgs_ls_finish': (_int, [ctypes.POINTER(BBProblem), ctypes.POINTER(LsState), _vp, _vp,
                                    _vp]),
    'bsls_comm_id_bytes': (_sz, []),
    'bsls_comm_unique_id': (_int, [_vp]),
    'bsls_comm_create': (_int, [_vp, _int, _int, ctypes.POINTER(_vp)]),
    'bsls_comm_create_callback': (_int, [_int, _int, _vp, _vp, ctypes.POINTER(_vp)]),
    'bsls_comm_destroy': (_int, [_vp]),
    'bsls_comm_all_reduce': (_int, [_vp, _vp, _i64, _vp]),
    'bsls_comm_count': (_int, [_vp, ctypes.POINTER(_int)]),
    'bsls_comm_force_collectives': (_int, [_vp, _int]),
    'bsls_bb_shard_iterate':(_int, [ctypes.POINTER(BBProblem), _vp, _i64, _i64, _int, _vp]),
    'bsls_bb_k2_part': (_int, [ctypes.POINTER(BBProblem), _i64, _int, _vp]),
    'bsls_bb_k1_rows': (_int, [ctypes.POINTER(BBProblem), _i64, _i64, _i64, _vp]),
    'bsls_bb_shard_iterate_parts': (_int, [ctypes.POINTER(BBProblem), _vp, _i64, _i64, _int, _vp,
                                           _vp, _vp]),
    'bsls_comm_create_model': (_int, [_int, _int, _dbl, _dbl, ctypes.POINTER(_vp)]),
    'bsls_bb_row_blocks': (_i64, [ctypes.POINTER(BBProblem), _vp]),
    'bsls_bb_residual_rows': (_int, [ctypes.POINTER(BBProblem), _i64, _i64, _i64, _vp]),
    'bsls_md_update_gated': (_int, [_vp, _vp, _vp, _i64, _i64, _dbl, _dbl, _i64, _vp, _vp, _sz,
                                    _vp]),
    'bsls_md_pack_workspace_size': (_sz, [_i64]),
    'bsls_md_update_packs': (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _dbl, _dbl, _i64, _vp, _vp,
                                    _sz, _vp]),
    'bsls_md_update': (_int, [_vp, _vp, _vp, _i64, _i64, _dbl, _vp, _vp, _sz, _vp]),
    'bsls_md_workspace_size': (_sz, [_i64]),
    'bsls_tiles_build': (_i64, [_i64, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp,
                                _i64]),
    'bsls_tiles_build_dealt': (_i64, [_i64, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp,
                                      _vp, _vp, _i64]),
    'bsls_tiles_build_dealt3': (_i64, [_i64, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp,
                                      _vp, _vp, _i64]),
    'bsls_version': (ctypes.c_char_p, []),
    'bsls_device_arch': (_int, [ctypes.c_char_p, _int]),
}


# ---- the host path (include/bsls_cpu.h, lib/libbsls_cpu.so) -------------------
# Selected explicitly only (BSLS_DEVICE=cpu, or set_device('cpu'); main.py
# --device cpu): BASELINE configs[0], the reference's CPU c_extensions path.
# Nothing falls back to it -- lib() still raises without a HIP device.
CPU_LIB_PATH = os.path.join(HERE, 'lib', 'libbsls_cpu.so')
CPU_HEADER = os.path.join(os.path.dirname(HERE), 'include', 'bsls_cpu.h')
_device = None

_CPU_SIGS = {
    'bsls_cpu_proj_simplex': (_int, [_vp, _i64, _i64]),
    'bsls_cpu_proj_multi_simplex': (_int, [_vp, _vp, _i64, _i64, _int]),
    'bsls_cpu_proj_multi_ball': (_int, [_vp, _vp, _i64, _i64, _int]),
    'bsls_cpu_isotonic_multi': (_int, [_int, _vp, _vp, _i64, _i64, _vp, _int, _int]),
    'bsls_cpu_quad_obj': (_dbl, [_vp, _vp, _vp, _vp, _i64]),
    'bsls_cpu_line_search': (_dbl, [_vp, _dbl, _vp, _vp, _dbl, _vp, _vp, _vp, _i64]),
    'bsls_cpu_x2z': (_int, [_vp, _vp, _vp, _i64, _i64]),
    'bsls_cpu_z2x': (_int, [_vp, _vp, _vp, _i64, _i64]),
    'bsls_cpu_version': (ctypes.c_char_p, []),
}
_cpu = None


def set_device(name):
    """'hip' (the default: every entry point on the MI355X) or 'cpu' (the
    host path of the c_extensions drop-in and the solvers' closures)."""
    global _device
    if name not in ('hip', 'cpu', None):
        raise ValueError("device must be 'hip' or 'cpu'")
    _device = name


def device_mode():
    if _device is not None:
        return _device
    d = os.environ.get('BSLS_DEVICE', 'hip').lower()
    return 'cpu' if d == 'cpu' else 'hip'


def cpu_threads():
    return int(os.environ.get('BSLS_CPU_THREADS') or os.environ.get('OMP_NUM_THREADS')
               or os.cpu_count() or 1)


def cpu_lib():
    """The host library (built with the HIP one by build())."""
    global _cpu
    if _cpu is None:
        if not os.path.exists(CPU_LIB_PATH):
            raise RuntimeError('bsls: %s is missing -- run __graft_entry__.build()'
                               % CPU_LIB_PATH)
        L = ctypes.CDLL(CPU_LIB_PATH)
        for name, (res, args) in _CPU_SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _cpu = L
    return _cpu


def declared_cpu_symbols():
    import re
    text = open(CPU_HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:double|int|const char \*)\s*(bsls_cpu_\w+)\s*\(',
                                 text, re.M)))


def build(force=False):
    """Compile csrc/*.hip for gfx950 into lib/libbsls_hip.so (hipcc via make)."""
    args = ['make', '-s', '-C', CSRC, '-j8']
    if force:
        subprocess.check_call(['make', '-s', '-C', CSRC, 'clean'])
    subprocess.check_call(args)
    return LIB_PATH


_lib = None


def load():
    """dlopen the library and bind every entry point (works without a GPU)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('bsls: %s is missing -- run __graft_entry__.build() '
                               '(or make -C %s)' % (LIB_PATH, CSRC))
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_checked_device = False


def lib():
    """The library, after checking that a HIP device is usable (raises if not)."""
    global _checked_device
    L = load()
    if not _checked_device:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError('bsls: no HIP device visible; this package has no CPU path '
                               '(the CPU oracle lives under oracle/ for tests only)')
        _checked_device = True
    return L


def check(rc, what='bsls call'):
    if rc != BSLS_OK:
        if rc == BSLS_E_ARG:
            raise ValueError('%s: invalid arguments (BSLS_E_ARG)' % what)
        if rc == BSLS_E_WORKSPACE:
            raise RuntimeError('%s: workspace too small' % what)
        raise RuntimeError('%s failed with hipError %d' % (what, rc))


def stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def pack_plan(starts, n):
    """Host pack plan of a block layout (bsls_isotonic_pack_plan, no GPU):
    dict(start, mask, len, longs) NumPy arrays -- runs of whole consecutive
    blocks with <= 64 elements, or one longer block (listed in longs)."""
    import numpy as np
    st = np.ascontiguousarray(starts, dtype=np.int64)
    L = load()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)
    nl = ctypes.c_int64(0)
    np_ = L.bsls_isotonic_pack_plan(vp(st), st.shape[0], int(n), None, None, None, None,
                                    ctypes.byref(nl), 0)
    if np_ < 0:
        raise ValueError('pack plan: invalid block starts')
    out = dict(start=np.zeros(np_, np.int64), mask=np.zeros(np_, np.int64),
               len=np.zeros(np_, np.int32), longs=np.zeros(max(nl.value, 1), np.int32))
    L.bsls_isotonic_pack_plan(vp(st), st.shape[0], int(n), vp(out['start']), vp(out['mask']),
                              vp(out['len']), vp(out['longs']), ctypes.byref(nl), np_)
    out['longs'] = out['longs'][:nl.value]
    return out


def plan_tiles(indptr, nzt=2048, rmax=1024, ends=None):
    """Row tiles for the CSR-stream kernels (bsls_csr_plan_tiles, host only)."""
    import numpy as np
    ip = np.ascontiguousarray(indptr, dtype=np.int64)
    m = ip.shape[0] - 1
    L = load()
    e = None if ends is None else np.ascontiguousarray(ends, dtype=np.int64)
    ep = ctypes.c_void_p(e.ctypes.data) if e is not None else ctypes.c_void_p(0)
    ne = 0 if e is None else e.shape[0]
    cnt = L.bsls_csr_plan_tiles(ctypes.c_void_p(ip.ctypes.data), m, nzt, rmax, ep, ne, None, 0)
    if cnt < 0:
        raise ValueError('tile planning failed (%d): a block spans more than %d rows'
                         % (cnt, rmax))
    out = np.zeros(cnt + 1, dtype=np.int64)
    L.bsls_csr_plan_tiles(ctypes.c_void_p(ip.ctypes.data), m, nzt, rmax, ep, ne,
                          ctypes.c_void_p(out.ctypes.data), cnt + 1)
    return out


def group_for_rows(mean_rows):
    """Lanes per row in the tile reduce: the largest power of two with
    G * mean_rows <= 256 (every thread of the tile busy)."""
    g = 64
    while g > 1 and g * mean_rows > 256:
        g //= 2
    return g


def declared_symbols():
    """Every function name declared in include/bsls_hip.h."""
    import re
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:size_t|int64_t|int|const char \*)\s*(bsls_\w+)\s*\(',
                                 text, re.M)))


def tiles_build(M, H, halo, group_col, values=True):
    """Host arrays of the tile image of CSR matrix M (bsls_tiles_build, host only):
    dict(wave_off, ent, val or None, nquads)."""
    import numpy as np
    ip = np.ascontiguousarray(M.indptr, dtype=np.int64)
    ix = np.ascontiguousarray(M.indices, dtype=np.int32)
    dv = np.ascontiguousarray(M.data, dtype=np.float64) if values else None
    gc = np.ascontiguousarray(group_col, dtype=np.int64)
    R, C = M.shape
    G = gc.shape[0] - 1
    L = load()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)
    nq = L.bsls_tiles_build(R, C, vp(ip), vp(ix), vp(dv), int(H), int(halo), G, vp(gc), None, None,
                            None, 0)
    if nq < 0:
        raise ValueError('tile image: invalid layout (H %d, halo %d, %d groups)' % (H, halo, G))
    nrb = -(-R // int(H))
    wo = np.zeros(nrb * G * 16 + 1, dtype=np.int64)
    ent = np.zeros(4 * nq + 256, dtype=np.uint32)
    val = np.zeros(4 * nq + 256, dtype=np.float64) if values else None
    rc = L.bsls_tiles_build(R, C, vp(ip), vp(ix), vp(dv), int(H), int(halo), G, vp(gc), vp(wo),
                            vp(ent), vp(val), nq)
    if rc != nq:
        raise RuntimeError('bsls_tiles_build failed (%d)' % rc)
    return dict(wave_off=wo, ent=ent, val=val, nquads=int(nq), nrb=nrb)


def tiles_build_dealt(M, H, halo, group_col, values=True, packed=False):
    """Host arrays of the layout-1 (dealt) tile image of CSR matrix M
    (bsls_tiles_build_dealt, host only), or with `packed` layout 2 (3-byte
    entries, bsls_tiles_build_dealt3): dict(wave_off, ent, base, val or None,
    nquads, nrb)."""
    import numpy as np
    ip = np.ascontiguousarray(M.indptr, dtype=np.int64)
    ix = np.ascontiguousarray(M.indices, dtype=np.int32)
    dv = np.ascontiguousarray(M.data, dtype=np.float64) if values else None
    gc = np.ascontiguousarray(group_col, dtype=np.int64)
    R, C = M.shape
    G = gc.shape[0] - 1
    L = load()
    vp = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)
    fn = L.bsls_tiles_build_dealt3 if packed else L.bsls_tiles_build_dealt
    nq = fn(R, C, vp(ip), vp(ix), vp(dv), int(H), int(halo), G, vp(gc), None, None, None, None, 0)
    if nq < 0:
        raise ValueError('dealt tile image: invalid layout (H %d, halo %d, %d groups)'
                         % (H, halo, G))
    nrb = -(-R // int(H))
    wo = np.zeros(nrb * G + 1, dtype=np.int64)
    ent = np.zeros((3 if packed else 4) * nq + 256, dtype=np.uint32)
    base = np.zeros(4 * nq // 64 + 64, dtype=np.int32)
    val = np.zeros(4 * nq + 256, dtype=np.float64) if values else None
    rc = fn(R, C, vp(ip), vp(ix), vp(dv), int(H), int(halo), G, vp(gc), vp(wo), vp(ent), vp(base),
            vp(val), nq)
    if rc != nq:
        raise RuntimeError('bsls_tiles_build_dealt failed (%d)' % rc)
    return dict(wave_off=wo, ent=ent, base=base, val=val, nquads=int(nq), nrb=nrb)
