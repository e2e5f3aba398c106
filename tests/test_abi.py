"""The C-ABI library loads and exports every symbol include/bsls_hip.h declares
(CPU only: dlopen needs no GPU; no compute call is made)."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def native():
    import _native
    if not os.path.exists(_native.LIB_PATH):
        _native.build()
    return _native


def test_header_declares_the_hot_path(native):
    syms = native.declared_symbols()
    for s in ('bsls_proj_multi_simplex', 'bsls_proj_multi_ball', 'bsls_isotonic_multi',
              'bsls_csr_spmv', 'bsls_bb_prologue', 'bsls_bb_iterate', 'bsls_bb_stage',
              'bsls_x2z', 'bsls_z2x', 'bsls_quad_obj', 'bsls_line_search', 'bsls_md_update'):
        assert s in syms


def test_library_exports_every_declared_symbol(native):
    L = native.load()
    missing = [s for s in native.declared_symbols() if not hasattr(L, s)]
    assert not missing
    out = subprocess.check_output(['nm', '-D', '--defined-only', native.LIB_PATH]).decode()
    exported = {ln.split()[-1] for ln in out.splitlines() if ' T ' in ln}
    assert set(native.declared_symbols()) <= exported


def test_library_is_gfx950_only(native):
    """Every device code object bundled in the library targets gfx950 (the
    rocPRIM host code the huge-block projection links carries a table of
    architecture names as data; only the offload targets count)."""
    import re
    blob = open(native.LIB_PATH, 'rb').read()
    targets = set(re.findall(rb'amdgcn-amd-amdhsa--(gfx[0-9a-z]+)', blob))
    assert targets == {b'gfx950'}, targets


def test_host_only_entry_points(native):
    L = native.load()
    assert L.bsls_version().startswith(b'bsls-hip')
    assert L.bsls_proj_workspace_size(3_200_000, 100_000, 60) > 0
    assert L.bsls_proj_workspace_size(100, 2, 50) < L.bsls_proj_workspace_size(100_000, 2, 50_000)
    assert L.bsls_isotonic_workspace_size(1000) >= 4000
    assert L.bsls_bb_workspace_size(100_000, 1_000_000, 950_000) > 4 * 950_000
    assert L.bsls_spmv_workspace_size(8000) > 8 * 8000
    assert L.bsls_md_workspace_size(50_000) > 0
    # nine 64-B ticket words (bsls_common.hpp TICKET_BYTES; DORE.py sizes its
    # ticket buffer from this, not from a literal)
    assert L.bsls_ticket_bytes() == 9 * 64


def _c_layout(tmp_path, struct, fields):
    """sizeof and offsetof as the C compiler lays the header's struct out."""
    src = tmp_path / 'lay.c'
    body = ''.join('printf("%%zu\\n", offsetof(%s, %s));' % (struct, f) for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "bsls_hip.h"\n'
                   'int main(void){printf("%%zu\\n", sizeof(%s));%s return 0;}\n' % (struct, body))
    exe = tmp_path / 'lay'
    subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


@pytest.mark.parametrize('struct,cls', [('bsls_bb_problem', 'BBProblem'), ('bsls_panels', 'Panels'),
                                        ('bsls_xbb_problem', 'XBBProblem'), ('bsls_csr', 'CSR'),
                                        ('bsls_tiles', 'Tiles'), ('bsls_dore_state', 'DoreState'),
                                        ('bsls_lsq_op', 'LsqOp')])
def test_struct_layout_matches_header(native, tmp_path, struct, cls):
    C = getattr(native, cls)
    names = [f[0] for f in C._fields_]
    want = _c_layout(tmp_path, struct, names)
    got = [ctypes.sizeof(C)] + [getattr(C, f).offset for f in names]
    assert got == want


def test_panel_limits_match_header(native):
    hdr = open(os.path.join(ROOT, 'include', 'bsls_hip.h')).read()
    assert '#define BSLS_PANEL_CHUNK %d' % native.PANEL_CHUNK in hdr
    assert '#define BSLS_PANEL_ROWS %d' % native.PANEL_ROWS in hdr
    assert '#define BSLS_PANEL_WAVES %d' % native.PANEL_WAVES in hdr
    assert '#define BSLS_TILE_THREADS %d' % native.TILE_THREADS in hdr
    assert '#define BSLS_TILE_NT 0x%x' % native.TILE_NT in hdr
    assert '#define BSLS_TILE_VAL32 0x%x' % native.TILE_VAL32 in hdr
    assert '#define BSLS_TILE_VAL16 0x%x' % native.TILE_VAL16 in hdr


def test_tile_planner(native):
    import numpy as np
    rs = np.random.RandomState(1)
    lens = rs.poisson(16, size=5000)
    lens[100] = 10_000                                   # one long row
    ip = np.concatenate(([0], np.cumsum(lens))).astype(np.int64)
    t = native.plan_tiles(ip)
    assert t[0] == 0 and t[-1] == 5000 and np.all(np.diff(t) > 0)
    nnz = ip[t[1:]] - ip[t[:-1]]
    rows = np.diff(t)
    assert np.all((nnz <= 2048) | (rows == 1)) and np.all(rows <= 1024)
    ends = np.cumsum(rs.randint(1, 40, size=400))
    ends = ends[ends < 5000]
    t2 = native.plan_tiles(ip, ends=ends)
    assert set(t2[1:-1]) <= set(ends.tolist())
    assert native.group_for_rows(12.8) == 16 and native.group_for_rows(128) == 2


def test_invalid_arguments_rejected_without_launch(native):
    L = native.load()
    assert L.bsls_proj_multi_simplex(None, None, 0, 0, 1, None, 0, None) == native.BSLS_E_ARG
    assert L.bsls_isotonic_multi(4, None, None, 1, 1, None, 1, 1, None, 0, None, None) == \
        native.BSLS_E_ARG
    assert L.bsls_bb_prologue(None, None) == native.BSLS_E_ARG
    # LBFGS.solve's history kernels (csrc/lbfgs.hip): argument and workspace
    # checks come before any launch
    p = ctypes.c_void_p(8)
    assert L.bsls_multi_dot(p, 0, p, 4, 10, p, p, 1 << 20, None) == native.BSLS_E_ARG
    assert L.bsls_multi_dot(p, 5, p, 4, 10, p, p, 1 << 20, None) == native.BSLS_E_ARG
    assert L.bsls_multi_dot(p, 3, p, 4, 10, p, p, 8, None) == native.BSLS_E_WORKSPACE
    assert L.bsls_multi_axpy(p, 257, p, 10, p, None) == native.BSLS_E_ARG
    assert L.bsls_lbfgs_coef(0, 0, p, p, None) == native.BSLS_E_ARG
    assert L.bsls_lbfgs_coef(128, 0, p, p, None) == native.BSLS_E_ARG
    assert L.bsls_lbfgs_coef(5, 5, p, p, None) == native.BSLS_E_ARG
    assert L.bsls_lbfgs_push(5, -1, 1.0, p, p, p, p, p, p, 10, None) == native.BSLS_E_ARG
    # sizes: rho, SY, YY, coef, scratch; multi-dot partials per column chunk
    assert L.bsls_lbfgs_state_size(50) == 8 * (50 + 2 * 50 * 50 + 101 + 150)
    assert L.bsls_multi_dot_workspace_size(3, 102) >= 8 * 3 * 102
    assert L.bsls_multi_dot_workspace_size(0, 10) == 0


def test_isotonic_pack_plan(native):
    """bsls_isotonic_pack_plan (host only): packs tile [starts[0], n) in order,
    each a run of whole blocks with <= 64 elements (mask bit i = a block starts
    at element i of the pack) or one longer block (listed in longs), greedy as
    K3's packs."""
    import numpy as np
    rs = np.random.RandomState(3)
    sizes = rs.randint(1, 50, size=3000)
    sizes[[5, 700, 2999]] = [65, 400, 64]
    first = 7
    starts = first + np.concatenate(([0], np.cumsum(sizes)[:-1]))
    n = int(first + sizes.sum())
    P = native.pack_plan(starts, n)
    assert P['start'][0] == first
    ends = P['start'] + P['len']
    assert np.array_equal(P['start'][1:], ends[:-1]) and ends[-1] == n
    blk = 0
    for q in range(P['start'].shape[0]):
        m, L = int(P['mask'][q]) & 0xFFFFFFFFFFFFFFFF, int(P['len'][q])
        nb = bin(m).count('1')
        assert m & 1
        assert np.array_equal(starts[blk:blk + nb] - P['start'][q],
                              [i for i in range(64) if (m >> i) & 1])
        if L > 64:
            assert nb == 1 and q in set(P['longs'].tolist())
        else:
            # greedy: the next block would not have fitted
            nxt = sizes[blk + nb] if blk + nb < sizes.size else 0
            assert blk + nb == sizes.size or L + nxt > 64 or nxt > 64
        blk += nb
    assert blk == sizes.size
    assert sorted(P['longs'].tolist()) == [q for q in range(P['len'].size) if P['len'][q] > 64]
