"""The C-ABI library loads and exports every symbol include/bsls_hip.h declares
(CPU only: dlopen needs no GPU; no compute call is made)."""
import ctypes
import os
import subprocess

import pytest


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
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '-n', native.LIB_PATH],
                         capture_output=True, text=True).stdout
    blob = open(native.LIB_PATH, 'rb').read()
    assert b'gfx950' in blob
    for other in (b'gfx942', b'gfx90a', b'gfx1100'):
        assert other not in blob


def test_host_only_entry_points(native):
    L = native.load()
    assert L.bsls_version().startswith(b'bsls-hip')
    assert L.bsls_proj_workspace_size(3_200_000, 100_000, 60) > 0
    assert L.bsls_proj_workspace_size(100, 2, 50) < L.bsls_proj_workspace_size(100_000, 2, 50_000)
    assert L.bsls_isotonic_workspace_size(1000) >= 4000
    assert L.bsls_bb_workspace_size(100_000, 1_000_000, 950_000) > 4 * 950_000
    assert L.bsls_spmv_workspace_size(100_000) > 8 * 25_000
    assert L.bsls_md_workspace_size(50_000) > 0


def test_bb_struct_layout_matches_header(native):
    # struct bsls_bb_problem: 4 int64, 10 + 2 + 2 + 4 pointers, 2 int64, 1 double, 3 int32
    assert ctypes.sizeof(native.BBProblem) == 8 * 4 + 8 * 18 + 8 * 2 + 8 + 4 * 3 + 4


def test_invalid_arguments_rejected_without_launch(native):
    L = native.load()
    assert L.bsls_proj_multi_simplex(None, None, 0, 0, 1, None, 0, None) == native.BSLS_E_ARG
    assert L.bsls_isotonic_multi(4, None, None, 1, 1, None, 1, 1, None, 0, None, None) == \
        native.BSLS_E_ARG
    assert L.bsls_bb_prologue(None, None) == native.BSLS_E_ARG
