"""Host-side logic (CPU only): drop-in argument checking, data preparation and
generators, pinned against the reference's fixtures."""
import os

import numpy as np
import pytest
import scipy.sparse as sps

from conftest import SEED


# ------------------------------------------------ c_extensions argument checks
# (they run before anything is launched, so they work without a GPU)

@pytest.fixture(scope='module')
def cx():
    from c_extensions import c_extensions
    return c_extensions


def test_bad_indices_raise_assertion(cx):
    # tests/fast/test_proj_simplex.py:36-42,54-59
    y = np.random.rand(7)
    for s, e in [(2, 8), (-1, 7), (-1, 4)]:
        with pytest.raises(AssertionError):
            cx.proj_simplex_c(y, s, e)
        with pytest.raises(AssertionError):
            cx.isotonic_regression_c(y, s, e)
    for b in (np.array([-1, 2, 4]), np.array([1, 3, 7]), np.array([0, 4, 2])):
        for fn in (cx.proj_multi_simplex_c, cx.proj_multi_ball_c, cx.isotonic_regression_multi_c,
                   cx.isotonic_regression_multi_c_2, cx.isotonic_regression_multi_c_3):
            with pytest.raises(AssertionError):
                fn(y, b)
    with pytest.raises(AssertionError):
        cx.x2z_c(np.random.rand(5), np.zeros(3), np.array([1, 3]))   # blocks[0] must be 0


def test_empty_range_is_a_no_op(cx):
    y = np.random.rand(7)
    y0 = y.copy()
    assert cx.proj_simplex_c(y, 4, 4) is None
    assert np.array_equal(y, y0)


def test_buffer_typing(cx):
    with pytest.raises(ValueError):
        cx.proj_multi_simplex_c(np.arange(7), np.array([0, 2]))          # int y
    with pytest.raises(ValueError):
        cx.proj_multi_simplex_c(np.random.rand(7), np.array([0, 2], dtype=np.int32))
    with pytest.raises(ValueError):
        cx.proj_multi_simplex_c(np.random.rand(2, 7), np.array([0, 2]))
    with pytest.raises(TypeError):
        cx.proj_multi_simplex_c([0.1, 0.2], np.array([0]))


def test_no_cpu_fallback(cx):
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is present')
    with pytest.raises(RuntimeError, match='no HIP device'):
        cx.proj_multi_simplex_c(np.random.rand(7), np.array([0, 2, 4]))


# ------------------------------------------------ bsls_utils

def test_particular_x0_kat():
    from bsls_utils import particular_x0
    assert list(particular_x0(np.array([1, 2, 3, 4]))) == [1, 0, 1, 0, 0, 1, 0, 0, 0, 1]


def test_generate_data_matches_reference(golden):
    import bsls_utils
    G = golden('solvers.npz')
    np.random.seed(SEED)
    d = bsls_utils.generate_data()
    for k in ('A', 'b', 'x_true', 'f', 'block_sizes'):
        assert np.array_equal(np.asarray(d[k]), G['gen_%s' % k]), k
    np.random.seed(SEED)
    d = bsls_utils.generate_data(n=300, m1=40, m2=12, A_sparse=0.3, alpha=0.5)
    for k in ('A', 'b', 'x_true', 'f', 'block_sizes'):
        assert np.array_equal(np.asarray(d[k]), G['gen2_%s' % k]), k
    assert abs(sum(d['f']) - sum(d['x_true'])) < 1e-10   # tests/fast/test_util.py:34-40


def test_N_and_x2z_match_oracle(orc):
    from bsls_utils import block_sizes_to_N, x2z
    rs = np.random.RandomState(SEED)
    bs = rs.randint(1, 9, size=50)
    N1, N2 = block_sizes_to_N(bs), orc.block_sizes_to_N(bs)
    assert (N1 != N2).nnz == 0
    x = rs.rand(int(bs.sum()))
    assert np.array_equal(x2z(x, bs), orc.x2z(x, bs))


def test_bsls_matrices_matches_reference(golden, tmp_path):
    """BSLSMatrices on the tests/fast/test_main.py .mat files reproduces the
    matrices the reference's pipeline handed to solve_in_z."""
    import bsls_utils
    from bsls_matrices import BSLSMatrices
    G = golden('solvers.npz')
    for vi, kw in enumerate([{}, {'alpha': 0.5}, {'A_sparse': 0.05}]):
        np.random.seed(SEED)
        fname = os.path.join(str(tmp_path), 'test_main.mat')
        bsls_utils.generate_data(fname=fname, **kw)
        bm = BSLSMatrices(fname=fname, full=True, L=True, OD=True, CP=True, LP=True, eq='CP')
        bm.degree_reduced_form()
        AA, bb, N, bsz, x_split, nz, scaling, rsort, x0 = bm.get_LS()
        AA = sps.csr_matrix(AA)
        AA.sort_indices()
        ref = sps.csr_matrix((G['main%d_A_data' % vi], G['main%d_A_indices' % vi],
                              G['main%d_A_indptr' % vi]), shape=tuple(G['main%d_A_shape' % vi]))
        ref.sort_indices()
        assert AA.shape == ref.shape and (AA != ref).nnz == 0, vi
        assert np.array_equal(bb, G['main%d_b' % vi])
        assert np.array_equal(bsz, G['main%d_block_sizes' % vi])
        assert np.array_equal(x_split, G['main%d_x_split' % vi])
        assert np.array_equal(scaling, G['main%d_scaling' % vi])


# ------------------------------------------------ synthetic generator + partition

def test_synthetic_shard_properties():
    from synthetic import make_shard
    sh = make_shard(20_000, 1_000, 2_000, per_col=16, seed=1)
    A, AT = sh['A'], sh['AT']
    assert A.shape == (2_000, 20_000) and A.nnz == 16 * 20_000
    assert (A.T.tocsr() != AT).nnz == 0
    assert sh['block_sizes'].sum() == 20_000 and sh['block_sizes'].min() >= 1
    # scaled incidence: one value per column; splits on the simplex
    C = A.tocsc()
    for j in range(0, 20_000, 997):
        v = C.data[C.indptr[j]:C.indptr[j + 1]]
        assert np.all(v == v[0]) and len(np.unique(C.indices[C.indptr[j]:C.indptr[j + 1]])) == 16
    ends = np.cumsum(sh['block_sizes'])
    sums = np.add.reduceat(sh['x_true'], ends - sh['block_sizes'])
    assert np.allclose(sums, 1.0)
    assert np.allclose(A.dot(sh['x_true']), sh['Ax'])
    sh2 = make_shard(20_000, 1_000, 2_000, per_col=16, seed=1)
    assert (sh2['A'] != A).nnz == 0                     # seeded


def test_partition_blocks_balanced():
    from distributed import partition_blocks
    rs = np.random.RandomState(SEED)
    bs = rs.multinomial(10_000 - 500, np.ones(500) / 500) + 1
    for world in (1, 2, 3, 8):
        bounds = partition_blocks(bs, bs * 16.0, world)
        assert bounds[0] == 0 and bounds[-1] == 500 and np.all(np.diff(bounds) > 0)
        loads = [bs[bounds[g]:bounds[g + 1]].sum() for g in range(world)]
        assert max(loads) - min(loads) <= 2 * bs.max()
    with pytest.raises(ValueError):
        partition_blocks(bs, bs, 501)


def _rand_csr(rs, R, C, dens):
    return sps.random(R, C, density=dens, random_state=rs, format='csr')


@pytest.mark.parametrize('R,C,dens,prow,halo,ngroups,chunk', [
    (300, 500, 0.05, 64, False, 1, None),
    (300, 500, 0.05, 7, True, 1, None),
    (1000, 40000, 0.001, 64, False, 8, 4000),     # K1 shape: chunk groups
    (2000, 70000, 0.0005, 100, True, 1, 4000),    # K2 shape: halo rows, many chunks
    (1, 5, 1.0, 1, False, 1, None),
    (64, 300, 0.9, 255, True, 1, 128),            # dense rows: > 64 diagonals per segment
])
def test_panel_image_walk_matches_scipy(R, C, dens, prow, halo, ngroups, chunk):
    """The panel image (device.build_panels) walked in the kernels' order
    (device.panels_matvec = panel_segment restated) gives SciPy's csr_matvec bit
    for bit with one chunk group (K2), and to rounding with several (K1)."""
    import device
    rs = np.random.RandomState(SEED)
    A = _rand_csr(rs, R, C, dens)
    ccol, gch = device.chunk_plan(C, ngroups, chunk=chunk)
    assert ccol[0] == 0 and ccol[-1] == C and np.all(ccol[:-1] % 2 == 0)
    assert np.all(np.diff(ccol) <= (chunk or 20224)) and gch[-1] == ccol.size - 1
    img = device.build_panels(A, prow, halo, ccol, gch)
    assert img['nnz'] == A.nnz + (halo and sum(A[p * prow].nnz for p in range(1, img['npanels'])))
    assert np.all(img['ent_off'] % 2 == 0)                # pair loads stay 4-B aligned
    # D_q = the slice's largest row count; one 64-byte count group per live slice
    info = img['seg_info']
    D = np.stack([(info >> (16 * q)) & 0xFFFF for q in range(4)], axis=1)
    assert img['cnt_off'][-1] == 64 * np.count_nonzero(D)
    groups = img['cnt'][:img['cnt_off'][-1]].astype(np.int64).reshape(-1, 64)
    padded = np.diff(np.concatenate([np.zeros((groups.shape[0], 1), np.int64), groups & ~1],
                                    axis=1), axis=1)
    assert np.all(padded >= 0) and np.all(padded % 2 == 0)
    assert (padded - (groups & 1)).sum() == img['nnz'] and padded.sum() == img['stored']
    x = rs.randn(C)
    y, acc = device.panels_matvec(img, x)
    ref = A.dot(x)
    if img['ngroups'] == 1:
        assert np.array_equal(y, ref)
    else:
        assert np.allclose(y, ref, rtol=1e-13, atol=1e-13)
    if halo:
        assert np.array_equal(acc[:-1, prow], acc[1:, 0])


def test_panel_image_scaled_incidence():
    """Scaled incidence: no values stored; K1 walks colv*x, K2 multiplies by its
    row's colv, bit-identical to SciPy's A'r (the products are the same)."""
    import device
    rs = np.random.RandomState(SEED)
    A = sps.random(500, 3000, density=0.01, random_state=rs, format='csc')
    A.data[:] = np.repeat(np.floor(rs.rand(3000) * 1000) + 1, np.diff(A.indptr))
    A = A.tocsr()
    colv = device.scaled_incidence_scale(A)
    assert colv is not None
    B = A.copy()
    B.data[0] += 1.0
    assert device.scaled_incidence_scale(B) is None
    x = rs.rand(3000)
    img = device.build_panels(A, 64, False, *device.chunk_plan(3000, 1, chunk=256), values=False)
    assert img['val'] is None
    y, _ = device.panels_matvec(img, colv * x)
    assert np.array_equal(y, A.dot(x))
    AT = A.T.tocsr()
    r = rs.randn(500)
    img = device.build_panels(AT, 64, True, *device.chunk_plan(500, 1, chunk=128), values=False)
    y, _ = device.panels_matvec(img, r, colv=colv)
    assert np.array_equal(y, AT.dot(r))


def test_panel_rows_choice():
    import device
    assert device.panel_rows(100_000, 32) == 196          # C3 K1: 8 groups x 32 workgroups
    assert device.panel_rows(1_000_000, 256) == 245       # C3 K2: 256 workgroups
    assert device.panel_rows(10, 256) == 10
    assert device.panel_rows(10_000_000, 256) == 255


def test_k1_plan_fits_one_round(monkeypatch):
    """The A-image plan: C3 gets 10 column groups x 25 row blocks of 250-row
    panels; every m stays within one workgroup per CU (256) and <= 255 rows."""
    import device
    monkeypatch.delenv('BSLS_K1_PLAN', raising=False)
    assert device.k1_plan(100_000) == (250, 10)
    for m in (1, 100, 5_000, 100_000, 200_000, 1_000_000, 4_000_000):
        prow, groups = device.k1_plan(m)
        assert 1 <= prow <= 255 and 1 <= groups <= 10
        rbs = -(-(-(-m // prow)) // 16)
        assert groups * rbs <= 256 or groups == 1, (m, prow, groups, rbs)
    monkeypatch.setenv('BSLS_K1_PLAN', '8,32')
    assert device.k1_plan(100_000) == (196, 8)


def test_batch_stopping_matches_oracle(orc):
    """algorithm_utils.stopping (python/algorithm_utils.py:158-172): the last
    true test names the reason."""
    from algorithm_utils import stopping
    cases = [(5, 5, 1.0, 2.0, 1e-6, 1e-12, None), (3, 5, 1.0, 1.0, 1e-6, 1e-12, None),
             (3, 5, 1.0, 2.0, 1e-6, 1e-12, 1.0 - 1e-9), (5, 5, 1.0, 1.0, 1e-6, 1e-12, 0.5),
             (2, 5, 1.0, np.inf, 1e-6, 1e-12, None)]
    for c in cases:
        assert stopping(*c) == orc.batch_stopping(*c)


def test_batch_modules_import_without_device():
    import BATCH
    import algorithm_utils
    assert BATCH.solve_BB.__code__.co_varnames[:8] == ('obj', 'proj', 'line_search', 'x_init',
                                                      'f_min', 'opt_tol', 'max_iter',
                                                      'prog_tol')
    with pytest.raises(RuntimeError):
        algorithm_utils.get_solver_parts((sps.eye(4).tocsr(), np.ones(4)), np.array([0]), 1.0,
                                         is_sparse=True)


def test_md_pack_blocks():
    """mirror_descent.pack_blocks: whole blocks, <= 64 entries per pack, longer
    blocks alone, masks of block starts."""
    from mirror_descent import pack_blocks
    sizes = [20, 30, 20, 70, 3, 64, 1, 1]
    x0, mask, ln = pack_blocks(sizes)
    assert list(x0) == [0, 50, 70, 140, 143, 207]
    assert list(mask.view(np.uint64)) == [1 + (1 << 20), 1, 1, 1, 1, 3]
    assert list(ln) == [50, 20, 70, 3, 64, 2]
    rs = np.random.RandomState(0)
    sizes = rs.randint(1, 90, 2000)
    x0, mask, ln = pack_blocks(sizes)
    assert ln.sum() == sizes.sum() and np.all(np.diff(x0) == ln[:-1])
    nblk = sum(bin(int(v)).count('1') for v in mask.view(np.uint64))
    assert nblk == sizes.size


def test_lbfgs_host_loop_matches_reference(orc, golden):
    """LBFGS.py (the host loop over whatever closures it is given) over the
    CPU restatement's closures reproduces the reference's LBFGS.solve
    trajectory bit for bit (tests/golden/plugins.npz, 25 iterations)."""
    import LBFGS
    import solvers
    G = golden('plugins.npz')
    A = sps.csr_matrix((G['lbfgs_A_data'], G['lbfgs_A_indices'], G['lbfgs_A_indptr']),
                       shape=tuple(G['lbfgs_A_shape']))
    P = orc.solve_in_z_parts(A, G['lbfgs_b'], G['lbfgs_block_sizes'])
    rec = {}

    def log(i, s, dt):
        rec[i] = np.array(s)
        return 0.0
    LBFGS.solve(P['z0'] + 1, P['f'], P['nabla_f'], solvers.stopping, record_every=1,
                proj=P['proj'], log=log, options={'max_iter': 25, 'verbose': 0, 'opt_tol': 1e-30})
    assert sorted(rec) == list(G['lbfgs_trace_iters'])
    for k, i in enumerate(G['lbfgs_trace_iters']):
        assert np.array_equal(rec[i], G['lbfgs_trace_states'][k]), i


def _dense_row_matrix(n=100_000, m=1000, dense=8, seed=3):
    """A network with a few links every route crosses (dense rows 0..dense-1)
    plus 16 random links per route: a 64-row slice then holds more entries per
    chunk than the panel format addresses."""
    rs = np.random.RandomState(seed)
    rows = np.concatenate([np.repeat(np.arange(dense), n),
                           rs.randint(dense, m, size=16 * n)])
    cols = np.concatenate([np.tile(np.arange(n), dense), np.repeat(np.arange(n), 16)])
    A = sps.csr_matrix((np.ones(rows.size), (rows, cols)), shape=(m, n))
    A.sum_duplicates()
    return A


def test_panel_overflow_is_typed():
    """build_panels refuses a dense-row slice with PanelOverflow (a ValueError),
    which BBEngine / lsq_operator catch to fall back."""
    import device
    A = _dense_row_matrix()
    prow, groups = device.k1_plan(A.shape[0])
    with pytest.raises(device.PanelOverflow):
        device.build_panels(A, prow, False, *device.chunk_plan(A.shape[1], groups),
                            values=False)
    assert issubclass(device.PanelOverflow, ValueError)


@pytest.mark.parametrize('layout', [0, 1, 2])
@pytest.mark.parametrize('halo', [0, 1])
@pytest.mark.parametrize('values', [True, False])
def test_tile_images_restate_scipy(layout, halo, values):
    """Both tile layouts (thread streams; dealt column-sorted instructions)
    hold every entry once: the host restatement of the kernels' walk over the
    image equals SciPy's A.dot to rounding (halo rows dropped), with several
    column groups, a short last row block and empty rows."""
    import _native
    import device
    rs = np.random.RandomState(9 + layout)
    m, n = 5000, 3000
    A = sps.random(m, n, density=0.004, random_state=rs, format='csr')
    A = sps.csr_matrix(A.toarray() * (rs.rand(m, 1) > 0.05))   # some empty rows
    A.data = rs.randn(A.nnz) if values else np.ones(A.nnz)
    gc = np.round(np.linspace(0, n, 4)).astype(np.int64)
    H = 1500
    if layout:
        img = _native.tiles_build_dealt(A, H, halo, gc, values=values, packed=layout == 2)
    else:
        img = _native.tiles_build(A, H, halo, gc, values=values)
    img.update(rows=m, cols=n, H=H, halo=halo, ngroups=3, order=0, group_col=gc, layout=layout)
    x = rs.randn(n)
    got = device.tiles_matvec(img, x)
    want = A.dot(x)
    assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))
    if layout == 1:
        # every entry once: the non-dummy entries count nnz (+ halo copies)
        e = img['ent'][:4 * img['nquads']].astype(np.int64)
        live = int(np.sum((e >> 16) != H + halo))
        extra = sum(int(A.indptr[r + 1] - A.indptr[r]) for r in range(H, m, H)) if halo else 0
        assert live == A.nnz + extra
    if layout == 2:
        # 3 words per 4 entries, rows above 24 - bit_width(H + halo) column bits
        w = img['ent'][:3 * img['nquads']].astype(np.int64).reshape(-1, 3)
        e = np.stack([w[:, 0] & 0xFFFFFF, (w[:, 0] >> 24) | ((w[:, 1] & 0xFFFF) << 8),
                      (w[:, 1] >> 16) | ((w[:, 2] & 0xFF) << 16), w[:, 2] >> 8], 1)
        cb = 24 - int(H + halo).bit_length()
        live = int(np.sum((e >> cb) != H + halo))
        extra = sum(int(A.indptr[r + 1] - A.indptr[r]) for r in range(H, m, H)) if halo else 0
        assert live == A.nnz + extra


def test_iso_plan_cache_by_content(monkeypatch):
    """device.iso_plan's cache (the pack plan of a block layout, made once):
    a fresh array with the same starts finds the cached plan, other starts or
    another length make a new one, and changing the caller's array in place
    after caching does not alias the cached entry (the cache keeps a copy)."""
    import device
    made = []

    class Stub:
        def __init__(self, st, n):
            made.append((st.copy(), n))
    monkeypatch.setattr(device, 'IsoPlan', Stub)
    monkeypatch.setattr(device, '_iso_plans', {})
    a = np.array([0, 3, 7, 12], dtype=np.int64)
    p1 = device.iso_plan(a, 20)
    assert device.iso_plan(a.copy(), 20) is p1
    assert device.iso_plan(list(a), 20) is p1            # converted, same content
    p2 = device.iso_plan(a, 21)                         # another length
    b = a.copy()
    b[2] = 8
    p3 = device.iso_plan(b, 20)                         # other starts, same count
    assert len({id(p1), id(p2), id(p3)}) == 3 and len(made) == 3
    a[1] = 4                                            # the caller mutates its array
    p4 = device.iso_plan(a, 20)
    assert p4 is not p1 and len(made) == 4
    assert device.iso_plan(np.array([0, 3, 7, 12]), 20) is p1
    # a plan's arrays live on one GPU: the same layout on another device is
    # planned again, and the first device still finds its own
    monkeypatch.setattr(device, '_cur_dev', lambda: 5)
    p5 = device.iso_plan(np.array([0, 3, 7, 12]), 20)
    assert p5 is not p1 and len(made) == 5
    monkeypatch.setattr(device, '_cur_dev', lambda: -1)
    assert device.iso_plan(np.array([0, 3, 7, 12]), 20) is p1
