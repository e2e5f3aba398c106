"""The x-space operator pair (csrc/lsq.hip, device.DeviceLSQ): r = A x + add,
||r||^2 and g = A' r -- sparse_least_squares_obj's two SciPy products
(python/algorithm_utils.py:88-94).  Needs an MI355X.

Bar: g bit-identical to SciPy's csr_matvec on A' (each row summed in CSR
order); r within 1e-12 relative of SciPy on both residual walks, and on the
panels (the default) bit-identical to the host restatement of the panel walk
(device.panels_matvec: 8 column-group partials summed in group order) and
run-to-run; the dealt tile residual (k1='tiles', LDS atomic sums) within
1e-12 run-to-run, and with fixed-point row sums (k1='tiles_fixed')
bit-identical run-to-run; ||r||^2 within 1e-12 relative.
"""
import numpy as np
import pytest
import scipy.sparse as sps

from conftest import SEED

pytestmark = pytest.mark.gpu


def exact(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def _scaled(m, n, per_col, rs):
    """Scaled incidence: per_col distinct rows per column, value colv[j]."""
    rows = np.concatenate([rs.choice(m, min(per_col, m), replace=False) for _ in range(n)])
    cols = np.repeat(np.arange(n), min(per_col, m))
    colv = np.floor(rs.rand(n) * 1000) + 1
    return sps.csr_matrix((colv[cols], (rows, cols)), shape=(m, n))


@pytest.mark.parametrize('m,n,per_col', [(1000, 9001, 5), (37, 300, 3), (20000, 150000, 12),
                                         (4096, 64, 40)])
@pytest.mark.parametrize('scaled', [True, False])
@pytest.mark.parametrize('k1,k2', [('tiles', 'panels'), ('panels', 'panels'), ('tiles', 'tiles'),
                                   ('tiles_fixed', 'panels')])
def test_lsq_operator(cuda, m, n, per_col, scaled, k1, k2):
    import torch
    from device import DeviceLSQ, panels_matvec
    rs = np.random.RandomState(SEED + m)
    A = _scaled(m, n, per_col, rs)
    if not scaled:
        A.data = rs.randn(A.nnz)
    # empty rows and columns
    A = sps.csr_matrix(sps.diags((rs.rand(m) > 0.05).astype(float)) @ A @
                       sps.diags((rs.rand(n) > 0.05).astype(float)))
    A.eliminate_zeros()
    AT = A.T.tocsr()
    op = DeviceLSQ(A, AT, general=not scaled, k1=k1, k2=k2)
    assert op.scaled == scaled and op.k1 == k1 and op.k2 == k2
    x = rs.randn(n)
    add = rs.randn(m)
    xd, ad = torch.from_numpy(x).cuda(), torch.from_numpy(add).cuda()
    r = torch.empty(m, dtype=torch.float64, device='cuda')
    sq = torch.zeros(1, dtype=torch.float64, device='cuda')
    op.residual(xd, r, add=ad, sq=sq)
    rh = r.cpu().numpy()
    ref = A.dot(x) + add
    np.testing.assert_allclose(rh, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    assert abs(float(sq.item()) - ref.dot(ref)) <= 1e-12 * ref.dot(ref)
    if m * n <= 10 ** 7 and k1 == 'panels':
        if scaled:
            colv = op.colv.cpu().numpy()
            want, _ = panels_matvec(op.A_pan.img, colv * x)
        else:
            want, _ = panels_matvec(op.A_pan.img, x)
        assert exact(rh, want + add)
    # residual without add / without ||r||^2
    r2 = torch.empty(m, dtype=torch.float64, device='cuda')
    op.residual(xd, r2)
    np.testing.assert_allclose(r2.cpu().numpy(), A.dot(x), rtol=1e-12,
                               atol=1e-12 * np.abs(ref).max())
    g = torch.empty(n, dtype=torch.float64, device='cuda')
    op.gradient(r, g)
    gref = AT.dot(rh)
    if k2 == 'panels':
        assert exact(g.cpu().numpy(), gref)
    else:
        # dealt tiles: LDS atomic row sums (scaled: colv times the row's sum)
        np.testing.assert_allclose(g.cpu().numpy(), gref, rtol=1e-12,
                                   atol=1e-12 * max(np.abs(gref).max(), 1.0))
    # repeated calls (tickets re-armed): bit for bit on the panels, to
    # rounding on the dealt tiles
    r3 = torch.empty(m, dtype=torch.float64, device='cuda')
    sq3 = torch.zeros(1, dtype=torch.float64, device='cuda')
    for _ in range(3):
        op.residual(xd, r3, add=ad, sq=sq3)
    if k1 in ('panels', 'tiles_fixed'):
        # (tiles_fixed: two-word fixed-point row sums, order-free)
        assert exact(r3.cpu().numpy(), rh) and float(sq3.item()) == float(sq.item())
    else:
        np.testing.assert_allclose(r3.cpu().numpy(), rh, rtol=1e-12,
                                   atol=1e-12 * np.abs(ref).max())
        assert abs(float(sq3.item()) - float(sq.item())) <= 1e-12 * float(sq.item())


def test_sparse_lsq_panel_and_csr_paths_agree(cuda):
    """SparseLSQ (the obj of get_solver_parts(is_sparse=True)) on panels and on
    the CSR kernels: same f to 1e-12, g within 1e-12 (its input r differs by
    the residual's group order only)."""
    import torch
    from algorithm_utils import SparseLSQ
    from synthetic import make_shard, add_noise
    sh = make_shard(60_000, 3_000, 6_000, 16, seed=5)
    b = add_noise(sh['Ax'], 0.02, seed=5)
    P = SparseLSQ(sh['A'], b, panels=True)
    C = SparseLSQ(sh['A'], b, panels=False)
    assert P.lsq is not None and P.lsq.scaled and C.lsq is None
    x = np.random.RandomState(1).rand(sh['A'].shape[1])
    gp = torch.empty(P.n, dtype=torch.float64, device='cuda')
    gc = torch.empty(P.n, dtype=torch.float64, device='cuda')
    fp, fc = P(torch.from_numpy(x).cuda(), gp), C(torch.from_numpy(x).cuda(), gc)
    assert abs(fp - fc) <= 1e-12 * abs(fc)
    tmp = sh['A'].dot(x) - b
    assert abs(fp - .5 * tmp.dot(tmp)) <= 1e-12 * abs(fp)
    gref = sh['A'].T.tocsr().dot(tmp)
    np.testing.assert_allclose(gp.cpu().numpy(), gref, rtol=1e-10,
                               atol=1e-12 * np.abs(gref).max())
    np.testing.assert_allclose(gc.cpu().numpy(), gref, rtol=1e-10,
                               atol=1e-12 * np.abs(gref).max())


@pytest.mark.parametrize('panels', [False, True])
def test_mirror_descent_vs_reference(cuda, golden, orc, panels):
    """mirror_descent.least_squares (python/mirror_descent.py:7-53) on the
    reference's own runs (tests/golden/solvers.npz): iterates at 1, 5 and 40
    iterations within 1e-10 (device exp and sequential block sums differ from
    NumPy's in the last bits); with a tolerance, the device-side stopping test
    ends at the oracle's iteration with the same x."""
    import mirror_descent
    G = golden('solvers.npz')
    A = sps.csr_matrix((G['md_A_data'], G['md_A_indices'], G['md_A_indptr']),
                       shape=tuple(G['md_A_shape']))
    blocks = list(G['md_blocks'])
    for it in (1, 5, 40):
        x, k = mirror_descent.least_squares(A, G['md_b'], blocks, iters=it, tolerance=0.0,
                                            return_iters=True, panels=panels, poll=7)
        assert k == it
        np.testing.assert_allclose(x, G['md_x_%d' % it], rtol=1e-10, atol=1e-14)
    for tol in (1e-3, 1e-5):
        xr, kr = orc.md_least_squares(A, G['md_b'], blocks, iters=500, tolerance=tol,
                                      return_iters=True)
        x, k = mirror_descent.least_squares(A, G['md_b'], blocks, iters=500, tolerance=tol,
                                            return_iters=True, panels=panels, poll=16)
        assert k == kr, (tol, k, kr)
        np.testing.assert_allclose(x, xr, rtol=1e-9, atol=1e-13)


def test_mirror_descent_ragged_blocks_vs_oracle(cuda, orc):
    """Ragged blocks, including blocks of 1 and blocks longer than a wave
    (packs of their own): the device iterates follow the oracle's restatement
    of mirror_descent.py within 1e-10."""
    import mirror_descent
    rs = np.random.RandomState(SEED)
    sizes = np.concatenate([[1, 1, 65, 200, 64, 63, 2], rs.randint(1, 40, 300)])
    n = int(sizes.sum())
    m = 400
    A = sps.random(m, n, density=8.0 / m, random_state=rs, format='csr')
    A.data = rs.rand(A.nnz)
    b = A.dot(np.repeat(1.0 / sizes, sizes)) * (1 + 0.05 * rs.randn(m))
    for it in (1, 7, 30):
        x = mirror_descent.least_squares(A, b, list(sizes), iters=it, tolerance=0.0, poll=5)
        xr = orc.md_least_squares(A, b, list(sizes), iters=it, tolerance=0.0)
        np.testing.assert_allclose(x, xr, rtol=1e-10, atol=1e-14)


def test_lsq_fixed_point_residual_edges(cuda):
    """k1='tiles_fixed': x = 0 (scale from a zero bound), huge and tiny
    magnitudes (1e150, 1e-150: the scale follows max|x|), a NaN in x (NaN
    residual rows, not a finite garbage sum), heavy cancellation (r ~ 1e-9 of
    the terms: the two-word sums keep it to 1e-12 of the terms), and the
    order-free sums: the same r after the input entries' dealing changes
    nothing but run order (three calls, bit-identical)."""
    import torch
    from device import DeviceLSQ
    rs = np.random.RandomState(SEED + 9)
    m, n = 3000, 40000
    A = _scaled(m, n, 6, rs)
    op = DeviceLSQ(A, A.T.tocsr(), k1='tiles_fixed', k2='panels')
    r = torch.empty(m, dtype=torch.float64, device='cuda')
    for scale in (0.0, 1e150, 1e-150, 1.0):
        x = rs.rand(n) * scale
        op.residual(torch.from_numpy(x).cuda(), r)
        ref = A.dot(x)
        np.testing.assert_allclose(r.cpu().numpy(), ref, rtol=1e-12,
                                   atol=1e-12 * max(np.abs(ref).max(), 1e-300))
    x = rs.rand(n)
    x[123] = np.nan
    op.residual(torch.from_numpy(x).cuda(), r)
    assert np.isnan(r.cpu().numpy()).any()
    # cancellation: add = -A x + tiny
    x = rs.rand(n)
    ax = A.dot(x)
    tiny = 1e-9 * np.abs(ax).max() * rs.randn(m)
    add = torch.from_numpy(tiny - ax).cuda()
    op.residual(torch.from_numpy(x).cuda(), r, add=add)
    got = r.cpu().numpy()
    assert np.max(np.abs(got - tiny)) <= 1e-12 * np.abs(ax).max()
    outs = []
    for _ in range(3):
        op.residual(torch.from_numpy(x).cuda(), r, add=add)
        outs.append(r.cpu().numpy().copy())
    assert all(exact(o, outs[0]) for o in outs)


def test_lsq_fixed_point_dense_row_lined_up_remainders(cuda):
    """k1='tiles_fixed' on a link that every route crosses (one row holding all
    600k columns) with x = 1/3 everywhere (blocks of 3 at their uniform
    point): every term has the same rounding remainder, so a low word scaled
    by 2^50 per term would take 75k x 2^48 > 2^63 in one tile row and wrap
    (ADVICE r04).  The low word's scale now follows the column count
    (tiles.hpp fx_lo_shift): r matches SciPy to 1e-12, and repeats bit for bit."""
    import torch
    from device import DeviceLSQ
    rs = np.random.RandomState(SEED + 10)
    m, n = 64, 600_000
    rows = [np.arange(n)]                                    # row 0: dense
    for _ in range(1, m):
        rows.append(np.sort(rs.choice(n, 4000, replace=False)))
    indptr = np.concatenate(([0], np.cumsum([len(r) for r in rows])))
    A = sps.csr_matrix((np.ones(indptr[-1]), np.concatenate(rows), indptr), shape=(m, n))
    op = DeviceLSQ(A, A.T.tocsr(), k1='tiles_fixed', k2='panels')
    assert op.k1 == 'tiles_fixed'
    x = np.full(n, 1.0 / 3.0)
    r = torch.empty(m, dtype=torch.float64, device='cuda')
    # the exact row sums (correctly rounded): SciPy's left-to-right sum of
    # 600k equal terms drifts by ~6e-12 relative, the fixed-point one does not
    import math
    ref = np.array([math.fsum(x[A.indices[A.indptr[i]:A.indptr[i + 1]]]) for i in range(m)])
    outs = []
    for _ in range(2):
        op.residual(torch.from_numpy(x).cuda(), r)
        outs.append(r.cpu().numpy().copy())
    np.testing.assert_allclose(outs[0], ref, rtol=1e-12, atol=0)
    assert exact(outs[0], outs[1])
    # and against the reference's own arithmetic (SciPy csr_matvec, main.py:53):
    # within the worst-case error of its left-to-right sum of a row's nnz
    # non-negative terms, gamma_nnz = nnz 2^-53 / (1 - nnz 2^-53) relative
    # (6.7e-11 for the dense row) -- the device's sum is the correctly rounded
    # one, so the gap is SciPy's rounding, bounded by that
    sp = A.dot(x)
    for i in range(m):
        nnz = A.indptr[i + 1] - A.indptr[i]
        gam = nnz * 2.0 ** -53 / (1 - nnz * 2.0 ** -53)
        assert abs(outs[0][i] - sp[i]) <= gam * abs(sp[i]), (i, outs[0][i], sp[i], gam)
