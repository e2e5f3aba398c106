"""Problem algebra and synthetic data (reference: python/bsls_utils.py).

Host-side set-up only (one-off per problem); nothing here runs per iteration.
Kept: the change of variables x = x0 + N z (particular_x0, block_sizes_to_N,
x2z), the reference's generator generate_data (same RNG call sequence, pinned
by tests/golden/solvers.npz gen_*), and lsv_operator for DORE.  Dropped: the
dense-QP experiment helpers (SURVEY.md §2 marks them out of scope).
"""
import logging

import numpy as np
import scipy.io
import scipy.linalg as ssla
import scipy.sparse as sps
import scipy.sparse.linalg as sla

# Constraint / reduction / method tags (bsls_utils.py:23-30)
PROB_SIMPLEX = 'probability simplex'
EQ_CONSTR_ELIM = 'equality constraint elimination'
L_BFGS = 'L-BFGS'
SPG = 'SPG'
ADMM = 'ADMM'


def array(x):
    return np.atleast_1d(np.squeeze(np.array(x)))


def block_e(I, N):
    """Stacked unit vectors: e_{I_k} of length N_k per block (bsls_utils.py:100-101)."""
    out = np.zeros(int(np.sum(N)))
    ends = np.cumsum(N)
    starts = ends - np.asarray(N)
    out[starts + np.asarray(I)] = 1
    return out


def particular_x0(block_sizes):
    """1 at every block's last entry (bsls_utils.py:327-328)."""
    bs = np.asarray(block_sizes)
    return block_e(bs - 1, bs)


def block_sizes_to_N(block_sizes):
    """Null-space basis N (n x (n - p)): +1 at (r+j, c+j), -1 at (r+j+1, c+j)
    (bsls_utils.py:139-162), built vectorised instead of a lil loop."""
    bs = np.asarray(block_sizes, dtype=np.int64).ravel()
    n = int(bs.sum())
    nz = n - bs.size
    xz = np.arange(n) - np.repeat(np.arange(bs.size), bs)
    inner = np.ones(n, dtype=bool)
    inner[np.cumsum(bs) - 1] = False
    i = np.nonzero(inner)[0]
    rows = np.concatenate((i, i + 1))
    cols = np.concatenate((xz[i], xz[i]))
    vals = np.concatenate((np.ones(i.size), -np.ones(i.size)))
    return sps.csr_matrix((vals, (rows, cols)), shape=(n, nz))


def block_starts_to_block_sizes(block_starts, n):
    block_starts = np.asarray(block_starts)
    assert False not in ((block_starts[1:] - block_starts[:-1]) > 0)
    assert block_starts[0] == 0 and block_starts[-1] < n
    return np.append(block_starts[1:], [n]) - block_starts


def x2z(x, block_sizes=None, block_starts=None, lasso=False):
    """z = per-block cumulative sums, each block's last entry dropped (lasso:
    kept) -- bsls_utils.py:267-287."""
    assert block_sizes is not None or block_starts is not None
    x = np.asarray(x)
    if block_sizes is None:
        block_sizes = np.append(block_starts[1:], [x.shape[0]]) - block_starts
    ends = np.cumsum(block_sizes)
    starts = np.hstack(([0], ends[:-1]))
    k = 0 if lasso else 1
    parts = [np.cumsum(x[i:j - k]) for i, j in zip(starts, ends) if i < j - k]
    return np.concatenate(parts) if parts else np.zeros(0)


def lsv_operator(A, N):
    """Largest singular value of A N (bsls_utils.py:334-369): sqrt of the top
    eigenvalue of N'A'AN by ARPACK, applied matrix-free.  A may be a
    device.DeviceCSR pair (then every matvec runs on the GPU and ARPACK only
    orchestrates, as the reference's closures do); N is implied by the layout."""
    if hasattr(A, 'lsv_matvec'):
        op = sla.LinearOperator((A.nz, A.nz), matvec=A.lsv_matvec, dtype=np.float64)
    else:
        op = sla.LinearOperator((N.shape[1], N.shape[1]),
                                matvec=lambda v: N.T.dot(A.T.dot(A.dot(N.dot(v)))),
                                dtype=A.dtype)
    ev = sla.eigs(op, k=1, tol=0, maxiter=None, ncv=10, which='LM', return_eigenvectors=False)
    return np.sqrt(ev)[0].real


def generate_data(fname=None, n=100, m1=5, m2=10, A_sparse=0.5, alpha=1.0, tolerance=1e-10,
                  permute=False, scale=True, in_z=False, distribution='uniform'):
    """The reference's synthetic generator (bsls_utils.py:590-655): A is m1 x n
    (0/1, density 1 - A_sparse), U the m2 x n block-incidence, x Dirichlet(alpha)
    per block scaled by the block flow f, b = A x.  Same RNG draws in the same
    order; block sizes cast to int (NumPy >= 2 refuses float sizes)."""
    if distribution == 'uniform':
        A = (np.random.random((m1, n)) > A_sparse).astype(float)
    elif distribution in ('affine', 'aggregated'):
        if distribution == 'affine':
            spread = 2 * (1 - A_sparse)
            line = (1 - spread) + spread * np.arange(n) / (n - 1)
        else:
            nzero = int(n * A_sparse)
            line = np.array([0.1] * nzero + [.9] * (n - nzero))
        lines = []
        for _ in range(m1):
            j = np.random.randint(n)
            lines.append(np.append(line[j:], line[:j]))
        A = (np.random.random((m1, n)) > np.array(lines)).astype(float)
    else:
        raise ValueError(distribution)
    block_sizes = (np.random.multinomial(n - m2, np.ones(m2) / m2) + np.ones(m2)).astype(int)
    assert sum(block_sizes) == n, 'all-zero row present!'
    block_starts = np.append([0], np.cumsum(block_sizes[:-1])).astype(int)
    x = np.concatenate([np.random.dirichlet(alpha * np.ones(k)) for k in block_sizes])
    U = ssla.block_diag(*[np.ones(k) for k in block_sizes])
    if scale:
        f = np.floor(np.random.random(m2) * 1000)
        x = U.T.dot(f) * x
    else:
        f = np.ones(len(U))
    b = A.dot(x)
    assert np.linalg.norm(U.dot(x) - f) < tolerance, 'Ux!=f'
    assert np.linalg.norm(A.dot(x) - b) < tolerance, 'Ax!=b'
    if permute:
        order = np.random.permutation(n)
        A, U, x = A[:, order], U[:, order], x[order]
    data = {'A': A, 'b': b, 'x_true': x, 'U': U, 'f': f, 'block_starts': block_starts,
            'block_sizes': block_sizes}
    if fname:
        scipy.io.savemat(fname, data, oned_as='column')
    return data


logging.getLogger(__name__).addHandler(logging.NullHandler())
