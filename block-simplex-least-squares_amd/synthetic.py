"""Seeded synthetic block-LSQ problems at benchmark scale.

The recipe follows the reference's generator bsls_utils.generate_data
(python/bsls_utils.py:590-655), made sparse so it scales to 10M routes:
  * block sizes  multinomial(n - p, 1/p) + 1          (bsls_utils.py:625)
  * block flows  f = floor(U * 1000), clamped to >= 1 (bsls_utils.py:635; zero-flow
                 blocks would be dropped by standard_simplex_form)
  * splits       x* ~ Dirichlet(1) per block          (bsls_utils.py:631)
  * A            every column has `per_col` distinct uniform rows out of m, value
                 = that block's f (a scaled incidence matrix, as
                 assert_scaled_incidence requires, bsls_utils.py:494-507)
  * b            A x* (+ multiplicative Gaussian noise for timing runs, as
                 python/main.py:164-166 does).
Host-side data preparation only (numpy); nothing here is on the hot path.

Column sharding (multi-GPU): shard `rank` of `world` owns a contiguous run of
whole blocks; every shard draws its own blocks/columns from its own stream
(seed, rank), rows from the global m.  The full problem is the column
concatenation of the shards.
"""
import numpy as np
import scipy.sparse as sps

SEED = 237423433


def _distinct_rows(rs, m, ncols, per_col):
    rows = rs.randint(0, m, size=(ncols, per_col)).astype(np.int64)
    rows.sort(axis=1)
    while True:
        dup = np.any(rows[:, 1:] == rows[:, :-1], axis=1)
        k = int(dup.sum())
        if k == 0:
            return rows
        fresh = rs.randint(0, m, size=(k, per_col)).astype(np.int64)
        fresh.sort(axis=1)
        rows[dup] = fresh


def make_shard(n, p, m, per_col=16, seed=SEED, rank=0):
    """One column shard: n routes in p blocks over m rows.

    Returns dict(A=csr m x n, AT=csr n x m, block_sizes, x_true, f, Ax=A x_true)."""
    rs = np.random.RandomState([seed, rank])
    sizes = rs.multinomial(n - p, np.ones(p) / p) + 1
    f = np.maximum(np.floor(rs.random_sample(p) * 1000), 1.0)
    # Dirichlet(1) per block == normalised exponentials, vectorised
    e = rs.standard_exponential(n)
    bid = np.repeat(np.arange(p), sizes)
    sums = np.bincount(bid, weights=e, minlength=p)
    x_split = e / sums[bid]
    rows = _distinct_rows(rs, m, n, per_col)
    vals = np.repeat(f[bid], per_col)
    # CSC of A (columns sorted) is exactly the CSR of A'
    indptr = np.arange(0, per_col * (n + 1), per_col, dtype=np.int64)
    AT = sps.csr_matrix((vals, rows.reshape(-1).astype(np.int32), indptr), shape=(n, m))
    A = AT.T.tocsr()
    A.sort_indices()
    Ax = A.dot(x_split)
    return dict(A=A, AT=AT, block_sizes=sizes, x_true=x_split, f=f, Ax=Ax, m=m, n=n, p=p)


def make_partitioned(n, p, m, per_col=16, rank=0, world=1, seed=SEED, gen_chunks=256,
                     need_csr_values=False):
    """Rank `rank`'s column shard of ONE problem that does not depend on `world`
    (strong scaling, BASELINE config C5): block sizes multinomial(n - p, 1/p) + 1
    from one stream; blocks split into `gen_chunks` fixed generation chunks,
    each drawing its flows, Dirichlet splits and rows from its own stream
    (seed, 1000 + k); the shard = the contiguous run of whole blocks that
    distributed.partition_blocks gives this rank (balanced by nnz = per_col x
    routes, bsls_matrices.py:109-126 keeps blocks whole).  The union of the
    shards is the same matrix for every world size.

    Returns dict(A, AT (CSR, scaled incidence: every stored entry of column j
    is colv[j]), colv, block_sizes, x_true, Ax (= A_g x_true_g: sum over ranks
    for b), bounds (block partition), col0 (first column), n, p, m, nnz)."""
    from distributed import partition_blocks
    rs = np.random.RandomState(seed)
    sizes = rs.multinomial(n - p, np.ones(p) / p) + 1
    bounds = partition_blocks(sizes, per_col * sizes.astype(np.float64), world)
    b0, b1 = int(bounds[rank]), int(bounds[rank + 1])
    cb = np.linspace(0, p, gen_chunks + 1).astype(np.int64)
    k0 = int(np.searchsorted(cb, b0, side='right') - 1)
    k1 = int(np.searchsorted(cb, b1, side='left'))
    f_l, x_l, rows_l = [], [], []
    for k in range(k0, k1):
        c0, c1 = int(cb[k]), int(cb[k + 1])
        sz = sizes[c0:c1]
        nk = int(sz.sum())
        crs = np.random.RandomState([seed, 1000 + k])
        f = np.maximum(np.floor(crs.random_sample(c1 - c0) * 1000), 1.0)
        e = crs.standard_exponential(nk)
        bid = np.repeat(np.arange(c1 - c0), sz)
        sums = np.bincount(bid, weights=e, minlength=c1 - c0)
        rows = _distinct_rows(crs, m, nk, per_col)
        # keep this rank's blocks of the chunk
        lo, hi = max(b0, c0) - c0, min(b1, c1) - c0
        xs = np.concatenate(([0], np.cumsum(sz)))
        f_l.append(np.repeat(f[lo:hi], sz[lo:hi]))
        x_l.append((e / sums[bid])[xs[lo]:xs[hi]])
        rows_l.append(rows[xs[lo]:xs[hi]])
    colv = np.concatenate(f_l)
    x_true = np.concatenate(x_l)
    rows = np.concatenate(rows_l)
    ng = colv.shape[0]
    indptr = np.arange(0, per_col * (ng + 1), per_col, dtype=np.int64)
    vals = np.repeat(colv, per_col)
    AT = sps.csr_matrix((vals, rows.reshape(-1).astype(np.int32), indptr), shape=(ng, m))
    A = AT.T.tocsr()
    A.sort_indices()
    Ax = A.dot(x_true)
    col0 = int(sizes[:b0].sum())
    return dict(A=A, AT=AT, colv=colv, block_sizes=sizes[b0:b1], x_true=x_true, Ax=Ax,
                bounds=bounds, col0=col0, n=ng, p=b1 - b0, m=m, nnz=int(A.nnz),
                n_total=n, p_total=p)


def add_noise(b, noise, seed=SEED):
    """b + N(0, (|b| noise)^2) elementwise (python/main.py:164-166)."""
    if not noise:
        return b
    rs = np.random.RandomState([seed, 7919])
    return b + rs.normal(size=b.shape[0]) * (np.abs(b) * noise)


# Benchmark configurations (BASELINE.json configs; SURVEY.md §8 notation)
CONFIGS = {
    'C2': dict(n=3_200_000, p=100_000),                    # proj_simplex in isolation
    'C3': dict(n=1_000_000, p=50_000, m=100_000, per_col=16),
    'C5': dict(n=10_000_000, p=500_000, m=1_000_000, per_col=16),
}


def make_problem(name='C3', noise=0.02, seed=SEED):
    c = CONFIGS[name]
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=seed)
    sh['b'] = add_noise(sh['Ax'], noise, seed)
    return sh


def proj_input(n=3_200_000, p=100_000, kind='unif', seed=SEED):
    """C2 input: y ~ U[0,1) (experiments/test_stress_proj_simplex.py:39) or 5 N(0,1);
    block starts from multinomial sizes (mean n/p)."""
    rs = np.random.RandomState(seed)
    sizes = rs.multinomial(n - p, np.ones(p) / p) + 1
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    y = rs.random_sample(n) if kind == 'unif' else 5.0 * rs.standard_normal(n)
    return y, starts
