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
