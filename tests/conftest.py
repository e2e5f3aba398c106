import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

SEED = 237423433  # the reference tests' seed


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device)')


@pytest.fixture(scope='session')
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
        return cache[name]
    return load


@pytest.fixture(scope='session')
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    return torch.device('cuda:0')


@pytest.fixture(scope='session')
def parity():
    """parity(tag, err, tol): assert err <= tol and, with BSLS_PARITY_LOG set,
    append {tag, err, tol} to that file (the measured errors the bounds were
    set from: profiles/r06_parity_errors.jsonl)."""
    import json
    path = os.environ.get('BSLS_PARITY_LOG')

    def check(tag, err, tol):
        if path:
            with open(path, 'a') as fh:
                fh.write(json.dumps({'tag': tag, 'err': float(err), 'tol': float(tol)}) + '\n')
        assert err <= tol, (tag, err, tol)
    return check
