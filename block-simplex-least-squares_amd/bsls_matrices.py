"""Load a network .mat and put the problem in standard block-simplex form
(reference: python/bsls_matrices.py).  Host-side one-off preparation (SciPy);
the result is uploaded once to HBM by device.BBEngine.

Pipeline (degree_reduced_form, bsls_matrices.py:51-86):
  consolidate         stack [A; V; T or U] into AA, pick C (U for eq='CP', T for 'OD')
  standard_simplex    scaling = C' d; drop zero-flow routes; x_split = x_true / scaling;
                      AA <- AA diag(scaling)
  cleanup             drop all-zero rows of AA and C
  blockify            sort the routes by block so every block is contiguous
  N, x0               null-space basis and particular solution (bsls_utils)
.mat schema (bsls_utils.generate_data writes it, oned_as='column'): A / A_full /
phi, b / b_full, x_true / real_a, U, f, T, d, V, g.
"""
import logging

import numpy as np
import scipy.io as sio
import scipy.sparse as sps
import scipy.sparse.linalg as sla

from bsls_utils import array, block_sizes_to_N, particular_x0


def _sparse(M):
    if M is None:
        return None
    return sps.csr_matrix(M)


def _present(data, key):
    return key in data and data[key] is not None and np.size(data[key]) > 0


def _stack(X, x, Y, y):
    if X is None:
        return Y, y
    if Y is None:
        return X, x
    return sps.vstack([X, Y]).tocsr(), np.append(x, y)


def _drop_zero_rows(M, v):
    # rows whose SUM is nonzero, as bsls_utils.remove_zero_rows (:55-57)
    keep = np.nonzero(np.asarray(M.sum(axis=1)).ravel())[0]
    return M[keep, :], v[keep], keep


def _assert_scaled_incidence(M, thresh=1e-12):
    """Every column's nonzeros share one value (bsls_utils.py:494-507)."""
    C = sps.csc_matrix(M)
    for j in range(C.shape[1]):
        v = C.data[C.indptr[j]:C.indptr[j + 1]]
        v = v[v != 0]
        if v.size:
            assert np.all(np.abs(v - v[0]) < thresh), \
                'Not a proper scaled incidence matrix, check column entries'


class BSLSMatrices:

    def __init__(self, data=None, fname=None, full=False, L=True, OD=False, CP=False, LP=False,
                 eq=None, init=False, thresh=1e-5, noisy=False):
        self.eq = eq
        if data is None and fname is not None:
            logging.debug('Loading %s...' % fname)
            data = sio.loadmat(fname)
        if data is None:
            raise ValueError('need data or fname')
        (self.rA, self.b, self.rx_true, self.rT, self.d, self.rU, self.f, self.rV, self.g,
         self.nz, self.info) = self.load_raw(data, full=full, L=L, OD=OD, CP=CP, LP=LP,
                                             thresh=thresh, noisy=noisy)
        self.A, self.T, self.U, self.V = self.rA, self.rT, self.rU, self.rV
        self.x_true, self.x_split = self.rx_true, self.rx_true
        self.block_sizes, self.rsort_index, self.scaling = None, None, None
        self.N, self.x0 = None, None
        self.AA = self.bb = self.C = None

    # -- stages ---------------------------------------------------------------
    def simple_simplex_form(self, thresh=1e-5, noisy=False):
        self.consolidate(eq=self.eq)
        self.standard_simplex_form(thresh=thresh, noisy=noisy)
        self.cleanup()
        self.blockify(noisy=noisy)
        if self.AA is None or self.x_split is None:
            self.info['error'] = 'AA,bb is empty'

    def degree_reduced_form(self, init=False):
        self.simple_simplex_form()
        if self.block_sizes is not None:
            self.N = block_sizes_to_N(self.block_sizes)
            self.x0 = self.initial_solution(init=init)
        else:
            self.N = None
            self.x0 = sla.lsmr(self.AA, self.bb)[0]

    def consolidate(self, eq=None):
        AA, bb = _stack(self.A, self.b, self.V, self.g)
        if eq == 'OD':
            self.AA, self.bb = _stack(AA, bb, self.U, self.f)
            self.C, self.d = self.T, self.d
        elif eq == 'CP':
            self.AA, self.bb = _stack(AA, bb, self.T, self.d)
            self.C, self.d = self.U, self.f
        else:
            AA, bb = _stack(AA, bb, self.T, self.d)
            self.AA, self.bb = _stack(AA, bb, self.U, self.f)
            self.C, self.d = None, None

    def standard_simplex_form(self, thresh=1e-30, noisy=False):
        scaling = np.asarray(self.C.T.dot(self.d)).ravel()
        nz = np.nonzero(scaling > thresh)[0]
        self.nz_cols = nz
        scaling = scaling[nz]
        with np.errstate(divide='ignore', invalid='ignore'):
            self.x_split = np.nan_to_num(self.x_true[nz] / scaling)
        self.C = sps.csc_matrix(self.C)[:, nz].tocsr()
        self.AA = (sps.csc_matrix(self.AA)[:, nz] @ sps.diags([scaling], [0])).tocsr()
        self.scaling = scaling

    def cleanup(self):
        self.AA, self.bb, _ = _drop_zero_rows(sps.csr_matrix(self.AA), self.bb)
        self.C, self.d, _ = _drop_zero_rows(sps.csr_matrix(self.C), self.d)

    def blockify(self, noisy=False):
        C = sps.csr_matrix(self.C)
        self.block_sizes = array((C > 0).sum(axis=1)).astype(int)
        rows, cols = C.nonzero()
        # the reference's default-kind argsort (bsls_matrices.py:116): its tie
        # order fixes the column order inside each block, hence the z coordinates
        order = cols[np.argsort(rows)]
        self.AA = sps.csc_matrix(self.AA)[:, order].tocsr()
        self.x_true = self.x_true[order]
        self.x_split = self.x_split[order]
        self.C = sps.csc_matrix(C)[:, order].tocsr()
        self.rsort_index = np.argsort(order)

    def initial_solution(self, init=False):
        if init and self.C is not None:
            return self.direct_solve(self.C, np.ones(self.d.shape), x_split=self.x_split)
        return particular_x0(self.block_sizes)

    @staticmethod
    def reconstruct(x_split, rsort_index=None, scaling=None, nz=None, n=None):
        x_true = np.zeros(n)
        x_true[nz] = x_split[rsort_index] * scaling
        return x_true

    @staticmethod
    def direct_solve(M, m, x_split=None):
        if M.shape[0] == M.shape[1]:
            x0 = sla.spsolve(sps.csc_matrix(M), m)
        else:
            x0 = sla.lsmr(M, m)[0]
        if x_split is not None:
            logging.info('direct solve error: %s' % np.linalg.norm(x0 - x_split))
        return x0

    # -- loading --------------------------------------------------------------
    def load_raw(self, data, full=False, L=True, OD=False, CP=False, LP=False, thresh=1e-5,
                 noisy=False, info=None):
        info = {} if info is None else info
        A = b = nz = None
        if L and full and 'A_full' in data and 'b_full' in data:
            A, b = _sparse(data['A_full']), array(data['b_full'])
        elif L and 'A' in data and 'b' in data:
            A, b = _sparse(data['A']), array(data['b'])
        elif 'phi' in data and 'b' in data:
            A, b = _sparse(data['phi']), array(data['b'])
        if A is not None:
            _assert_scaled_incidence(A)
        if 'b_full' in data:
            info['nAllLinks'] = array(data['b_full']).size
        if b is not None:
            info['nLinks'] = b.size
        if 'x_true' in data:
            x_true = array(data['x_true'])
        elif 'real_a' in data:
            x_true = array(data['real_a'])
        else:
            return NotImplemented
        if A is not None:
            rownnz = np.diff(sps.csr_matrix(A).indptr)
            nz = list(np.nonzero(rownnz == 0)[0])
            keep = np.nonzero(rownnz > 0)[0]
            A, b = A[keep, :], b[keep]
            if not noisy:
                res = np.linalg.norm(A.dot(x_true) - b)
                assert res < thresh, 'Check data input: Ax != b, norm: %s' % res
        T = d = U = f = V = g = None
        if OD and _present(data, 'T') and _present(data, 'd'):
            T, d = _sparse(data['T']), array(data['d'])
            info['nOD'] = d.size
        if CP and _present(data, 'U') and _present(data, 'f'):
            U, f = _sparse(data['U']), array(data['f'])
            info['nCP'] = f.size
        if LP and _present(data, 'V') and _present(data, 'g'):
            V, g = _sparse(data['V']), array(data['g'])
            info['nLP'] = g.size
        return A, b, x_true, T, d, U, f, V, g, nz, info

    def load_data(self, filename, full=True, L=True, OD=True, CP=True, LP=True, thresh=1e-5,
                  noisy=False):
        return self.load_raw(sio.loadmat(filename), full=full, L=L, OD=OD, CP=CP, LP=LP,
                             thresh=thresh, noisy=noisy)

    # -- accessors (bsls_matrices.py:297-322) ----------------------------------
    def get_LSQR(self):
        self.consolidate(eq=None)
        return self.AA, self.bb, self.x_true, self.nz_cols

    def get_CS(self):
        return (self.AA, self.bb, self.N, self.block_sizes, self.x_split, self.nz_cols,
                self.scaling, self.rsort_index, self.x0, self.C)

    def get_BI(self):
        return self.AA, self.bb, self.C, self.x_split, self.scaling, self.block_sizes

    def get_LS(self):
        return (self.AA, self.bb, self.N, self.block_sizes, self.x_split, self.nz_cols,
                self.scaling, self.rsort_index, self.x0)
