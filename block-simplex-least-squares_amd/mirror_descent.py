"""Entropic mirror descent over block simplices (reference:
python/mirror_descent.py:7-53), on MI355X.

least_squares(A, b, blocks, iters=1000, tolerance=1e-9) -> x (NumPy), with
`blocks` the list of block sizes.  Per iteration: r = A x - b and g = A' r
(CSR SpMV kernels, explicit A'), then one fused kernel does
x <- x * exp(-t_k g), t_k = sqrt(2 ln k_b) / (sqrt(k) Lf), the per-block
normalisation and ||x_new - x||_inf.  Lf = sigma_max(A) from ARPACK (svds)
driving device matvecs.  The reference's ragged np.array at :10-11 (which
NumPy >= 1.24 rejects) is not reproduced: blocks of any sizes work.
"""
import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as sla

import _native
from _native import check, ptr, stream_handle


def least_squares(A, b, blocks, iters=1000, tolerance=1e-9, return_iters=False):
    import torch
    from device import DeviceCSR
    L = _native.lib()
    A = sps.csr_matrix(A)
    sizes = np.asarray(blocks, dtype=np.int64)
    n = int(sizes.sum())
    if A.shape[1] != n:
        raise ValueError('blocks cover %d entries, A has %d columns' % (n, A.shape[1]))
    Ad, ATd = DeviceCSR(A), DeviceCSR(A.T.tocsr())
    starts = torch.from_numpy(np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)).cuda()
    x = torch.from_numpy(np.repeat(1.0 / sizes.astype(float), sizes)).cuda()
    bd = torch.from_numpy(np.asarray(b, dtype=np.float64).ravel()).cuda()

    def mv(v):
        return Ad.matvec(torch.from_numpy(np.ascontiguousarray(np.real(v).ravel())).cuda()
                         ).cpu().numpy()

    def rmv(v):
        return ATd.matvec(torch.from_numpy(np.ascontiguousarray(np.real(v).ravel())).cuda()
                          ).cpu().numpy()
    op = sla.LinearOperator(A.shape, matvec=mv, rmatvec=rmv, dtype=np.float64)
    Lf = sla.svds(op, 1, return_singular_vectors=False)[0]
    ws = torch.zeros(L.bsls_md_workspace_size(len(sizes)), dtype=torch.uint8, device='cuda')
    dx = torch.zeros(1, dtype=torch.float64, device='cuda')
    r = torch.empty(A.shape[0], dtype=torch.float64, device='cuda')
    g = torch.empty(n, dtype=torch.float64, device='cuda')
    it = 0
    for it in range(1, iters + 1):
        Ad.matvec(x, out=r, add=-bd)
        ATd.matvec(r, out=g)
        check(L.bsls_md_update(ptr(x), ptr(g), ptr(starts), len(sizes), n,
                               float(np.sqrt(it) * Lf), ptr(dx), ptr(ws), ws.numel(),
                               stream_handle()), 'bsls_md_update')
        if float(dx.item()) < tolerance:
            break
    out = x.cpu().numpy()
    return (out, it) if return_iters else out
