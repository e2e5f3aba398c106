"""Entropic mirror descent over block simplices (reference:
python/mirror_descent.py:7-53), on MI355X.

least_squares(A, b, blocks, iters=1000, tolerance=1e-9) -> x (NumPy), with
`blocks` the list of block sizes.  Per iteration: r = A x - b and g = A' r
(panel operator csrc/lsq.hip for large A, CSR SpMV kernels otherwise), then
one fused kernel (one wave per pack of whole blocks, bsls_md_update_packs)
does x <- x * exp(-t_k g), t_k = sqrt(2 ln k_b) / (sqrt(k) Lf), the per-block
normalisation, ||x_new - x||_inf and the stopping test.  Lf = sigma_max(A) from ARPACK (svds)
driving device matvecs.  The reference's ragged np.array at :10-11 (which
NumPy >= 1.24 rejects) is not reproduced: blocks of any sizes work.
"""
import os

import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as sla

import _native
from _native import check, ptr, stream_handle


def pack_blocks(sizes):
    """Packs of consecutive whole blocks with <= 64 entries for one wave (one
    entry per lane), or a single longer block: (first entry, block-start mask,
    length) per pack (bsls_md_update_packs)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    starts = np.concatenate(([0], np.cumsum(sizes)[:-1]))
    x0, mask, ln = [], [], []
    b, p = 0, sizes.size
    while b < p:
        if sizes[b] > 64:
            x0.append(starts[b]); mask.append(1); ln.append(int(sizes[b]))
            b += 1
            continue
        tot, m = 0, 0
        while b < p and sizes[b] <= 64 and tot + sizes[b] <= 64:
            if tot == 0:
                x0.append(starts[b])
            m |= 1 << tot
            tot += int(sizes[b])
            b += 1
        mask.append(m); ln.append(tot)
    return (np.array(x0, dtype=np.int64), np.array(mask, dtype=np.uint64).view(np.int64),
            np.array(ln, dtype=np.int32))


class MirrorDescent:
    """Device state of mirror_descent.least_squares: A (the x-space operator
    from 2^20 nonzeros up -- `panels` overrides -- else CSR), b, the block
    starts, x, and Lf = sigma_max(A) from ARPACK driving device mat-vecs.
    The operator's residual and gradient walk dealt tile images (BSLS_LSQ_K1 /
    BSLS_LSQ_K2 override): the loop's only test is ||x_new - x||_inf <
    tolerance (mirror_descent.py:50), which never asks f or g to repeat bit for
    bit, so the faster walks with LDS atomic row sums are safe here (BATCH's
    solvers keep the panels)."""

    def __init__(self, A, b, blocks, panels=None):
        import torch
        from device import DeviceCSR, lsq_operator
        L = _native.lib()
        A = sps.csr_matrix(A)
        sizes = np.asarray(blocks, dtype=np.int64)
        n = int(sizes.sum())
        if A.shape[1] != n:
            raise ValueError('blocks cover %d entries, A has %d columns' % (n, A.shape[1]))
        AT = A.T.tocsr()
        self.n, self.sizes = n, sizes
        self.Ad, self.ATd = DeviceCSR(A), DeviceCSR(AT)
        if panels is None:
            panels = A.nnz >= (1 << 20)
        self.lsq = (lsq_operator(A, AT, k1=os.environ.get('BSLS_LSQ_K1', 'tiles'),
                                 k2=os.environ.get('BSLS_LSQ_K2', 'tiles'))
                    if panels else None)
        self.starts = torch.from_numpy(
            np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)).cuda()
        bd = torch.from_numpy(np.asarray(b, dtype=np.float64).ravel()).cuda()
        self.neg_b = -bd
        dev = dict(dtype=torch.float64, device='cuda')
        self.x = torch.empty(n, **dev)
        self.r = torch.empty(A.shape[0], **dev)
        self.g = torch.empty(n, **dev)
        self.state = torch.zeros(3, **dev)
        x0, mask, ln = pack_blocks(sizes)
        self.pk = [torch.from_numpy(a).cuda() for a in (x0, mask, ln)]
        self.npacks = int(x0.size)
        self.ws = torch.zeros(L.bsls_md_pack_workspace_size(self.npacks), dtype=torch.uint8,
                              device='cuda')

        def mv(v):
            return self.Ad.matvec(torch.from_numpy(np.ascontiguousarray(np.real(v).ravel()))
                                  .cuda()).cpu().numpy()

        def rmv(v):
            return self.ATd.matvec(torch.from_numpy(np.ascontiguousarray(np.real(v).ravel()))
                                   .cuda()).cpu().numpy()
        op = sla.LinearOperator(A.shape, matvec=mv, rmatvec=rmv, dtype=np.float64)
        self.Lf = sla.svds(op, 1, return_singular_vectors=False)[0]

    def start(self):
        """x = 1 / block size (mirror_descent.py:9-16), stopping state cleared."""
        import torch
        self.x.copy_(torch.from_numpy(np.repeat(1.0 / self.sizes.astype(float), self.sizes)))
        self.state.zero_()

    def iterate(self, first, count, tolerance):
        """Enqueue iterations first .. first + count - 1 (no host sync)."""
        L = _native.lib()
        for it in range(first, first + count):
            if self.lsq is not None:
                self.lsq.residual(self.x, self.r, add=self.neg_b)
                self.lsq.gradient(self.r, self.g)
            else:
                self.Ad.matvec(self.x, out=self.r, add=self.neg_b)
                self.ATd.matvec(self.r, out=self.g)
            check(L.bsls_md_update_packs(ptr(self.x), ptr(self.g), ptr(self.pk[0]),
                                         ptr(self.pk[1]), ptr(self.pk[2]), self.npacks,
                                         float(np.sqrt(it) * self.Lf), float(tolerance), it,
                                         ptr(self.state), ptr(self.ws), self.ws.numel(),
                                         stream_handle()), 'bsls_md_update_packs')


def least_squares(A, b, blocks, iters=1000, tolerance=1e-9, return_iters=False, poll=16,
                  panels=None):
    """x after at most `iters` steps, stopping at the first whose
    ||x - x_prev||_inf < tolerance (mirror_descent.py:37-51).  The stopping test
    runs on the device (bsls_md_update_gated) and the host reads it every
    `poll` iterations -- iterations enqueued past the stop leave x unchanged."""
    md = MirrorDescent(A, b, blocks, panels=panels)
    md.start()
    poll = max(1, int(poll))
    it = 0
    done = 0
    while done < iters:
        k = min(poll, iters - done)
        md.iterate(done + 1, k, tolerance)
        done += k
        it = done
        st = md.state.cpu().numpy()
        if st[0] != 0.0:
            it = int(st[2])
            break
    out = md.x.cpu().numpy()
    return (out, it) if return_iters else out
