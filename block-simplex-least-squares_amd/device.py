"""Device-resident problem state for the block-simplex LSQ hot path (MI355X).

HBM layout of one z-space problem (python/main.py:41-79 restated for the GPU):
  A      CSR, m x n: int64 indptr, int32 indices, fp64 data     (SpMV,  K1)
  A'     CSR, n x m: the explicit transpose (no atomics)         (SpMV', K2)
  target m fp64 = A x0 - b (python/main.py:48)
  x      n fp64 = N z (never materialised N: per-block differences; x0 is in target)
  r      m fp64 residual
  z[2], g[2]   ping-pong iterate / gradient buffers, n_z = n - p fp64 each
  xstarts, zstarts  p int64 block starts in x and z; xz n int32 (z index of an
               x entry, -1 for a block's last entry) -- the N' adjacency
  scal   16 fp64 device scalars (t, f, BB sums, stop flag, iteration)
All compute is in lib/libbsls_hip.so; this module only owns buffers and
sequences calls.
"""
import time

import numpy as np
import scipy.sparse as sps

import _native
from _native import BBProblem, check, ptr, stream_handle


def _torch():
    import torch
    return torch


class DeviceCSR:
    """A CSR matrix resident in HBM (int64 indptr, int32 indices, fp64 data) plus
    its CSR-stream row tiles (<= 2048 nonzeros, <= 1024 rows each; with
    `tile_ends` tiles end only at those rows)."""

    def __init__(self, A, tile_ends=None, group=None):
        torch = _torch()
        A = sps.csr_matrix(A)
        A.sort_indices()
        self.shape = A.shape
        self.m, self.n = A.shape
        self.nnz = int(A.nnz)
        if self.n >= 2 ** 31:
            raise ValueError('column count exceeds int32 indices; shard the columns')
        ip = A.indptr.astype(np.int64)
        self.indptr = torch.from_numpy(ip).cuda()
        self.indices = torch.from_numpy(A.indices.astype(np.int32)).cuda()
        self.data = torch.from_numpy(A.data.astype(np.float64)).cuda()
        tiles = _native.plan_tiles(ip, ends=tile_ends)
        self.ntiles = int(tiles.shape[0] - 1)
        self.tiles = torch.from_numpy(tiles).cuda()
        self.group = group or _native.group_for_rows(self.m / max(self.ntiles, 1))
        self._work = None

    def matvec(self, x, out=None, add=None, alpha=1.0, want_sq=False):
        """out = alpha * (A x) + add ; returns (out, sq) with sq = ||out||^2 (device
        scalar tensor) when want_sq."""
        torch = _torch()
        L = _native.lib()
        if out is None:
            out = torch.empty(self.m, dtype=torch.float64, device='cuda')
        sq = torch.zeros(1, dtype=torch.float64, device='cuda') if want_sq else None
        if self._work is None:
            self._work = torch.zeros(L.bsls_spmv_workspace_size(self.ntiles), dtype=torch.uint8,
                                     device='cuda')
        check(L.bsls_csr_spmv(self.m, ptr(self.indptr), ptr(self.indices), ptr(self.data),
                              ptr(self.tiles), self.ntiles, ptr(x), ptr(add), float(alpha),
                              ptr(out), ptr(sq), self.group, ptr(self._work), self._work.numel(),
                              stream_handle()), 'bsls_csr_spmv')
        return (out, sq) if want_sq else out


def build_sell(A, window=0, col_lo=None, col_hi=None, C=64):
    """SELL-C-64 image of the CSR matrix A (rows of A restricted to columns
    [col_lo, col_hi), global column indices kept).  window > 0 sorts rows by
    length (longest first) inside windows of that many rows to cut padding;
    window = 0 keeps the row order.  Returns host arrays
    (sidx int32 with -1 padding, sval f64, sptr int64 per slice, slot_row int32)."""
    A = sps.csr_matrix(A)
    A.sort_indices()
    m, n = A.shape
    if col_lo is not None:
        A = A[:, col_lo:col_hi].tocsr()
        A.sort_indices()
        A.indices = A.indices + col_lo
    ip = A.indptr.astype(np.int64)
    lens = np.diff(ip)
    if window > 0:
        key = (np.arange(m) // window) * (int(lens.max(initial=0)) + 1) - lens
        order = np.argsort(key, kind='stable')
    else:
        order = np.arange(m)
    nsl = (m + C - 1) // C
    slot_row = np.full(nsl * C, -1, dtype=np.int32)
    slot_row[:m] = order
    slot_len = np.zeros(nsl * C, dtype=np.int64)
    slot_len[:m] = lens[order]
    W = slot_len.reshape(nsl, C).max(axis=1)
    sptr = np.concatenate(([0], np.cumsum(W * C))).astype(np.int64)
    sidx = np.full(int(sptr[-1]), -1, dtype=np.int32)
    sval = np.zeros(int(sptr[-1]), dtype=np.float64)
    inv = np.empty(m, dtype=np.int64)
    inv[order] = np.arange(m)
    rows = np.repeat(np.arange(m, dtype=np.int64), lens)
    k = np.arange(A.nnz, dtype=np.int64) - ip[rows]
    slot = inv[rows]
    dest = sptr[slot // C] + k * C + slot % C
    sidx[dest] = A.indices
    sval[dest] = A.data
    return sidx, sval, sptr, slot_row


class SellChunked:
    """A for K1: SELL-C-64 per column chunk (rows length-sorted in windows),
    concatenated; chunk c is processed by workgroups b with b % nchunk == c."""

    def __init__(self, A, nchunk=8, window=4096):
        torch = _torch()
        A = sps.csr_matrix(A)
        m, n = A.shape
        nchunk = max(1, min(int(nchunk), n))
        bounds = np.linspace(0, n, nchunk + 1).astype(np.int64)
        parts = [build_sell(A, window, bounds[c], bounds[c + 1]) for c in range(nchunk)]
        off = 0
        sptrs, coff = [], [0]
        for (_, _, sp, _) in parts:
            sptrs.append(sp[:-1] + off)
            off += int(sp[-1])
            coff.append(coff[-1] + sp.shape[0] - 1)
        sptr = np.concatenate(sptrs + [np.array([off], dtype=np.int64)])
        self.nchunk = nchunk
        self.maxsl = int(max(sp.shape[0] - 1 for (_, _, sp, _) in parts))
        self.sidx = torch.from_numpy(np.concatenate([p[0] for p in parts])).cuda()
        self.sval = torch.from_numpy(np.concatenate([p[1] for p in parts])).cuda()
        self.sptr = torch.from_numpy(sptr).cuda()
        self.perm = torch.from_numpy(np.concatenate([p[3] for p in parts])).cuda()
        self.coff = torch.from_numpy(np.array(coff, dtype=np.int64)).cuda()
        self.padded = off
        self.nnz = int(A.nnz)


class SellRows:
    """A' for K2: SELL-C-64 with rows in order."""

    def __init__(self, AT):
        torch = _torch()
        sidx, sval, sptr, _ = build_sell(AT, 0)
        self.sidx = torch.from_numpy(sidx).cuda()
        self.sval = torch.from_numpy(sval).cuda()
        self.sptr = torch.from_numpy(sptr).cuda()
        self.padded = int(sptr[-1])


class BlockLayout:
    """Block structure of x (sizes k_b) and of z (sizes k_b - 1), on device."""

    def __init__(self, block_sizes):
        torch = _torch()
        bs = np.asarray(block_sizes, dtype=np.int64)
        if bs.ndim != 1 or bs.size == 0 or np.any(bs < 1):
            raise ValueError('block_sizes must be positive')
        self.sizes = bs
        self.p = int(bs.size)
        self.n = int(bs.sum())
        self.nz = self.n - self.p
        self.xstarts_h = np.concatenate(([0], np.cumsum(bs)[:-1])).astype(np.int64)
        self.zstarts_h = self.xstarts_h - np.arange(self.p, dtype=np.int64)
        xz = np.arange(self.n, dtype=np.int64)
        xz -= np.repeat(np.arange(self.p, dtype=np.int64), bs)
        xz[np.cumsum(bs) - 1] = -1
        self.xstarts = torch.from_numpy(self.xstarts_h).cuda()
        self.zstarts = torch.from_numpy(self.zstarts_h).cuda()
        self.xz = torch.from_numpy(xz.astype(np.int32)).cuda()
        self.max_block = int(bs.max())
        self.max_zblock = self.max_block - 1
        self._packs = None

    def packs(self):
        """K3 packs (csrc/bb.hip): consecutive whole z-blocks with <= 64 z entries
        for one wave, or a single longer block.  Host-planned once."""
        if self._packs is None:
            torch = _torch()
            kz = self.sizes - 1
            z0, b0, mask, ln = [], [], [], []
            b = 0
            p = self.p
            zst = self.zstarts_h
            while b < p:
                if kz[b] > 64:
                    z0.append(zst[b]); b0.append(b); mask.append(1); ln.append(int(kz[b]))
                    b += 1
                    continue
                tot, m_, e = 0, 0, b
                while e < p and kz[e] <= 64 and tot + kz[e] <= 64:
                    m_ |= 1 << tot
                    tot += int(kz[e])
                    e += 1
                z0.append(zst[b]); b0.append(b); mask.append(m_); ln.append(tot)
                b = e
            mask = np.array(mask, dtype=np.uint64).view(np.int64)
            self._packs = dict(
                z0=torch.from_numpy(np.array(z0, dtype=np.int64)).cuda(),
                b0=torch.from_numpy(np.array(b0, dtype=np.int64)).cuda(),
                mask=torch.from_numpy(mask).cuda(),
                len=torch.from_numpy(np.array(ln, dtype=np.int32)).cuda(),
                n=len(z0))
        return self._packs


class BBEngine:
    """Fused z-space projected BB (python/BB.py:7-45 over python/main.py:53-65).

    The device runs K2 -> K3 -> K1 per iteration (bsls_bb_iterate); the stop
    test, the BB step and every reduction stay on the device.  The host polls
    the scalar block every `poll` iterations and at each `record_every`
    boundary, to log states exactly where BB.solve logs them.
    """

    def __init__(self, A, b, block_sizes, options=None, early_exit=True, A_dev=None,
                 AT_dev=None, AT=None, target=None, x0=None):
        torch = _torch()
        L = _native.lib()
        self.layout = lay = BlockLayout(block_sizes)
        A = sps.csr_matrix(A)
        if A.shape[1] != lay.n:
            raise ValueError('A has %d columns but the blocks cover %d' % (A.shape[1], lay.n))
        AT = sps.csr_matrix(AT) if AT is not None else A.T.tocsr()
        self.A = A_dev or DeviceCSR(A)
        self.AT = AT_dev or DeviceCSR(AT)
        # the fused kernels' images: A chunked by columns (K1), A' by rows (K2)
        self.A_sell = SellChunked(A)
        self.AT_sell = SellRows(AT)
        self.m, self.n, self.nz = A.shape[0], lay.n, lay.nz
        opts = options or {}
        self.options = dict(opts)
        dev = dict(dtype=torch.float64, device='cuda')
        x = x0
        # x0 = particular_x0 (bsls_utils.py:327-328): 1 at each block's last entry
        x0 = torch.zeros(lay.n, **dev)
        x0[torch.from_numpy(np.cumsum(lay.sizes) - 1).cuda()] = 1.0
        self.x0 = x0
        if target is not None:
            # column-sharded: the caller formed sum_g A_g x0_g - b (distributed.py)
            self.target = torch.as_tensor(target, dtype=torch.float64).cuda().contiguous()
        else:
            # target = A x0 - b (python/main.py:48), on the device; x0 defaults
            # to the particular solution, as BSLSMatrices.initial_solution does
            xin = x0 if x is None else torch.as_tensor(np.asarray(x, dtype=np.float64)).cuda()
            b_dev = torch.as_tensor(np.asarray(b, dtype=np.float64)).cuda()
            self.target = torch.empty(self.m, **dev)
            self.A.matvec(xin, out=self.target, add=-b_dev)
        self.z = [torch.zeros(max(self.nz, 1), **dev) for _ in range(2)]
        self.g = [torch.zeros(max(self.nz, 1), **dev) for _ in range(2)]
        self.x = torch.empty(lay.n, **dev)
        self.r = torch.empty(self.m, **dev)
        self.scal = torch.zeros(_native.S_COUNT, **dev)
        self.work = torch.zeros(L.bsls_bb_workspace_size(self.m, self.n, self.nz),
                                dtype=torch.uint8, device='cuda')
        self.rpart = torch.zeros(self.A_sell.nchunk * self.m, **dev)
        P = BBProblem()
        P.m, P.n, P.nz, P.nblocks = self.m, lay.n, lay.nz, lay.p
        S = self.A_sell
        P.A_sidx, P.A_sval, P.A_sptr = S.sidx.data_ptr(), S.sval.data_ptr(), S.sptr.data_ptr()
        P.A_perm, P.A_coff = S.perm.data_ptr(), S.coff.data_ptr()
        P.A_nchunk, P.A_maxsl, P.rpart = S.nchunk, S.maxsl, self.rpart.data_ptr()
        T = self.AT_sell
        P.AT_sidx, P.AT_sval, P.AT_sptr = T.sidx.data_ptr(), T.sval.data_ptr(), T.sptr.data_ptr()
        P.target = self.target.data_ptr()
        P.xstarts, P.zstarts, P.xz = (lay.xstarts.data_ptr(), lay.zstarts.data_ptr(),
                                      lay.xz.data_ptr())
        if np.any(lay.sizes < 2):
            # a one-route block has no z coordinate; the reference's projection
            # asserts on it too (strictly increasing z-starts, c_extensions.pyx:78)
            raise ValueError('every block needs at least 2 routes')
        pk = lay.packs()
        P.pk_z0, P.pk_b0, P.pk_mask, P.pk_len = (pk['z0'].data_ptr(), pk['b0'].data_ptr(),
                                                 pk['mask'].data_ptr(), pk['len'].data_ptr())
        P.npacks = pk['n']
        P.z[0], P.z[1] = self.z[0].data_ptr(), self.z[1].data_ptr()
        P.g[0], P.g[1] = self.g[0].data_ptr(), self.g[1].data_ptr()
        P.x, P.r, P.scal, P.work = (self.x.data_ptr(), self.r.data_ptr(), self.scal.data_ptr(),
                                    self.work.data_ptr())
        P.max_zblock = lay.max_zblock
        P.max_iter = int(opts.get('max_iter', 300000))
        P.opt_tol = float(opts.get('opt_tol', 1e-6))
        P.early_exit = 1 if early_exit else 0
        self.P = P
        self.z0 = None

    # -- raw device steps ------------------------------------------------------
    def set_z0(self, z0):
        torch = _torch()
        z0 = torch.as_tensor(z0, dtype=torch.float64).cuda().reshape(-1)
        if z0.numel() != self.nz:
            raise ValueError('z0 has %d entries, expected %d' % (z0.numel(), self.nz))
        self.z[0][:self.nz].copy_(z0)
        self.z0 = z0

    def prologue(self):
        check(_native.lib().bsls_bb_prologue(self.P, stream_handle()), 'bsls_bb_prologue')

    def iterate(self, first, count):
        check(_native.lib().bsls_bb_iterate(self.P, int(first), int(count), stream_handle()),
              'bsls_bb_iterate')

    def stage(self, k, it):
        """One building block of an iteration (bsls_bb_stage, include/bsls_hip.h)."""
        check(_native.lib().bsls_bb_stage(self.P, int(k), int(it), stream_handle()),
              'bsls_bb_stage %d' % k)

    # -- closures of main.solve_in_z (python/main.py:53-65), on the device ------
    def n_apply(self, z, with_x0=False, out=None):
        """N z (or x0 + N z) without materialising N."""
        torch = _torch()
        if out is None:
            out = torch.empty(self.n, dtype=torch.float64, device='cuda')
        check(_native.lib().bsls_n_apply(ptr(out), ptr(z), ptr(self.layout.xstarts),
                                         self.layout.p, self.n, 1 if with_x0 else 0,
                                         stream_handle()), 'bsls_n_apply')
        return out

    def nt_apply(self, w, out=None):
        """N' w."""
        torch = _torch()
        if out is None:
            out = torch.empty(max(self.nz, 1), dtype=torch.float64, device='cuda')
        check(_native.lib().bsls_nt_apply(ptr(w), ptr(out), ptr(self.layout.xstarts),
                                          self.layout.p, self.n, stream_handle()),
              'bsls_nt_apply')
        return out[:self.nz]

    def residual(self, z, alpha=1.0):
        """alpha A N z + alpha target (DORE scales A and target by alpha)."""
        r = self.A.matvec(self.n_apply(z), alpha=alpha)
        return r.add_(self.target, alpha=alpha) if alpha != 1.0 else r.add_(self.target)

    def f(self, z):
        """0.5 ||A N z + target||^2 (main.py:53)."""
        nr = float(self.residual(z).norm())
        return 0.5 * nr ** 2

    def nabla_f(self, z):
        """N' A' (A N z + target) (main.py:54)."""
        return self.nt_apply(self.AT.matvec(self.residual(z)))

    def proj(self, z):
        """isotonic_regression_multi_c on the z-blocks, then clip to [0, 1]
        (main.py:61-65); returns a new tensor like np.maximum(np.minimum(..))."""
        torch = _torch()
        L = _native.lib()
        if self.layout.max_zblock < 1 or np.any(self.layout.sizes < 2):
            raise AssertionError   # the reference's strictly-increasing z-starts assert
        y = z.clone()
        if not hasattr(self, '_iso_ws'):
            self._iso_ws = torch.zeros(L.bsls_isotonic_workspace_size(self.nz),
                                       dtype=torch.uint8, device='cuda')
        check(L.bsls_isotonic_multi(1, ptr(y), ptr(self.layout.zstarts), self.layout.p, self.nz,
                                    None, 1, self.layout.max_zblock, ptr(self._iso_ws),
                                    self._iso_ws.numel(), None, stream_handle()),
              'bsls_isotonic_multi')
        return torch.clamp(y, 0.0, 1.0)

    def lsv_matvec(self, v):
        """N'A'A N v for ARPACK (bsls_utils.lsv_operator), on the device."""
        torch = _torch()
        vd = torch.from_numpy(np.ascontiguousarray(np.real(v), dtype=np.float64)).cuda()
        w = self.AT.matvec(self.A.matvec(self.n_apply(vd)))
        return self.nt_apply(w).cpu().numpy()

    def scalars(self):
        return self.scal.cpu().numpy()

    def current_z(self, zbuf):
        return self.z[int(zbuf)][:self.nz]

    # -- BB.solve semantics ------------------------------------------------------
    def solve(self, z0=None, log=None, record_every=500, poll=50, to_host=True):
        """Run BB to its stopping rule; log(i, state, dt) exactly where
        python/BB.py:10,40-44 logs.  Returns the final z (device tensor)."""
        torch = _torch()
        if z0 is None:
            z0 = torch.zeros(self.nz, dtype=torch.float64)   # x2z(particular_x0) == 0
        self.set_z0(z0)
        keep = (lambda t: t.cpu().numpy().copy()) if to_host else (lambda t: t.clone())
        if log is None:
            log = lambda i, s, d: time.time()
        start = log(0, keep(self.z0), 0)
        self.prologue()
        i = 0
        max_iter = self.P.max_iter
        warned = 0
        while True:
            nxt = min((i // record_every + 1) * record_every, i + poll, max_iter)
            if nxt <= i:
                nxt = i + 1
            self.iterate(i + 1, nxt - i)
            i = nxt
            s = self.scalars()
            if s[_native.S_WARN] > warned:
                print('BB update is having some trouble, implement fix! t=%8.5e'
                      % s[_native.S_T])
                warned = s[_native.S_WARN]
            stop = int(s[_native.S_STOP])
            last = int(s[_native.S_ITER]) if stop else i
            zb = int(s[_native.S_ZBUF]) if stop else (i & 1)
            if stop != _native.STOP_NOCHANGE and last % record_every == 0:
                start = log(last, keep(self.current_z(zb)), time.time() - start)
            if stop:
                if stop == _native.STOP_NOCHANGE:
                    print('Exiting... no change in gradient')
                self.stop_reason = stop
                self.iterations = last
                log(last, keep(self.current_z(zb)), time.time() - start)
                return self.current_z(zb)

    def run_fixed(self, iters):
        """Enqueue exactly `iters` iterations (no host sync, no logging)."""
        self.iterate(1, iters)
