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
import ctypes
import time

import os

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


def even_bounds(lo, hi, parts):
    """parts + 1 increasing even column bounds from lo to hi (hi itself may be odd):
    chunk starts stay 16-B aligned for the LDS staging (panels.hpp)."""
    b = np.round(np.linspace(lo, hi, parts + 1) / 2.0).astype(np.int64) * 2
    b[0], b[-1] = lo, hi
    return np.unique(b)


def chunk_plan(ncols, ngroups, chunk=None):
    """Column chunks (<= chunk wide) nested in `ngroups` groups of near-equal
    width.  Returns (chunk_col, group_chunk)."""
    chunk = int(chunk or _native.PANEL_CHUNK)
    ngroups = max(1, min(int(ngroups), (ncols + 1) // 2))
    gb = even_bounds(0, ncols, ngroups)
    cols, gch = [0], [0]
    for g in range(gb.size - 1):
        w = int(gb[g + 1] - gb[g])
        k = max(1, -(-w // chunk))
        cb = even_bounds(int(gb[g]), int(gb[g + 1]), k)
        while np.any(np.diff(cb) > chunk):
            k += 1
            cb = even_bounds(int(gb[g]), int(gb[g + 1]), k)
        cols.extend(cb[1:].tolist())
        gch.append(len(cols) - 1)
    return np.array(cols, dtype=np.int64), np.array(gch, dtype=np.int64)


class PanelOverflow(ValueError):
    """A 64-row slice holds more entries in one chunk than the panel format's
    16-bit running counts address (dense rows): the caller falls back to
    another format (BBEngine: streamed tiles; DeviceLSQ users: the CSR kernels)."""


def build_panels(M, prow, halo=False, chunk_col=None, group_chunk=None, values=True):
    """Panel image of the CSR matrix M (include/bsls_hip.h struct bsls_panels,
    csrc/panels.hpp).  Host arrays in a dict; `values=False` drops the entry
    values (scaled incidence).  Vectorised: two sorts over the entries."""
    M = sps.csr_matrix(M)
    M.sort_indices()
    R, C = M.shape
    PW = _native.PANEL_WAVES
    prow = int(prow)
    if not 1 <= prow <= _native.PANEL_ROWS or prow + int(halo) > 256:
        raise ValueError('prow out of range')
    if chunk_col is None:
        chunk_col, group_chunk = chunk_plan(C, 1)
    chunk_col = np.asarray(chunk_col, dtype=np.int64)
    group_chunk = np.asarray(group_chunk, dtype=np.int64)
    widths = np.diff(chunk_col)
    if np.any(widths > _native.PANEL_CHUNK) or np.any(chunk_col[:-1] % 2):
        raise ValueError('bad chunk plan')
    nch = chunk_col.size - 1
    npan = max(1, -(-R // prow))
    nrb = -(-npan // PW)
    nsegs = nrb * nch * PW
    ip = M.indptr.astype(np.int64)
    rows = np.repeat(np.arange(R, dtype=np.int64), np.diff(ip))
    cols = M.indices.astype(np.int64)
    vals = M.data
    pn = rows // prow
    lr = rows - pn * prow
    if halo:
        # row 0 of panel p > 0 is also local row prow of panel p - 1
        h = np.nonzero((lr == 0) & (pn > 0))[0]
        pn = np.concatenate([pn, pn[h] - 1])
        lr = np.concatenate([lr, np.full(h.size, prow, dtype=np.int64)])
        cols = np.concatenate([cols, cols[h]])
        vals = np.concatenate([vals, vals[h]])
    ch = np.searchsorted(chunk_col, cols, side='right') - 1
    seg = ((pn // PW) * nch + ch) * PW + pn % PW
    # storage order: segment, row (slice-major), then the row's entries by
    # column, each row's run padded to an even length (aligned pair loads)
    key = seg * 256 + lr
    order = np.argsort(key, kind='stable')
    key, cols, ch, vals = key[order], cols[order], ch[order], vals[order]
    E = key.size
    cnt_all = np.bincount(key, minlength=nsegs * 256).reshape(nsegs, 4, 64)
    D = cnt_all.max(axis=2)                       # nsegs x 4 (<= chunk width < 2^16)
    live = D > 0
    padc = cnt_all + (cnt_all & 1)
    incl = np.cumsum(padc, axis=2)                # per slice, inclusive over lanes
    if incl[:, :, 63].max(initial=0) > 0xFFFE:
        raise PanelOverflow('a 64-row slice has more than 65534 entries in one chunk')
    cnt = (incl | (cnt_all & 1))[live].astype(np.uint16).reshape(-1)
    cnt_off = np.concatenate(([0], np.cumsum(64 * live.sum(axis=1)))).astype(np.int64)
    ne = padc.sum(axis=(1, 2))
    ent_off = np.concatenate(([0], np.cumsum(ne))).astype(np.int64)
    seg_info = (D[:, 0] | (D[:, 1] << 16) | (D[:, 2] << 32) | (D[:, 3] << 48)).astype(np.int64)
    Ep = int(ent_off[-1])
    slack = 64
    ent = np.zeros(Ep + slack, dtype=np.uint16)
    val = np.zeros(Ep + slack, dtype=np.float64) if values else None
    if E:
        flat = padc.reshape(nsegs, 256)
        excl = (np.cumsum(flat, axis=1) - flat).reshape(-1)       # per (seg, row)
        newp = np.empty(E, dtype=bool)
        newp[0] = True
        np.not_equal(key[1:], key[:-1], out=newp[1:])
        pstart = np.nonzero(newp)[0]
        k = np.arange(E, dtype=np.int64) - np.repeat(pstart, np.diff(np.append(pstart, E)))
        dest = ent_off[key >> 8] + excl[key] + k
        ent[dest] = (cols - chunk_col[ch]).astype(np.uint16)
        if values:
            val[dest] = vals
    return dict(rows=R, cols=C, prow=prow, halo=int(bool(halo)), npanels=npan, nchunks=nch,
                ngroups=group_chunk.size - 1, tab_cap=max(64, int(widths.max(initial=2))),
                chunk_col=chunk_col, group_chunk=group_chunk, ent_off=ent_off, cnt_off=cnt_off,
                seg_info=seg_info, cnt=np.concatenate([cnt, np.zeros(64, np.uint16)]),
                ent=ent, val=val, nnz=E, stored=Ep)


def panels_matvec(img, x, colv=None):
    """Host restatement of the kernels' walk over a panel image (panel_segment
    in csrc/panels.hpp): per chunk group, row sums entry by entry in storage
    order; the group partials then added in group order (K1b).  Returns the
    kernels' bit pattern and, for the last group, the per-panel sums including
    halo rows.  Test helper (numpy, vectorised per diagonal)."""
    R, prow, halo = img['rows'], img['prow'], img['halo']
    nch = img['nchunks']
    PW = _native.PANEL_WAVES
    x = np.asarray(x, dtype=np.float64)
    parts = []
    for g in range(img['ngroups']):
        acc = np.zeros((img['npanels'], 256))
        for c in range(img['group_chunk'][g], img['group_chunk'][g + 1]):
            c0 = img['chunk_col'][c]
            for p in range(img['npanels']):
                sgi = ((p // PW) * nch + c) * PW + p % PW
                info = int(img['seg_info'][sgi])
                e = int(img['ent_off'][sgi])
                co = int(img['cnt_off'][sgi])
                for q in range(4):
                    Dq = (info >> (16 * q)) & 0xFFFF
                    if Dq == 0:
                        continue
                    st = img['cnt'][co:co + 64].astype(np.int64)
                    co += 64
                    inc = st & ~1
                    cnp = np.diff(np.concatenate(([0], inc)))          # padded counts
                    start = e + inc - cnp
                    cn = cnp - (st & 1)
                    rr = 64 * q + np.arange(64)
                    for k in range(Dq):
                        a = cn > k
                        t = x[c0 + img['ent'][start[a] + k].astype(np.int64)]
                        if img['val'] is not None:
                            acc[p, rr[a]] = acc[p, rr[a]] + img['val'][start[a] + k] * t
                        elif colv is not None:
                            acc[p, rr[a]] = acc[p, rr[a]] + colv[p * prow + rr[a]] * t
                        else:
                            acc[p, rr[a]] = acc[p, rr[a]] + t
                    e += int(cnp.sum())
        parts.append(acc)
    out = parts[0][:, :prow].reshape(-1)[:R].copy()
    for acc in parts[1:]:
        out = out + acc[:, :prow].reshape(-1)[:R]
    return out, parts[-1][:, :prow + halo]


def scaled_incidence_scale(A):
    """colv with A[i, j] == colv[j] for every stored entry, or None
    (bsls_utils.assert_scaled_incidence, bsls_utils.py:494-507, made exact)."""
    C = sps.csc_matrix(A)
    C.sort_indices()
    n = C.shape[1]
    lens = np.diff(C.indptr)
    colv = np.zeros(n)
    has = lens > 0
    colv[has] = C.data[C.indptr[:-1][has]]
    if C.nnz and not np.array_equal(C.data, np.repeat(colv, lens)):
        return None
    return colv


class DevicePanels:
    """A panel image on the device + the ctypes struct pointing at it."""

    def __init__(self, M, prow, halo=False, ngroups=1, values=True, img=None, chunk=None):
        torch = _torch()
        img = img or build_panels(M, prow, halo, *chunk_plan(M.shape[1], ngroups, chunk=chunk),
                                  values=values)
        self.img = img
        self.nnz = img['nnz']
        self.t = {}
        for k in ('chunk_col', 'group_chunk', 'ent_off', 'cnt_off', 'seg_info'):
            self.t[k] = torch.from_numpy(np.ascontiguousarray(img[k], dtype=np.int64)).cuda()
        self.t['cnt'] = torch.from_numpy(img['cnt'].view(np.int16)).cuda()
        self.t['ent'] = torch.from_numpy(img['ent'].view(np.int16)).cuda()
        if img['val'] is not None:
            self.t['val'] = torch.from_numpy(img['val']).cuda()
        S = _native.Panels()
        for k in ('rows', 'cols', 'prow', 'halo', 'npanels', 'nchunks', 'ngroups', 'tab_cap'):
            setattr(S, k, int(img[k]))
        for k, v in self.t.items():
            setattr(S, k, v.data_ptr())
        self.struct = S

    def bytes(self):
        return sum(v.numel() * v.element_size() for v in self.t.values())


def tile_plan(rows, cols, halo=0, colv_lds=False, cus=256, l2_slice=None, env=None, layout=0,
              nnz=None):
    """(H, ngroups, order) of a tile image (include/bsls_hip.h struct bsls_tiles,
    csrc/tiles.hpp): column groups (a power of two) until one group's slice of
    the gathered vector fits an XCD's L2 (order 1, XCD-sequential, past 8
    groups); row blocks as tall as the LDS holds (half of it when K2 keeps the
    column scales beside the sums: scaled incidence, one group), at least one
    workgroup per CU, the grid rounded up to whole rounds of `cus` workgroups.
    The environment variable `env` ("H,groups") overrides it."""
    plan = os.environ.get(env) if env else None
    if plan:
        v = [int(a) for a in plan.split(',')]
        H, G = v[0], v[1]
        return H, G, (v[2] if len(v) > 2 else (1 if G > 8 else 0))
    if layout in (1, 2):
        # dealt image: one round of workgroups (one per CU); K1 with as many
        # column groups, up to 8, as keep its row blocks within the LDS -- a
        # narrower group puts more of a tile's entries on each gathered line,
        # past 8 the last-arriving workgroups' group sums make a tail.
        # Measured (tools/stage_time.py): C3 K1 G x row blocks 8 x 32 34.0 us
        # (4 x 64: 36.5, 16 x 16: 51.8, 2 x 128: 46.9, 8 x 64: 46.6, 32 x 8:
        # 126); C5 K1 4 x 64 374 us (the most the LDS allows in one round;
        # 8 x 64: 400, 16: 526, 32: 812; 2 / 1 groups leave CUs idle: 698 /
        # 1303).  K2 (the routes' rows: partial sums of n rows are dear) one
        # group: C3 256 row blocks 36.9 us (128: 48.9, 500: 47.0), C5 512
        # row blocks 370 us (before the row-sum scaling: 2 groups 611, 4: 775
        # against 503).
        mult = 2 if colv_lds else 1
        hmax = _native.TILE_LDS_BYTES // (8 * mult) - 1 - halo
        G = 1
        if not halo:
            G = 8
            while G > 1 and (-(-rows * G // cus) > hmax or G > cols):
                G //= 2
        nmin = -(-rows // hmax)
        nrb = max(nmin, cus // G)
        nrb = -(-(nrb * G) // cus) * cus // G if nrb * G > cus else nrb
        H = max(64, -(-rows // nrb))
        # (K2 tiles as sparse as a C5 shard over 8 GPUs, 0.08 entries per
        # column, were given two groups of twice the rows until round 4: the
        # kernel alone 78.0 -> 72.5 us, but the rehearsed iteration is faster
        # with one group -- 160.7 against 149.6 us, 162.5 against 154.4 in an
        # earlier session -- the groups' partial row sums (2 x 10 MB through the
        # Infinity Cache) cost K1 and K3 more than K2 gains; tools/shard_ab_r04.sh)
        return int(H), int(G), 0
    if l2_slice is None:
        # measured on the C5 shard (tools/stage_time.py): K1 fastest with
        # 2.5-MB slices of x (4 groups: 112 us, 8: 148 us), K2 with the whole
        # 8-MB r in one group (117 us; 2: 122, 4: 150) -- one group also keeps
        # K2 bit-identical to SciPy
        l2_slice = (8 << 20) if halo else (3 << 20)
    G = 1
    while 8 * cols / G > l2_slice and G < 64:
        G *= 2
    G = max(1, min(G, cols))
    order = 1 if G > 8 else 0
    mult = 2 if (colv_lds and G == 1) else 1
    if layout == 1:
        hmax = _native.TILE_LDS_BYTES // (8 * mult) - 1 - halo      # rows + the dummy row
    else:
        per = _native.TILE_LDS_BYTES // (8 * _native.TILE_THREADS * mult) - 1
        hmax = per * _native.TILE_THREADS - halo
    nrb = max(-(-rows // hmax), -(-cus // G))
    nrb = -(-(nrb * G) // cus) * cus // G if nrb * G > cus else nrb
    H = max(64, -(-rows // nrb))
    return int(H), int(G), int(order)


def spmv_format(M, fmt=None, dealt=True):
    """'panels' or 'tiles' for the fused SpMV over matrix M (rows x cols).
    With the dealt tile layout available (`dealt`, i.e. not a deterministic
    engine) always tiles: measured on C3 (tools/stage_time.py --fmt) K1 34.0
    against the panels' 43.0 us, K2 36.9 against 41.4; on C5 the panels idle
    (0.3 entries per row per chunk).  Deterministic engines keep the panels
    while a panel chunk (BSLS_PANEL_CHUNK columns) holds at least one entry
    per row on average (C3: 3.2), the thread-stream tiles below that
    (csrc/tiles.hpp).  fmt / BSLS_SPMV_FORMAT force one."""
    fmt = fmt or os.environ.get('BSLS_SPMV_FORMAT') or 'auto'
    if fmt != 'auto':
        if fmt not in ('panels', 'tiles'):
            raise ValueError('unknown SpMV format %r' % fmt)
        return fmt
    if dealt:
        return 'tiles'
    R, C = M.shape
    lam = (M.nnz / max(R, 1)) * min(_native.PANEL_CHUNK, C) / max(C, 1)
    return 'tiles' if lam < 1.0 else 'panels'


def tiles_matvec(img, x, colv=None, group_sums=False):
    """Host restatement of the tile kernels' walk (csrc/tiles.hpp) over an image
    from _native.tiles_build: per (row block, group) each row summed entry by
    entry in stream order, the groups then added in group order.  Returns the
    row sums (halo rows dropped).  Test helper (NumPy, vectorised per quad)."""
    R, H, halo, G = img['rows'], img['H'], img['halo'], img['ngroups']
    T = _native.TILE_THREADS
    gc = img['group_col']
    x = np.asarray(x, dtype=np.float64)
    if img.get('layout', 0) in (1, 2):
        return _dealt_matvec(img, x, colv, group_sums)
    nslots = -(-(H + halo) // T)
    out = np.zeros(R)
    parts = []
    for g in range(G):
        acc = np.zeros(R)
        for rb in range(img['nrb']):
            rows = np.zeros((nslots + 1) * T)
            for w in range(16):
                s = (rb * G + g) * 16 + w
                q0, q1 = int(img['wave_off'][s]), int(img['wave_off'][s + 1])
                lanes = w * 64 + np.arange(64)
                for q in range(q0, q1, 64):
                    for j in range(4):
                        e = img['ent'][4 * (q + np.arange(64)) + j].astype(np.int64)
                        lr = (e >> 24) * T + lanes
                        xv = x[gc[g] + (e & 0xFFFFFF)]
                        if img['val'] is not None:
                            t = img['val'][4 * (q + np.arange(64)) + j] * xv
                        elif colv is not None:
                            rr = np.minimum(rb * H + lr, R - 1)
                            t = np.where(lr < H + halo, colv[rr], 0.0) * xv
                        else:
                            t = xv
                        rows[lr] = rows[lr] + t
            r0 = rb * H
            r1 = min(r0 + H, R)
            acc[r0:r1] = rows[:r1 - r0]
        parts.append(acc)
    out = parts[0].copy()
    for a in parts[1:]:
        out = out + a
    return (out, parts) if group_sums else out


def _dealt_matvec(img, x, colv=None, group_sums=False):
    """tiles_matvec for a layout-1 (dealt) image: every (quad-step, wave, slot,
    lane) entry added to its row (the device adds them with LDS atomics in no
    fixed order; the sums agree to rounding)."""
    R, H, halo, G = img['rows'], img['H'], img['halo'], img['ngroups']
    gc, wo = img['group_col'], img['wave_off']
    ent = img['ent'].astype(np.int64)
    cb = 16
    if img.get('layout', 1) == 2:
        # 3-byte entries: unpack every lane's 3 words into the 4-per-lane form
        cb = 24 - int(H + halo).bit_length()
        nl = int(wo[-1]) * 1024
        w = ent[:3 * nl].reshape(-1, 3)
        u = np.empty((nl, 4), dtype=np.int64)
        u[:, 0] = w[:, 0] & 0xFFFFFF
        u[:, 1] = (w[:, 0] >> 24) | ((w[:, 1] & 0xFFFF) << 8)
        u[:, 2] = (w[:, 1] >> 16) | ((w[:, 2] & 0xFF) << 16)
        u[:, 3] = w[:, 2] >> 8
        ent = u.reshape(-1)
    cmask = (1 << cb) - 1
    parts = []
    for g in range(G):
        acc = np.zeros(R)
        for rb in range(img['nrb']):
            t = rb * G + g
            q0, q1 = int(wo[t]), int(wo[t + 1])
            if q1 == q0:
                continue
            rows = np.zeros(H + halo + 1)
            lanes = np.arange(64)
            for q in range(q0, q1):
                for w in range(16):
                    u = ((q * 16 + w) * 64 + lanes) * 4
                    for j in range(4):
                        e = ent[u + j]
                        lr = e >> cb
                        col = gc[g] + int(img['base'][(q * 16 + w) * 4 + j]) + (e & cmask)
                        xv = x[np.minimum(col, x.size - 1)]
                        if img['val'] is not None:
                            term = img['val'][u + j] * xv
                        elif colv is not None:
                            rr = np.minimum(rb * H + lr, R - 1)
                            term = np.where(lr < H + halo, colv[rr], 0.0) * xv
                        else:
                            term = xv
                        np.add.at(rows, lr, term)
            r0 = rb * H
            r1 = min(r0 + H, R)
            acc[r0:r1] = rows[:r1 - r0]
        parts.append(acc)
    out = parts[0].copy()
    for a in parts[1:]:
        out = out + a
    return (out, parts) if group_sums else out


NT_BYTES = 256 << 20


def value_codec(val, layout):
    """(flag, array) for a dealt image's stored values: _Float16 or float when
    every value (padding zeros included) converts to that type exactly -- the
    kernels widen them back to the same doubles, so the products do not change
    (BSLS_TILE_VAL16 / VAL32, include/bsls_hip.h) -- else the doubles.
    BSLS_VAL_CODEC=f64|f32|f16 forces the choice down to the exact ones."""
    if val is None or layout not in (1, 2):
        return 0, val
    want = os.environ.get('BSLS_VAL_CODEC', 'auto')
    order = {'auto': ('f16', 'f32'), 'f16': ('f16', 'f32'), 'f32': ('f32',), 'f64': ()}[want]
    for c in order:
        dt = np.float16 if c == 'f16' else np.float32
        with np.errstate(over='ignore', invalid='ignore'):
            nv = val.astype(dt)
        if np.array_equal(nv.astype(np.float64), val):
            return (_native.TILE_VAL16 if c == 'f16' else _native.TILE_VAL32), nv
    return 0, val


def self_bytes(img):
    """Bytes of a tile image's entry stream (+ values)."""
    b = img['ent'].nbytes
    if img.get('val') is not None:
        b += img.get('val_dev', img['val']).nbytes
    return b


class DeviceTiles:
    """A tile image on the device + the ctypes struct pointing at it."""

    def __init__(self, M, halo=0, values=True, colv_lds=False, plan=None, layout=0,
                 group_col=None):
        torch = _torch()
        M = sps.csr_matrix(M)
        M.sort_indices()
        R, C = M.shape
        H, G, order = plan or tile_plan(R, C, halo, colv_lds,
                                        env='BSLS_TILE_PLAN_AT' if halo else 'BSLS_TILE_PLAN_A',
                                        layout=layout, nnz=M.nnz)
        if group_col is not None:
            # the caller's column groups (the sharded K2's link parts, aligned
            # with K1's row-block parts)
            gc = np.asarray(group_col, dtype=np.int64)
            G = gc.shape[0] - 1
            if gc[0] != 0 or gc[-1] != C:
                raise ValueError('column groups must cover [0, %d)' % C)
        else:
            gc = np.round(np.linspace(0, C, G + 1)).astype(np.int64)
        if np.any(np.diff(gc) < 1):
            raise ValueError('more column groups than columns')
        if layout in (1, 2):
            img = _native.tiles_build_dealt(M, H, halo, gc, values=values, packed=layout == 2)
        else:
            img = _native.tiles_build(M, H, halo, gc, values=values)
        img.update(rows=R, cols=C, H=H, halo=halo, ngroups=G, order=order, group_col=gc,
                   layout=layout)
        self.img = img
        self.nnz = int(M.nnz)
        self.t = {'group_col': torch.from_numpy(gc).cuda(),
                  'wave_off': torch.from_numpy(img['wave_off']).cuda(),
                  'ent': torch.from_numpy(img['ent'].view(np.int32)).cuda()}
        vflag, vdev = value_codec(img['val'], layout)
        self.val_codec = {0: 'f64', _native.TILE_VAL32: 'f32', _native.TILE_VAL16: 'f16'}[vflag]
        if img['val'] is not None:
            img['val_dev'] = vdev
            self.t['val'] = torch.from_numpy(vdev).cuda()
        if layout in (1, 2):
            self.t['base'] = torch.from_numpy(img['base']).cuda()
        S = _native.Tiles()
        # dealt images larger than the Infinity Cache stream their entries
        # non-temporally (csrc/tiles.hpp tq_load)
        nt = self_bytes(img) > NT_BYTES
        if os.environ.get('BSLS_TILE_NT'):          # A/B override of the policy
            nt = os.environ['BSLS_TILE_NT'] == '1'
        S.layout = layout | (_native.TILE_NT if layout in (1, 2) and nt else 0) | vflag
        S.base = self.t['base'].data_ptr() if layout in (1, 2) else None
        S.rows, S.cols, S.H, S.halo = R, C, H, halo
        S.nrb, S.ngroups, S.order, S.nquads = img['nrb'], G, order, img['nquads']
        S.group_col = self.t['group_col'].data_ptr()
        S.wave_off = self.t['wave_off'].data_ptr()
        S.ent = self.t['ent'].data_ptr()
        S.val = self.t['val'].data_ptr() if 'val' in self.t else None
        self.struct = S

    def bytes(self):
        return sum(v.numel() * v.element_size() for v in self.t.values())


def panel_rows(rows, workgroups_per_group, waves=16):
    """Rows per panel so one launch is about `workgroups_per_group` workgroups of
    16 panels per group (one per CU), within 64 .. BSLS_PANEL_ROWS."""
    want = -(-rows // (workgroups_per_group * waves))
    return int(min(_native.PANEL_ROWS, max(min(64, rows), want)))


def k1_plan(m, cus=256, max_groups=10):
    """(rows per panel, column groups) of the A image (K1, lsq_k1): as many
    column groups as keep the launch (groups x row blocks of 16 panels) within
    one workgroup per CU with panels as tall as they go (<= BSLS_PANEL_ROWS),
    i.e. full 64-row slices and fewer chunks per workgroup.  C3 (m = 100k):
    10 groups x 25 row blocks of 250-row panels, K1 42.8 us against 45.8 us
    for 8 x 32 of 196 rows (whose fourth slice held 4 rows).
    BSLS_K1_PLAN="groups,wg" overrides it (A/B timing of plans)."""
    plan = os.environ.get('BSLS_K1_PLAN')
    if plan:
        groups, wg = (int(v) for v in plan.split(','))
        return panel_rows(m, wg), groups
    rbs_min = -(-m // (16 * _native.PANEL_ROWS))
    groups = max(1, min(max_groups, cus // max(1, rbs_min)))
    rbs = max(rbs_min, cus // groups)
    return panel_rows(m, rbs), groups


class DeviceLSQ:
    """The x-space operator pair (csrc/lsq.hip, struct bsls_lsq_op): residual
    r = A x + add with ||r||^2, gradient g = A' r -- sparse_least_squares_obj's
    two SciPy products (algorithm_utils.py:88-94).  The residual walks column
    groups of panels (fixed order: f repeats bit for bit at the same x, which
    the reference's exits rely on -- BATCH.solve_LBFGS's revert stops on
    |f_old - f| < prog_tol with delta_x = 0); k1='tiles' (or
    BSLS_LSQ_K1=tiles) walks a dealt tile image of A instead (the z-space
    K1's walk: LDS atomic row sums, faster, the same sums to rounding only);
    k1='tiles_fixed' walks it with 64-bit fixed-point row sums (order-free:
    bit-repeatable like the panels, at the dealt walk's speed).
    A' is one group of panels (every row in CSR order: g bit-identical to
    SciPy's csr_matvec); k2='tiles' (or BSLS_LSQ_K2=tiles) walks a dealt tile
    image of A' instead (one group, LDS atomic row sums scaled by colv once per
    row: the same sums to rounding).  A scaled incidence drops the values
    (colv * x formed once per residual, A' entries scaled by colv row by row)."""

    def __init__(self, A, AT=None, general=False, k1=None, k2=None):
        torch = _torch()
        L = _native.lib()
        A = sps.csr_matrix(A)
        AT = sps.csr_matrix(AT) if AT is not None else A.T.tocsr()
        self.m, self.n = A.shape
        colv = None if general else scaled_incidence_scale(A)
        self.scaled = colv is not None
        k1 = k1 or os.environ.get('BSLS_LSQ_K1', 'panels')
        self.A_pan = self.A_til = None
        if k1 in ('tiles', 'tiles_fixed'):
            # (the fixed-point walk keeps two words per row: plan for twice the LDS)
            plan = (tile_plan(self.m, self.n, 0, colv_lds=True, layout=2, nnz=A.nnz)
                    if k1 == 'tiles_fixed' else None)
            self.A_til = DeviceTiles(A, 0, values=not self.scaled, layout=2, plan=plan)
            groups, npanels = self.A_til.img['ngroups'], 0
        else:
            prow, groups = k1_plan(self.m)
            self.A_pan = DevicePanels(A, prow, False, groups, values=not self.scaled)
            groups, npanels = self.A_pan.img['ngroups'], self.A_pan.img['npanels']
        self.k1 = k1
        k2 = k2 or os.environ.get('BSLS_LSQ_K2', 'panels')
        self.AT_pan = self.AT_til = None
        if k2 == 'tiles':
            # one group of row blocks as tall as the LDS holds, whole rounds of
            # 256 workgroups (the z-space K2's plan)
            hmax = _native.TILE_LDS_BYTES // 8 - 1
            nrb = -(-max(256, -(-self.n // hmax)) // 256) * 256
            # (a tile holds at least 64 rows: bsls_tiles_build_dealt3)
            self.AT_til = DeviceTiles(AT, 0, values=not self.scaled,
                                      plan=(max(64, -(-self.n // nrb)), 1, 0), layout=2)
        else:
            self.AT_pan = DevicePanels(AT, panel_rows(self.n, 256), False, 1,
                                       values=not self.scaled)
        self.k2 = k2
        dev = dict(dtype=torch.float64, device='cuda')
        self.colv = torch.from_numpy(colv).cuda() if self.scaled else None
        # max |colv| (1 unscaled): with |x| <= 1, the bound on the gathered colv * x
        self.colv_max = float(np.max(np.abs(colv))) if (self.scaled and colv.size) else 1.0
        self.xs = torch.empty(self.n, **dev) if self.scaled else None
        self.rpart = torch.zeros(groups * self.m, **dev)
        self.work = torch.zeros(L.bsls_lsq_workspace_size(self.m, npanels),
                                dtype=torch.uint8, device='cuda')
        op = _native.LsqOp()
        op.m, op.n = self.m, self.n
        if self.A_pan is not None:
            op.A = self.A_pan.struct
        else:
            op.At = self.A_til.struct
        if self.AT_pan is not None:
            op.AT = self.AT_pan.struct
        else:
            op.ATt = self.AT_til.struct
        op.colv = ptr(self.colv)
        op.rpart = self.rpart.data_ptr()
        op.xs = ptr(self.xs)
        op.work, op.work_bytes = self.work.data_ptr(), self.work.numel()
        if k1 == 'tiles_fixed':
            # fixed-point row sums: the bound of a row's |terms| per unit of
            # max|x| -- its entry count for a scaled incidence (the walk
            # gathers colv * x), else sum_j |A_ij|
            op.fixed = 1
            if self.scaled:
                op.fx_amax = float(max(1, int(np.max(np.diff(A.indptr))) if A.nnz else 1))
            else:
                rows = np.repeat(np.arange(self.m), np.diff(A.indptr))
                ra = np.bincount(rows, weights=np.abs(A.data), minlength=self.m)
                op.fx_amax = float(max(np.max(ra) if ra.size else 0.0, 1e-300))
        self.op = op

    def residual(self, x, out, add=None, sq=None):
        check(_native.lib().bsls_lsq_residual(self.op, ptr(x), ptr(add), ptr(out), ptr(sq),
                                              stream_handle()), 'bsls_lsq_residual')
        return out

    def gradient(self, r, out):
        check(_native.lib().bsls_lsq_gradient(self.op, ptr(r), ptr(out), stream_handle()),
              'bsls_lsq_gradient')
        return out


def lsq_operator(A, AT=None, general=False, k1=None, k2=None):
    """DeviceLSQ (residual walk `k1`, gradient walk `k2`: 'panels' or 'tiles',
    see DeviceLSQ), or None (the caller keeps the general CSR kernels) when the
    panel format cannot hold the matrix (dense rows)."""
    try:
        return DeviceLSQ(A, AT, general=general, k1=k1, k2=k2)
    except PanelOverflow:
        return None


class IsoPlan:
    """A block layout's pack plan on the device (bsls_isotonic_pack_plan /
    bsls_isotonic_packs): isotonic_regression_multi_c's variant-1 call
    (weight=None, update=1) in one launch, planned once per layout."""

    def __init__(self, starts, n):
        torch = _torch()
        L = _native.lib()
        P = _native.pack_plan(starts, n)
        self.device = _cur_dev()                      # the plan's arrays live there
        self.n = int(n)
        self.npacks = int(P['start'].shape[0])
        self.nlong = int(P['longs'].shape[0])
        self.host = P
        self.start = torch.from_numpy(P['start']).cuda()
        self.mask = torch.from_numpy(P['mask']).cuda()
        self.len = torch.from_numpy(P['len']).cuda()
        self.longs = torch.from_numpy(P['longs'] if self.nlong else np.zeros(1, np.int32)).cuda()
        self.work = (torch.zeros(L.bsls_isotonic_workspace_size(self.n), dtype=torch.uint8,
                                 device='cuda') if self.nlong else None)

    def apply(self, y, stream=None):
        """PAVA v1 (expanded) of every block of y[:n], in place."""
        L = _native.lib()
        if y.device.index != self.device:
            raise ValueError('IsoPlan built on cuda:%d applied to a tensor on %s'
                             % (self.device, y.device))
        check(L.bsls_isotonic_packs(ptr(y), ptr(self.start), ptr(self.mask), ptr(self.len),
                                    self.npacks, ptr(self.longs), self.nlong, self.n,
                                    ptr(self.work), self.work.numel() if self.work is not None
                                    else 0, stream_handle(stream)), 'bsls_isotonic_packs')
        return y


_iso_plans = {}


def _cur_dev():
    """Index of the current GPU (-1 without one: host-only tests of the cache)."""
    torch = _torch()
    return torch.cuda.current_device() if torch.cuda.is_available() else -1


def iso_plan(starts_h, n):
    """IsoPlan of a host block-start array, cached by content (a few layouts):
    an entry matches when its own copy of the starts equals these (a compare
    of the arrays, ~30 us at 50k blocks -- hashing them took ~0.5-1 ms a
    call, more than the projection it planned)."""
    st = np.ascontiguousarray(starts_h, dtype=np.int64)
    n = int(n)
    dev = _cur_dev()                         # a plan's arrays belong to one GPU
    for key, (ref, plan) in _iso_plans.items():
        if key[:3] == (st.shape[0], n, dev) and (ref is st or np.array_equal(ref, st)):
            return plan
    if len(_iso_plans) >= 8:
        _iso_plans.pop(next(iter(_iso_plans)))
    plan = IsoPlan(st, n)
    # keyed by (count, n) plus insertion order; the copy guards against a
    # caller that changes its array in place later
    k = (st.shape[0], n, dev)
    while k in _iso_plans:
        k = k + (len(_iso_plans),)
    _iso_plans[k] = (st.copy(), plan)
    return plan


class LineSearch:
    """LBFGS.solve's weak Wolfe line search (python/LBFGS.py:9-53) on a BBEngine,
    decided on the device (bsls_lbfgs_ls_begin / _trials): trials enqueued in
    chunks, the state read once per chunk.  search() returns (t, exit, trials,
    ||d||); after the accepted exit take() gives x_next, nabla_f(x_next) and
    f(x_next)."""

    CHUNK = int(os.environ.get('BSLS_LS_CHUNK', '4'))   # trials per state read

    def __init__(self, eng, c1=1e-3, c2=0.9):
        torch = _torch()
        L = _native.lib()
        nz = eng.nz
        f64 = dict(dtype=torch.float64, device='cuda')
        self.eng = eng
        self.pt = torch.empty(nz, **f64)
        self.gpt = torch.empty(nz, **f64)
        self.zero = torch.zeros(nz, **f64)
        self.fx = torch.zeros(1, **f64)
        self.st = torch.zeros(_native.LS_COUNT, **f64)
        self.S = torch.zeros(2, _native.S_COUNT, **f64)
        self.part = torch.zeros(max(1, L.bsls_lbfgs_ls_work_size(nz) // 8), **f64)
        self.tickets = torch.zeros(max(1, L.bsls_ticket_bytes() // 4), dtype=torch.int32,
                                   device='cuda')
        self.c1, self.c2 = float(c1), float(c2)

    def _state(self, x, d, gx, fx):
        return _native.LsState(x.data_ptr(), d.data_ptr(), gx.data_ptr(), self.pt.data_ptr(),
                               self.gpt.data_ptr(), self.zero.data_ptr(), fx.data_ptr(),
                               self.st.data_ptr(), self.S[0].data_ptr(), self.S[1].data_ptr(),
                               self.part.data_ptr(), self.tickets.data_ptr(), self.c1, self.c2)

    def search(self, x, d, gx, fx, y_out=None, s_out=None):
        """x (projected), d, gx = nabla_f(x): contiguous device vectors of nz;
        fx: f(x) as a one-element device tensor.  Returns (t, exit, trials,
        ||d||) after one host read per chunk of trials.  On the accepted exit
        the same read also brings f(x_next), y.s and g(x_next).g(x_next)
        (self.last = (f, ys, gg); bsls_lbfgs_ls_finish), with y = g(x_next) -
        gx and s = t d written into y_out / s_out when given."""
        L = _native.lib()
        S = self._state(x, d, gx, fx)
        P = self.eng.P
        st_h = stream_handle()
        yp = y_out.data_ptr() if y_out is not None else None
        sp = s_out.data_ptr() if s_out is not None else None
        self.last = None
        check(L.bsls_lbfgs_ls_begin(P, S, st_h), 'bsls_lbfgs_ls_begin')
        while True:
            check(L.bsls_lbfgs_ls_trials(P, S, self.CHUNK, st_h), 'bsls_lbfgs_ls_trials')
            check(L.bsls_lbfgs_ls_finish(P, S, yp, sp, st_h), 'bsls_lbfgs_ls_finish')
            st = self.st.cpu().numpy()
            if st[_native.LS_STOP] != 0:
                if st[_native.LS_DONE] != 0:
                    self.last = (float(st[_native.LS_FT]), float(st[_native.LS_YS]),
                                 float(st[_native.LS_GG]))
                return (float(st[_native.LS_T]), int(st[_native.LS_STOP]),
                        int(st[_native.LS_NTRIAL]), float(st[_native.LS_DNORM]))

    def take(self):
        """(x_next, nabla_f(x_next), f(x_next) as a one-element device tensor)
        of the accepted trial: the search's own buffers, handed over (fresh
        ones are allocated for the next search, no copies); f(x_next) is a
        view of the state's f(pt) slot, which the next search reads first."""
        torch = _torch()
        pt, gpt = self.pt, self.gpt
        self.pt, self.gpt = torch.empty_like(pt), torch.empty_like(gpt)
        return pt, gpt, self.st[_native.LS_FT:_native.LS_FT + 1]


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
        for one wave, or a single longer block.  Host-planned once
        (bsls_isotonic_pack_plan over the z-block starts; every z-block holds
        >= 1 entry)."""
        if self._packs is None:
            torch = _torch()
            P = _native.pack_plan(self.zstarts_h, self.nz)
            b0 = np.searchsorted(self.zstarts_h, P['start']).astype(np.int64)
            self._packs = dict(
                z0=torch.from_numpy(P['start']).cuda(),
                b0=torch.from_numpy(b0).cuda(),
                mask=torch.from_numpy(P['mask']).cuda(),
                len=torch.from_numpy(P['len']).cuda(),
                n=int(P['start'].shape[0]))
        return self._packs

    def iso_plan(self):
        """The z-layout's IsoPlan (PAVA v1 over the z-blocks, BBEngine.proj),
        kept by the layout: the content-keyed cache hashes the whole start
        array (C3: 400 KB, ~0.3 ms a call -- most of an LBFGS.solve iteration,
        whose line search projects ~20 times)."""
        plan = getattr(self, '_iso', None)
        if plan is None or getattr(plan, 'device', None) != _cur_dev():
            plan = self._iso = iso_plan(self.zstarts_h, self.nz)
        return plan


class BBEngine:
    """Fused z-space projected BB (python/BB.py:7-45 over python/main.py:53-65).

    The device runs K2 -> K3 -> K1 per iteration (bsls_bb_iterate); the stop
    test, the BB step and every reduction stay on the device.  The host polls
    the scalar block every `poll` iterations and at each `record_every`
    boundary, to log states exactly where BB.solve logs them.
    """

    def __init__(self, A, b, block_sizes, options=None, early_exit=True, A_dev=None,
                 AT_dev=None, AT=None, target=None, x0=None, general=False, fmt=None,
                 tile_plans=(None, None), colv=None, deterministic=False, tile_layouts=None,
                 link_parts=None):
        torch = _torch()
        L = _native.lib()
        self.layout = lay = BlockLayout(block_sizes)
        A = sps.csr_matrix(A)
        if A.shape[1] != lay.n:
            raise ValueError('A has %d columns but the blocks cover %d' % (A.shape[1], lay.n))
        AT = sps.csr_matrix(AT) if AT is not None else A.T.tocsr()
        # the general CSR copies (closures f / nabla_f, DORE, LBFGS, LS_postprocess)
        # are uploaded on first use: the fused loop never reads them
        self._A_host, self._AT_host = A, AT
        self._A_dev, self._AT_dev = A_dev, AT_dev
        self.m, self.n, self.nz = A.shape[0], lay.n, lay.nz
        # the fused kernels' images: A (K1), A' with halo rows (K2), each as
        # panels or streamed tiles (spmv_format); values dropped for a scaled
        # incidence (colv: the caller's column scales, else detected)
        if colv is None and not general:
            colv = scaled_incidence_scale(A)
        elif general:
            colv = None
        self.scaled = colv is not None
        # tile layouts (K1, K2): the dealt images (column-sorted gathers, LDS
        # atomic sums: the same sums to rounding, not run-to-run bit-identical;
        # C5 K1 1334 -> 374 us, K2 984 -> 503 us), with 3-byte entries (layout
        # 2: C5 K1 359 -> 331, K2 358 -> 345 us against 4-byte layout 1)
        # unless `deterministic`, which keeps the thread streams (every row
        # summed in CSR order: K2 bit-identical to SciPy with one group).
        # BSLS_TILE_LAYOUT="a,at" overrides.
        if tile_layouts is None:
            env = os.environ.get('BSLS_TILE_LAYOUT')
            tile_layouts = (tuple(int(v) for v in env.split(',')) if env
                            else ((0, 0) if deterministic else (2, 2)))
        self.tile_layouts = tile_layouts
        # per matrix: panels or streamed tiles (spmv_format)
        self.fmt_A = spmv_format(A, fmt, dealt=tile_layouts[0] in (1, 2))
        self.fmt_AT = spmv_format(AT, fmt, dealt=tile_layouts[1] in (1, 2))
        self.A_pan = self.AT_pan = self.A_til = self.AT_til = None
        if self.fmt_A == 'panels':
            prow, groups = k1_plan(self.m)
            try:
                self.A_pan = DevicePanels(A, prow, False, groups, values=not self.scaled)
            except PanelOverflow:
                self.fmt_A = 'tiles'      # dense rows: the tiles have no such limit
        if self.fmt_A == 'tiles':
            self.A_til = DeviceTiles(A, 0, values=not self.scaled, plan=tile_plans[0],
                                     layout=tile_layouts[0])
        if self.fmt_AT == 'panels':
            try:
                self.AT_pan = DevicePanels(AT, panel_rows(self.n, 256), True, 1,
                                           values=not self.scaled)
            except PanelOverflow:
                self.fmt_AT = 'tiles'
        # link parts (the sharded schedule's exchange pipelined behind the
        # walks, bsls_bb_shard_iterate_parts): K1's row blocks cut into
        # `link_parts` runs, and K2's image in as many column groups over the
        # same link ranges, so K2 part q reads only the rows of r part q's
        # exchange delivered
        self.k1_part_bounds = None
        k2_gc = None
        if link_parts is not None and int(link_parts) > 1:
            if self.fmt_A != 'tiles' or self.fmt_AT != 'tiles' or tile_layouts[1] not in (1, 2):
                raise ValueError('link parts need dealt tile images for K1 and K2')
            from distributed import row_parts
            nrb, H = self.A_til.img['nrb'], self.A_til.img['H']
            self.k1_part_bounds = np.array(row_parts(nrb, int(link_parts)), dtype=np.int64)
            if len(self.k1_part_bounds) - 1 != int(link_parts):
                raise ValueError('%d link parts need as many K1 row blocks (%d)'
                                 % (int(link_parts), nrb))
            k2_gc = np.minimum(self.k1_part_bounds * H, self.m)
        if self.fmt_AT == 'tiles':
            # (the thread-stream K2 keeps each row's colv in LDS beside its sum:
            # every term colv_i * r_j, SciPy's product; the dealt K2 scales
            # the row sum once, so its LDS holds twice the rows)
            plan_at = tile_plans[1]
            if k2_gc is not None and plan_at is None:
                H2, _, _ = tile_plan(self.n, self.m, 1, False, layout=tile_layouts[1], nnz=AT.nnz)
                plan_at = (H2, len(k2_gc) - 1, 0)
            self.AT_til = DeviceTiles(AT, 1, values=not self.scaled,
                                      colv_lds=self.scaled and tile_layouts[1] == 0,
                                      plan=plan_at, layout=tile_layouts[1], group_col=k2_gc)
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
            xin = None
        else:
            # target = A x0 - b (python/main.py:48), formed after the images are
            # up by the engine's own K1; x0 defaults to the particular solution,
            # as BSLSMatrices.initial_solution does
            xin = x0 if x is None else torch.as_tensor(np.asarray(x, dtype=np.float64)).cuda()
            self.target = -torch.as_tensor(np.asarray(b, dtype=np.float64)).cuda()
        self.z = [torch.zeros(max(self.nz, 1), **dev) for _ in range(2)]
        self.g = [torch.zeros(max(self.nz, 1), **dev) for _ in range(2)]
        self.x = torch.empty(lay.n, **dev)
        self.r = torch.empty(self.m, **dev)
        self.scal = torch.zeros(_native.S_COUNT, **dev)
        self.work = torch.zeros(L.bsls_bb_workspace_size(self.m, self.n, self.nz),
                                dtype=torch.uint8, device='cuda')
        ga = (self.A_pan or self.A_til).img['ngroups']
        self.rpart = torch.zeros(ga * self.m if ga > 1 or self.A_pan else 1, **dev)
        self.wpart = None
        if self.AT_til is not None and self.AT_til.img['ngroups'] > 1:
            ti = self.AT_til.img
            # + one slot per (group, row block): stage 8's r^2 slices
            self.wpart = torch.zeros(ti['ngroups'] * ti['nrb'] * (ti['H'] + 2), **dev)
        self.colv = torch.from_numpy(colv).cuda() if self.scaled else None
        # max |colv| (1 unscaled): with |x| <= 1, the bound on the gathered colv * x
        self.colv_max = float(np.max(np.abs(colv))) if (self.scaled and colv.size) else 1.0
        # the scales as the kernels read them every iteration: the narrowest
        # exact type (flows are integers: _Float16; value_codec)
        self.colv_codec, self.colv_n = 0, None
        if self.scaled:
            flag, cn = value_codec(np.asarray(colv, dtype=np.float64), 2)
            if flag:
                self.colv_codec = 2 if flag == _native.TILE_VAL16 else 1
                self.colv_n = torch.from_numpy(cn).cuda()
        P = BBProblem()
        P.m, P.n, P.nz, P.nblocks = self.m, lay.n, lay.nz, lay.p
        if self.A_pan is not None:
            P.A = self.A_pan.struct
        else:
            P.At = self.A_til.struct
        if self.AT_pan is not None:
            P.AT = self.AT_pan.struct
        else:
            P.ATt = self.AT_til.struct
        P.wpart = self.wpart.data_ptr() if self.wpart is not None else None
        P.work_bytes = self.work.numel()
        P.colv = self.colv.data_ptr() if self.scaled else None
        P.colv_n = self.colv_n.data_ptr() if self.colv_n is not None else None
        P.colv_codec = self.colv_codec
        P.rpart = self.rpart.data_ptr()
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
        # packs of one z-block longer than a wave: a workgroup each (bb_k3_long)
        ln = pk['len'].cpu().numpy()
        longs = np.nonzero(ln > 64)[0].astype(np.int32)
        self.long_packs = None
        if longs.size:
            off = np.concatenate(([0], np.cumsum(ln[longs]))).astype(np.int64)
            self.long_packs = torch.from_numpy(longs).cuda()
            self.long_off = torch.from_numpy(off).cuda()
            self.long_scratch = torch.zeros(L.bsls_bb_long_scratch_size(int(off[-1])),
                                            dtype=torch.uint8, device='cuda')
            P.long_packs, P.nlong = self.long_packs.data_ptr(), int(longs.size)
            P.long_off, P.long_scratch = self.long_off.data_ptr(), self.long_scratch.data_ptr()
        P.z[0], P.z[1] = self.z[0].data_ptr(), self.z[1].data_ptr()
        P.g[0], P.g[1] = self.g[0].data_ptr(), self.g[1].data_ptr()
        P.x, P.r, P.scal, P.work = (self.x.data_ptr(), self.r.data_ptr(), self.scal.data_ptr(),
                                    self.work.data_ptr())
        P.max_zblock = lay.max_zblock
        P.max_iter = int(opts.get('max_iter', 300000))
        P.opt_tol = float(opts.get('opt_tol', 1e-6))
        P.early_exit = 1 if early_exit else 0
        # K3's warm start (pava_wave.hpp pava_warm: within ulps of the reference
        # PAVA, not bit-identical): on unless deterministic; BSLS_K3_WARM=0/1
        warm = os.environ.get('BSLS_K3_WARM')
        P.pava_warm = int(warm) if warm is not None else (0 if deterministic else 1)
        # K1's group sums by atomics (column shards) / K3's pack form: the
        # defaults unless BSLS_K1_ATOMIC / BSLS_K3_MERGE = 0 / 1 (read here,
        # once, not per launch)
        for field, env in (('k1_atomic', 'BSLS_K1_ATOMIC'), ('k3_merge', 'BSLS_K3_MERGE')):
            v = os.environ.get(env)
            setattr(P, field, 0 if v is None else (2 if int(v) else 1))
        self.P = P
        self.z0 = None
        if xin is not None:
            self.x.copy_(self.colv * xin if self.scaled else xin)
            self.stage(7, 0)                       # r = A x0 + (-b)
            self.target.copy_(self.r)

    @property
    def A(self):
        if self._A_dev is None:
            self._A_dev = DeviceCSR(self._A_host)
        return self._A_dev

    @property
    def AT(self):
        if self._AT_dev is None:
            self._AT_dev = DeviceCSR(self._AT_host)
        return self._AT_dev

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

    def set_rr_slice(self, lo, hi):
        """Rows [lo, hi) of r whose ||r||^2 stage 10 sums (the sliced sharded
        schedule: each rank its 1/world share)."""
        if not (0 <= lo <= hi <= self.m):
            raise ValueError('slice out of range')
        self.P.rr_lo, self.P.rr_hi = int(lo), int(hi)

    def fixed_r_ok(self):
        """Whether this column shard can keep r in 64-bit fixed point
        (bsls_bb_problem.r_fx): its K1 adds its column groups' sums by
        atomics with the init folded into K3 (a dealt K1 image of several
        groups on shard_role 1 / 2) and its K2 walks a dealt image."""
        P = self.P
        atomic = (P.k1_atomic == 2) if P.k1_atomic else P.shard_role != 0
        return bool(self.A_til is not None and self.A_til.img['ngroups'] > 1 and atomic
                    and self.AT_til is not None and self.tile_layouts[1] in (1, 2)
                    and P.shard_role != 0)

    def set_r_fixed(self, scale):
        """r in 64-bit fixed point at `scale` (a power of two; 0: doubles):
        the atomic K1's group sums then add as integers (order-free) and the
        r exchange sums int64 words (exact) -- the same r bits however the
        groups and ranks land.  Every |partial sum of r| must stay below
        2^62 / scale (distributed.ShardedBB sizes it)."""
        scale = float(scale)
        if scale < 0 or (scale > 0 and not self.fixed_r_ok()):
            raise ValueError('fixed-point r needs an atomic sharded K1 (fixed_r_ok)')
        self.P.r_fx = scale

    @property
    def r_exchange(self):
        """r as the exchange sums it: int64 words under a fixed-point r."""
        torch = _torch()
        return self.r.view(torch.int64) if self.P.r_fx > 0 else self.r

    def residual_value(self):
        """r as doubles (a copy), whatever its representation."""
        torch = _torch()
        if self.P.r_fx > 0:
            return self.r.view(torch.int64).to(torch.float64) / self.P.r_fx
        return self.r.clone()

    def set_shard_role(self, role):
        """bsls_bb_problem.shard_role: 0 the whole problem here, 1 a column
        shard that adds target to its partial residual, 2 another column shard
        (distributed.ShardedBB)."""
        if role not in (0, 1, 2):
            raise ValueError('shard role must be 0, 1 or 2')
        self.P.shard_role = int(role)

    def row_blocks(self):
        """(K1 row blocks, rows per block): the granule of residual_rows."""
        R = ctypes.c_int64(0)
        nb = _native.lib().bsls_bb_row_blocks(self.P, ctypes.byref(R))
        if nb < 0:
            check(int(nb), 'bsls_bb_row_blocks')
        return int(nb), int(R.value)

    def k2_part(self, it, part, stream=None):
        """Stage 10 on K2 column group `part` (bsls_bb_k2_part; link-part engines)."""
        check(_native.lib().bsls_bb_k2_part(self.P, int(it), int(part), stream_handle(stream)),
              'bsls_bb_k2_part')

    def k1_rows(self, it, rb0, rb1, stream=None):
        """Stage 14 on K1 row blocks [rb0, rb1) (bsls_bb_k1_rows)."""
        check(_native.lib().bsls_bb_k1_rows(self.P, int(it), int(rb0), int(rb1),
                                            stream_handle(stream)), 'bsls_bb_k1_rows')

    def residual_rows(self, it, rb0, rb1, stream=None):
        """Stage 1 on K1 row blocks [rb0, rb1) (bsls_bb_residual_rows)."""
        check(_native.lib().bsls_bb_residual_rows(self.P, int(it), int(rb0), int(rb1),
                                                  stream_handle(stream)),
              'bsls_bb_residual_rows')

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

    # The closures run on the fused kernels' images (K1 / K2 stages), not on
    # general CSR copies: z goes through z[0] (stage 6: x = colv * N z), K1
    # (stage 1: A x; stage 7: A x + target, ||r||^2, f) and K2 (stage 3 at
    # iteration 0: N'A'r).  They share the engine's buffers with the fused BB
    # loop, so they must not run while a solve() is in flight.
    def _x_of(self, z):
        torch = _torch()
        z = torch.as_tensor(z, dtype=torch.float64, device='cuda').reshape(-1)
        if z.numel() != self.nz:
            raise ValueError('z has %d entries, expected %d' % (z.numel(), self.nz))
        self.z[0][:self.nz].copy_(z)
        self.stage(6, 0)

    def apply_A(self, z, alpha=1.0):
        """alpha A N z (DORE's linop with A scaled by alpha, gradient_descent.py:57-63)."""
        self._x_of(z)
        self.stage(1, 0)
        return self.r * alpha if alpha != 1.0 else self.r.clone()

    def apply_AT(self, r, alpha=1.0):
        """alpha N' A' r (DORE's linop_T)."""
        self.r.copy_(r)
        self.stage(3, 0)
        g = self.g[0][:self.nz]
        return g * alpha if alpha != 1.0 else g.clone()

    def residual(self, z, alpha=1.0):
        """alpha (A N z + target) (DORE scales A and target by alpha)."""
        self._x_of(z)
        self.stage(7, 0)
        return self.r * alpha if alpha != 1.0 else self.r.clone()

    def f(self, z):
        """0.5 ||A N z + target||^2 (main.py:53), f as K1's finish forms it."""
        self._x_of(z)
        self.stage(7, 0)
        return float(self.scal[_native.S_FX].item())

    def nabla_f(self, z):
        """N' A' (A N z + target) (main.py:54)."""
        self._x_of(z)
        self.stage(7, 0)
        self.stage(3, 0)
        return self.g[0][:self.nz].clone()

    def line_search(self):
        """This engine's device weak Wolfe line search (LBFGS.solve)."""
        ls = getattr(self, '_ls', None)
        if ls is None:
            ls = self._ls = LineSearch(self)
        return ls

    def apply_A_x(self, x):
        """A x for an x-space vector (LS_postprocess's A x_true)."""
        torch = _torch()
        x = torch.as_tensor(x, dtype=torch.float64, device='cuda').reshape(-1)
        self.x.copy_(self.colv * x if self.scaled else x)
        self.stage(1, 0)
        return self.r.clone()

    def proj(self, z):
        """isotonic_regression_multi_c on the z-blocks, then clip to [0, 1]
        (main.py:61-65); returns a new tensor like np.maximum(np.minimum(..))."""
        torch = _torch()
        L = _native.lib()
        if self.layout.max_zblock < 1 or np.any(self.layout.sizes < 2):
            raise AssertionError   # the reference's strictly-increasing z-starts assert
        y = z.clone()
        self.layout.iso_plan().apply(y)
        return torch.clamp(y, 0.0, 1.0)

    def lsv_matvec(self, v):
        """N'A'A N v for ARPACK (bsls_utils.lsv_operator), on the fused images."""
        torch = _torch()
        vd = torch.from_numpy(np.ascontiguousarray(np.real(v), dtype=np.float64)).cuda()
        return self.apply_AT(self.apply_A(vd)).cpu().numpy()

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


class XBBEngine:
    """Fused x-space projected BB (python/BATCH.py:55-106 over
    algorithm_utils.get_solver_parts(is_sparse=True), python/algorithm_utils.py:
    182-271): the step, projection, objective, Armijo backtracking
    (line_search_np, :113-137) and stopping test (:158-172) run as device rounds
    (csrc/xbb.hip, bsls_xbb_rounds); the host polls the mode every `poll`
    rounds."""

    def __init__(self, obj, proj, A_dev=None, lbfgs=0):
        """lbfgs = C > 0: BATCH.solve_LBFGS (python/BATCH.py:110-214) with C
        corrections -- the BB step of iterations i > 5 replaced by
        LBFGS_helper's two-loop recursion on the device (csrc/xbb.hip
        xlb_step / xlb_dir)."""
        torch = _torch()
        L = _native.lib()
        self.obj, self.proj = obj, proj
        m, n = obj.m, obj.n
        if proj.n != n:
            raise ValueError('projection covers %d entries, A has %d columns' % (proj.n, n))
        dev = dict(dtype=torch.float64, device='cuda')
        self.m, self.n = m, n
        self.x = torch.zeros(n, **dev)
        self.g = torch.zeros(n, **dev)
        self.xn = torch.zeros(n, **dev)
        self.gn = torch.zeros(n, **dev)
        self.r = torch.zeros(m, **dev)
        self.scal = torch.zeros(_native.XS_COUNT, **dev)
        self.work = torch.zeros(L.bsls_xbb_workspace_size(m, n, obj.A.ntiles, obj.AT.ntiles),
                                dtype=torch.uint8, device='cuda')
        self.hist = None
        P = _native.XBBProblem()
        P.m, P.n, P.nblocks, P.max_block = m, n, proj.p, proj.max_block
        # bit 0: the l1 ball; bit 1: the sort-free projection (BSLS_PROJ=fast,
        # as c_extensions' proj_multi_*_c take it: 1e-12, not bit-identical)
        P.ball = ((1 if proj.kind == 'ball' else 0)
                  | (2 if os.environ.get('BSLS_PROJ', 'exact') == 'fast' else 0))
        for dst, M in ((P.A, obj.A), (P.AT, obj.AT)):
            dst.rows = M.m
            dst.indptr, dst.indices, dst.data = (M.indptr.data_ptr(), M.indices.data_ptr(),
                                                 M.data.data_ptr())
            dst.tiles, dst.ntiles, dst.group = M.tiles.data_ptr(), M.ntiles, M.group
        P.neg_b = obj.neg_b.data_ptr()
        P.starts = proj.starts.data_ptr()
        P.x, P.g, P.xn, P.gn = (self.x.data_ptr(), self.g.data_ptr(), self.xn.data_ptr(),
                                self.gn.data_ptr())
        P.r, P.scal = self.r.data_ptr(), self.scal.data_ptr()
        P.proj_work, P.proj_work_bytes = proj.ws.data_ptr(), proj.ws.numel()
        P.work, P.work_bytes = self.work.data_ptr(), self.work.numel()
        lsq = getattr(obj, 'lsq', None)
        P.lsq = ctypes.pointer(lsq.op) if lsq is not None else None
        self._lsq, self._xb = lsq, 0.0
        self.lbfgs = int(lbfgs)
        if self.lbfgs < 0:
            raise ValueError('corrections must be >= 0')
        if self.lbfgs:
            self.s = torch.zeros(n, **dev)
            self.y = torch.zeros(n, **dev)
            self.lb = torch.zeros(max(1, L.bsls_xbb_lbfgs_size(self.lbfgs) // 8), **dev)
            P.lbfgs, P.s, P.y, P.lb = (self.lbfgs, self.s.data_ptr(), self.y.data_ptr(),
                                       self.lb.data_ptr())
        self.P = P

    def start(self, x_init, f_min=None, opt_tol=1e-6, max_iter=2000, prog_tol=1e-12,
              hist_cap=None):
        torch = _torch()
        x0 = torch.as_tensor(np.asarray(x_init, dtype=np.float64) if not hasattr(x_init, 'cpu')
                             else x_init, dtype=torch.float64).cuda().reshape(-1)
        if x0.numel() != self.n:
            raise ValueError('x_init has %d entries, expected %d' % (x0.numel(), self.n))
        self.x.copy_(x0)
        # every iterate the rounds evaluate is x_init, a projection onto the
        # simplex / l1 ball (entries within [-1, 1]) or a convex combination of
        # those: its entries stay within max(1, max|x_init|), which lets a
        # fixed-point residual skip its per-call max pass (bsls_lsq_op.x_bound)
        self._xb = 0.0
        lsq = self._lsq
        if lsq is not None and lsq.op.fixed:
            xm = float(x0.abs().max()) if x0.numel() else 0.0
            if np.isfinite(xm):
                self._xb = max(1.0, xm) * lsq.colv_max
        cap = int(hist_cap if hist_cap is not None else min(max(int(max_iter), 1) + 1, 1 << 22))
        if self.hist is None or self.hist.numel() < cap:
            self.hist = torch.zeros(cap, dtype=torch.float64, device='cuda')
        P = self.P
        P.hist, P.hist_cap = self.hist.data_ptr(), cap
        P.max_iter = int(min(max_iter, 2 ** 62))
        P.opt_tol, P.prog_tol = float(opt_tol), float(prog_tol)
        P.has_fmin = 0 if f_min is None else 1
        P.f_min = 0.0 if f_min is None else float(f_min)
        self.f_min = f_min
        check(_native.lib().bsls_xbb_init(P, stream_handle()), 'bsls_xbb_init')

    def rounds(self, count):
        lsq = self._lsq
        if lsq is not None and self._xb > 0.0:
            lsq.op.x_bound = self._xb          # read by the launches enqueued below only
        try:
            check(_native.lib().bsls_xbb_rounds(self.P, int(count), stream_handle()),
                  'bsls_xbb_rounds')
        finally:
            if lsq is not None:
                lsq.op.x_bound = 0.0

    def scalars(self):
        return self.scal.cpu().numpy()

    def solve(self, x_init, f_min=None, opt_tol=1e-6, max_iter=2000, prog_tol=1e-12, poll=8):
        """BATCH.solve_BB's result dict: f, x (NumPy), stop, iterations, progress
        ([time, f] per iteration; the time is the wall clock of the poll that
        saw the iteration finish), plus rounds / backtracks."""
        self.start(x_init, f_min, opt_tol, max_iter, prog_tol)
        t0 = time.time()
        seen, times = 0, [0.0]
        while True:
            self.rounds(poll)
            s = self.scalars()
            it = int(s[_native.XS_ITER])
            now = time.time() - t0
            times.extend([now] * max(0, it - 1 - seen))
            seen = max(seen, it - 1)
            if int(s[_native.XS_MODE]) == _native.XM_STOPPED:
                break
        f, f_old = float(s[_native.XS_F]), float(s[_native.XS_FOLD])
        reason = int(s[_native.XS_STOP])
        if reason == _native.XSTOP_MAXITER:
            stop = 'max_iter'
        elif reason == _native.XSTOP_OPT:
            stop = 'f-f_min = {} < opt_tol'.format(f - f_min)
        else:
            stop = '|f_old-f| = {} < prog_tol'.format(abs(f_old - f))
        k = min(it, self.P.hist_cap)
        fh = self.hist[:k].cpu().numpy()
        progress = [[times[j] if j < len(times) else times[-1], float(fh[j])] for j in range(k)]
        return {'f': f, 'x': self.xn.cpu().numpy(), 'stop': stop, 'iterations': it,
                'progress': progress, 'rounds': int(s[_native.XS_ROUNDS]),
                'backtracks': int(s[_native.XS_BACKTRACKS])}
