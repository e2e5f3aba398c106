"""Column-sharded BB across GPUs of one node (one process per GPU).

The reference has no parallelism at all; its only natural
decomposition is by block: blocks are independent in the projection and
blockify() already makes each block's columns contiguous
(python/bsls_matrices.py:109-126).  So rank g owns a contiguous run of whole
blocks = a column slice A_g (m x n_g), its transpose, and its slices of
z, g, x.  Per BB iteration:

    stage 10  g_g = N_g' A_g' r  and the four local BB sums, and this rank's
              1/world slice of ||r||^2 (r is the same all-reduced vector on
              every rank)
    all-reduce(sum) of the 4 BB sums and ||r||^2  (40 bytes)
    stage 15  f and the stopping test of the previous iteration (every rank
              tests the same summed values, so every rank decides alike), then
              t, z_g <- clip01(PAVA(z_g - t g_g)), x_g = x0_g + N_g z_g  (K3),
              and -- where K1 adds its column groups' sums by atomics -- r set
              to target (rank 0) / 0 for them
    stage 14  r_g = A_g x_g, + target on rank 0 (partial residual, length m)
    all-reduce(sum) of r_g  (8 m bytes: the one real exchange of the algorithm)
and after the last iteration of a call stage 9 (||r||^2, f, stopping test of
that iteration).  Once the run has stopped, ranks other than 0 write r = 0 and
rank 0 leaves its r (the final residual) alone, so the all-reduce keeps the
final residual intact (csrc/bb.hip k1_stopped_rows), and ranks other than 0
zero their BB sums before the five-sum all-reduce (k2_stopped_sums).  The
Python loop below and the C++ driver (bsls_bb_shard_iterate) enqueue the same
stages; the C++ one takes RCCL (RcclComm) or any transport through a callback
(CallbackComm).

The collectives go through torch.distributed: backend "nccl" is RCCL over xGMI
on MI355X; "gloo" runs the same orchestration in CPU tests with a fake stage
backend.  Results depend on the rank count only through the summation order of
the r all-reduce (within the 1e-6 iterate contract).
"""
import os

import numpy as np


def partition_blocks(block_sizes, col_weights, world):
    """Split blocks into `world` contiguous runs balancing the per-block weight
    (nnz of the block's columns).  Returns block boundaries [b_0=0, ..., b_W=p]."""
    bs = np.asarray(block_sizes, dtype=np.int64)
    w = np.asarray(col_weights, dtype=np.float64)
    if w.shape[0] != bs.shape[0]:
        raise ValueError('one weight per block expected')
    p = bs.shape[0]
    if world < 1 or world > p:
        raise ValueError('need 1 <= world <= number of blocks')
    cum = np.concatenate(([0.0], np.cumsum(w)))
    total = cum[-1]
    bounds = [0]
    for g in range(1, world):
        target = total * g / world
        b = int(np.searchsorted(cum, target, side='left'))
        b = min(max(b, bounds[-1] + 1), p - (world - g))
        bounds.append(b)
    bounds.append(p)
    return np.array(bounds, dtype=np.int64)


def row_parts(nblocks, parts):
    """parts + 1 row-block bounds splitting K1's row blocks into `parts` runs."""
    parts = max(1, min(int(parts), int(nblocks)))
    return [int(v) for v in np.round(np.linspace(0, nblocks, parts + 1)).astype(np.int64)]


def _world_size():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size()
    except ImportError:
        pass
    return 1


def _shard_rank(rank):
    """The rank that decides the shard role: the caller's, else the initialized
    default process group's.  Without either there is no safe default -- every
    rank taking role 1 would add target world times over -- so it raises."""
    if rank is not None:
        return int(rank)
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except ImportError:
        pass
    raise ValueError('ShardedBB needs rank= (no torch.distributed process group is '
                     'initialized to take it from)')


class ShardedBB:
    """Drive one rank's stages with the all-reduces between them.

    `engine` exposes stage(k, it), r (m-vector), scal (BSLS_S_COUNT vector) --
    device.BBEngine on GPUs; a numpy/torch fake in the gloo tests -- and, for
    the overlapped residual, row_blocks() and residual_rows(it, rb0, rb1).
    `all_reduce(t)` sums a tensor in place across ranks; `all_reduce_async(t)`
    starts that sum and returns a handle with wait().

    With parts > 1 the residual's all-reduce is pipelined behind K1 (SURVEY.md
    §8(e)): K1 runs on row parts one after the other on the compute stream; as
    soon as part p is enqueued its rows of r are all-reduced asynchronously
    (RCCL on its own stream, ordered after part p only), so the exchange of
    part p overlaps the computation of part p + 1; the compute stream waits
    for every part before stage 2."""

    SUMS = slice(5, 9)      # scal[SUMDG..GG]
    SUMS_RR = slice(5, 10)  # scal[SUMDG..RR]

    def __init__(self, engine, all_reduce, parts=1, all_reduce_async=None, rank=None,
                 fuse=None, native=None, slices=None):
        self.e = engine
        rank = _shard_rank(rank)
        # link parts: an engine built with link_parts = parts (K2's image in
        # column groups over K1's row-block parts) runs the exchange pipelined
        # behind both walks (bsls_bb_shard_iterate_parts); other engines with
        # parts > 1 pipeline it behind K1 only, from Python
        lb = getattr(engine, 'k1_part_bounds', None)
        self.link = (lb is not None and int(parts) > 1 and len(lb) - 1 == int(parts))
        # native: an RcclComm / CallbackComm / ModelComm -- iterate() then
        # enqueues the whole schedule from C++ (bsls_bb_shard_iterate[_parts]:
        # the stages and the all-reduces of an iteration, no Python per
        # iteration); row parts without link parts stay Python-driven
        self.native = native if (native is not None and (int(parts) <= 1 or self.link)) else None
        self._cstream = None
        # fuse 2 (default): K2 sums this rank's slice of ||r||^2 beside the BB
        # sums (stage 10), all-reduced with them, then f / stopping test
        # (stage 12); 1: K2 reads all of r for it and tests in its last
        # workgroup (stage 8); 0: stage 3 and a stage-9 launch after every
        # residual exchange.  BSLS_SHARD_FUSE=0|1|2 (A/B).
        if fuse is None:
            fuse = int(os.environ.get('BSLS_SHARD_FUSE', '2'))
        self.fuse = int(fuse)
        if self.fuse not in (0, 1, 2):
            raise ValueError('fuse must be 0, 1 or 2')
        if self.fuse == 2:
            # rows [lo, hi) of r: this rank's share of ||r||^2.  slices: the
            # rank count (the process group's); a one-GPU rehearsal of rank 0
            # of N passes N (its ||r||^2 is then 1/N of the true one: timing
            # only)
            if slices is None:
                slices = _world_size()
            m = engine.r.shape[0]
            engine.set_rr_slice(rank * m // slices, (rank + 1) * m // slices)
        # rank 0 adds target to its partial residual; the others zero theirs
        # once the run has stopped (bsls_bb_problem.shard_role)
        engine.set_shard_role(1 if rank == 0 else 2)
        self._rank = rank
        self.all_reduce = all_reduce
        self.all_reduce_async = all_reduce_async
        self.parts = int(parts) if (all_reduce_async is not None or self.native) else 1
        if self.link and self.parts < 2:
            # (the link pipeline needs its exchanges asynchronous: from Python
            # through all_reduce_async, or the native driver's comm stream)
            raise ValueError('link parts need all_reduce_async or a native communicator')
        if self.link and self.fuse != 2:
            raise ValueError('link parts run the sliced schedule (fuse 2)')
        self._slices = None
        self._works = []
        if self.parts > 1:
            nb, R = engine.row_blocks()
            m = engine.r.shape[0]
            b = row_parts(nb, self.parts)
            self._slices = [(b[k], b[k + 1], b[k] * R, min(b[k + 1] * R, m))
                            for k in range(len(b) - 1)]

    def _rx(self):
        """r as exchanged: the int64 words of a fixed-point r."""
        return getattr(self.e, 'r_exchange', self.e.r)

    def residual(self, it):
        """r = sum over ranks of A_g x_g (before stage 2)."""
        e = self.e
        if not self._slices or self.all_reduce_async is None:
            # (stage 14: K1 after stage 15, which may have initialised r)
            e.stage(14 if (self.fuse == 2 and it > 0) else 1, it)
            self.all_reduce(self._rx())
            return
        works = []
        for rb0, rb1, r0, r1 in self._slices:
            e.residual_rows(it, rb0, rb1)
            works.append(self.all_reduce_async(self._rx()[r0:r1]))
        for w in works:
            w.wait()

    def _fix_r(self):
        """The fixed-point r (bsls_bb_problem.r_fx) of an atomic-K1 shard:
        every |partial sum| of a row is at most |target_i| + |N z|max * sum_j
        |A_ij| over all ranks' columns (|N z| <= 2 (max|z0| + 1) in the
        prologue, <= 1 once K3 has clipped z), so the scale 2^k puts that bound
        B below 2^61.  Collective: every rank computes the same B, and the
        choice itself is all-reduced first -- fixed point only if every rank's
        engine can take it (fixed_r_ok depends on the rank's own shard: its K1
        plan, its formats), else every rank keeps doubles; ranks that decided
        alone would skip the others' all-reduces, or sum int64 words into
        doubles.  BSLS_SHARD_RFX=0 keeps r in doubles.

        Precision: one scale for all rows resolves every row to 2^-61 B
        absolute; a row far below the largest bound carries more rounding than
        a double sum would (|row| 2^-53) -- below 2^-61 B it is still within
        the 1e-12 relative contract of any row above ~2^-21 B.  Measured on
        rows spanning six orders (test_gpu_shard_native's uneven-rows cases,
        b's first links x 10^6): the iterates sit ~1e-11 from the oracle
        with the fixed point and ~5e-12 with doubles at iteration 1 -- the
        problem's conditioning, not the representation, sets it -- and
        1e-14 at a spread of 65; so the fixed point stays (doubles would
        give back the run-dependent exits it fixes)."""
        import torch
        e = self.e
        ok = (os.environ.get('BSLS_SHARD_RFX', '1') != '0' and hasattr(e, 'fixed_r_ok')
              and bool(e.fixed_r_ok()))
        dev = getattr(e.r, 'device', 'cpu')
        world = max(1, _world_size())
        flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev)
        if world > 1:
            self.all_reduce(flag)
        if float(flag.item()) != float(world):
            return
        import math
        A = e._A_host
        S = np.asarray(abs(A).sum(axis=1)).ravel()
        t = torch.from_numpy(S).to(e.r.device)
        self.all_reduce(t)
        world, rank = max(1, _world_size()), self._rank
        zv = torch.zeros(world, dtype=torch.float64, device=e.r.device)
        zv[rank % world] = float(e.z0.abs().max()) if e.z0 is not None and e.z0.numel() else 0.0
        self.all_reduce(zv)
        nzb = 2.0 * (float(zv.max()) + 1.0)
        B = float((e.target.abs() + nzb * t).max()) if t.numel() else 0.0
        k = 61 - int(math.ceil(math.log2(B))) if B > 0 else 61
        e.set_r_fixed(math.ldexp(1.0, max(-1000, min(1000, k))))

    def prologue(self):
        e = self.e
        self._fix_r()
        e.stage(0, 0)
        e.stage(5, 0)            # z[1] = z0 + 1, x = x0 + N z[1]
        self.residual(0)         # r(z0 + 1)
        e.stage(3, 0)            # g_prev = grad(z0 + 1) -> g[0]
        e.stage(6, 0)            # x = x0 + N z0
        self.residual(0)         # r(z0)
        e.stage(9, 0)            # f(z0)

    def iterate(self, first, count):
        e = self.e
        if self.native is not None:
            import ctypes
            import _native
            from _native import check, stream_handle
            if count > 0 and self.link:
                import torch
                if self._cstream is None:
                    self._cstream = torch.cuda.Stream()
                lb = (ctypes.c_int64 * (self.parts + 1))(*[int(v) for v in e.k1_part_bounds])
                rc = _native.lib().bsls_bb_shard_iterate_parts(
                    e.P, self.native.handle, int(first), int(count), self.parts, lb,
                    ctypes.c_void_p(self._cstream.cuda_stream), stream_handle())
            elif count > 0:
                rc = _native.lib().bsls_bb_shard_iterate(e.P, self.native.handle, int(first),
                                                         int(count), int(self.fuse),
                                                         stream_handle())
            if count > 0:
                err = getattr(self.native, 'error', None)
                if rc != 0 and err is not None:
                    raise RuntimeError('bsls_bb_shard_iterate: all-reduce callback failed') from err
                check(rc, 'bsls_bb_shard_iterate')
            return
        if self.link:
            self._iterate_link(first, count)
            return
        for i in range(first, first + count):
            if self.fuse == 2:
                e.stage(10, i)   # K2 + this rank's slice of ||r||^2
                self.all_reduce(e.scal[self.SUMS_RR])
                # K3 after f / the stopping test of iteration i - 1; stage 15
                # also sets r to target / 0 for stage 14's atomic K1 where the
                # library folds that in (what bsls_bb_shard_iterate enqueues);
                # row parts keep stage 13 (each part initialises its rows)
                e.stage(13 if self._slices else 15, i)
            else:
                e.stage(8 if self.fuse else 3, i)   # (8: + f / stop test of i - 1)
                self.all_reduce(e.scal[self.SUMS])
                e.stage(4, i)
            self.residual(i)
            if not self.fuse:
                e.stage(9, i)    # f / stopping test of iteration i
        if count > 0 and self.fuse:
            e.stage(9, first + count - 1)   # f / stopping test of the last one

    def _iterate_link(self, first, count):
        """The link-part pipeline from Python: what bsls_bb_shard_iterate_parts
        enqueues, with torch.distributed's asynchronous all-reduces."""
        e = self.e
        lb = e.k1_part_bounds
        for i in range(first, first + count):
            for q in range(self.parts):
                if self._works:
                    self._works[q].wait()     # this part's rows of r are summed
                e.k2_part(i, q)
            self._works = []
            self.all_reduce(e.scal[self.SUMS_RR])
            e.stage(15, i)
            for q, (rb0, rb1, r0, r1) in enumerate(self._slices):
                e.k1_rows(i, rb0, rb1)
                self._works.append(self.all_reduce_async(self._rx()[r0:r1]))
        if count > 0:
            for w in self._works:
                w.wait()
            self._works = []
            e.stage(9, first + count - 1)


def comm_count(handle):
    """bsls_comm_count: the ranks a C-ABI communicator spans."""
    import ctypes
    import _native
    from _native import check
    n = ctypes.c_int(0)
    check(_native.lib().bsls_comm_count(handle, ctypes.byref(n)), 'bsls_comm_count')
    return int(n.value)


def torch_all_reduce(group=None):
    import torch.distributed as dist

    def f(t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return f


def torch_all_reduce_async(group=None):
    import torch.distributed as dist

    def f(t):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)
    return f


class CallbackComm:
    """A C-ABI communicator whose all-reduce is a Python callable
    (bsls_comm_create_callback, csrc/shard.hip): the native driver
    bsls_bb_shard_iterate then runs its world > 1 loop -- both shard roles, the
    five-sum and r all-reduces between its stages -- over any transport, e.g.
    gloo ranks sharing one GPU in the tests.  `all_reduce(t)` sums a float64
    device tensor in place across the ranks; `views` are the tensors the
    driver reduces (the engine's scal and r), found by their device address.
    The callback synchronises the stream before reducing, so the sum sees the
    stages enqueued before it, and returns before the next stage is enqueued."""

    def __init__(self, all_reduce, views=None, rank=None, world=None, engine=None):
        import ctypes
        import _native
        from _native import check
        self.rank = _shard_rank(rank)
        self.world = int(world) if world is not None else _world_size()
        # an engine's scal and r (r as its exchange sums it: int64 words under
        # a fixed-point r, whose scale the prologue sets), else the tensors given
        if engine is not None:
            views = [lambda: engine.scal, lambda: engine.r_exchange]
        self._views = [v if callable(v) else (lambda v=v: v) for v in views]
        self._fn = all_reduce
        self.error = None

        def cb(buf, count, stream, user):
            try:
                import torch
                t = None
                for view in self._views:
                    v = view()
                    base = int(v.data_ptr())
                    off = (int(buf) - base) // 8
                    if 0 <= off and off + count <= v.numel() and int(buf) == base + 8 * off:
                        t = v[off:off + count]
                        break
                if t is None:
                    raise ValueError('all-reduce of an unknown buffer 0x%x' % int(buf))
                torch.cuda.synchronize()
                self._fn(t)
                return 0
            except Exception as exc:      # reported as BSLS_E_COMM by the driver
                self.error = exc
                return 1
        self._cb = _native.ALL_REDUCE_FN(cb)    # kept alive with the communicator
        h = ctypes.c_void_p()
        check(_native.lib().bsls_comm_create_callback(self.world, self.rank, self._cb, None,
                                                      ctypes.byref(h)),
              'bsls_comm_create_callback')
        self.handle = h

    def count(self):
        return comm_count(self.handle)

    def close(self):
        import _native
        if self.handle is not None:
            _native.lib().bsls_comm_destroy(self.handle)
            self.handle = None


class ModelComm:
    """A modelled exchange (bsls_comm_create_model) for one-GPU rehearsals of
    rank `rank` of `world`: every all-reduce moves nothing and holds its stream
    for fixed_us + us_per_mb per MB (timing only)."""

    def __init__(self, world, rank, fixed_us=0.0, us_per_mb=0.0):
        import ctypes
        import _native
        from _native import check
        self.world, self.rank = int(world), int(rank)
        h = ctypes.c_void_p()
        check(_native.lib().bsls_comm_create_model(self.world, self.rank, float(fixed_us),
                                                   float(us_per_mb), ctypes.byref(h)),
              'bsls_comm_create_model')
        self.handle = h

    def close(self):
        import _native
        if self.handle is not None:
            _native.lib().bsls_comm_destroy(self.handle)
            self.handle = None


class RcclComm:
    """A C-ABI communicator (bsls_comm_*, csrc/shard.hip) over the ranks of the
    initialized torch.distributed group: rank 0 makes the RCCL id, a broadcast
    over the group hands it to the others, every rank joins on its current
    device.  In a torch process csrc/shard.hip resolves the RCCL torch loaded,
    so both drive the same library.  force: the native driver runs its
    collectives at world 1 too (bsls_comm_force_collectives; a one-rank sum is
    the identity) -- every RCCL call of the loop executes on a one-GPU box."""

    def __init__(self, group=None, force=False):
        import ctypes
        import torch
        import torch.distributed as dist
        import _native
        from _native import check
        L = _native.lib()
        nb = int(L.bsls_comm_id_bytes())
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        buf = ctypes.create_string_buffer(nb)
        if self.rank == 0:
            check(L.bsls_comm_unique_id(buf), 'bsls_comm_unique_id')
        t = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        if dist.get_backend(group) == 'nccl':
            t = t.cuda()
        dist.broadcast(t, src=0, group=group)
        raw = bytes(t.cpu().numpy().tobytes())
        h = ctypes.c_void_p()
        check(L.bsls_comm_create(raw, self.world, self.rank, ctypes.byref(h)), 'bsls_comm_create')
        self.handle = h
        if force:
            check(L.bsls_comm_force_collectives(h, 1), 'bsls_comm_force_collectives')

    def count(self):
        """The ranks RCCL says this communicator spans (ncclCommCount)."""
        return comm_count(self.handle)

    def all_reduce(self, t):
        """In-place sum of a float64 device tensor over the ranks (current stream)."""
        import _native
        from _native import check, ptr, stream_handle
        check(_native.lib().bsls_comm_all_reduce(self.handle, ptr(t), t.numel(),
                                                 stream_handle()), 'bsls_comm_all_reduce')

    def close(self):
        import _native
        if self.handle is not None:
            _native.lib().bsls_comm_destroy(self.handle)
            self.handle = None
