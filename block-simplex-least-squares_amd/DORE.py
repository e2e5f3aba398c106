"""DORE: projected Landweber step + two residual extrapolations
(reference: python/DORE.py:6-90).

`solve`: same signature and control flow; linop / linop_T / proj are device
closures, the vectors HIP-resident torch tensors, and the scalar branch
decisions (dp > 0, ||err_2||^2 / ||err||^2 < 1) are made on the host, one
small device->host read per decision.

`solve_engine`: the same loop with every step and decision on the device
(bsls_dore_iterate over a BBEngine's K1 / K2 / K3 images; what
gradient_descent's 'DORE' runs); the host only enqueues iterations and reads
the state at the reference's log points.
"""
import logging
import time

from _arr import copy, dot, norm


def solve(x0, linop, linop_T, target, record_every=5, proj=None, log=None, options=None,
          i=10000, eps=10 ** -16):
    start = log(0, x0, 0)
    if options and 'max_iter' in options:
        i = options['max_iter']
    if options and 'opt_tol' in options:
        eps = options['opt_tol']
    b = -copy(target)
    x = copy(x0)
    x_prev = x
    Ax = 0
    Ax_prev = 0
    iter_ = 0
    err = None
    for iter_ in range(i):
        Ax_prev_prev = Ax_prev
        Ax_prev = Ax
        Ax = linop(x)
        err = b - Ax
        nc = norm(x - x_prev)
        norm_change = nc * nc
        if iter_ > 0 and norm_change <= eps:
            break
        x_new = x + linop_T(err)
        x_new = proj(x_new)
        Ax = linop(x_new)
        err = b - Ax
        x_select = x_new
        if iter_ > 2:
            delta_Ax = Ax - Ax_prev
            dp = dot(delta_Ax, delta_Ax)
            if dp > 0:
                a1 = dot(delta_Ax, err) / dp
                Ax_1 = (1 + a1) * Ax - a1 * Ax_prev
                x_1 = x_new + a1 * (x_new - x)
                err_1 = b - Ax_1
                delta_Ax = Ax_1 - Ax_prev_prev
                dp = dot(delta_Ax, delta_Ax)
                if dp > 0:
                    a2 = dot(delta_Ax, err_1) / dp
                    x_2 = x_1 + a2 * (x_1 - x_prev)
                    x_2 = proj(x_2)
                    Ax_2 = linop(x_2)
                    err_2 = b - Ax_2
                    if dot(err_2, err_2) / dot(err, err) < 1:
                        x_select = x_2
                        Ax = Ax_2
        x_prev = x
        x = x_select
        if iter_ % record_every == 0:
            start = log(iter_, x, time.time() - start)
        if options and options.get('verbose', 0) >= 1 and iter_ % 100 == 0:
            logging.debug('iter=%d: %e %e %e' % (iter_, dot(err, err), norm_change, norm(x)))
    log(iter_, x, time.time() - start)
    return x


def solve_engine(engine, z0, scale, target, record_every=5, log=None, options=None, i=10000,
                 eps=10 ** -16, chunk=25):
    """DORE.solve with linop = scale * A N, linop_T = scale * N'A' and proj =
    PAVA v1 + clip on `engine` (device.BBEngine), b = -target (the caller's
    target, already scaled as gradient_descent.py:57-63 scales it).  Logs at
    the reference's points (0, every iteration with iter % record_every == 0,
    the last); iterations are enqueued `chunk` at a time between reads of the
    device's stop flag, and those enqueued past a norm-change break leave the
    iterate as it was."""
    import torch
    import _native
    from _native import ptr, stream_handle, check
    start = log(0, z0, 0)
    if options and 'max_iter' in options:
        i = options['max_iter']
    if options and 'opt_tol' in options:
        eps = options['opt_tol']
    e = engine
    L = _native.lib()
    dev = dict(dtype=torch.float64, device='cuda')
    nz, m = e.nz, e.m
    x0 = torch.as_tensor(z0).to(**dev).reshape(-1)
    if x0.numel() != nz:
        raise ValueError('z0 has %d entries, expected %d' % (x0.numel(), nz))
    bufs = dict(X=[x0.clone(), torch.zeros(nz, **dev), x0.clone()],
                X1=torch.zeros(nz, **dev), D=torch.zeros(nz, **dev), X2=torch.zeros(nz, **dev),
                AX=[torch.zeros(m, **dev) for _ in range(3)], AX2=torch.zeros(m, **dev),
                err=torch.zeros(m, **dev),
                b=-torch.as_tensor(target).to(**dev).reshape(-1),
                S=torch.zeros(_native.S_COUNT, **dev), S2=torch.zeros(_native.S_COUNT, **dev),
                dsc=torch.zeros(_native.DORE_COUNT, **dev),
                part=torch.zeros(L.bsls_dore_work_size(nz, m), dtype=torch.uint8, device='cuda'),
                tickets=torch.zeros(L.bsls_ticket_bytes(), dtype=torch.uint8, device='cuda'))
    bufs['S'][_native.S_SUMDG] = 1.0
    bufs['S'][_native.S_DZDG] = -scale      # K3: x - (-scale) g = x + linop_T(err)
    bufs['S'][_native.S_DGDG] = 1.0
    d = _native.DoreState()
    for k in range(3):
        d.X[k] = bufs['X'][k].data_ptr()
        d.AX[k] = bufs['AX'][k].data_ptr()
    for nm in ('X1', 'D', 'X2', 'AX2', 'err', 'b', 'S', 'S2', 'dsc', 'part', 'tickets'):
        setattr(d, nm, bufs[nm].data_ptr())
    d.scale, d.eps = float(scale), float(eps)
    X = bufs['X']
    it = 0
    while it < i:
        nxt = it if it % record_every == 0 else (it // record_every + 1) * record_every
        end = min(i, it + chunk, nxt + 1)
        check(L.bsls_dore_iterate(e.P, d, it, end - it, stream_handle()), 'bsls_dore_iterate')
        sc = bufs['S'].cpu().numpy()
        if sc[_native.S_STOP] != 0:
            s = int(bufs['dsc'][_native.DORE_STOPIT].item())
            x = X[s % 3].clone()
            log(s, x, time.time() - start)
            e.dore_scalars = bufs['dsc'].cpu().numpy()
            return x
        if (end - 1) % record_every == 0:
            start = log(end - 1, X[end % 3].clone(), time.time() - start)
        it = end
    x = X[i % 3].clone()
    # the reference's loop variable after the loop: i - 1, or 0 when it never ran
    log(max(i - 1, 0), x, time.time() - start)
    e.dore_scalars = bufs['dsc'].cpu().numpy()
    return x
