"""Closed-loop simulation on the GPU (bqp_closed_loop_ocp): the MPC loop of the reference's
tracking-LMPC examples - solve at the measured state, apply the first move to the true plant,
repeat - for a whole batch of initial states at once.

Reference: ``examples/DMS_tracking_LMPC_casadi.m:153-189`` / ``DSS_tracking_LMPC_casadi.m``
(``solver(...)`` then ``xmeasure = dynamic(delta, xmeasure, u_OL(1:m))``), with the
Moore-Greitzer plant ``system`` (:215-221) integrated by one RK4 step (``dynamic``, :297-304).
"""
import ctypes as C

import numpy as np

from . import _lib
from .ocp import OcpResult, _default_handle, pack

BQP_PLANT_MG_RK4 = 1
BQP_PLANT_MG_ODE23 = 2
_PLANTS = {'rk4': BQP_PLANT_MG_RK4, 'ode23': BQP_PLANT_MG_ODE23}


class ClosedLoop(C.Structure):
    _fields_ = [('plant', C.c_int), ('steps', C.c_int), ('delta', C.c_double),
                ('x_eq', _lib._PD), ('u_eq', _lib._PD)]


class Learning(C.Structure):
    _fields_ = [('q', C.c_int), ('mask', C.c_int), ('bandwidth', C.c_double),
                ('lambda_', C.c_double), ('XL', _lib._PD), ('window', _lib._PD)]


class _Dev:
    """device=... path of the closed loops: the inputs of a packed ctypes
    structure moved to the GPU (each pointer field replaced by a device copy of the numpy array it
    pointed to) and the outputs allocated there, so that the _device entry points run on device
    memory and the trajectories stay in HBM for bqp.dist.gather_rows (RCCL all-gather) - no host
    round trip between the loop and the collective."""

    def __init__(self, device):
        import torch
        self.torch = torch
        self.dev = torch.device('cuda', device) if isinstance(device, int) else torch.device(device)
        self.keep = []

    def inputs(self, st, arrays):
        by_addr = {a.ctypes.data: a for a in arrays if a is not None}
        for name, typ in st._fields_:
            if typ not in (_lib._PD, _lib._PI):
                continue
            p = getattr(st, name)
            if not p:
                continue
            a = by_addr[C.cast(p, C.c_void_p).value]
            t = self.torch.from_numpy(a).to(self.dev)
            self.keep.append(t)
            setattr(st, name, C.cast(C.c_void_p(t.data_ptr()), typ))

    def array(self, a):
        t = self.torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)
        self.keep.append(t)
        return t

    def out(self, shape, dtype=np.float64):
        t = self.torch.zeros(shape, dtype=self.torch.float64 if dtype == np.float64 else self.torch.int32,
                             device=self.dev)
        return t

    @staticmethod
    def p(t, typ=None):
        if t is None:
            return None
        return C.cast(C.c_void_p(t.data_ptr()), typ or (_lib._PD if t.dtype.is_floating_point else _lib._PI))

    def stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)


def closed_loop(mpc, x_init, steps, delta=0.01, handle=None, learning=None, plant='rk4',
                x_eq=None, u_eq=None, device=None, **opts):
    """mpc: a TrackingLMPC / TrackingLBMPC (deviation coordinates around mpc.x_eq, mpc.u_eq), or
    an LMPC with the working point passed as x_eq / u_eq (functions/ocpLMPC.m: x_wp, u_wp);
    x_init (batch, n) absolute initial states.  Returns X (batch, steps+1, n), U (batch, steps,
    m) absolute, and the per-step exit flags (batch, steps).
    plant: 'rk4' - one RK4 step per period (`dynamic` of the CasADi scripts); 'ode23' - MATLAB's
    ode23 at its default options (models/trueModel.m behind transitionTrue.m, the plant of the
    fmincon loops ocpLMPC.m / ocpLBMPC.m).

    learning=dict(q=100, mask=1[, bandwidth, lambda_]) also keeps the learned model's data window
    per instance (bqp_closed_loop_lbmpc: LBMPC_casadi.m:193-198 / DMS_LBMPC_casadi.m:198-207)
    and returns XL (batch, steps+1, n), the learned one-step predictions, and window
    (batch, q, 8), the final windows [X; Y; v] per point in ring order (iteration it's sample
    in point it mod q).

    device (a GPU index or torch device): run on device memory through the _device entry points
    (bqp_closed_loop_ocp_device / _lbmpc_device) on torch's current stream of that device; the
    results are torch tensors there (the trajectories stay in HBM, e.g. for bqp.dist.gather_rows)."""
    lib = _lib.load()
    h = handle or _default_handle()
    x_init = np.ascontiguousarray(np.atleast_2d(x_init), dtype=np.float64)
    b = x_init.shape[0]
    prob = mpc.prob
    xeq = np.ascontiguousarray(mpc.x_eq if x_eq is None else np.ravel(x_eq), dtype=np.float64)
    ueq = np.ascontiguousarray(mpc.u_eq if u_eq is None else np.ravel(u_eq), dtype=np.float64)
    dims, data, batch, keep = pack(prob, x_init - xeq)
    cl = ClosedLoop(_PLANTS[plant], int(steps), float(delta), _lib.ptr(xeq), _lib.ptr(ueq))
    if device is not None:
        return _closed_loop_device(lib, h, mpc, dims, data, keep, cl, [xeq, ueq], x_init, b, steps,
                                   learning, device, opts)
    X = np.zeros((b, steps + 1, prob.nx)); U = np.zeros((b, steps, prob.nu))
    flags = np.zeros((b, steps), np.int32)
    o = _lib.options(**opts)
    if learning is None:
        rc = lib.bqp_closed_loop_ocp(h.value, C.byref(dims), b, C.byref(data), C.byref(o),
                                     C.byref(cl), _lib.ptr(x_init), _lib.ptr(X), _lib.ptr(U),
                                     _lib.iptr(flags))
        _lib.check(rc, 'bqp_closed_loop_ocp')
        return OcpResult(X=X, U=U, exitflag=flags)
    q = int(learning.get('q', 100))
    XL = np.zeros_like(X)
    win = np.zeros((b, q, 8))
    lw = Learning(q, int(learning.get('mask', 1)), float(learning.get('bandwidth', 0.0)),
                  float(learning.get('lambda_', 0.0)), _lib.ptr(XL), _lib.ptr(win))
    rc = lib.bqp_closed_loop_lbmpc(h.value, C.byref(dims), b, C.byref(data), C.byref(o),
                                   C.byref(cl), C.byref(lw), _lib.ptr(x_init), _lib.ptr(X),
                                   _lib.ptr(U), _lib.iptr(flags))
    _lib.check(rc, 'bqp_closed_loop_lbmpc')
    return OcpResult(X=X, U=U, exitflag=flags, XL=XL, window=win)


def _closed_loop_device(lib, h, mpc, dims, data, keep, cl, wp, x_init, b, steps, learning, device,
                        opts):
    prob = mpc.prob
    d = _Dev(device)
    d.inputs(data, keep)
    d.inputs(cl, wp)
    xi = d.array(x_init)
    X = d.out((b, steps + 1, prob.nx)); U = d.out((b, steps, prob.nu))
    flags = d.out((b, steps), np.int32)
    o = _lib.options(**opts)
    if learning is None:
        rc = lib.bqp_closed_loop_ocp_device(h.value, C.byref(dims), b, C.byref(data), C.byref(o),
                                            C.byref(cl), d.p(xi), d.p(X), d.p(U), d.p(flags),
                                            d.stream())
        _lib.check(rc, 'bqp_closed_loop_ocp_device')
        d.torch.cuda.current_stream(d.dev).synchronize()
        return OcpResult(X=X, U=U, exitflag=flags)
    q = int(learning.get('q', 100))
    XL = d.out((b, steps + 1, prob.nx)); win = d.out((b, q, 8))
    lw = Learning(q, int(learning.get('mask', 1)), float(learning.get('bandwidth', 0.0)),
                  float(learning.get('lambda_', 0.0)), d.p(XL), d.p(win))
    rc = lib.bqp_closed_loop_lbmpc_device(h.value, C.byref(dims), b, C.byref(data), C.byref(o),
                                          C.byref(cl), C.byref(lw), d.p(xi), d.p(X), d.p(U),
                                          d.p(flags), d.stream())
    _lib.check(rc, 'bqp_closed_loop_lbmpc_device')
    d.torch.cuda.current_stream(d.dev).synchronize()
    return OcpResult(X=X, U=U, exitflag=flags, XL=XL, window=win)


def closed_loop_sqp(mpc, x_init, steps, learning=None, warm=True, delta=0.01, handle=None,
                    max_iter=200, tol=1e-8, log_z=False, plant='rk4', x_eq=None,
                    u_eq=None, polish=0, device=None):
    """Learned-model NLP closed loop on the GPU (bqp_closed_loop_sqp): per step the batched
    Gauss-Newton SQP of mpc (a DMSLBMPC - DMS_LBMPC_casadi.m:163-218 -, HybridLBMPC -
    hybrid_LBMPC_casadi.m:163-204 - or LBMPC) at the measured states, one RK4 plant step with the
    first move, and get_data.m's window update.  x_init (batch, n) absolute.
    learning=dict(q=100, mask=1[, bandwidth, lambda_]): mask 1 is DMS_LBMPC_casadi.m's 8 x q
    window (only the first, zero point valid at the start), mask 0 counts every point (the 7-row
    window of hybrid_LBMPC_casadi.m).  warm: the scripts' shifted guess (previous inputs moved one
    stage, zero last move, theta kept); otherwise z = 0 each step.
    plant: 'rk4' (the CasADi scripts' `dynamic`) or 'ode23' (models/trueModel.m, the fmincon loop
    functions/ocpLBMPC.m; its update_data.m window of q points equals this ring with q - 1: the
    initial zero point leaves when the q-th sample arrives).  polish: the QP sub-problems'
    active-set polish (bqp_options.polish encoding; 0 = the loop's default 3, polish only once the
    SQP stalls at a step; 1 also after -8 sub-problem exits; -1 off).
    Returns X (batch, steps+1, n), U (batch, steps, m) absolute, exitflag and iterations (batch,
    steps), XL (batch, steps+1, n) the learned one-step predictions, window (batch, q, 8) the
    final windows in ring order, and with log_z every step's solution Z (batch, steps, nz).
    device (a GPU index or torch device): bqp_closed_loop_sqp_device on device memory and torch's
    current stream there; every result is a torch tensor on that device."""
    lib = _lib.load()
    h = handle or _default_handle()
    learning = dict(learning or {})
    x_init = np.ascontiguousarray(np.atleast_2d(x_init), dtype=np.float64)
    b = x_init.shape[0]
    q = int(learning.get('q', 100))
    mask = int(learning.get('mask', 1))
    # working point: the caller's (LBMPC, ocpLBMPC.m's x_wp / u_wp), else the shim's own
    x_eq = np.ascontiguousarray(getattr(mpc, 'x_eq', np.zeros(mpc.n)) if x_eq is None else np.ravel(x_eq),
                                dtype=np.float64)
    u_eq = np.ascontiguousarray(getattr(mpc, 'u_eq', np.zeros(mpc.m)) if u_eq is None else np.ravel(u_eq),
                                dtype=np.float64)
    mrows = mpc.Ain.shape[0]
    keep = [np.ascontiguousarray(a, dtype=np.float64) for a in
            (mpc.A.T, mpc.B.T, mpc.K.T, mpc.Lq, mpc.Lr, mpc.Lp, mpc.Lt, mpc.LAMBDA.T, mpc.PSI.T,
             mpc.xs)]
    bin0 = np.ascontiguousarray(mpc.b0, dtype=np.float64)
    Bx = np.ascontiguousarray(mpc.Bx.T, dtype=np.float64)        # column-major m x n
    dims = _lib.LbmpcDims(mpc.n, mpc.m, mpc.p, mpc.N, mpc.n_run, int(mpc.term_learned), q, mrows, 1,
                          int(getattr(mpc, 'hessian', 'exact') == 'exact'))
    dd = _lib.LbmpcData(*[_lib.ptr(a) for a in keep], None, 0, None, 0, _lib.ptr(mpc.Ain_cm), None,
                        0, mpc.bandwidth, mpc.lam)
    if device is not None:
        return _closed_loop_sqp_device(lib, h, mpc, dims, dd, keep, bin0, Bx, x_eq, u_eq, x_init, b,
                                       steps, q, mask, learning, warm, delta, plant, max_iter, tol,
                                       log_z, polish, device)
    X = np.zeros((b, steps + 1, mpc.n)); U = np.zeros((b, steps, mpc.m))
    XL = np.zeros_like(X); win = np.zeros((b, q, 8))
    flags = np.zeros((b, steps), np.int32); its = np.zeros((b, steps), np.int32)
    Z = np.zeros((b, steps, mpc.nz)) if log_z else None
    sl = _lib.SqpLoop(_lib.ptr(bin0), _lib.ptr(Bx), int(bool(warm)), _lib.ptr(Z), _lib.iptr(its))
    cl = ClosedLoop(_PLANTS[plant], int(steps), float(delta), _lib.ptr(x_eq), _lib.ptr(u_eq))
    lw = Learning(q, mask, float(learning.get('bandwidth', 0.0)), float(learning.get('lambda_', 0.0)),
                  _lib.ptr(XL), _lib.ptr(win))
    o = _lib.options(max_iter=max_iter, tol_stat=tol, polish=polish)
    rc = lib.bqp_closed_loop_sqp(h.value, C.byref(dims), b, C.byref(dd), C.byref(sl), C.byref(o),
                                 C.byref(cl), C.byref(lw), _lib.ptr(x_init), _lib.ptr(X),
                                 _lib.ptr(U), _lib.iptr(flags))
    _lib.check(rc, 'bqp_closed_loop_sqp')
    out = OcpResult(X=X, U=U, exitflag=flags, iterations=its, XL=XL, window=win)
    if log_z:
        out.update(Z=Z)
    return out


def _closed_loop_sqp_device(lib, h, mpc, dims, dd, keep, bin0, Bx, x_eq, u_eq, x_init, b, steps, q,
                            mask, learning, warm, delta, plant, max_iter, tol, log_z, polish,
                            device):
    d = _Dev(device)
    d.inputs(dd, keep + [mpc.Ain_cm])
    X = d.out((b, steps + 1, mpc.n)); U = d.out((b, steps, mpc.m))
    XL = d.out((b, steps + 1, mpc.n)); win = d.out((b, q, 8))
    flags = d.out((b, steps), np.int32); its = d.out((b, steps), np.int32)
    Z = d.out((b, steps, mpc.nz)) if log_z else None
    sl = _lib.SqpLoop(d.p(d.array(bin0)), d.p(d.array(Bx)), int(bool(warm)), d.p(Z), d.p(its))
    cl = ClosedLoop(_PLANTS[plant], int(steps), float(delta), d.p(d.array(x_eq)), d.p(d.array(u_eq)))
    lw = Learning(q, mask, float(learning.get('bandwidth', 0.0)), float(learning.get('lambda_', 0.0)),
                  d.p(XL), d.p(win))
    o = _lib.options(max_iter=max_iter, tol_stat=tol, polish=polish)
    xi = d.array(x_init)
    rc = lib.bqp_closed_loop_sqp_device(h.value, C.byref(dims), b, C.byref(dd), C.byref(sl), C.byref(o),
                                        C.byref(cl), C.byref(lw), d.p(xi), d.p(X), d.p(U), d.p(flags),
                                        d.stream())
    _lib.check(rc, 'bqp_closed_loop_sqp_device')
    d.torch.cuda.current_stream(d.dev).synchronize()
    out = OcpResult(X=X, U=U, exitflag=flags, iterations=its, XL=XL, window=win)
    if log_z:
        out.update(Z=Z)
    return out
