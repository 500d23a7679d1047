"""Structured batched OCP solve (bqp_solve_ocp_batched) — the fast path.

``OcpProblem`` holds one stage-wise problem description (shared by the whole batch unless a
per-instance array is given); ``solve_ocp`` solves a batch of instances that differ in x0 (and
optionally the linear terms w, the polytope right-hand side hp, or the model A/B).

Dimensions without a compiled structured kernel ((nx, nu, np) other than the MG (4, 1, 1) and
DI (2, 2, 2) families, or N + 1 > 128) take the condensed route: the states are eliminated on
the host once per problem (bqp.condense) and the batch runs through bqp_quadprog_batched, the
dense GPU kernels — same iterate semantics (exit flags, iterations), no CPU solve.
"""
import ctypes as C

import numpy as np

from . import _lib


class OcpProblem:
    """x_{k+1} = A x_k + B u_k + c; cost sum 0.5 v'W_k v + w_k'v, v = [x; u; theta];
    box bounds on x_k (k>=1), u_k; polytope Fp [x_kp; u_kp; theta] <= hp.

    Arrays use natural numpy shapes (row-major): W (N+1, nv, nv), w (N+1, nv),
    xlb/xub (N+1, nx), ulb/uub (N, nu), Fp (mp, nv), hp (mp,)."""

    def __init__(self, A, B, W, N, np_, w=None, c=None, xlb=None, xub=None, ulb=None, uub=None,
                 Fp=None, hp=None, poly_stage=None, const=0.0):
        self.A = np.asarray(A, float)
        self.B = np.asarray(B, float)
        self.nx, self.nu = self.B.shape
        self.np = int(np_)
        self.N = int(N)
        nv = self.nx + self.nu + self.np
        self.nv = nv
        self.W = np.asarray(W, float).reshape(self.N + 1, nv, nv)
        self.w = np.zeros((self.N + 1, nv)) if w is None else np.asarray(w, float).reshape(self.N + 1, nv)
        self.c = np.zeros(self.nx) if c is None else np.asarray(c, float)
        inf = np.inf
        self.xlb = np.full((self.N + 1, self.nx), -inf) if xlb is None else np.asarray(xlb, float)
        self.xub = np.full((self.N + 1, self.nx), inf) if xub is None else np.asarray(xub, float)
        self.ulb = np.full((self.N, self.nu), -inf) if ulb is None else np.asarray(ulb, float)
        self.uub = np.full((self.N, self.nu), inf) if uub is None else np.asarray(uub, float)
        self.Fp = np.zeros((0, nv)) if Fp is None else np.asarray(Fp, float).reshape(-1, nv)
        self.hp = np.zeros(0) if hp is None else np.asarray(hp, float).ravel()
        self.poly_stage = self.N if poly_stage is None else int(poly_stage)
        self.const = const

    @property
    def mp(self):
        return self.Fp.shape[0]


def _cm(a):
    """Column-major flattening of the trailing two axes (MATLAB layout)."""
    return np.ascontiguousarray(np.swapaxes(a, -1, -2), dtype=np.float64)


class OcpResult(dict):
    __getattr__ = dict.__getitem__


def pack(prob, x0, w=None, hp=None, A=None, B=None, Fp=None, W=None):
    """Builds (dims, data, keepalive) for a batch.  x0: (batch, nx); per-instance overrides
    w (batch, N+1, nv), hp (batch, mp), A (batch, nx, nx), B (batch, nx, nu) and the polytope
    Fp (batch, mp, nv) (same row count and stage as prob's) and the stage costs W (batch, N+1, nv,
    nv)."""
    x0 = np.ascontiguousarray(np.atleast_2d(x0), dtype=np.float64)
    batch = x0.shape[0]
    keep = [x0]

    def arr(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        keep.append(a)
        return a

    nx, nu, nv, N, mp = prob.nx, prob.nu, prob.nv, prob.N, prob.mp
    Aa = arr(_cm(prob.A if A is None else A))
    Ba = arr(_cm(prob.B if B is None else B))
    Wa = arr(_cm(prob.W if W is None else W))
    wa = arr(prob.w if w is None else w)
    Fa = arr(_cm(prob.Fp if Fp is None else Fp)) if mp else None
    ha = arr(prob.hp if hp is None else hp) if mp else None
    ca = arr(prob.c)
    xlb, xub, ulb, uub = arr(prob.xlb), arr(prob.xub), arr(prob.ulb), arr(prob.uub)
    dims = _lib.OcpDims(nx, nu, prob.np, N, mp, prob.poly_stage)
    data = _lib.OcpData(
        A=_lib.ptr(Aa), B=_lib.ptr(Ba), c=_lib.ptr(ca), W=_lib.ptr(Wa), w=_lib.ptr(wa),
        xlb=_lib.ptr(xlb), xub=_lib.ptr(xub), ulb=_lib.ptr(ulb), uub=_lib.ptr(uub),
        Fp=_lib.ptr(Fa), hp=_lib.ptr(ha), x0=_lib.ptr(x0),
        sA=0 if A is None else nx * nx, sB=0 if B is None else nx * nu, sc=0,
        sW=0 if W is None else (N + 1) * nv * nv,
        sw=0 if w is None else (N + 1) * nv, sxb=0, sub=0, sFp=0 if Fp is None else mp * nv,
        shp=0 if hp is None else mp, sx0=nx)
    return dims, data, batch, keep


def solve_ocp(prob, x0, w=None, hp=None, A=None, B=None, handle=None, want_duals=False, Fp=None,
              W=None, route='auto', **opts):
    """Solve a batch on the GPU.  Returns OcpResult(x (b,N+1,nx), u (b,N,nu), theta (b,np),
    fval, exitflag, iterations, firstorderopt, constrviolation, mu[, pi, lam_x, lam_u, lam_p]).
    route: 'auto' (structured kernel; condensed when the C ABI reports the dimensions
    unsupported), 'structured' (no condensed route) or 'condensed'."""
    if route not in ('auto', 'structured', 'condensed'):
        raise ValueError("route must be 'auto', 'structured' or 'condensed', not %r" % (route,))
    lib = _lib.load()
    h = handle or _default_handle()
    dims, data, batch, keep = pack(prob, x0, w, hp, A, B, Fp, W)
    N, nx, nu, npar, mp = prob.N, prob.nx, prob.nu, prob.np, prob.mp
    x = np.zeros((batch, N + 1, nx)); u = np.zeros((batch, N, nu)); th = np.zeros((batch, npar))
    fval = np.zeros(batch); flag = np.zeros(batch, np.int32)
    out = (_lib.Output * batch)()
    duals = None
    dd = {}
    if want_duals:
        dd = dict(pi=np.zeros((batch, N, nx)), lam_x=np.zeros((batch, N + 1, 2, nx)),
                  lam_u=np.zeros((batch, N, 2, nu)), lam_p=np.zeros((batch, max(mp, 1))))
        duals = _lib.OcpDuals(*(_lib.ptr(dd[k]) for k in ('pi', 'lam_x', 'lam_u', 'lam_p')))
    if route == 'condensed':
        return solve_ocp_condensed(prob, x0, w, hp, A, B, handle, want_duals, Fp, W, **opts)
    o = _lib.options(**opts)
    rc = lib.bqp_solve_ocp_batched(h.value, C.byref(dims), batch, C.byref(data), C.byref(o),
                                   _lib.ptr(x), _lib.ptr(u), _lib.ptr(th), _lib.ptr(fval),
                                   _lib.iptr(flag), out, C.byref(duals) if duals else None)
    # the condensed route takes only x0 and hp per instance: anything else keeps the structured
    # solver's own error (an LDS fit failure is not a reason to change the algorithm)
    condensable = all(v is None for v in (w, A, B, Fp, W)) and not want_duals
    if rc == _lib.BQP_E_UNSUPPORTED and route == 'auto' and condensable and \
            not _lib.ocp_dims_supported(prob.nx, prob.nu, prob.np, prob.N, prob.mp):
        return solve_ocp_condensed(prob, x0, w, hp, A, B, handle, want_duals, Fp, W, **opts)
    _lib.check(rc, 'bqp_solve_ocp_batched')
    res = OcpResult(x=x, u=u, theta=th, fval=fval + prob.const, exitflag=flag,
                    iterations=np.array([o_.iterations for o_ in out]),
                    firstorderopt=np.array([o_.firstorderopt for o_ in out]),
                    constrviolation=np.array([o_.constrviolation for o_ in out]),
                    mu=np.array([o_.mu for o_ in out]),
                    polished=np.array([o_.polished for o_ in out], dtype=np.int32))
    if want_duals:
        dd['lam_p'] = dd['lam_p'][:, :mp]
        res.update(dd)
    return res


_handles = {}


def _default_handle(device=-1):
    h = _handles.get(device)
    if h is None:
        h = _lib.Handle(device)
        _handles[device] = h
    return h


def condensed_rhs(prob, X0, hp=None):
    """per-instance (f, b) of the condensed QP (bqp.condense) for states X0 (batch, nx) and
    optional per-instance polytope right-hand sides hp (batch, mp); the polytope rows are the
    last mp rows of Condensed.A"""
    from .condense import Condensed
    cd = getattr(prob, '_condensed', None)
    if cd is None:
        cd = prob._condensed = Condensed(prob)
    f, b = cd.rhs(X0)
    if hp is not None and prob.mp:
        b = b.copy()
        b[:, -prob.mp:] += np.asarray(hp, float).reshape(len(b), prob.mp) - prob.hp
    return cd, f, b


def solve_ocp_condensed(prob, x0, w=None, hp=None, A=None, B=None, handle=None, want_duals=False,
                        Fp=None, W=None, **opts):
    """The condensed route of solve_ocp: one host condensing per problem, the batch on the dense
    GPU kernels (bqp_quadprog_batched), trajectories recovered through the dynamics.  Per-instance
    x0 and hp; the model, costs and polytope matrix are shared (they define the dense H and A)."""
    from .quadprog import quadprog
    if any(a is not None for a in (w, A, B, Fp, W)):
        raise ValueError('condensed route: only x0 and hp may vary per instance')
    if want_duals:
        raise ValueError('condensed route: stage-wise multipliers are not returned '
                         '(bqp.quadprog gives the condensed rows\' multipliers)')
    X0 = np.ascontiguousarray(np.atleast_2d(x0), dtype=np.float64)
    cd, f, b = condensed_rhs(prob, X0, hp)
    z, _, flag, out, _ = quadprog(cd.H, f, cd.A, b, options=opts or None,
                                  handle=handle or _default_handle())
    N, nx, nu = prob.N, prob.nx, prob.nu
    V = np.einsum('kaj,bj->bka', cd.S, z) + np.einsum('kax,bx->bka', cd.T, X0) + cd.const_e[None]
    Wc = prob.W.copy(); wc = prob.w.copy()
    Wc[N, nx:nx + nu, :] = 0.0; Wc[N, :, nx:nx + nu] = 0.0; wc[N, nx:nx + nu] = 0.0
    fval = 0.5 * np.einsum('bka,kac,bkc->b', V, Wc, V) + np.einsum('bka,ka->b', V, wc)
    return OcpResult(x=V[:, :, :nx], u=V[:, :N, nx:nx + nu], theta=z[:, N * nu:],
                     fval=fval + prob.const, exitflag=flag, iterations=out['iterations'],
                     firstorderopt=out['firstorderopt'], constrviolation=out['constrviolation'],
                     mu=np.full(len(X0), np.nan))
