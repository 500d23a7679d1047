"""MATLAB-quadprog-compatible batched dense solve (bqp_quadprog_batched).

    x, fval, exitflag, output, lam = quadprog(H, f, A, b, Aeq, beq, lb, ub)

Each argument may carry a leading batch axis (per-instance) or not (shared by the batch);
matrices use numpy's natural (rows, cols) shape and are passed column-major to the C ABI.
lam has quadprog's fields: ineqlin, eqlin, lower, upper.
"""
import ctypes as C

import numpy as np

from . import _lib


def _prep(a, shape, batch):
    """(array or None, stride) in column-major per-instance layout."""
    if a is None:
        return None, 0
    a = np.asarray(a, dtype=np.float64)
    nd = len(shape)
    if a.ndim == nd + 1:
        if a.shape[0] != batch:
            raise ValueError('batch mismatch')
        per = True
    elif a.ndim == nd:
        per = False
        a = a[None]
    else:
        raise ValueError('bad shape %s, want %s' % (a.shape, shape))
    if nd == 2:
        a = np.swapaxes(a, -1, -2)
    a = np.ascontiguousarray(a)
    size = int(np.prod(shape)) if nd else 1
    return a, (size if per else 0)


def _fixed_to_equalities(n, Aeq, beq, lb, ub, batch):
    """quadprog accepts lb == ub (fixed variables); the kernel takes them as equality rows."""
    if lb is None or ub is None:
        return Aeq, beq, lb, ub, None
    L = np.broadcast_to(np.asarray(lb, float), (batch, n))
    U = np.broadcast_to(np.asarray(ub, float), (batch, n))
    fixed = np.isfinite(L) & np.isfinite(U) & (L == U)
    if not fixed.any():
        return Aeq, beq, lb, ub, None
    if not (fixed == fixed[0]).all():
        raise ValueError('fixed variables (lb == ub) must be the same for every instance')
    idx = np.flatnonzero(fixed[0])
    E = np.zeros((idx.size, n)); E[np.arange(idx.size), idx] = 1.0
    me0 = 0 if Aeq is None else np.shape(Aeq)[-2]
    if Aeq is None:
        Aeq2 = E
        beq2 = L[:, idx]
    else:
        Ae = np.asarray(Aeq, float)
        Aeq2 = np.concatenate([np.broadcast_to(Ae, (batch,) + Ae.shape[-2:]),
                               np.broadcast_to(E, (batch,) + E.shape)], axis=1)
        beq2 = np.concatenate([np.broadcast_to(np.asarray(beq, float), (batch, me0)), L[:, idx]], axis=1)
    lb2 = np.where(fixed, -np.inf, L)
    ub2 = np.where(fixed, np.inf, U)
    return Aeq2, beq2, lb2, ub2, (idx, me0)


def quadprog(H, f, A=None, b=None, Aeq=None, beq=None, lb=None, ub=None, x0=None, options=None,
             handle=None):
    from .ocp import _default_handle
    lib = _lib.load()
    H = np.asarray(H, float)
    f = np.asarray(f, float)
    n = H.shape[-1]
    b0 = max(H.shape[0] if H.ndim == 3 else 1, f.shape[0] if f.ndim == 2 else 1)
    for a_, nd in ((A, 2), (b, 1), (Aeq, 2), (beq, 1), (lb, 1), (ub, 1)):
        if a_ is not None and np.ndim(a_) == nd + 1:
            b0 = max(b0, np.shape(a_)[0])
    Aeq, beq, lb, ub, fixinfo = _fixed_to_equalities(n, Aeq, beq, lb, ub, b0)
    batch = max(H.shape[0] if H.ndim == 3 else 1, f.shape[0] if f.ndim == 2 else 1)
    for a, nd in ((A, 2), (b, 1), (Aeq, 2), (beq, 1), (lb, 1), (ub, 1)):
        if a is not None and np.ndim(a) == nd + 1:
            batch = max(batch, np.shape(a)[0])
    m = 0 if A is None else np.shape(A)[-2]
    me = 0 if Aeq is None else np.shape(Aeq)[-2]
    Hc, sH = _prep(H, (n, n), batch)
    fc, sf = _prep(f, (n,), batch)
    Ac, sA = _prep(A, (m, n), batch) if m else (None, 0)
    bc, sb = _prep(b, (m,), batch) if m else (None, 0)
    Ec, sE = _prep(Aeq, (me, n), batch) if me else (None, 0)
    ec, se = _prep(beq, (me,), batch) if me else (None, 0)
    lc, sl = _prep(lb, (n,), batch)
    uc, su = _prep(ub, (n,), batch)
    dims = _lib.Dims(n, m, me)
    st = _lib.Strides(sH, sf, sA, sb, sE, se, sl, su)
    x = np.zeros((batch, n)); fval = np.zeros(batch); flag = np.zeros(batch, np.int32)
    li = np.zeros((batch, max(m, 1))); le = np.zeros((batch, max(me, 1)))
    ll = np.zeros((batch, n)); lu = np.zeros((batch, n))
    out = (_lib.Output * batch)()
    o = _lib.options(**(options or {}))
    h = handle or _default_handle()
    rc = lib.bqp_quadprog_batched(h.value, C.byref(dims), batch, C.byref(st), _lib.ptr(Hc),
                                  _lib.ptr(fc), _lib.ptr(Ac), _lib.ptr(bc), _lib.ptr(Ec),
                                  _lib.ptr(ec), _lib.ptr(lc), _lib.ptr(uc), None, C.byref(o),
                                  _lib.ptr(x), _lib.ptr(fval), _lib.iptr(flag), _lib.ptr(li),
                                  _lib.ptr(le), _lib.ptr(ll), _lib.ptr(lu), out)
    _lib.check(rc, 'bqp_quadprog_batched')
    output = dict(iterations=np.array([q.iterations for q in out]),
                  constrviolation=np.array([q.constrviolation for q in out]),
                  firstorderopt=np.array([q.firstorderopt for q in out]))
    lam = dict(ineqlin=li[:, :m], eqlin=le[:, :me], lower=ll, upper=lu)
    if fixinfo is not None:
        idx, me0 = fixinfo
        yf = le[:, me0:me]
        lam['eqlin'] = le[:, :me0]
        # multiplier of a fixed variable reported on lower/upper by sign (quadprog convention)
        lam['upper'][:, idx] = np.maximum(yf, 0.0)
        lam['lower'][:, idx] = np.maximum(-yf, 0.0)
    return x, fval, flag, output, lam
