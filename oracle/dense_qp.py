"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Ground-truth dense QP solver for the restated reference QPs:

    min 0.5 z'Hz + f'z  s.t.  A z <= b,  Aeq z = beq,  lb <= z <= ub.

Stage 1: a plain fp64 primal-dual Mehrotra IPM on the full KKT (numpy dense LU).
Stage 2: exact active-set polish — rows with lambda_i > slack_i are taken as active, the
equality-constrained KKT on that set is solved directly, and the result is accepted only if it
is primal feasible and dual feasible (lambda >= 0) to 1e-12.  This is the "exact active-set
KKT refinement" of SURVEY.md §8(c); it does not depend on any iterate of the solver under
test.

Multiplier conventions follow MATLAB quadprog: ``lam['ineqlin']``, ``lam['eqlin']``,
``lam['lower']``, ``lam['upper']`` with  H z + f + A'l_in + Aeq'l_eq - l_lo + l_up = 0.
"""
import numpy as np


def _rows(qp):
    H, f = qp['H'], qp['f']
    n = H.shape[0]
    A, b = qp['A'], qp['b']
    Aeq, beq = qp['Aeq'], qp['beq']
    lb, ub = qp['lb'], qp['ub']
    fixed = np.isfinite(lb) & np.isfinite(ub) & (lb == ub)
    E = [Aeq]; e = [beq]
    if fixed.any():
        idx = np.flatnonzero(fixed)
        M = np.zeros((idx.size, n)); M[np.arange(idx.size), idx] = 1.0
        E.append(M); e.append(lb[idx])
    E = np.vstack(E); e = np.concatenate(e)
    G = [A]; h = [b]; kind = [np.zeros(A.shape[0], int)]; src = [np.arange(A.shape[0])]
    iu = np.flatnonzero(np.isfinite(ub) & ~fixed)
    il = np.flatnonzero(np.isfinite(lb) & ~fixed)
    if iu.size:
        M = np.zeros((iu.size, n)); M[np.arange(iu.size), iu] = 1.0
        G.append(M); h.append(ub[iu]); kind.append(np.full(iu.size, 2)); src.append(iu)
    if il.size:
        M = np.zeros((il.size, n)); M[np.arange(il.size), il] = -1.0
        G.append(M); h.append(-lb[il]); kind.append(np.full(il.size, 1)); src.append(il)
    return (H, f, np.vstack(G), np.concatenate(h), np.concatenate(kind),
            np.concatenate(src), E, e, fixed)


def solve(qp, tol=1e-12, max_iter=200, polish=True):
    H, f, G, h, kind, src, E, e, fixed = _rows(qp)
    n = H.shape[0]
    m = G.shape[0]
    p = E.shape[0]
    # --- stage 1: Mehrotra predictor-corrector on [H E' G'; E 0 0; G 0 -D^{-1}] ----------
    z = np.zeros(n)
    y = np.zeros(p)
    s = np.ones(m)
    lam = np.ones(m)
    # initial point: least squares with unit scaling (CVXOPT-style)
    K = np.block([[H + G.T @ G, E.T], [E, np.zeros((p, p))]])
    sol = np.linalg.lstsq(K, np.concatenate([-f + G.T @ h, e]), rcond=None)[0]
    z = sol[:n]
    r = h - G @ z
    s = np.maximum(r, 1.0)
    lam = np.ones(m)
    scale = max(1.0, np.abs(f).max(initial=0), np.abs(h).max(initial=0))
    it = 0
    for it in range(max_iter):
        rd = H @ z + f + E.T @ y + G.T @ lam
        re = E @ z - e
        ri = G @ z + s - h
        mu = s @ lam / max(m, 1)
        if (np.abs(rd).max(initial=0) < tol * scale and np.abs(re).max(initial=0) < tol * scale
                and np.abs(ri).max(initial=0) < tol * scale and mu < tol * 1e-2):
            break
        d = lam / s

        def kkt(rc):
            Kr = np.block([[H + G.T @ (d[:, None] * G), E.T], [E, np.zeros((p, p))]])
            rhs = np.concatenate([-rd - G.T @ ((lam * ri - rc) / s), -re])
            dd = np.linalg.solve(Kr, rhs)
            dz, dy = dd[:n], dd[n:]
            ds = -ri - G @ dz
            dl = (-rc - lam * ds) / s
            return dz, dy, ds, dl

        def step(v, dv):
            neg = dv < 0
            return min(1.0, (-v[neg] / dv[neg]).min()) if neg.any() else 1.0

        dz, dy, ds, dl = kkt(s * lam)
        a = min(step(s, ds), step(lam, dl))
        mua = (s + a * ds) @ (lam + a * dl) / m
        sig = (mua / mu) ** 3
        dz, dy, ds, dl = kkt(s * lam + ds * dl - sig * mu)
        a = min(1.0, 0.99 * min(step(s, ds), step(lam, dl)))
        z += a * dz; y += a * dy; s += a * ds; lam += a * dl
    info = dict(iterations=it, polished=False)
    # --- stage 2: active-set polish ------------------------------------------------------
    if polish and m > 0:
        act = lam > s
        Ga = G[act]
        na = Ga.shape[0]
        Kp = np.block([[H, E.T, Ga.T],
                       [E, np.zeros((p, p)), np.zeros((p, na))],
                       [Ga, np.zeros((na, p)), np.zeros((na, na))]])
        rhs = np.concatenate([-f, e, h[act]])
        try:
            solp = np.linalg.lstsq(Kp, rhs, rcond=1e-14)[0]   # degenerate active sets allowed
            zp = solp[:n]; yp = solp[n:n + p]; lp = np.zeros(m); lp[act] = solp[n + p:]
            feas = (G @ zp - h).max(initial=-1) <= 1e-12 * scale
            dual = lp.min(initial=0) >= -1e-12 * max(1.0, np.abs(lp).max(initial=0))
            if feas and dual and np.isfinite(zp).all():
                z, y, lam = zp, yp, np.maximum(lp, 0.0)
                s = h - G @ z
                info['polished'] = True
                info['n_active'] = int(na)
        except np.linalg.LinAlgError:
            pass
    # --- multipliers in quadprog layout ---------------------------------------------------
    nA = qp['A'].shape[0]
    lam_out = dict(ineqlin=lam[kind == 0][:nA].copy(), lower=np.zeros(n), upper=np.zeros(n),
                   eqlin=y[:qp['Aeq'].shape[0]].copy())
    lam_out['upper'][src[kind == 2]] = lam[kind == 2]
    lam_out['lower'][src[kind == 1]] = lam[kind == 1]
    if fixed.any():
        # multiplier of a fixed variable: reported on lower/upper by sign (quadprog convention)
        yf = y[qp['Aeq'].shape[0]:]
        idx = np.flatnonzero(fixed)
        lam_out['upper'][idx] = np.maximum(yf, 0)
        lam_out['lower'][idx] = np.maximum(-yf, 0)
    fval = 0.5 * z @ H @ z + f @ z
    info['kkt'] = kkt_residual(qp, z, lam_out)
    return z, fval, lam_out, info


def kkt_residual(qp, z, lam):
    """inf-norms (stationarity, primal eq, primal ineq, complementarity)."""
    H, f, A, b, Aeq, beq, lb, ub = (qp[k] for k in ('H', 'f', 'A', 'b', 'Aeq', 'beq', 'lb', 'ub'))
    g = H @ z + f + A.T @ lam['ineqlin'] + Aeq.T @ lam['eqlin'] - lam['lower'] + lam['upper']
    st = np.abs(g).max(initial=0)
    peq = np.abs(Aeq @ z - beq).max(initial=0)
    viol = [np.maximum(A @ z - b, 0).max(initial=0)]
    fl = np.isfinite(lb); fu = np.isfinite(ub)
    viol.append(np.maximum(lb[fl] - z[fl], 0).max(initial=0))
    viol.append(np.maximum(z[fu] - ub[fu], 0).max(initial=0))
    comp = [np.abs(lam['ineqlin'] * (b - A @ z)).max(initial=0)]
    fixed = fl & fu & (lb == ub)
    ml = fl & ~fixed; mu_ = fu & ~fixed
    comp.append(np.abs(lam['lower'][ml] * (z[ml] - lb[ml])).max(initial=0))
    comp.append(np.abs(lam['upper'][mu_] * (ub[mu_] - z[mu_])).max(initial=0))
    return dict(stationarity=st, primal_eq=peq, primal_ineq=max(viol), complementarity=max(comp))
