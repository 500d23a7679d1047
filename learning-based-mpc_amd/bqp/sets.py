"""Terminal sets per model - the offline set construction of the
tracking MPC (trackingMPC/compute_MPIS.m:7-22, RunExample.m:77-108) for a whole batch of
(perturbed / learned) models, packed for the structured solver's per-instance polytope blocks
(bqp_ocp_data.sFp != 0, rows padded with 0 <= 1 to a common count).

Host-side and offline (scipy HiGHS LPs, as the reference's MPT3 calls are); the solve that uses
the sets runs on the GPU.  Per model the maximal positively invariant set of the extended
closed loop w+ = Ak w, w = [x; theta], inside the extended constraint polytope X_ext
(lambda-tightened steady states) is grown one prediction step at a time: the rows F Ak^i whose
support over the current set exceeds 1 are added, and the recursion ends at the first step
that adds none (compute_MPIS.m's O_{i+1} == O_i); implied rows are then dropped.
"""
import numpy as np
from scipy.optimize import linprog


def _support(F, h, c):
    """max c'w over {F w <= h} (None if unbounded / infeasible)"""
    res = linprog(-c, A_ub=F, b_ub=h, bounds=[(None, None)] * F.shape[1], method='highs')
    return -res.fun if res.status == 0 else None


def _prune(F, h, tol):
    """drop the rows implied by the others (one LP per row, last rows first)"""
    keep = np.ones(len(h), bool)
    for i in range(len(h) - 1, -1, -1):
        keep[i] = False
        s = _support(F[keep], h[keep], F[i])
        keep[i] = s is None or s > h[i] + tol
    return F[keep], h[keep]


def mpis(F_w, h_w, Ak, max_steps=500, tol=1e-9):
    """Maximal positively invariant subset of {F_w w <= h_w} under w+ = Ak w, as (F, h) with
    h = 1 (compute_MPIS.m normalises the rows), minimal H-representation."""
    G = np.asarray(F_w, float) / np.asarray(h_w, float)[:, None]
    F, h = _prune(G, np.ones(len(G)), tol)
    Ai = np.eye(Ak.shape[0])
    for _ in range(max_steps):
        Ai = Ai @ Ak
        add = []
        for r in G @ Ai:
            s = _support(F, h, r)
            if s is None or s > 1.0 + tol:
                add.append(r)
        if not add:
            return _prune(F, h, tol)
        F = np.vstack([F, np.array(add)])
        h = np.concatenate([h, np.ones(len(add))])
    raise RuntimeError('terminal set not finitely determined within %d steps' % max_steps)


def tracking_terminal_set(A, B, K, LAMBDA, PSI, F_x, h_x, F_u, h_u, lam=0.99):
    """RunExample.m:77-108 for one model: the extended-state constraints (x in X, LAMBDA theta
    in lam X, K x + L theta in U, PSI theta in lam U with L = PSI - K LAMBDA) and the closed
    loop Ak = [A + B K, B L; 0, I]; returns its MPIS over [x; theta]."""
    A = np.asarray(A, float); B = np.asarray(B, float)
    n, m = B.shape
    K = np.asarray(K, float).reshape(m, n)
    LAMBDA = np.asarray(LAMBDA, float).reshape(n, -1)
    PSI = np.asarray(PSI, float).reshape(m, -1)
    p = LAMBDA.shape[1]
    L = PSI - K @ LAMBDA
    F_x = np.asarray(F_x, float); F_u = np.asarray(F_u, float)
    F_w = np.block([[F_x, np.zeros((len(F_x), p))],
                    [np.zeros((len(F_x), n)), F_x @ LAMBDA],
                    [F_u @ K, F_u @ L],
                    [np.zeros((len(F_u), n)), F_u @ PSI]])
    h_w = np.concatenate([h_x, lam * np.asarray(h_x, float), h_u, lam * np.asarray(h_u, float)])
    Ak = np.block([[A + B @ K, B @ L], [np.zeros((p, n)), np.eye(p)]])
    return mpis(F_w, h_w, Ak)


def pack_sets(sets, nx, nu, rows=None):
    """Per-model sets [(F_i (m_i, nx + np), h_i)] -> (Fp (batch, rows, nv), hp (batch, rows)) in
    the structured problem's [x; u; theta] columns; missing rows are 0 <= 1 (inactive)."""
    rows = rows or max(len(h) for _, h in sets)
    npar = sets[0][0].shape[1] - nx
    nv = nx + nu + npar
    Fp = np.zeros((len(sets), rows, nv))
    hp = np.ones((len(sets), rows))
    for i, (F, h) in enumerate(sets):
        if len(h) > rows:
            raise ValueError('set %d has %d rows > %d' % (i, len(h), rows))
        Fp[i, :len(h), :nx] = F[:, :nx]
        Fp[i, :len(h), nx + nu:] = F[:, nx:]
        hp[i, :len(h)] = h
    return Fp, hp
