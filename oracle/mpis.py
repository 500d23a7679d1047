"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the offline terminal-set construction of the tracking MPC:

* ``compute_mpis`` — ``trackingMPC/compute_MPIS.m:7-22``: with F the rows of Xc normalised to
  right-hand side 1, intersect {w : F Ak^i w <= 1} for i = 0, 1, ... until the set stops
  changing.  MPT3's polytope equality test is replaced by an LP redundancy test of the new rows
  (scipy HiGHS): a new row is kept only if max over the current set exceeds 1.  The returned
  H-representation describes the same set (it is not row-for-row MPT's output, which the
  reference never stores for the DI).
* ``di_terminal_set`` — ``trackingMPC/RunExample.m:77-108``: the extended-state constraint
  polytope X_ext (lambda = 0.99) and Ak = [A+BK, BL; 0, I], L = PSI - K LAMBDA.
"""
import numpy as np
from scipy.optimize import linprog


def _redundant(F, h, row, rhs, tol=1e-9):
    res = linprog(-row, A_ub=F, b_ub=h, bounds=[(None, None)] * F.shape[1], method='highs')
    if res.status != 0:
        return False
    return -res.fun <= rhs + tol


def min_hrep(F, h, tol=1e-9):
    """Drop rows implied by the others (LP test per row)."""
    keep = np.ones(F.shape[0], bool)
    for i in range(F.shape[0]):
        keep[i] = False
        if not _redundant(F[keep], h[keep], F[i], h[i], tol):
            keep[i] = True
    return F[keep], h[keep]


def compute_mpis(Fc, hc, Ak, max_iter=500):
    F = Fc / hc[:, None]                                   # compute_MPIS.m:14-15
    Fs, hs = min_hrep(F, np.ones(F.shape[0]))
    Ai = np.eye(Ak.shape[0])
    for i in range(1, max_iter + 1):                        # compute_MPIS.m:20-29
        Ai = Ai @ Ak
        new = F @ Ai
        added = False
        for r in new:
            if not _redundant(Fs, hs, r, 1.0):
                Fs = np.vstack([Fs, r]); hs = np.append(hs, 1.0)
                added = True
        if not added:
            return min_hrep(Fs, hs) + (i,)
    raise RuntimeError('MPIS not finitely determined within %d steps' % max_iter)


def di_terminal_set(di, lam=0.99):
    A, B, K = di['A'], di['B'], di['K']
    LAM, PSI = di['LAMBDA'], di['PSI']
    F_x, h_x, F_u, h_u = di['F_x'], di['h_x'], di['F_u'], di['h_u']
    n, m = B.shape
    L = PSI - K @ LAM
    F_w = np.block([[F_x, np.zeros((F_x.shape[0], m))],
                    [np.zeros((F_x.shape[0], n)), F_x @ LAM],
                    [F_u @ K, F_u @ L],
                    [np.zeros((F_u.shape[0], n)), F_u @ PSI]])
    h_w = np.concatenate([h_x, lam * h_x, h_u, lam * h_u])  # LAMBDA_0 = PSI_0 = 0 (d_0 = 0)
    Ak = np.block([[A + B @ K, B @ L], [np.zeros((m, n)), np.eye(m)]])
    F, h, _ = compute_mpis(F_w, h_w, Ak)
    return F, h
