"""Maps the structured solver's multipliers onto the rows of the reference's own QP forms (as
restated by oracle/qp_forms.py), so duals can be compared with the dense ground truth lambda*
and the KKT conditions checked in the reference's variable layout.

Structured duals (bqp.solve_ocp(..., want_duals=True)): lam_x (b, N+1, 2, nx) [lower, upper],
lam_u (b, N, 2, nu), lam_p (b, mp), pi (b, N, nx) with pi[:, k-1] the multiplier of
x_k = A x_{k-1} + B u_{k-1} + c (Lagrangian + pi'(A x + B u + c - x_next)).
"""
import numpy as np


def f1_ineqlin(N, lam_x, lam_u, lam_p):
    """constraintsLMPC.m row order: for k = 1..N-1: F_x x_k (upper nx, lower nx), F_u u_{k-1}
    (upper nu, lower nu); then the terminal set (on x_{N-1})."""
    rows = []
    for k in range(1, N):
        rows += [lam_x[k, 1], lam_x[k, 0], lam_u[k - 1, 1], lam_u[k - 1, 0]]
    rows.append(lam_p)
    return np.concatenate(rows)


def f2_duals(N, lam_x, lam_u, lam_p, pi):
    """DMS_tracking_LMPC_casadi.m:254-287 row order: for k = 0..N-1: F_x (x_{k+1} - x_eq)
    (upper, lower), F_u (u_k - u_eq) (upper, lower); then the terminal set.  Equality rows
    x_{k+1} - A x_k - B u_k = 0 carry y_k = -pi_{k+1}."""
    rows = []
    for k in range(N):
        rows += [lam_x[k + 1, 1], lam_x[k + 1, 0], lam_u[k, 1], lam_u[k, 0]]
    rows.append(lam_p)
    return np.concatenate(rows), -pi.reshape(-1)


def from_statement(r, N, nx, nu):
    """The numpy algorithm statement's (oracle/ocp_ipm.py) multipliers in the API layout."""
    lam = r['lam']
    lam_x = np.stack([lam['xl'], lam['xu']], axis=1)
    lam_u = np.stack([lam['ul'], lam['uu']], axis=1)
    # absent bounds carry no multiplier
    return lam_x, lam_u, lam['p'], r['pi'][1:, :nx]


def f1_kkt(qp, z, lam):
    """stationarity, complementarity, min multiplier, max violation of the dense F1 QP."""
    H, f, A, b = qp['H'], qp['f'], qp['A'], qp['b']
    g = H @ z + f + A.T @ lam
    sl = b - A @ z
    return (np.abs(g).max() / (1 + np.abs(H @ z + f).max()), np.abs(lam * sl).max(), lam.min(),
            -sl.min())


def f2_kkt(qp, z, lin, y, n):
    """as f1_kkt for the dense F2 QP; the x_0 entries (fixed by lb == ub) are left out of the
    stationarity test (their multipliers are the fixed-variable ones)."""
    H, f, A, b, E = qp['H'], qp['f'], qp['A'], qp['b'], qp['Aeq']
    g = H @ z + f + A.T @ lin + E.T @ y
    sl = b - A @ z
    return (np.abs(g[n:]).max() / (1 + np.abs(H @ z + f).max()), np.abs(lin * sl).max(),
            lin.min(), -sl.min())


def licq(A, lam_a, lam_b, thr=1e-9):
    """True when the rows active in either multiplier vector are linearly independent (the
    multipliers are then unique, so two solvers' lambda must agree)."""
    act = np.union1d(np.flatnonzero(lam_a > thr), np.flatnonzero(lam_b > thr))
    return act.size == 0 or np.linalg.matrix_rank(A[act]) == act.size
