"""Per-model tracking-MPC ingredients (trackingMPC/RunExample.m:42-60): the steady-state
parametrisation M_theta = null([A - I, B, 0; C, 0, -I]) (LAMBDA, PSI), the LQR gain
K = -dlqr(A, B, Q, R), the terminal weight P (DARE of the closed loop) and T = 100 P.  Host-side and
offline (scipy), for batches of perturbed / learned models whose costs (bqp_ocp_data.sW != 0) and
terminal sets (bqp.sets) are then built per model; the solve runs on the GPU.
"""
import numpy as np
import scipy.linalg as sla


def tracking_design(A, B, C, Q, R, t_factor=100.0):
    A = np.asarray(A, float); B = np.asarray(B, float); C = np.atleast_2d(np.asarray(C, float))
    n, m = B.shape
    o = C.shape[0]
    M = np.block([[A - np.eye(n), B, np.zeros((n, o))],
                  [C, np.zeros((o, m)), -np.eye(o)]])
    Mth = sla.null_space(M)
    # the sign of each basis vector is fixed by its first non-negligible entry (positive), so that
    # a model and its slight perturbation get the same orientation of theta
    for j in range(Mth.shape[1]):
        nz = np.flatnonzero(np.abs(Mth[:, j]) > 1e-12)
        if nz.size and Mth[nz[0], j] < 0:
            Mth[:, j] = -Mth[:, j]
    X = sla.solve_discrete_are(A, B, Q, R)
    K = -np.linalg.solve(R + B.T @ X @ B, B.T @ X @ A)
    P = sla.solve_discrete_are(A + B @ K, B, Q, R)
    return dict(K=K, P=P, T=t_factor * P, LAMBDA=Mth[:n], PSI=Mth[n:n + m], Mtheta=Mth)
