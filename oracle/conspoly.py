"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the LBMPC constraint-set construction:

* ``pdiff`` - ``utilities/pdiff.m:10-17`` (Kolmanovsky-Gilbert): Pontryagin difference of
  {F_u x <= h_u} and {F_v x <= h_v}: h_i -= max_{F_v x <= h_v} F_u(i,:) x (one LP per row, scipy
  HiGHS in place of MATLAB linprog).
* ``get_conspoly`` - ``functions/getCONSPOLY.m:17-69``: box constraints shifted to the working
  point, the tightened state set X - D (MPT3 ``minus`` + ``minHRep``), the terminal feedback
  K_t = -dlqr(A, B, Q, 10 R), the extended-state constraint polytope F_w/h_w (lambda = 0.99) and
  its Pontryagin difference with the disturbance set [D; theta = 0], reduced by an LP redundancy
  test (``mpis.min_hrep``, in place of MPT3 ``minHRep``).

Pinned (tests/test_conspoly.py) to the sets of the R2019a workspace dump examples/DSS_NMPC.m
(tests/golden/lbmpc_instance.npz: F_x_d 8x4, F_w_N 16x5) up to row order, which MPT3 does not
define.
"""
import numpy as np
import scipy.linalg as sla
from scipy.optimize import linprog

from .mpis import min_hrep


def pdiff(F_u, h_u, F_v, h_v):
    h = np.zeros(len(h_u))
    for i in range(len(h_u)):
        res = linprog(-F_u[i], A_ub=F_v, b_ub=h_v, bounds=[(None, None)] * F_v.shape[1],
                      method='highs')
        if res.status != 0:
            raise RuntimeError('pdiff: LP for row %d failed (%s)' % (i, res.message))
        h[i] = -res.fun
    return F_u.copy(), h_u - h


def dlqr_gain(A, B, Q, R):
    X = sla.solve_discrete_are(A, B, Q, R)
    return np.linalg.solve(R + B.T @ X @ B, B.T @ X @ A)


def get_conspoly(A, B, Q, R, LAMBDA, PSI, xmax, xmin, umax, umin, state_uncert, x_wp, u_wp,
                 lam=0.99):
    n, m = B.shape
    LAMBDA = LAMBDA.reshape(n, -1); PSI = PSI.reshape(m, -1)
    LAMBDA_0 = np.zeros((n, 1)); PSI_0 = np.zeros((m, 1))      # matOCP.m:21-24, d_0 = 0
    F_u = np.vstack([np.eye(m), -np.eye(m)]); h_u = np.concatenate([umax - u_wp, -umin + u_wp])
    F_x = np.vstack([np.eye(n), -np.eye(n)]); h_x = np.concatenate([xmax - x_wp, -xmin + x_wp])
    F_d = np.vstack([np.eye(n), -np.eye(n)]); h_d = np.concatenate([state_uncert, state_uncert])
    F_x_d, h_x_d = pdiff(F_x, h_x, F_d, h_d)                   # getCONSPOLY.m:28-30
    F_x_d, h_x_d = min_hrep(F_x_d, h_x_d)
    K_t = -dlqr_gain(A, B, Q, 10.0 * R)                          # :38-39
    L = PSI - K_t @ LAMBDA
    L0 = PSI_0 - K_t @ LAMBDA_0
    nx_d = F_x_d.shape[0]
    F_w = np.block([[F_x, np.zeros((2 * n, m))],                 # :46-55
                    [np.zeros((2 * n, n)), F_x @ LAMBDA],
                    [F_u @ K_t, F_u @ L],
                    [np.zeros((2 * m, n)), F_u @ PSI],
                    [F_x_d @ (A + B @ K_t), F_x_d @ B @ L]])
    h_w = np.concatenate([h_x, lam * (h_x - (F_x @ LAMBDA_0).ravel()),
                          h_u - (F_u @ L0).ravel(), lam * (h_u - (F_u @ PSI_0).ravel()),
                          h_x_d - (F_x_d @ B @ (PSI_0 - K_t @ LAMBDA_0)).ravel()])
    F_d_w = np.block([[F_d, np.zeros((2 * n, m))],               # :58-62
                      [np.zeros((m, n)), np.eye(m)],
                      [np.zeros((m, n)), -np.eye(m)]])
    h_d_w = np.concatenate([h_d, np.zeros(2 * m)])
    F_w_N0, h_w_N0 = pdiff(F_w, h_w, F_d_w, h_d_w)               # :65
    F_w_N, h_w_N = min_hrep(F_w_N0, h_w_N0)                      # :67-69
    return dict(F_x=F_x, h_x=h_x, F_u=F_u, h_u=h_u, F_w_N=F_w_N, h_w_N=h_w_N, F_x_d=F_x_d,
                h_x_d=h_x_d, K_t=K_t)


def mg_conspoly(mg):
    """getCONSPOLY with the Moore-Greitzer data of LBMPC_RunExample.m:24-56."""
    xmax = np.array([1.0, 2.1875, 2.1547, 20.0]); xmin = np.array([0.0, 1.1875, 0.1547, -20.0])
    umax = np.array([2.1547]); umin = np.array([0.1547])
    state_uncert = np.array([0.02, 5e-4, 0.0, 0.0])
    return get_conspoly(mg['A'], mg['B'].reshape(4, 1), mg['Q'], np.atleast_2d(mg['R']),
                        mg['LAMBDA'], mg['PSI'], xmax, xmin, umax, umin, state_uncert,
                        mg['x_wp'], np.atleast_1d(mg['u_wp']))
