"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the reference's offline model/controller design:

* ``mgcm_dlti``  — ``matlab/LBMPC/functions/mgcmDLTI.m:6-41``: Jacobian linearisation of the
  Moore-Greitzer compressor at x=[0.5 1.6875 1.1547 0] and exact ZOH with Ts=0.01.
* ``mat_ocp``    — ``matlab/LBMPC/functions/matOCP.m:7-31``: K=-place(A,B,p), Mtheta=null(M),
  Q=I, R=I, P=dare(A+BK,B,Q,R), T=1000.
* ``di_model``   — ``matlab/trackingMPC/RunExample.m:20-60``: sampled double integrator,
  K=-dlqr(A,B,I,I), P=dare(A+BK,B,I,I), T=100P.
* ``mg_constraints`` — ``functions/getCONS.m:15-16`` with the bounds of
  ``examples/LMPC_RunExample.m:24-32``.
"""
import numpy as np
import scipy.linalg as sla
import scipy.signal as ssig

# Working point (examples/LMPC_RunExample.m:48-52, DMS_tracking_LMPC_casadi.m:73-74)
X_WP = np.array([0.5, 1.6875, 1.1547, 0.0])
U_WP = 1.1547
TS = 0.01


def mgcm_dlti():
    """functions/mgcmDLTI.m:12-41 — returns (Ad, Bd, Ts)."""
    wn = np.sqrt(1000.0)
    zeta = 1.0 / np.sqrt(2.0)
    x1, x2, x3 = 0.5, 1.6875, 1.1547
    # jacobian([f1,f2,f3,f4],[x1..x4]) evaluated at the equilibrium (mgcmDLTI.m:18-31)
    A = np.array([
        [1.5 - 1.5 * x1 ** 2, -1.0, 0.0, 0.0],
        [1.0, -x3 / (2.0 * np.sqrt(x2)), -np.sqrt(x2), 0.0],
        [0.0, 0.0, 0.0, 1.0],
        [0.0, 0.0, -wn ** 2, -2.0 * zeta * wn],
    ])
    B = np.array([[0.0], [0.0], [0.0], [wn ** 2]])
    Ad = sla.expm(A * TS)                                    # mgcmDLTI.m:38
    Bd = (Ad - np.eye(4)) @ np.linalg.inv(A) @ B             # mgcmDLTI.m:39
    return Ad, Bd, TS


def null_space_signed(M):
    """MATLAB ``null`` (orthonormal SVD basis); sign fixed so that the first entry is > 0,
    matching the stored Mtheta (examples/DSS_NMPC.m:88-90)."""
    Z = sla.null_space(M)
    for j in range(Z.shape[1]):
        i = np.flatnonzero(np.abs(Z[:, j]) > 1e-12)[0]
        if Z[i, j] < 0:
            Z[:, j] = -Z[:, j]
    return Z


def mat_ocp(A, B, C=None):
    """functions/matOCP.m:7-31 -> dict(K, Q, R, P, T, Mtheta, LAMBDA, PSI)."""
    n, m = B.shape
    if C is None:
        C = np.eye(n)
    o = C.shape[0]
    p = [0.75, 0.78, 0.98, 0.99]                             # matOCP.m:7
    Kp = ssig.place_poles(A, B, p).gain_matrix               # matOCP.m:8
    K = -Kp                                                  # matOCP.m:9
    M = np.block([[A - np.eye(n), B, np.zeros((n, o))],
                  [C, np.zeros((o, m)), -np.eye(o)]])        # matOCP.m:12-13
    Mtheta = null_space_signed(M)                            # matOCP.m:14
    LAMBDA = Mtheta[:n, :]
    PSI = Mtheta[n:n + m, :]
    Q = np.eye(n)
    R = np.eye(m)
    P = sla.solve_discrete_are(A + B @ K, B, Q, R)           # matOCP.m:30
    return dict(K=K, Q=Q, R=R, P=P, T=1000.0 * np.eye(n), Tscalar=1000.0,
                Mtheta=Mtheta, LAMBDA=LAMBDA, PSI=PSI)


def mg_constraints():
    """getCONS.m:15-16 with LMPC_RunExample.m:24-32 bounds (deviation coordinates)."""
    xmax = np.array([1.0, 2.1875, 2.1547, 20.0])
    xmin = np.array([0.0, 1.1875, 0.1547, -20.0])
    umax, umin = 2.1547, 0.1547
    F_u = np.array([[1.0], [-1.0]])
    h_u = np.array([umax - U_WP, -umin + U_WP])
    F_x = np.vstack([np.eye(4), -np.eye(4)])
    h_x = np.concatenate([xmax - X_WP, -xmin + X_WP])
    return F_x, h_x, F_u, h_u


def mg_problem():
    """Everything a Moore-Greitzer LMPC needs, restated from the reference."""
    A, B, Ts = mgcm_dlti()
    d = mat_ocp(A, B)
    F_x, h_x, F_u, h_u = mg_constraints()
    d.update(A=A, B=B, Ts=Ts, F_x=F_x, h_x=h_x, F_u=F_u, h_u=h_u,
             x_wp=X_WP.copy(), u_wp=U_WP)
    return d


def di_model():
    """trackingMPC/RunExample.m:20-108: double integrator + tracking ingredients."""
    A = np.array([[1.0, 1.0], [0.0, 1.0]])
    B = np.array([[0.0, 0.5], [1.0, 0.5]])
    C = np.array([[1.0, 0.0]])
    n, m, o = 2, 2, 1
    Q = np.eye(n)
    R = np.eye(m)
    M = np.block([[A - np.eye(n), B, np.zeros((n, o))],
                  [C, np.zeros((o, m)), -np.eye(o)]])        # RunExample.m:42-43
    Mtheta = null_space_signed(M)                            # RunExample.m:44
    LAMBDA = Mtheta[:n, :]
    PSI = Mtheta[n:n + m, :]
    # K = -dlqr(A,B,Q,R) (RunExample.m:56)
    X = sla.solve_discrete_are(A, B, Q, R)
    Klqr = np.linalg.solve(R + B.T @ X @ B, B.T @ X @ A)
    K = -Klqr
    P = sla.solve_discrete_are(A + B @ K, B, Q, R)           # RunExample.m:58
    T = 100.0 * P                                            # RunExample.m:60
    u_min = np.array([-0.3, -0.3]); u_max = np.array([0.3, 0.3])
    x_min = np.array([-5.0, -5.0]); x_max = np.array([5.0, 5.0])
    F_u = np.vstack([np.eye(m), -np.eye(m)]); h_u = np.concatenate([u_max, -u_min])
    F_x = np.vstack([np.eye(n), -np.eye(n)]); h_x = np.concatenate([x_max, -x_min])
    return dict(A=A, B=B, C=C, Q=Q, R=R, K=K, P=P, T=T, Mtheta=Mtheta, LAMBDA=LAMBDA,
                PSI=PSI, F_u=F_u, h_u=h_u, F_x=F_x, h_x=h_x)


def mg_rhs(x, u):
    """Continuous MG dynamics, DMS_tracking_LMPC_casadi.m:215-221 (`system`)."""
    return np.array([
        -x[1] + 1 + 3 * (x[0] / 2) - (x[0] ** 3 / 2),
        (x[0] + 1 - x[2] * np.sqrt(x[1])),
        x[3],
        -1000 * x[2] - 2 * np.sqrt(500) * x[3] + 1000 * u,
    ])


def mg_rk4(delta, x, u):
    """RK4 plant step, DMS_tracking_LMPC_casadi.m:297-304 (`dynamic`)."""
    k1 = mg_rhs(x, u)
    k2 = mg_rhs(x + delta / 2 * k1, u)
    k3 = mg_rhs(x + delta / 2 * k2, u)
    k4 = mg_rhs(x + delta * k3, u)
    return x + delta / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


def mg_ode23(delta, x, u, rtol=1e-3, atol=1e-6):
    """True-plant step of the fmincon loops: models/trueModel.m:14/48 (simulate_cont) integrates
    the MG model over [0, delta] with MATLAB's ode23 at its default options.  Restated from the
    published algorithm (Bogacki-Shampine 3(2) pair, FSAL, local extrapolation; the MATLAB ODE
    suite's initial step and step-size control, Shampine & Reichelt 1997): MaxStep 0.1 delta,
    threshold AbsTol/RelTol, error h |f E ./ max(|y|, |ynew|, thr)|_inf, E = [-5/72 1/12 1/9
    -1/8], the last step stretched when within 10 % of the end.  Pinned: it reproduces every
    stored transition of LMPC_N{20,40,50}_sys_full.mat and LBMPC_N{40,50}_sys_full.mat to
    1.4e-15 (tests/test_oracle.py).  Returns x(delta)."""
    f = lambda y: mg_rhs(y, u)                                    # noqa: E731
    t, y = 0.0, np.array(x, float)
    T = float(delta)
    hmax, thr, pw = 0.1 * T, atol / rtol, 1.0 / 3.0
    Bt = np.array([[1 / 2, 0, 2 / 9], [0, 3 / 4, 1 / 3], [0, 0, 4 / 9], [0, 0, 0]])
    E = np.array([-5 / 72, 1 / 12, 1 / 9, -1 / 8])
    F = np.zeros((4, 4))
    F[:, 0] = f(y)
    absh = min(hmax, T)
    rh = np.max(np.abs(F[:, 0] / np.maximum(np.abs(y), thr))) / (0.8 * rtol ** pw)
    if absh * rh > 1:
        absh = 1 / rh
    done = False
    while not done:
        hmin = 16 * np.spacing(t)
        absh = min(hmax, max(hmin, absh))
        h = absh
        if 1.1 * absh >= abs(T - t):
            h = T - t
            absh = abs(h)
            done = True
        nofailed = True
        while True:
            hB = h * Bt
            F[:, 1] = f(y + F @ hB[:, 0])
            F[:, 2] = f(y + F @ hB[:, 1])
            tnew = T if done else t + h
            h = tnew - t
            ynew = y + F @ (h * Bt[:, 2])
            F[:, 3] = f(ynew)
            err = absh * np.max(np.abs((F @ E) / np.maximum(np.maximum(np.abs(y), np.abs(ynew)), thr)))
            if not err > rtol:
                break
            if absh <= hmin:
                break                                             # MATLAB warns and returns
            absh = max(hmin, absh * max(0.5, 0.8 * (rtol / err) ** pw)) if nofailed \
                else max(hmin, 0.5 * absh)
            nofailed = False
            h = absh
            done = False
        if not done and nofailed:
            temp = 1.25 * (err / rtol) ** pw
            absh = absh / temp if temp > 0.2 else 5.0 * absh
        t, y = tnew, ynew
        F[:, 0] = F[:, 3]
    return y
