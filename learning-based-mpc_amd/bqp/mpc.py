"""Reference-facing MPC problem shims: the host-side mirror of the reference's per-step OCP
interfaces, mapped onto the structured solver (bqp_solve_ocp_batched).

Each class takes the same design data the reference passes to its solve call and returns what
the reference reads back from it:

* ``LMPC``        ``ocpLMPC.m:20-27``: fmincon over ``var = [c_0..c_{N-1}; theta]`` with
                  ``costLMPC.m`` / ``constraintsLMPC.m``  ->  ``opt_var`` (c, theta), art_ref.
* ``TrackingLMPC`` ``DMS_tracking_LMPC_casadi.m:122-172``: IPOPT over
                  ``y = [x_0..x_N; u_0..u_{N-1}; theta]``  ->  ``y_OL``.
* ``TrackingMPC`` ``trackingMPC/RunExample.m:134-139``: fmincon over ``[u_0..u_{N-1}; theta]``
                  with ``costFunction.m`` / ``constraintsFunction.m``.

The change of variables used (u_k = K x_k + c_k for F1, deviation coordinates for F2) is a
bijection, so the optimum is exactly the reference problem's optimum (tests compare against
the oracle's dense restatement of the reference loops).
"""
import numpy as np

from .ocp import OcpProblem, solve_ocp


def _split_box(F, h, n):
    """[I; -I] x <= h  ->  (lb, ub) (getCONS.m:15-16 layout)."""
    F = np.asarray(F, float)
    h = np.asarray(h, float).ravel()
    ub = np.full(n, np.inf)
    lb = np.full(n, -np.inf)
    for r in range(F.shape[0]):
        nz = np.flatnonzero(np.abs(F[r]) > 0)
        if nz.size != 1:
            raise ValueError('box constraint rows must have one non-zero')
        j = nz[0]
        if F[r, j] > 0:
            ub[j] = min(ub[j], h[r] / F[r, j])
        else:
            lb[j] = max(lb[j], h[r] / F[r, j])
    return lb, ub


def _tracking_blocks(n, m, p, LAMBDA, PSI):
    Ex = np.hstack([np.eye(n), np.zeros((n, m)), -LAMBDA])     # x - LAMBDA th
    Eu = np.hstack([np.zeros((m, n)), np.eye(m), -PSI])        # u - PSI th
    Eth = np.hstack([np.zeros((n, n + m)), LAMBDA])            # LAMBDA th
    return Ex, Eu, Eth


def _poly(F_T, n, m, p):
    F_T = np.asarray(F_T, float)
    Fp = np.zeros((F_T.shape[0], n + m + p))
    Fp[:, :n] = F_T[:, :n]
    Fp[:, n + m:] = F_T[:, n:n + p]
    return Fp


class LMPC:
    """fmincon LMPC (functions/ocpLMPC.m, costLMPC.m, constraintsLMPC.m), deviation coordinates.

    Reproduces the reference's quirks: running cost only for prediction steps k < N-1
    (costLMPC.m:30), terminal set imposed on [x_{N-1}; theta] (constraintsLMPC.m:37)."""

    def __init__(self, A, B, Kstabil, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N,
                 N, xs=None):
        A = np.asarray(A, float); B = np.asarray(B, float).reshape(A.shape[0], -1)
        n, m = B.shape
        LAMBDA = np.asarray(LAMBDA, float).reshape(n, -1)
        p = LAMBDA.shape[1]
        PSI = np.asarray(PSI, float).reshape(m, p)
        self.K = np.asarray(Kstabil, float).reshape(m, n)
        Tm = np.asarray(T, float) * np.eye(n) if np.ndim(T) == 0 else np.asarray(T, float)
        Q = np.atleast_2d(Q); R = np.atleast_2d(R); P = np.atleast_2d(P)
        xs = np.zeros(n) if xs is None else np.asarray(xs, float)
        nv = n + m + p
        Ex, Eu, Eth = _tracking_blocks(n, m, p, LAMBDA, PSI)
        W = np.zeros((N + 1, nv, nv)); w = np.zeros((N + 1, nv))
        for k in range(N):
            if k + 1 < N - 1:                                   # costLMPC.m:30 (k is 1-based)
                W[k] = 2 * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)
        W[N] = 2 * (Ex.T @ P @ Ex + Eth.T @ Tm @ Eth)           # costLMPC.m:37-38
        w[N] = -2 * Eth.T @ Tm @ xs
        xlb, xub = _split_box(F_x, h_x, n)
        ulb, uub = _split_box(F_u, h_u, m)
        XL = np.full((N + 1, n), -np.inf); XU = np.full((N + 1, n), np.inf)
        UL = np.full((N, m), -np.inf); UU = np.full((N, m), np.inf)
        XL[1:N], XU[1:N] = xlb, xub                             # x_1..x_{N-1}
        UL[:N - 1], UU[:N - 1] = ulb, uub                       # u_0..u_{N-2}
        self.prob = OcpProblem(A, B, W, N, p, w=w, xlb=XL, xub=XU, ulb=UL, uub=UU,
                               Fp=_poly(F_w_N, n, m, p), hp=h_w_N, poly_stage=N - 1,
                               const=float(xs @ Tm @ xs))
        self.N, self.n, self.m, self.p = N, n, m, p
        self.LAMBDA, self.PSI = LAMBDA, PSI

    def solve(self, dx, **kw):
        """dx: (batch, n) states w.r.t. the working point.  Returns dict with
        opt_var (batch, N*m + p) = [c_0..c_{N-1}; theta] (ocpLMPC.m:24 layout), c0, theta,
        du0 = K dx + c_0 (the applied move w.r.t. u_wp, transitionTrue.m:11) and the solver
        status."""
        r = solve_ocp(self.prob, dx, **kw)
        N, m = self.N, self.m
        c = r.u - np.einsum('ij,bkj->bki', self.K, r.x[:, :N, :])
        opt_var = np.concatenate([c.reshape(c.shape[0], N * m), r.theta], axis=1)
        r.update(opt_var=opt_var, c0=c[:, 0, :], du0=r.u[:, 0, :])
        return r


class TrackingLMPC:
    """CasADi DMS tracking LMPC (examples/DMS_tracking_LMPC_casadi.m:223-291), absolute
    coordinates handled by the shift x~ = x - x_eq, u~ = u - u_eq."""

    def __init__(self, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, x_eq,
                 u_eq, N, delta=0.01):
        A = np.asarray(A, float); B = np.asarray(B, float).reshape(A.shape[0], -1)
        n, m = B.shape
        LAMBDA = np.asarray(LAMBDA, float).reshape(n, -1)
        p = LAMBDA.shape[1]
        PSI = np.asarray(PSI, float).reshape(m, p)
        Tm = np.asarray(T, float) * np.eye(n) if np.ndim(T) == 0 else np.asarray(T, float)
        Q = np.atleast_2d(Q); R = np.atleast_2d(R); P = np.atleast_2d(P)
        nv = n + m + p
        Ex, Eu, Eth = _tracking_blocks(n, m, p, LAMBDA, PSI)
        W = np.zeros((N + 1, nv, nv))
        for k in range(N):
            W[k] = 2 * delta * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)  # runningcosts :242-246
        W[N] = 2 * (Ex.T @ P @ Ex + Eth.T @ Tm @ Eth)           # terminalcosts :248-251
        xlb, xub = _split_box(F_x, h_x, n)
        ulb, uub = _split_box(F_u, h_u, m)
        XL = np.full((N + 1, n), -np.inf); XU = np.full((N + 1, n), np.inf)
        XL[1:], XU[1:] = xlb, xub                               # F_x (x_{k+1} - x_eq) <= h_x
        UL = np.tile(ulb, (N, 1)); UU = np.tile(uub, (N, 1))
        self.prob = OcpProblem(A, B, W, N, p, xlb=XL, xub=XU, ulb=UL, uub=UU,
                               Fp=_poly(F_w_N, n, m, p), hp=h_w_N, poly_stage=N)
        self.x_eq = np.asarray(x_eq, float).ravel()
        self.u_eq = np.atleast_1d(np.asarray(u_eq, float)).ravel()
        self.N, self.n, self.m, self.p = N, n, m, p

    def solve(self, xmeasure, **kw):
        """xmeasure: (batch, n) absolute states.  Returns y_OL (batch, (N+1)n + Nm + p) in the
        reference's layout (:168-171), u0 (applied input) and status."""
        xm = np.atleast_2d(xmeasure)
        r = solve_ocp(self.prob, xm - self.x_eq, **kw)
        b = xm.shape[0]
        X = r.x + self.x_eq
        U = r.u + self.u_eq
        y = np.concatenate([X.reshape(b, -1), U.reshape(b, -1), r.theta], axis=1)
        r.update(y_OL=y, u0=U[:, 0, :])
        return r


class TrackingLBMPC(TrackingLMPC):
    """CasADi LBMPC (examples/LBMPC_casadi.m:240-304; the nominal part of DMS_LBMPC_casadi.m):
    the DMS tracking cost of TrackingLMPC (delta-weighted running cost, terminal P and T) with
    the LBMPC constraint sets of getCONSPOLY.m - boxes F_x on x_1..x_N and F_u on every input,
    and at k = 1 the tightened state set F_x_d x_1 <= h_x_d and the robust terminal set
    F_w_N [x_1; theta] <= h_w_N (:285-289) - on the nominal model (the learned dynamics are
    commented out of the constraints there, :292).  The polytope block is [F_x_d; F_w_N] at
    stage 1.  closed_loop(..., learning=dict(q=100)) adds the script's data window
    (update_data.m)."""

    def __init__(self, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d,
                 h_x_d, x_eq, u_eq, N, delta=0.01):
        super().__init__(A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, x_eq,
                         u_eq, N, delta)
        pr = self.prob
        n, m, p = self.n, self.m, self.p
        Fd = np.zeros((np.shape(F_x_d)[0], n + m + p))
        Fd[:, :n] = np.asarray(F_x_d, float)
        Fp = np.vstack([Fd, _poly(F_w_N, n, m, p)])
        hp = np.concatenate([np.asarray(h_x_d, float).ravel(), np.asarray(h_w_N, float).ravel()])
        self.prob = OcpProblem(pr.A, pr.B, pr.W, N, p, xlb=pr.xlb, xub=pr.xub, ulb=pr.ulb,
                               uub=pr.uub, Fp=Fp, hp=hp, poly_stage=1)


class TrackingMPC:
    """trackingMPC/RunExample.m (double integrator): costFunction.m + constraintsFunction.m.
    The constant rows on x_0 (constraintsFunction.m:291, k=1) do not involve the decision and
    are checked on the host: an x0 outside them makes the reference problem infeasible
    (exitflag -2)."""

    def __init__(self, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, N):
        A = np.asarray(A, float); B = np.asarray(B, float)
        n, m = B.shape
        LAMBDA = np.asarray(LAMBDA, float).reshape(n, -1)
        p = LAMBDA.shape[1]
        PSI = np.asarray(PSI, float).reshape(m, p)
        T = np.asarray(T, float); P = np.asarray(P, float)
        Q = np.atleast_2d(Q); R = np.atleast_2d(R)
        nv = n + m + p
        Ex, Eu, Eth = _tracking_blocks(n, m, p, LAMBDA, PSI)
        W = np.zeros((N + 1, nv, nv))
        for k in range(N - 1):
            W[k] = 2 * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)          # costFunction.m:247-258
        W[N - 1] = 2 * (Ex.T @ P @ Ex)                          # :260 terminal on x_{N-1}
        W[N] = 2 * (Eth.T @ T @ Eth)                            # :261 (LAMBDA th - xs)'T(.)
        self.T, self.Eth = T, Eth
        xlb, xub = _split_box(F_x, h_x, n)
        ulb, uub = _split_box(F_u, h_u, m)
        XL = np.full((N + 1, n), -np.inf); XU = np.full((N + 1, n), np.inf)
        XL[1:N], XU[1:N] = xlb, xub                             # x_1..x_{N-1}
        UL = np.tile(ulb, (N, 1)); UU = np.tile(uub, (N, 1))
        self.xlb0, self.xub0 = xlb, xub
        self.prob = OcpProblem(A, B, W, N, p, xlb=XL, xub=XU, ulb=UL, uub=UU,
                               Fp=_poly(F_w_N, n, m, p), hp=h_w_N, poly_stage=N)
        self.N, self.n, self.m, self.p = N, n, m, p

    def linear_terms(self, xs):
        xs = np.atleast_2d(xs)
        w = np.zeros((xs.shape[0], self.N + 1, self.n + self.m + self.p))
        w[:, self.N, :] = -2 * (self.Eth.T @ self.T @ xs.T).T
        const = np.einsum('bi,ij,bj->b', xs, self.T, xs)
        return w, const

    def solve(self, x, xs, **kw):
        """x: (batch, n) states, xs: (batch, n) references.  Returns opt_var (batch, N*m + p)
        = [u_0..u_{N-1}; theta] (RunExample.m:136 layout), u0 and status."""
        x = np.atleast_2d(x)
        xs = np.broadcast_to(np.atleast_2d(xs), x.shape)
        w, const = self.linear_terms(xs)
        r = solve_ocp(self.prob, x, w=w, **kw)
        b = x.shape[0]
        r['fval'] = r.fval + const
        bad = np.any((x > self.xub0 + 1e-12) | (x < self.xlb0 - 1e-12), axis=1)
        r.exitflag[bad] = -2
        opt_var = np.concatenate([r.u.reshape(b, -1), r.theta], axis=1)
        r.update(opt_var=opt_var, u0=r.u[:, 0, :])
        return r
