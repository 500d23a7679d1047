"""Learning-based MPC shims (forms F3/F4): the host-side mirror of the reference's LBMPC solve
calls, mapped onto bqp_lbmpc_solve_batched (Gauss-Newton SQP on the GPU) and the batched
Nadaraya-Watson oracle (bqp_nw_oracle).

* ``nw_oracle``   ``functions/oracleL2NW.m``: g(xi) and dg/dxi for a batch of query points.
* ``LBMPC``       ``functions/ocpLBMPC.m:27-31``: fmincon over ``var = [c_0..c_{N-1}; theta]``
                  with ``costLBMPC.m`` (learned rollout u = K x + c, running cost for k < N-1,
                  terminal on the learned x_N) and ``constraintsLBMPC.m`` (nominal model; at
                  k = 1 the tightened set F_x_d and the robust terminal set on [x_1; theta]).
* ``HybridLBMPC`` ``examples/hybrid_LBMPC_casadi.m:250-311``: IPOPT over
                  ``y = [x_0..x_N; u_0..u_{N-1}; theta]`` with the learned rollout in the
                  running cost (delta-weighted) and the nominal decision x_N in the terminal cost.
* ``DMSLBMPC``    ``examples/DMS_LBMPC_casadi.m:121-129, 223-292``: IPOPT over
                  ``y = [xl_0..xl_N; x_0..x_N; u; theta]`` - the cost reads the LEARNED states
                  xl (running and terminal), the learned dynamics tie xl to u, the nominal x
                  carries the constraints; the 8 x q window with the validity row of
                  casadiL2NW.m.  Closed loop: ``bqp.closed_loop_sqp``.

This module only marshals data: the nominal-model constraints are condensed once per problem
(A_in is shared; b_in is affine in the measured state), everything iterative runs on the GPU.
"""
import ctypes as C

import numpy as np

from . import _lib
from .ocp import OcpResult, _default_handle


def _window(data):
    """7 x q NW window (rows X = [dx1; dx2; du], Y = 4 rows) -> (q, 7) C-order (= 7 x q
    column-major).  Accepts the 7-row matrix of hybrid_LBMPC_casadi.m or the struct form
    {X: 3 x q, Y: 4 x q} of oracleL2NW.m / update_data.m; an 8-row matrix is the window of
    DMS_LBMPC_casadi.m with casadiL2NW.m's validity row -> (q, 8).  Returns the array and the
    per-instance stride (0 = shared)."""
    if isinstance(data, dict):
        data = np.vstack([np.atleast_2d(data['X']), np.atleast_2d(data['Y'])])
    d = np.asarray(data, float)
    if d.shape[-2] not in (7, 8):
        raise ValueError('the NW window has 7 rows [X; Y] or 8 rows [X; Y; v], not %d' % d.shape[-2])
    if d.ndim == 2:
        return np.ascontiguousarray(d.T), 0
    return np.ascontiguousarray(np.swapaxes(d, 1, 2)), d.shape[1] * d.shape[2]


def nw_oracle(data, xi, handle=None, bandwidth=0.5, lam=1e-3):
    """g (b, 4), dg (b, 4, 3) of oracleL2NW at query points xi (b, 3) = [x1; x2; u]."""
    lib = _lib.load()
    h = handle or _default_handle()
    xi = np.ascontiguousarray(np.atleast_2d(xi), dtype=np.float64)
    b = xi.shape[0]
    w, sd = _window(data)
    q = w.shape[-2]
    g = np.zeros((b, 4)); dg = np.zeros((b, 4, 3))
    rc = lib.bqp_nw_oracle(h.value, b, q, _lib.ptr(w), sd, _lib.ptr(xi), _lib.ptr(g),
                           _lib.ptr(dg), bandwidth, lam)
    _lib.check(rc, 'bqp_nw_oracle')
    return g, dg


def _upper_factor(M):
    """U upper-triangular with U'U = M (row-major)."""
    M = np.atleast_2d(np.asarray(M, float))
    return np.ascontiguousarray(np.linalg.cholesky(M).T)


class _LearnedOCP:
    """Common condensing of the nominal-model constraints and the solve call."""

    def __init__(self, A, B, K, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_T, h_T, F_x_d,
                 h_x_d, N, w_run, n_run, term_learned, n_box, xs=None, bandwidth=0.5, lam=1e-3):
        self.A = np.asarray(A, float)
        n = self.A.shape[0]
        self.B = np.asarray(B, float).reshape(n, -1)
        m = self.B.shape[1]
        self.K = np.asarray(K, float).reshape(m, n)
        self.LAMBDA = np.asarray(LAMBDA, float).reshape(n, -1)
        p = self.LAMBDA.shape[1]
        self.PSI = np.asarray(PSI, float).reshape(m, p)
        Tm = np.asarray(T, float) * np.eye(n) if np.ndim(T) == 0 else np.asarray(T, float)
        self.Lq = _upper_factor(w_run * np.atleast_2d(Q))
        self.Lr = _upper_factor(w_run * np.atleast_2d(R))
        self.Lp = _upper_factor(P)
        self.Lt = _upper_factor(Tm)
        self.xs = np.zeros(n) if xs is None else np.asarray(xs, float).ravel()
        self.N, self.n, self.m, self.p = N, n, m, p
        self.nz = N * m + p
        self.n_run, self.term_learned = n_run, term_learned
        self.bandwidth, self.lam = bandwidth, lam
        # SQP model: 'exact' adds the second-order term of the learned dynamics whenever the
        # Hessian stays positive definite (bqp_lbmpc_dims.hessian), 'gn' is Gauss-Newton alone
        self.hessian = 'exact'
        # ---- condensed nominal constraints Ain z <= b0 + Bx x0 ---------------------------
        # nominal closed rollout x_{k+1} = A x_k + B (K x_k + v_k): x_k = Mx_k x0 + Sx_k z
        nz = self.nz
        Acl = self.A + self.B @ self.K
        Mx = [np.eye(n)]; Sx = [np.zeros((n, nz))]
        Mu, Su = [], []
        for k in range(N):
            Ev = np.zeros((m, nz)); Ev[:, k * m:(k + 1) * m] = np.eye(m)
            Mu.append(self.K @ Mx[k]); Su.append(self.K @ Sx[k] + Ev)
            Mx.append(Acl @ Mx[k]); Sx.append(self.A @ Sx[k] + self.B @ Su[k])
        Et = np.zeros((p, nz)); Et[:, N * m:] = np.eye(p)
        F_T = np.asarray(F_T, float)
        rows, r0, rx = [], [], []

        def add(F, h, S, M):
            rows.append(F @ S); r0.append(np.asarray(h, float).ravel()); rx.append(-F @ M)
        F_x_d = np.asarray(F_x_d, float)
        add(F_x_d, h_x_d, Sx[1], Mx[1])                            # constraintsLBMPC.m:27
        rows.append(F_T[:, :n] @ Sx[1] + F_T[:, n:] @ Et)           # :29 terminal set on x_1
        r0.append(np.asarray(h_T, float).ravel()); rx.append(-F_T[:, :n] @ Mx[1])
        for k in range(1, n_box + 1):
            add(np.asarray(F_x, float), h_x, Sx[k], Mx[k])        # :35 state rows
            add(np.asarray(F_u, float), h_u, Su[k - 1], Mu[k - 1])  # :38 input rows
        self.Ain = np.vstack(rows)
        self.b0 = np.concatenate(r0)
        self.Bx = np.vstack(rx)
        self.Ain_cm = np.ascontiguousarray(self.Ain.T)             # column-major m x nz

    def _solve(self, x0, data, z0, handle, max_iter, tol, polish=0):
        lib = _lib.load()
        h = handle or _default_handle()
        x0 = np.ascontiguousarray(np.atleast_2d(x0), dtype=np.float64)
        b = x0.shape[0]
        w, sd = _window(data)
        q, mask = w.shape[-2], int(w.shape[-1] == 8)
        bin_ = np.ascontiguousarray(self.b0[None, :] + x0 @ self.Bx.T)
        mrows = self.Ain.shape[0]
        z = np.zeros((b, self.nz)) if z0 is None else \
            np.ascontiguousarray(np.broadcast_to(np.atleast_2d(z0), (b, self.nz)), dtype=np.float64).copy()
        lam = np.zeros((b, mrows)); cost = np.zeros(b)
        flag = np.zeros(b, np.int32); it = np.zeros(b, np.int32)
        keep = [np.ascontiguousarray(a, dtype=np.float64) for a in
                (self.A.T, self.B.T, self.K.T, self.Lq, self.Lr, self.Lp, self.Lt,
                 self.LAMBDA.T, self.PSI.T, self.xs)]
        dims = _lib.LbmpcDims(self.n, self.m, self.p, self.N, self.n_run, int(self.term_learned), q,
                              mrows, mask, int(self.hessian == 'exact'))
        dd = _lib.LbmpcData(*[_lib.ptr(a) for a in keep], _lib.ptr(w), sd, _lib.ptr(x0), self.n,
                            _lib.ptr(self.Ain_cm), _lib.ptr(bin_), mrows, self.bandwidth, self.lam)
        o = _lib.options(max_iter=max_iter, tol_stat=tol, polish=polish)
        rc = lib.bqp_lbmpc_solve_batched(h.value, C.byref(dims), b, C.byref(dd), C.byref(o),
                                         _lib.ptr(z), _lib.ptr(lam), _lib.ptr(cost),
                                         _lib.iptr(flag), _lib.iptr(it))
        _lib.check(rc, 'bqp_lbmpc_solve_batched')
        return OcpResult(z=z, lam=lam, cost=cost, exitflag=flag, iterations=it)


class LBMPC(_LearnedOCP):
    """fmincon LBMPC (ocpLBMPC.m, costLBMPC.m, constraintsLBMPC.m), deviation coordinates."""

    def __init__(self, A, B, Kstabil, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N,
                 F_x_d, h_x_d, N, xs=None, bandwidth=0.5, lam=1e-3):
        super().__init__(A, B, Kstabil, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N,
                         F_x_d, h_x_d, N, w_run=1.0, n_run=max(N - 2, 0), term_learned=True,
                         n_box=N - 1, xs=xs, bandwidth=bandwidth, lam=lam)

    def solve(self, dx, data, opt_var0=None, handle=None, max_iter=50, tol=1e-8, polish=0):
        """dx (batch, n) states w.r.t. the working point, data the NW window (7 x q, or batch
        x 7 x q, or {X, Y}), opt_var0 the warm start (ocpLBMPC.m:31 passes the previous
        opt_var).  polish: the QP sub-problems' active-set polish (bqp_options.polish: 0/1/2
        after 0 / -8 sub-problem exits, every sub-problem once the SQP stalls; 3 only once it
        stalls; -1 off).  Returns opt_var (batch, N*m + m) = [c; theta], c0, du0 = K dx + c0."""
        r = self._solve(dx, data, opt_var0, handle, max_iter, tol, polish)
        dx = np.atleast_2d(dx)
        c0 = r.z[:, :self.m]
        r.update(opt_var=r.z, c0=c0, theta=r.z[:, self.N * self.m:],
                 du0=dx @ self.K.T + c0)
        return r


class HybridLBMPC(_LearnedOCP):
    """CasADi hybrid LBMPC (hybrid_LBMPC_casadi.m:250-311), absolute coordinates handled by the
    shift x~ = x - x_eq, u~ = u - u_eq."""

    def __init__(self, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d,
                 h_x_d, x_eq, u_eq, N, delta=0.01, bandwidth=0.5, lam=1e-3):
        Bm = np.asarray(B, float).reshape(np.shape(A)[0], -1)
        super().__init__(A, Bm, np.zeros((Bm.shape[1], Bm.shape[0])), Q, R, P, T, LAMBDA, PSI,
                         F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d, h_x_d, N, w_run=delta, n_run=N,
                         term_learned=False, n_box=N, bandwidth=bandwidth, lam=lam)
        self.x_eq = np.asarray(x_eq, float).ravel()
        self.u_eq = np.atleast_1d(np.asarray(u_eq, float)).ravel()

    def solve(self, xmeasure, data, y0=None, handle=None, max_iter=50, tol=1e-8, polish=0):
        """xmeasure (batch, n) absolute states, data the 7 x q window (or 8 x q with the validity
        row).  Returns y_OL (batch, (N+1)n + Nm + p) in the reference's layout (nominal state
        trajectory, inputs, theta) and u0."""
        xm = np.atleast_2d(xmeasure)
        x0 = xm - self.x_eq
        N, n, m = self.N, self.n, self.m
        z0 = None
        if y0 is not None:
            y0 = np.atleast_2d(y0)
            z0 = np.concatenate([y0[:, (N + 1) * n:(N + 1) * n + N * m] - np.tile(self.u_eq, N),
                                 y0[:, -self.p:]], axis=1)
        r = self._solve(x0, data, z0, handle, max_iter, tol, polish)
        b = xm.shape[0]
        u = r.z[:, :N * m].reshape(b, N, m)
        X = np.zeros((b, N + 1, n)); X[:, 0] = x0
        for k in range(N):
            X[:, k + 1] = X[:, k] @ self.A.T + u[:, k] @ self.B.T
        y = np.concatenate([(X + self.x_eq).reshape(b, -1), (u + self.u_eq).reshape(b, -1),
                            r.z[:, N * m:]], axis=1)
        r.update(y_OL=y, u0=u[:, 0, :] + self.u_eq, theta=r.z[:, N * m:])
        return r


class DMSLBMPC(HybridLBMPC):
    """CasADi DMS LBMPC (DMS_LBMPC_casadi.m:121-129): the running cost (delta-weighted, stages
    k = 0..N-1, :229-233) and the terminal cost (:234, terminalcosts :245-247) on the LEARNED
    states xl, which the learned dynamics xl_{k+1} = x_eq + A dxl + B du + casadiL2NW(dxl, du,
    data) tie to the inputs (:268); the nominal states x carry the constraints (:262-276): at
    k = 1 F_x_d and the robust terminal set on [x_1; theta], boxes on x_1..x_N and u_0..u_{N-1}.
    Eliminating both state chains leaves z = [u - u_eq; theta] with the learned rollout in the
    whole cost: the GN-SQP of HybridLBMPC with the terminal term on the learned x_N.  The window
    is the 8 x q matrix [X; Y; v] (get_data.m; v = 1 on the valid points)."""

    def __init__(self, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d,
                 h_x_d, x_eq, u_eq, N, delta=0.01, bandwidth=0.5, lam=1e-3):
        super().__init__(A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d,
                         h_x_d, x_eq, u_eq, N, delta=delta, bandwidth=bandwidth, lam=lam)
        self.term_learned = True

    def solve(self, xmeasure, data, y0=None, handle=None, max_iter=200, tol=1e-8, polish=0):
        """as HybridLBMPC.solve, data the 8 x q window [X; Y; v] (or 7 x q: every point valid);
        with hessian = 'gn' the iteration converges linearly on these learned costs (about 60 SQP
        iterations on the second step of the stored DMS_tLBMPC_q100 run, 5 with the exact
        Hessian), hence the larger default max_iter"""
        return super().solve(xmeasure, data, y0=y0, handle=handle, max_iter=max_iter, tol=tol,
                             polish=polish)
