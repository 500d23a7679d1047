"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the reference's per-step OCPs as quadprog-form QPs

    min 0.5 z'Hz + f'z   s.t.  A z <= b,  Aeq z = beq,  lb <= z <= ub

in the reference's OWN variable layout, built by replaying the reference's loops on affine
expressions (so every off-by-one quirk of the MATLAB code is reproduced literally):

* F1 ``lmpc_dense``   — fmincon LMPC: ``functions/costLMPC.m:20-45``,
  ``functions/constraintsLMPC.m:15-41``, ``transitionNominal.m:12-13``, decision
  ``var = [c_0..c_{N-1}; theta]`` (``ocpLMPC.m:20-24``).
* F2 ``dms_dense``    — CasADi DMS tracking LMPC: ``examples/DMS_tracking_LMPC_casadi.m:223-291``,
  bounds ``:107-119,161-162``, decision ``y = [x_0..x_N; u_0..u_{N-1}; theta]``.
* F5 ``track_dense``  — fmincon tracking MPC (double integrator):
  ``trackingMPC/costFunction.m:20-39``, ``trackingMPC/constraintsFunction.m:20-38``,
  decision ``var = [u_0..u_{N-1}; theta]`` (``RunExample.m:134-136``).

and the equivalent *structured* OCP (``*_ocp``) consumed by the batched solver:

    x_{k+1} = A x_k + B u_k + c,  x_0 given,  theta free (global),
    sum_k 0.5 v_k' W_k v_k + w_k' v_k   with  v_k = [x_k; u_k; theta]  (v_N = [x_N; theta]),
    box bounds on x_k (k=1..N) and u_k (k=0..N-1),
    one polytope block  Fp [x_kp; u_kp; theta] <= hp  at stage kp.

The structured form is what ``bqp_solve_ocp_batched`` (include/bqp.h) takes; the dense form is
what ``bqp_quadprog_batched`` takes.  Their optima coincide (tested).
"""
import numpy as np


class Aff:
    """Affine expression value = M @ z + v (M: d x nz)."""

    def __init__(self, M, v):
        self.M = np.atleast_2d(np.asarray(M, dtype=float))
        self.v = np.asarray(v, dtype=float).reshape(-1)

    @staticmethod
    def const(v, nz):
        v = np.asarray(v, dtype=float).reshape(-1)
        return Aff(np.zeros((v.size, nz)), v)

    @staticmethod
    def var(idx, nz):
        idx = np.atleast_1d(idx)
        M = np.zeros((idx.size, nz))
        M[np.arange(idx.size), idx] = 1.0
        return Aff(M, np.zeros(idx.size))

    def __add__(self, o):
        return Aff(self.M + o.M, self.v + o.v)

    def __sub__(self, o):
        return Aff(self.M - o.M, self.v - o.v)

    def lmul(self, L):
        L = np.atleast_2d(L)
        return Aff(L @ self.M, L @ self.v)

    def vstack(self, o):
        return Aff(np.vstack([self.M, o.M]), np.concatenate([self.v, o.v]))


class QuadAcc:
    """Accumulates J = sum (e' W e) for affine e into 0.5 z'Hz + f'z + const."""

    def __init__(self, nz):
        self.H = np.zeros((nz, nz))
        self.f = np.zeros(nz)
        self.c = 0.0

    def add(self, e, W):
        W = np.atleast_2d(W)
        self.H += 2.0 * e.M.T @ W @ e.M
        self.f += 2.0 * e.M.T @ W @ e.v
        self.c += float(e.v @ W @ e.v)


class IneqAcc:
    """Accumulates rows e <= 0  ->  A z <= b."""

    def __init__(self, nz):
        self.A = np.zeros((0, nz))
        self.b = np.zeros(0)

    def add(self, e):
        self.A = np.vstack([self.A, e.M])
        self.b = np.concatenate([self.b, -e.v])


def dense_qp(H, f, A=None, b=None, Aeq=None, beq=None, lb=None, ub=None, const=0.0):
    n = H.shape[0]
    return dict(H=H, f=f,
                A=np.zeros((0, n)) if A is None else A, b=np.zeros(0) if b is None else b,
                Aeq=np.zeros((0, n)) if Aeq is None else Aeq,
                beq=np.zeros(0) if beq is None else beq,
                lb=np.full(n, -np.inf) if lb is None else lb,
                ub=np.full(n, np.inf) if ub is None else ub, const=const)


# ----------------------------------------------------------------------------------------
# F1: fmincon LMPC (costLMPC.m / constraintsLMPC.m)
# ----------------------------------------------------------------------------------------
def lmpc_dense(mg, N, dx, F_T, h_T, xs=None):
    """F1 at state dx (deviation coordinates). Decision var = [c_0..c_{N-1}; theta] (m=1)."""
    A, B, K = mg['A'], mg['B'], mg['K']
    Q, R, P, T = mg['Q'], mg['R'], mg['P'], mg['Tscalar']
    LAM, PSI = mg['LAMBDA'], mg['PSI']
    n, m = B.shape
    nz = N * m + m
    xs = np.zeros(n) if xs is None else xs
    theta = Aff.var(np.arange(N * m, N * m + m), nz)
    c = [Aff.var(np.arange(k * m, (k + 1) * m), nz) for k in range(N)]
    lam_th = theta.lmul(LAM)
    psi_th = theta.lmul(PSI)

    def trans(xk, ck):                     # transitionNominal.m:12-13 / nominalModel.m:28
        uk = xk.lmul(K) + ck
        return xk.lmul(A) + uk.lmul(B), uk

    # costLMPC.m:20-45 (loop k=1..N, running cost only while k < N-1)
    J = QuadAcc(nz)
    xk = Aff.const(dx, nz)
    ck = c[0]
    for k in range(1, N + 1):
        xk1, uk = trans(xk, ck)
        if k < N - 1:
            J.add(xk - lam_th, Q)
            J.add(uk - psi_th, R)
        if k == N:
            J.add(xk1 - lam_th, P)
            J.add(lam_th - Aff.const(xs, nz), T * np.eye(n))
        xk = xk1
        if k < N:
            ck = c[k]
    # constraintsLMPC.m:15-41
    G = IneqAcc(nz)
    xk = Aff.const(dx, nz)
    ck = c[0]
    for k in range(1, N + 1):
        if k < N:
            xk1, uk = trans(xk, ck)
            G.add(xk1.lmul(mg['F_x']) - Aff.const(mg['h_x'], nz))
            G.add(uk.lmul(mg['F_u']) - Aff.const(mg['h_u'], nz))
            xk = xk1
            ck = c[k]
        else:
            G.add(xk1.vstack(theta).lmul(F_T) - Aff.const(h_T, nz))   # on x_{N-1} (:37)
    return dense_qp(J.H, J.f, G.A, G.b, const=J.c)


def lmpc_ocp(mg, N, F_T, h_T, xs=None):
    """F1 as a structured OCP in (x, u, theta) with u = K x + c (bijective re-parametrisation:
    the optimum maps back by c_k = u_k - K x_k).  Stage cost weights reproduce the
    ``if k < N-1`` quirk (costLMPC.m:30) and the terminal set sits on x_{N-1}
    (constraintsLMPC.m:37)."""
    A, B = mg['A'], mg['B']
    n, m = B.shape
    p = mg['LAMBDA'].shape[1]
    xs = np.zeros(n) if xs is None else xs
    nv = n + m + p
    W = np.zeros((N + 1, nv, nv))
    w = np.zeros((N + 1, nv))
    Q, R, P, T = mg['Q'], mg['R'], mg['P'], mg['Tscalar'] * np.eye(n)
    LAM, PSI = mg['LAMBDA'], mg['PSI']
    Ex = np.hstack([np.eye(n), np.zeros((n, m)), -LAM])          # x - LAM th
    Eu = np.hstack([np.zeros((m, n)), np.eye(m), -PSI])          # u - PSI th
    for k in range(N):
        if k + 1 < N - 1:                                        # costLMPC.m:30 (1-based k)
            W[k] += 2 * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)
    ExN = np.hstack([np.eye(n), np.zeros((n, m)), -LAM])
    EthN = np.hstack([np.zeros((n, n + m)), LAM])
    W[N] += 2 * (ExN.T @ P @ ExN + EthN.T @ T @ EthN)
    w[N] += -2 * EthN.T @ T @ xs
    const = float(xs @ T @ xs)
    hx_up, hx_lo = mg['h_x'][:n], -mg['h_x'][n:]
    hu_up, hu_lo = mg['h_u'][:m], -mg['h_u'][m:]
    xlb = np.full((N + 1, n), -np.inf); xub = np.full((N + 1, n), np.inf)
    ulb = np.full((N, m), -np.inf); uub = np.full((N, m), np.inf)
    for k in range(1, N):                                        # x_1..x_{N-1}, u_0..u_{N-2}
        xlb[k], xub[k] = hx_lo, hx_up
        ulb[k - 1], uub[k - 1] = hu_lo, hu_up
    # polytope F_T [x_{N-1}; theta] <= h_T  (columns over [x; u; theta])
    Fp = np.zeros((F_T.shape[0], nv))
    Fp[:, :n] = F_T[:, :n]
    Fp[:, n + m:] = F_T[:, n:]
    return dict(nx=n, nu=m, np=p, N=N, A=A, B=B, c=np.zeros(n), W=W, w=w, const=const,
                xlb=xlb, xub=xub, ulb=ulb, uub=uub, Fp=Fp, hp=np.asarray(h_T, float).ravel(),
                kp=N - 1)


# ----------------------------------------------------------------------------------------
# F2: DMS tracking LMPC (CasADi/IPOPT), DMS_tracking_LMPC_casadi.m:223-291
# ----------------------------------------------------------------------------------------
def dms_dense(mg, N, xmeas, F_T, h_T, delta=0.01):
    A, B = mg['A'], mg['B']
    n, m = B.shape
    x_eq, u_eq = mg['x_wp'], np.atleast_1d(mg['u_wp'])
    Q, R, P, T = mg['Q'], mg['R'], mg['P'], mg['Tscalar'] * np.eye(n)
    LAM, PSI = mg['LAMBDA'], mg['PSI']
    nz = (N + 1) * n + N * m + m
    X = [Aff.var(np.arange(k * n, (k + 1) * n), nz) for k in range(N + 1)]
    U = [Aff.var(np.arange((N + 1) * n + k * m, (N + 1) * n + (k + 1) * m), nz) for k in range(N)]
    th = Aff.var(np.arange(nz - m, nz), nz)
    xeq = Aff.const(x_eq, nz)
    ueq = Aff.const(u_eq, nz)
    x_art = th.lmul(LAM) + xeq
    u_art = th.lmul(PSI) + ueq
    J = QuadAcc(nz)
    for k in range(N):                                           # costfunction :233-237
        Jk = QuadAcc(nz)
        Jk.add(X[k] - x_art, Q)
        Jk.add(U[k] - u_art, R)
        J.H += delta * Jk.H; J.f += delta * Jk.f; J.c += delta * Jk.c
    J.add(X[N] - x_art, P)                                       # terminalcosts :248-251
    J.add(xeq - x_art, T)
    Geq = IneqAcc(nz)
    Gin = IneqAcc(nz)
    for k in range(N):                                           # nonlinearconstraints :264-282
        xn = xeq + (X[k] - xeq).lmul(A) + (U[k] - ueq).lmul(B)
        Geq.add(X[k + 1] - xn)
        Gin.add((X[k + 1] - xeq).lmul(mg['F_x']) - Aff.const(mg['h_x'], nz))
        Gin.add((U[k] - ueq).lmul(mg['F_u']) - Aff.const(mg['h_u'], nz))
    Gin.add((X[N] - xeq).vstack(th).lmul(F_T) - Aff.const(h_T, nz))   # :285
    lb = np.full(nz, -np.inf); ub = np.full(nz, np.inf)
    lb[:n] = xmeas; ub[:n] = xmeas                               # :161-162
    return dense_qp(J.H, J.f, Gin.A, Gin.b, Geq.A, Geq.b, lb, ub, const=J.c)


def dms_ocp(mg, N, F_T, h_T, delta=0.01):
    """F2 as a structured OCP in deviation coordinates (x~ = x - x_eq, u~ = u - u_eq)."""
    A, B = mg['A'], mg['B']
    n, m = B.shape
    p = mg['LAMBDA'].shape[1]
    nv = n + m + p
    Q, R, P, T = mg['Q'], mg['R'], mg['P'], mg['Tscalar'] * np.eye(n)
    LAM, PSI = mg['LAMBDA'], mg['PSI']
    Ex = np.hstack([np.eye(n), np.zeros((n, m)), -LAM])
    Eu = np.hstack([np.zeros((m, n)), np.eye(m), -PSI])
    Eth = np.hstack([np.zeros((n, n + m)), LAM])
    W = np.zeros((N + 1, nv, nv)); w = np.zeros((N + 1, nv))
    for k in range(N):
        W[k] = 2 * delta * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)
    W[N] = 2 * (Ex.T @ P @ Ex + Eth.T @ T @ Eth)
    hx_up, hx_lo = mg['h_x'][:n], -mg['h_x'][n:]
    hu_up, hu_lo = mg['h_u'][:m], -mg['h_u'][m:]
    xlb = np.full((N + 1, n), -np.inf); xub = np.full((N + 1, n), np.inf)
    xlb[1:], xub[1:] = hx_lo, hx_up
    ulb = np.tile(hu_lo, (N, 1)); uub = np.tile(hu_up, (N, 1))
    Fp = np.zeros((F_T.shape[0], nv))
    Fp[:, :n] = F_T[:, :n]
    Fp[:, n + m:] = F_T[:, n:]
    return dict(nx=n, nu=m, np=p, N=N, A=A, B=B, c=np.zeros(n), W=W, w=w, const=0.0,
                xlb=xlb, xub=xub, ulb=ulb, uub=uub, Fp=Fp, hp=np.asarray(h_T, float).ravel(),
                kp=N)


# ----------------------------------------------------------------------------------------
# F5: tracking MPC, double integrator (trackingMPC/costFunction.m, constraintsFunction.m)
# ----------------------------------------------------------------------------------------
def track_dense(di, N, x, xs, F_T, h_T):
    A, B = di['A'], di['B']
    n, m = B.shape
    P, T, Q, R = di['P'], di['T'], di['Q'], di['R']
    LAM, PSI = di['LAMBDA'], di['PSI']
    p = LAM.shape[1]
    nz = N * m + p
    U = [Aff.var(np.arange(k * m, (k + 1) * m), nz) for k in range(N)]
    th = Aff.var(np.arange(N * m, N * m + p), nz)
    lam_th = th.lmul(LAM); psi_th = th.lmul(PSI)
    J = QuadAcc(nz)
    xk = Aff.const(x, nz)
    uk = U[0]
    for k in range(1, N):                                        # costFunction.m:247-258
        J.add(xk - lam_th, Q)
        J.add(uk - psi_th, R)
        xk = xk.lmul(A) + uk.lmul(B)
        uk = U[k]
    J.add(xk - lam_th, P)                                        # costFunction.m:260-261
    J.add(lam_th - Aff.const(xs, nz), T)
    run_F = np.block([[di['F_x'], np.zeros((2 * n, m))], [np.zeros((2 * m, n)), di['F_u']]])
    run_h = np.concatenate([di['h_x'], di['h_u']])
    G = IneqAcc(nz)
    xk = Aff.const(x, nz)
    uk = U[0]
    for k in range(1, N + 1):                                    # constraintsFunction.m:287-302
        xk1 = xk.lmul(A) + uk.lmul(B)
        G.add(xk.vstack(uk).lmul(run_F) - Aff.const(run_h, nz))
        xk = xk1
        if k < N:
            uk = U[k]
        if k == N:
            G.add(xk.vstack(th).lmul(F_T) - Aff.const(h_T, nz))
    # rows of the constant x_0 block (k=1) do not depend on z: keep them (reference does)
    return dense_qp(J.H, J.f, G.A, G.b, const=J.c)


def track_ocp(di, N, F_T, h_T):
    """F5 structured: running cost k=0..N-2, terminal P on x_{N-1}, T on (LAM th - xs),
    boxes on x_1..x_{N-1}... (x_0 rows are constant and dropped), u_0..u_{N-1}, polytope
    on [x_N; theta].  xs enters only the per-instance linear term of stage N (``track_w``)."""
    A, B = di['A'], di['B']
    n, m = B.shape
    p = di['LAMBDA'].shape[1]
    nv = n + m + p
    Q, R, P, T = di['Q'], di['R'], di['P'], di['T']
    LAM, PSI = di['LAMBDA'], di['PSI']
    Ex = np.hstack([np.eye(n), np.zeros((n, m)), -LAM])
    Eu = np.hstack([np.zeros((m, n)), np.eye(m), -PSI])
    Eth = np.hstack([np.zeros((n, n + m)), LAM])
    W = np.zeros((N + 1, nv, nv)); w = np.zeros((N + 1, nv))
    for k in range(N - 1):
        W[k] = 2 * (Ex.T @ Q @ Ex + Eu.T @ R @ Eu)
    W[N - 1] = 2 * (Ex.T @ P @ Ex)
    W[N] = 2 * (Eth.T @ T @ Eth)
    hx_up, hx_lo = di['h_x'][:n], -di['h_x'][n:]
    hu_up, hu_lo = di['h_u'][:m], -di['h_u'][m:]
    xlb = np.full((N + 1, n), -np.inf); xub = np.full((N + 1, n), np.inf)
    xlb[1:N], xub[1:N] = hx_lo, hx_up                           # x_1..x_{N-1}
    ulb = np.tile(hu_lo, (N, 1)); uub = np.tile(hu_up, (N, 1))
    Fp = np.zeros((F_T.shape[0], nv))
    Fp[:, :n] = F_T[:, :n]
    Fp[:, n + m:] = F_T[:, n:]
    return dict(nx=n, nu=m, np=p, N=N, A=A, B=B, c=np.zeros(n), W=W, w=w, const=0.0,
                xlb=xlb, xub=xub, ulb=ulb, uub=uub, Fp=Fp, hp=np.asarray(h_T, float).ravel(),
                kp=N)


def track_w(di, N, xs):
    """Per-instance linear term of F5 stage N for reference xs (and the constant)."""
    n, m = di['B'].shape
    p = di['LAMBDA'].shape[1]
    nv = n + m + p
    Eth = np.hstack([np.zeros((n, n + m)), di['LAMBDA']])
    w = np.zeros((N + 1, nv))
    w[N] = -2 * Eth.T @ di['T'] @ xs
    return w, float(xs @ di['T'] @ xs)


# ----------------------------------------------------------------------------------------
# structured OCP -> dense (for cross-checking the structured description itself)
# ----------------------------------------------------------------------------------------
def ocp_to_dense(ocp, x0, w=None):
    """Dense quadprog form of a structured OCP over z = [x_0..x_N; u_0..u_{N-1}; theta]."""
    n, m, p, N = ocp['nx'], ocp['nu'], ocp['np'], ocp['N']
    nz = (N + 1) * n + N * m + p
    w = ocp['w'] if w is None else w
    ix = lambda k: np.arange(k * n, (k + 1) * n)
    iu = lambda k: np.arange((N + 1) * n + k * m, (N + 1) * n + (k + 1) * m)
    ith = np.arange(nz - p, nz)
    H = np.zeros((nz, nz)); f = np.zeros(nz)
    for k in range(N + 1):
        idx = np.concatenate([ix(k), iu(k) if k < N else np.zeros(0, int), ith])
        Wk = ocp['W'][k]; wk = w[k]
        if k == N:
            sel = np.concatenate([np.arange(n), np.arange(n + m, n + m + p)])
            Wk = Wk[np.ix_(sel, sel)]; wk = wk[sel]
        H[np.ix_(idx, idx)] += Wk
        f[idx] += wk
    Aeq = []; beq = []
    for k in range(N):
        row = np.zeros((n, nz))
        row[:, ix(k + 1)] = np.eye(n)
        row[:, ix(k)] = -ocp['A']
        row[:, iu(k)] = -ocp['B']
        Aeq.append(row); beq.append(ocp['c'])
    Aeq = np.vstack(Aeq); beq = np.concatenate(beq)
    lb = np.full(nz, -np.inf); ub = np.full(nz, np.inf)
    for k in range(1, N + 1):
        lb[ix(k)] = ocp['xlb'][k]; ub[ix(k)] = ocp['xub'][k]
    for k in range(N):
        lb[iu(k)] = ocp['ulb'][k]; ub[iu(k)] = ocp['uub'][k]
    lb[ix(0)] = x0; ub[ix(0)] = x0
    kp = ocp['kp']
    Fp = ocp['Fp']
    Ain = np.zeros((Fp.shape[0], nz))
    Ain[:, ix(kp)] = Fp[:, :n]
    if kp < N:
        Ain[:, iu(kp)] = Fp[:, n:n + m]
    Ain[:, ith] = Fp[:, n + m:]
    return dense_qp(H, f, Ain, ocp['hp'].copy(), Aeq, beq, lb, ub, const=ocp.get('const', 0.0))
