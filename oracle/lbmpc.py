"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the learning-based MPC problems (forms F3/F4) and of the
algorithm the GPU path uses for them: a Gauss-Newton SQP whose QP sub-problems go through the
batched dense solver.  numpy, one instance at a time - the checker for the HIP path.

Reference anchors
-----------------
* Nadaraya-Watson oracle: ``functions/oracleL2NW.m:26-36`` (struct data X 3xn, Y 4xn) and
  ``examples/hybrid_LBMPC_casadi.m:331-358`` (7xq matrix data, no validity mask: zero columns
  enter the normaliser).  g(xi) = sum_i Y_i k_i / (lambda + sum_j k_j),
  k_i = exp(-|X_i - xi|^2 / h^2), h = 0.5, lambda = 1e-3, xi = [x_1; x_2; u].
* learned model ``models/learnedModel.m:25``: x+ = A x + B u + g(x, u).
* F3 (fmincon LBMPC): ``functions/costLBMPC.m:20-45`` (rollout u = K x + c on the LEARNED
  model; running cost for k < N-1 on (x_{k-1}, u_{k-1}); terminal P, T on x_N),
  ``functions/constraintsLBMPC.m:18-45`` (NOMINAL model; at k = 1 F_x_d x_1 <= h_x_d and
  F_w_N [x_1; theta] <= h_w_N; F_x x_k <= h_x, F_u u_{k-1} <= h_u for k = 1..N-1).
* F4 (hybrid LBMPC, CasADi/IPOPT): ``examples/hybrid_LBMPC_casadi.m:250-311`` (running cost
  delta * (...) on the learned rollout from x_0 for k = 0..N-1, terminal cost on the NOMINAL
  decision x_N, nominal dynamics as equalities, the same stage-1 sets, boxes for k = 1..N).
  Golden instance: ``examples/DSS_NMPC.m`` (IPOPT optimum y_OL, :1147; tests/golden/
  lbmpc_instance.npz).

Algorithm (shared with the HIP path, bqp/lbmpc.py + csrc/bqp_lbmpc.hip)
----------------------------------------------------------------------
Decision z = [v_0..v_{N-1}; theta] (v = c for F3, v = u - u_eq for F4), deviation coordinates.
Nominal states/inputs are affine in z (exact condensing, constraints A_in z <= b_in).  At the
iterate z: learned rollout + forward sensitivities S_k = dx^L_k/dz, U_k = du^L_k/dz;
GN model H = 2 sum J'WJ, f = 2 sum J'W e of the quadratic cost in the residuals e; QP
min 0.5 d'Hd + f'd s.t. A_in (z + d) <= b_in; Armijo backtracking on the true cost over the
trial steps alpha = 2^-j (j = 0..7), sufficient-decrease 1e-4; stop when |d|_inf <= tol_step
(1 + |z|_inf) and the NLP stationarity |grad J + A_in' lam|_inf <= tol_stat (1 + |grad J|_inf).
"""
import numpy as np

from . import dense_qp

H_BW = 0.5
LAM_NW = 1e-3


def nw(xi, data):
    """g (4,), dg/dxi (4, 3) of the NW oracle at xi (3,); data 7 x q."""
    X, Y = data[:3], data[3:]
    d = X - xi[:, None]                                  # (3, q)
    k = np.exp(-(d * d).sum(0) / H_BW ** 2)              # (q,)
    s = k.sum()
    den = LAM_NW + s
    sy = Y @ k                                           # (4,)
    g = sy / den
    # dk_i/dxi = k_i * 2 (X_i - xi) / h^2
    dk = (k[None, :] * d) * (2.0 / H_BW ** 2)            # (3, q)
    dsy = Y @ dk.T                                       # (4, 3)
    ds = dk.sum(1)                                       # (3,)
    dg = dsy / den - np.outer(sy, ds) / den ** 2
    return g, dg


def rollout(p, x0, z, learned=True, jac=False):
    """x (N+1, nx), u (N, nu) of the (learned or nominal) closed rollout u_k = K x_k + v_k, and
    optionally the sensitivities S (N+1, nx, n), U (N, nu, n) w.r.t. z."""
    N, nx, nu = p['N'], p['nx'], p['nu']
    n = N * nu + p['np']
    A, B, K = p['A'], p['B'], p['K']
    v = z[:N * nu].reshape(N, nu)
    x = np.zeros((N + 1, nx)); u = np.zeros((N, nu))
    x[0] = x0
    S = np.zeros((N + 1, nx, n)); U = np.zeros((N, nu, n))
    for k in range(N):
        u[k] = K @ x[k] + v[k]
        Ak, Bk = A, B
        xn = A @ x[k] + B @ u[k]
        if learned:
            g, dg = nw(np.concatenate([x[k][:2], u[k]]), p['data'])
            xn = xn + g
            Gx = np.zeros((nx, nx)); Gx[:, :2] = dg[:, :2]
            Ak, Bk = A + Gx, B + dg[:, 2:2 + nu]
        x[k + 1] = xn
        if jac:
            U[k] = K @ S[k]
            U[k][:, k * nu:(k + 1) * nu] += np.eye(nu)
            S[k + 1] = Ak @ S[k] + Bk @ U[k]
    return (x, u, S, U) if jac else (x, u)


def _theta(p, z):
    return z[p['N'] * p['nu']:]


def cost(p, x0, z):
    xL, uL = rollout(p, x0, z, learned=True)
    th = _theta(p, z)
    LAM, PSI, Q, R = p['LAMBDA'], p['PSI'], p['Q'], p['R']
    J = 0.0
    for k in range(p['n_run']):
        ex = xL[k] - LAM @ th
        eu = uL[k] - PSI @ th
        J += p['w_run'] * (ex @ Q @ ex + eu @ R @ eu)
    xT = xL[p['N']] if p['term_learned'] else rollout(p, x0, z, learned=False)[0][p['N']]
    eT = xT - LAM @ th
    es = LAM @ th - p['xs']
    return J + eT @ p['P'] @ eT + es @ p['T'] @ es


def gn_model(p, x0, z):
    """GN Hessian H, exact gradient f of the cost at z."""
    N, nu, npar = p['N'], p['nu'], p['np']
    n = N * nu + npar
    LAM, PSI, Q, R = p['LAMBDA'], p['PSI'], p['Q'], p['R']
    xL, uL, S, U = rollout(p, x0, z, learned=True, jac=True)
    th = _theta(p, z)
    Et = np.zeros((npar, n)); Et[:, N * nu:] = np.eye(npar)
    H = np.zeros((n, n)); f = np.zeros(n)
    w = p['w_run']
    for k in range(p['n_run']):
        Jx = S[k] - LAM @ Et
        Ju = U[k] - PSI @ Et
        ex = xL[k] - LAM @ th
        eu = uL[k] - PSI @ th
        H += 2 * w * (Jx.T @ Q @ Jx + Ju.T @ R @ Ju)
        f += 2 * w * (Jx.T @ Q @ ex + Ju.T @ R @ eu)
    if p['term_learned']:
        xT, ST = xL[N], S[N]
    else:
        xn, _, Sn, _ = rollout(p, x0, z, learned=False, jac=True)
        xT, ST = xn[N], Sn[N]
    JT = ST - LAM @ Et
    eT = xT - LAM @ th
    H += 2 * (JT.T @ p['P'] @ JT)
    f += 2 * (JT.T @ p['P'] @ eT)
    Js = LAM @ Et
    es = LAM @ th - p['xs']
    H += 2 * (Js.T @ p['T'] @ Js)
    f += 2 * (Js.T @ p['T'] @ es)
    return H, f


def nw_hess(xi, data):
    """g (4,), dg (4, 3) and the second derivatives d2g (4, 3, 3) of the NW sums at xi over a 7-row
    window (every point counts) or an 8-row window [X; Y; v] (casadiL2NW.m normaliser).
    With c = 2/h^2: dk_j = c k_j d_j, d2k_j = k_j (c^2 d_j d_j' - c I), d_j = X_j - xi;
    g = N / D, dg = (dN - g dD') / D, d2g_i = (d2N_i - g_i d2D - dg_i dD' - dD dg_i') / D."""
    X, Y = data[:3], data[3:7]
    v = data[7] if data.shape[0] == 8 else np.ones(data.shape[1])
    d = X - xi[:, None]                                  # (3, q)
    k = np.exp(-(d * d).sum(0) / H_BW ** 2)
    c = 2.0 / H_BW ** 2
    D = LAM_NW + k @ v
    Nn = Y @ k
    g = Nn / D
    dk = c * k[None, :] * d                              # (3, q)
    dN = Y @ dk.T                                        # (4, 3)
    dD = dk @ v                                          # (3,)
    dg = (dN - np.outer(g, dD)) / D
    ddk = (c * c) * np.einsum('j,aj,bj->jab', k, d, d) - c * k[:, None, None] * np.eye(3)[None]
    d2N = np.einsum('ij,jab->iab', Y, ddk)               # (4, 3, 3)
    d2D = np.einsum('j,jab->ab', v, ddk)
    d2g = (d2N - g[:, None, None] * d2D[None] - np.einsum('ia,b->iab', dg, dD)
           - np.einsum('a,ib->iab', dD, dg)) / D
    return g, dg, d2g


def pd_cholesky(H, rel=1e-10, tol=None):
    """right-looking Cholesky of H with every pivot required above rel max_i |H_ii| (or above the
    absolute tol)"""
    K = np.array(H, float)
    n = K.shape[0]
    if tol is None:
        tol = rel * np.abs(np.diag(K)).max()
    for j in range(n):
        d = K[j, j]
        if not d > tol:
            return False
        K[j + 1:, j] /= np.sqrt(d)
        K[j + 1:, j + 1:] -= np.outer(K[j + 1:, j], K[j + 1:, j])
    return True


def hess_shift(H):
    """regularised exact Hessian (round 5, oracle/cpu_lbmpc.c hess_shift_k): the smallest grid
    shift delta_k = 1e-12 hd 4^k (k = 0..20, hd = max|H_ii|) with H + delta_k I positive definite
    under pd_cholesky's test (pivots above 1e-10 hd), by bisection over k (definiteness is
    monotone in the shift); None if even k = 20 fails"""
    hd = np.abs(np.diag(H)).max()
    tol = 1e-10 * hd
    n = H.shape[0]
    sh = lambda k: np.ldexp(1e-12 * hd, 2 * k)
    lo, hi = -1, 20
    if not pd_cholesky(H + sh(hi) * np.eye(n), tol=tol):
        return None
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if pd_cholesky(H + sh(mid) * np.eye(n), tol=tol):
            hi = mid
        else:
            lo = mid
    return sh(hi)


def psd_part(W):
    """the positive semidefinite part of a symmetric 3 x 3 matrix (eigenvalues clipped at 0)"""
    w, V = np.linalg.eigh(0.5 * (W + W.T))
    return (V * np.maximum(w, 0.0)) @ V.T


def newton_model(p, x0, z, clip=True):
    """H, f of the SQP model with the second-order term of the learned dynamics:
    H = H_GN + sum_k Xi_k' [sum_i p_{k+1,i} d2g_i(xi_k)]_+ Xi_k, with the costate
    p_k = dJ/dx_k (backward recursion through the learned rollout) and Xi_k = dxi_k/dz; the
    per-stage 3 x 3 curvature is clipped to its PSD part so that the QP stays convex."""
    N, nu, npar, nx = p['N'], p['nu'], p['np'], p['nx']
    n = N * nu + npar
    H, f = gn_model(p, x0, z)
    xL, uL, S, U = rollout(p, x0, z, learned=True, jac=True)
    th = _theta(p, z)
    LAM, PSI, Q, R, K, A, B = p['LAMBDA'], p['PSI'], p['Q'], p['R'], p['K'], p['A'], p['B']
    Gx, d2 = [], []
    for k in range(N):
        xi = np.concatenate([xL[k][:2], uL[k]])
        _, dg, d2g = nw_hess(xi, p['data'])
        Gx.append(dg); d2.append(d2g)
    pk = np.zeros(nx)
    if p['term_learned']:
        pk = 2.0 * p['P'] @ (xL[N] - LAM @ th)
    w = p['w_run']
    for k in range(N - 1, -1, -1):
        # W_k from p_{k+1}
        Wk = np.einsum('i,iab->ab', pk, d2[k])
        Xi = np.vstack([S[k][:2], U[k]])                  # (3, n)
        H += Xi.T @ (psd_part(Wk) if clip else 0.5 * (Wk + Wk.T)) @ Xi
        # p_k = dphi_k/dx_k + (dx_{k+1}/dx_k)' p_{k+1}
        dg = Gx[k]
        Jx = A + B @ K
        Jx = Jx + np.hstack([dg[:, :2], np.zeros((nx, nx - 2))]) + np.outer(dg[:, 2], K[0]) if nu == 1 else Jx
        pn = Jx.T @ pk
        if k < p['n_run']:
            ex = xL[k] - LAM @ th
            eu = uL[k] - PSI @ th
            pn = pn + 2 * w * (Q @ ex + K.T @ (R @ eu))
        pk = pn
    return H, f


def constraints(p, x0):
    """A_in z <= b_in from the nominal rollout (exact: affine in z)."""
    N, nu, npar = p['N'], p['nu'], p['np']
    n = N * nu + npar
    z0 = np.zeros(n)
    x, u, S, U = rollout(p, x0, z0, learned=False, jac=True)
    Et = np.zeros((npar, n)); Et[:, N * nu:] = np.eye(npar)
    rows, rhs = [], []
    # stage 1 sets (constraintsLBMPC.m:26-30, hybrid_LBMPC_casadi.m:296-300)
    rows.append(p['F_x_d'] @ S[1]); rhs.append(p['h_x_d'] - p['F_x_d'] @ x[1])
    FT = p['F_T']
    nxT = p['nx']
    rows.append(FT[:, :nxT] @ S[1] + FT[:, nxT:] @ Et)
    rhs.append(p['h_T'] - FT[:, :nxT] @ x[1])
    for k in range(1, p['n_box'] + 1):
        rows.append(p['F_x'] @ S[k]); rhs.append(p['h_x'] - p['F_x'] @ x[k])
        rows.append(p['F_u'] @ U[k - 1]); rhs.append(p['h_u'] - p['F_u'] @ u[k - 1])
    return np.vstack(rows), np.concatenate(rhs)


def sqp(p, x0, z0=None, max_iter=100, tol_step=1e-10, tol_stat=1e-9, trace=None, hessian='gn'):
    """SQP with parallel-trial Armijo line search (see module doc).  hessian: 'gn' Gauss-Newton;
    'exact' adds the second-order term of the learned dynamics (newton_model) whenever the result
    is positive definite (pd_cholesky), else Gauss-Newton for that iteration - the product's
    default (GN alone converges linearly, rate ~0.5, on the learned-state costs of
    DMS_LBMPC_casadi.m: 60-200 iterations against 4-6); 'newton' clips each stage's curvature to
    its PSD part (no faster than GN there: the curvature that matters is negative).
    Returns z, lam_in, info."""
    N, nu, npar = p['N'], p['nu'], p['np']
    n = N * nu + npar
    Ain, bin_ = constraints(p, x0)
    z = np.zeros(n) if z0 is None else np.array(z0, float)
    if np.any(Ain @ z > bin_ + 1e-12):
        # feasible start: the QP's own solution with the model at z (first iterate)
        pass
    lam = np.zeros(Ain.shape[0])
    J = cost(p, x0, z)
    it = 0
    stat = np.inf
    for it in range(1, max_iter + 1):
        if hessian == 'gn':
            H, f = gn_model(p, x0, z)
        else:
            H, f = newton_model(p, x0, z, clip=hessian == 'newton')
            if hessian == 'exact' and not pd_cholesky(H):
                # the exact Hessian of the learned cost when it is positive definite (Cholesky
                # pivots above 1e-10 max|H_ii|, the test of bqp_lbmpc.hip lbmpc_hess_kernel),
                # else shifted by the smallest grid delta that makes it so (hess_shift), the
                # Gauss-Newton matrix only if no shift does
                dsh = hess_shift(H)
                if dsh is None:
                    H, f = gn_model(p, x0, z)
                else:
                    H = H + dsh * np.eye(H.shape[0])
        qp = dict(H=H, f=f, A=Ain, b=bin_ - Ain @ z, Aeq=np.zeros((0, n)), beq=np.zeros(0),
                  lb=np.full(n, -np.inf), ub=np.full(n, np.inf))
        d, _, lamq, info = dense_qp.solve(qp)
        lam = lamq['ineqlin']
        if not (np.all(np.isfinite(d)) and np.all(np.isfinite(lam))):
            # the dense IPM broke down (it does on some well-conditioned learned-cost
            # sub-problems, eig(H) in [0.5, 1.2e3]): the exact LDP/NNLS solve of the same QP
            from . import exact_qp
            r = exact_qp.solve(H, f, Ain, bin_ - Ain @ z)
            d, lam = r['z'], r['lam']
        stat = np.abs(f + Ain.T @ lam).max()
        feas_start = np.all(Ain @ z <= bin_ + 1e-9)
        if trace is not None:
            trace.append(dict(it=it, J=J, step=np.abs(d).max(), stat=stat))
        if feas_start and np.abs(d).max() <= tol_step * (1 + np.abs(z).max()) and \
                stat <= tol_stat * (1 + np.abs(f).max()):
            break
        slope = f @ d
        acc = False
        for j in range(8):
            a = 0.5 ** j
            Jt = cost(p, x0, z + a * d)
            if not feas_start or Jt <= J + 1e-4 * a * slope:
                z = z + a * d
                J = Jt
                acc = True
                break
        if not acc:
            z = z + 0.5 ** 7 * d
            J = cost(p, x0, z)
    return z, lam, dict(iterations=it, cost=J, stat=stat)


# ----------------------------------------------------------------------------------------
# problem builders
# ----------------------------------------------------------------------------------------
def _common(mg, N, data, F_T, h_T, F_x_d, h_x_d):
    return dict(nx=4, nu=1, np=1, N=N, A=mg['A'], B=mg['B'].reshape(4, 1),
                Q=mg['Q'], R=np.atleast_2d(mg['R']), P=mg['P'],
                T=float(mg['Tscalar']) * np.eye(4), LAMBDA=mg['LAMBDA'].reshape(4, 1),
                PSI=np.atleast_2d(mg['PSI']).reshape(1, 1), xs=np.zeros(4),
                F_x=mg['F_x'], h_x=mg['h_x'], F_u=mg['F_u'], h_u=mg['h_u'],
                F_T=np.asarray(F_T, float), h_T=np.asarray(h_T, float).ravel(),
                F_x_d=np.asarray(F_x_d, float), h_x_d=np.asarray(h_x_d, float).ravel(),
                data=np.asarray(data, float))


def f3_problem(mg, N, data, F_T, h_T, F_x_d, h_x_d):
    """fmincon LBMPC (costLBMPC.m / constraintsLBMPC.m), decision [c; theta]."""
    p = _common(mg, N, data, F_T, h_T, F_x_d, h_x_d)
    p.update(K=np.asarray(mg['K'], float).reshape(1, 4), w_run=1.0, n_run=max(N - 2, 0),
             term_learned=True, n_box=N - 1)
    return p


def f4_problem(mg, N, data, F_T, h_T, F_x_d, h_x_d, delta=0.01):
    """hybrid LBMPC (hybrid_LBMPC_casadi.m:250-311), decision [u - u_eq; theta]."""
    p = _common(mg, N, data, F_T, h_T, F_x_d, h_x_d)
    p.update(K=np.zeros((1, 4)), w_run=delta, n_run=N, term_learned=False, n_box=N)
    return p


def f4_to_y(p, x0, z, x_eq, u_eq):
    """y_OL layout of hybrid_LBMPC_casadi.m (absolute [x_0..x_N; u; theta])."""
    x, u = rollout(p, x0, z, learned=False)
    return np.concatenate([(x + x_eq).ravel(), (u + u_eq).ravel(), _theta(p, z)])


# ----------------------------------------------------------------------------------------
# closed-loop data window (LBMPC_casadi.m:193-198 with utilities/update_data.m;
# DMS_LBMPC_casadi.m:198-207 with utilities/get_data.m and functions/casadiL2NW.m)
# ----------------------------------------------------------------------------------------
def nw_masked(xi, data, h=0.5, lam=1e-3):
    """casadiL2NW.m:14-28: g = sum_i Y_i k_i / (lambda + sum_j k_j v_j) over an 8 x q window
    [X; Y; v], k_i = exp(-|X_i - xi|^2 / h^2)."""
    d = data[:3] - np.asarray(xi, float)[:, None]
    k = np.exp(-np.sum(d * d, axis=0) / h ** 2)
    return data[3:7] @ k / (lam + k @ data[7])


def window_replay(X, U, A, B, x_eq, u_eq, q, mask=True, h=0.5, lam=1e-3):
    """Replays the data acquisition of the reference's LBMPC loop on a closed-loop record
    (X (T+1, 4) and U (T,) absolute): per iteration it = 1..T the learned prediction
    xl = x_eq + A dx + B du + g(xi) with the window before the update (DMS_LBMPC_casadi.m:199),
    then X = [dx1; dx2; du], Y = (x+ - x_eq) - (A dx + B du) appended by get_data.m (a column
    per iteration, the oldest dropped once the q columns are full).  The window starts as zeros
    with only the first point valid (mask, :160-161), or with every point valid (7-row window
    without validity row).  Returns XL (T+1, 4) with XL[0] = X[0], and the final 8 x q window in
    the reference's column order."""
    X = np.asarray(X, float); U = np.asarray(U, float).ravel()
    A = np.asarray(A, float); B = np.asarray(B, float).reshape(4)
    x_eq = np.asarray(x_eq, float); u_eq = float(np.ravel(u_eq)[0])
    data = np.zeros((8, q))
    if mask:
        data[7, 0] = 1.0
    else:
        data[7, :] = 1.0
    XL = [X[0].copy()]
    for it in range(1, len(U) + 1):
        t = it - 1
        dx = X[t] - x_eq
        du = U[t] - u_eq
        nom = A @ dx + B * du
        xi = np.array([dx[0], dx[1], du])
        XL.append(x_eq + nom + nw_masked(xi, data, h, lam))
        col = np.concatenate([xi, (X[t + 1] - x_eq) - nom, [1.0]])
        if it < q:                                          # get_data.m:3-6
            data[:, it] = col
        else:                                               # get_data.m:7-9
            data = np.hstack([data[:, 1:], col[:, None]])
    return np.array(XL), data


# ----------------------------------------------------------------------------------------
# learned-model NLP closed loop (DMS_LBMPC_casadi.m:163-218)
# ----------------------------------------------------------------------------------------
def nw_window(xi, data):
    """casadiL2NW.m:14-28 on an 8 x q window [X; Y; v] with dg/dxi:
    g = sum_i Y_i k_i / (lambda + sum_j v_j k_j) (numerator not masked: the points that are not
    yet valid hold Y = 0).  A 7-row window counts every point (v = 1), as nw()."""
    X, Y = data[:3], data[3:7]
    v = data[7] if data.shape[0] == 8 else np.ones(data.shape[1])
    d = X - xi[:, None]
    k = np.exp(-(d * d).sum(0) / H_BW ** 2)
    den = LAM_NW + k @ v
    sy = Y @ k
    dk = (k[None, :] * d) * (2.0 / H_BW ** 2)
    return sy / den, (Y @ dk.T) / den - np.outer(sy, dk @ v) / den ** 2


def dms_problem(mg, N, data, F_T, h_T, F_x_d, h_x_d, delta=0.01):
    """DMS_LBMPC_casadi.m:121-129 after eliminating both state chains: decision z = [u - u_eq;
    theta]; running cost (delta-weighted, k = 0..N-1, :229-233) and terminal cost (:234) on the
    learned rollout, constraints on the nominal rollout (:262-276) - the F4 problem with the
    terminal term on the learned x_N.  data: the 8 x q window (or 7 x q)."""
    p = f4_problem(mg, N, data, F_T, h_T, F_x_d, h_x_d, delta)
    p['term_learned'] = True
    return p


def dms_lbmpc_loop(mg, sets, N, q, steps, mask=True, term_learned=True, warm=True,
                   x_init=(0.15, 1.2875, 1.1547, 0.0), max_iter=200, hessian='exact'):
    """Closed loop of DMS_LBMPC_casadi.m:157-218: per iteration the NLP at the measured state
    (GN-SQP to a KKT point), u_0 to the RK4 plant (`dynamic`, :297-304), the sample
    [dx1; dx2; du; Y; 1] into the window by get_data.m, and the shifted warm start (:209-213,
    tail move 0).  mask: the 8 x q window with only the first (zero) point valid at the start
    (:158-161); mask=False counts every point (7-row window).  Returns X (steps+1, 4) absolute,
    U (steps,) absolute, Z (steps, N+1) and the SQP iteration counts."""
    from .mg_model import mg_rk4
    global nw
    x_eq = np.asarray(mg['x_wp'], float); u_eq = float(np.ravel(mg['u_wp'])[0])
    A = np.asarray(mg['A'], float); B = np.asarray(mg['B'], float).reshape(4)
    data = np.zeros((8, q))
    data[7, :] = 0.0 if mask else 1.0
    data[7, 0] = 1.0
    x = np.array(x_init, float)
    X, U, Z, IT = [x.copy()], [], [], []
    z = None
    saved = nw
    nw = nw_window
    try:
        for it in range(1, steps + 1):
            p = dms_problem(mg, N, data, sets['F_w_N'], sets['h_w_N'], sets['F_x_d'], sets['h_x_d'])
            p['term_learned'] = term_learned
            z, _, info = sqp(p, x - x_eq, z0=z if warm else None, max_iter=max_iter, hessian=hessian)
            du = z[0]
            xn = mg_rk4(0.01, x, du + u_eq)
            dx = x - x_eq
            nom = A @ dx + B * du
            col = np.concatenate([[dx[0], dx[1], du], (xn - x_eq) - nom, [1.0]])
            if it < q:                                      # get_data.m:3-6
                data[:, it] = col
            else:                                           # get_data.m:7-9
                data = np.hstack([data[:, 1:], col[:, None]])
            Z.append(z.copy()); IT.append(info['iterations']); U.append(du + u_eq)
            z = np.concatenate([z[1:N], [0.0], z[N:]])
            x = xn
            X.append(x.copy())
    finally:
        nw = saved
    return np.array(X), np.array(U), np.array(Z), np.array(IT)
