"""Dense (quadprog-form) condensing of a stage-wise OCP: the states are eliminated through the
dynamics, leaving min 0.5 z'Hz + f'z s.t. A z <= b over z = [u_0..u_{N-1}; theta].  This is the
form the reference's fmincon LMPC solves (functions/ocpLMPC.m:20-24 over costLMPC.m /
constraintsLMPC.m, form F1: 21 variables and 806 rows at N = 20), and what a MATLAB caller of
quadprog_gpu builds once per run.  H and A do not depend on the measured
state; f and b are affine in it, so a batch shares H and A (stride 0) and carries f and b.

Host-side numpy (runs once per design, not per solve); the solve is bqp.quadprog on the GPU.
"""
import numpy as np


class Condensed:
    """H (nz, nz), A (m, nz) shared; f(x0) = f0 + Fx x0, b(x0) = b0 + Bx x0 per instance."""

    def __init__(self, prob):
        N, nx, nu, npar = prob.N, prob.nx, prob.nu, prob.np
        nz = N * nu + npar
        Am, Bm, c = prob.A, prob.B, prob.c
        # x_k = Px[k] x0 + Gx[k] z + cx[k]
        Px = np.zeros((N + 1, nx, nx)); Gx = np.zeros((N + 1, nx, nz)); cx = np.zeros((N + 1, nx))
        Px[0] = np.eye(nx)
        for k in range(N):
            Px[k + 1] = Am @ Px[k]
            Gx[k + 1] = Am @ Gx[k]
            Gx[k + 1][:, k * nu:(k + 1) * nu] += Bm
            cx[k + 1] = Am @ cx[k] + c
        # v_k = [x_k; u_k; theta] = S[k] z + T[k] x0 + e[k]
        nv = nx + nu + npar
        S = np.zeros((N + 1, nv, nz)); T = np.zeros((N + 1, nv, nx)); e = np.zeros((N + 1, nv))
        for k in range(N + 1):
            S[k, :nx] = Gx[k]
            if k < N:
                S[k, nx:nx + nu, k * nu:(k + 1) * nu] = np.eye(nu)
            S[k, nx + nu:, N * nu:] = np.eye(npar)
            T[k, :nx] = Px[k]
            e[k, :nx] = cx[k]
        W = prob.W.copy()
        w = prob.w.copy()
        W[N, nx:nx + nu, :] = 0.0; W[N, :, nx:nx + nu] = 0.0; w[N, nx:nx + nu] = 0.0
        self.H = np.einsum('kai,kab,kbj->ij', S, W, S)
        self.H = 0.5 * (self.H + self.H.T)
        self.Fx = np.einsum('kai,kab,kbj->ij', S, W, T)
        self.f0 = np.einsum('kai,kab,kb->i', S, W, e) + np.einsum('kai,ka->i', S, w)
        rows, Bx, b0 = [], [], []

        def add(sel, Gz, Tx, ex, h, sign):
            rows.append(sign * Gz[sel]); Bx.append(-sign * Tx[sel]); b0.append(sign * h[sel] - sign * ex[sel])

        for k in range(1, N + 1):                       # state boxes (stage 0 is x0, fixed)
            up, lo = np.isfinite(prob.xub[k]), np.isfinite(prob.xlb[k])
            add(up, Gx[k], Px[k], cx[k], np.where(up, prob.xub[k], 0.0), 1.0)
            add(lo, Gx[k], Px[k], cx[k], np.where(lo, prob.xlb[k], 0.0), -1.0)
        for k in range(N):                              # input boxes
            up, lo = np.isfinite(prob.uub[k]), np.isfinite(prob.ulb[k])
            Gu = S[k, nx:nx + nu]
            zero = np.zeros((nu, nx)); ze = np.zeros(nu)
            add(up, Gu, zero, ze, np.where(up, prob.uub[k], 0.0), 1.0)
            add(lo, Gu, zero, ze, np.where(lo, prob.ulb[k], 0.0), -1.0)
        if prob.mp:
            kp = prob.poly_stage
            Fp = prob.Fp.copy()
            if kp == N:
                Fp[:, nx:nx + nu] = 0.0
            sel = np.ones(prob.mp, bool)
            add(sel, Fp @ S[kp], Fp @ T[kp], Fp @ e[kp], prob.hp, 1.0)
        self.A = np.vstack(rows)
        self.Bx = np.vstack(Bx)
        self.b0 = np.concatenate(b0)
        self.prob = prob
        self.const_e = e
        self.T, self.S = T, S

    @property
    def n(self):
        return self.H.shape[0]

    @property
    def m(self):
        return self.A.shape[0]

    def rhs(self, X0):
        """per-instance (f, b) for measured states X0 (batch, nx)"""
        X0 = np.atleast_2d(X0)
        return X0 @ self.Fx.T + self.f0, X0 @ self.Bx.T + self.b0

    def recover(self, Z, X0):
        """z (batch, nz) -> u (batch, N, nu), theta (batch, np), x (batch, N+1, nx)"""
        p = self.prob
        N, nx, nu = p.N, p.nx, p.nu
        Z = np.atleast_2d(Z); X0 = np.atleast_2d(X0)
        V = np.einsum('kaj,bj->bka', self.S, Z) + np.einsum('kax,bx->bka', self.T, X0) + self.const_e[None]
        return Z[:, :N * nu].reshape(-1, N, nu), Z[:, N * nu:], V[:, :, :nx]
