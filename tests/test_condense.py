"""bqp.condense: the stage-wise OCP condensed to quadprog form (z = [u; theta]) - for the C2
problem exactly fmincon's F1 (21 variables, 806 rows); its optimum (oracle dense solve) maps
back to the exact z* of the fixtures."""
import numpy as np

from conftest import golden


def test_condensed_f1_matches_z_star(mg, term_set):
    import bqp
    from bqp.condense import Condensed
    from oracle import dense_qp
    g = golden('lmpc_N20.npz')
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                  mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                  term_set[0], term_set[1], N=20)
    cd = Condensed(lm.prob)
    assert (cd.n, cd.m) == (21, 806)
    X0 = g['dx'][g['idx'][:6]]
    f, b = cd.rhs(X0)
    for i in range(len(X0)):
        qp = dict(H=cd.H, f=f[i], A=cd.A, b=b[i], Aeq=np.zeros((0, cd.n)), beq=np.zeros(0),
                  lb=np.full(cd.n, -np.inf), ub=np.full(cd.n, np.inf))
        z, fv, lam, info = dense_qp.solve(qp)
        u, th, x = cd.recover(z[None], X0[i:i + 1])
        c = u[0, :, 0] - (x[0, :20] @ lm.K.T)[:, 0]
        assert np.abs(np.concatenate([c, th[0]]) - g['z_star'][i]).max() < 1e-10


def odd_dims_problem(N=12, seed=3):
    """an (nx, nu, np) = (3, 1, 1) problem - no compiled structured kernel, so bqp.solve_ocp
    takes the condensed route - with boxes on x and u and a terminal polytope on [x_N; theta];
    returns (OcpProblem, the oracle's stage-wise dict, x0 batch, per-instance hp batch)"""
    import bqp
    rng = np.random.default_rng(seed)
    nx, nu, npar = 3, 1, 1
    nv = nx + nu + npar
    M = rng.standard_normal((nx, nx))
    A = 0.8 * M / np.abs(np.linalg.eigvals(M)).max()
    B = rng.standard_normal((nx, nu))
    c = 0.05 * rng.standard_normal(nx)
    W = np.zeros((N + 1, nv, nv))
    for k in range(N + 1):
        W[k] = np.diag(np.concatenate([rng.uniform(0.5, 2.0, nx), [0.3], [0.05]]))
    w = 1.5 * rng.standard_normal((N + 1, nv))
    xlb = np.full((N + 1, nx), -2.0); xub = np.full((N + 1, nx), 2.0)
    ulb = np.full((N, nu), -0.3); uub = np.full((N, nu), 0.3)
    Fp = rng.standard_normal((6, nv)); Fp[:, nx:nx + nu] = 0.0
    Fp /= np.linalg.norm(Fp, axis=1, keepdims=True)
    Fp[:2] = 0.0; Fp[0, -1] = 1.0; Fp[1, -1] = -1.0    # |theta| <= hp: binds (theta* ~ -0.2)
    hp = np.full(6, 0.1)
    prob = bqp.OcpProblem(A, B, W, N, npar, w=w, c=c, xlb=xlb, xub=xub, ulb=ulb, uub=uub,
                          Fp=Fp, hp=hp, poly_stage=N)
    d = dict(nx=nx, nu=nu, np=npar, N=N, W=W, w=w, A=A, B=B, c=c, xlb=xlb, xub=xub, ulb=ulb,
             uub=uub, kp=N, Fp=Fp, hp=hp)
    X0 = rng.uniform(-1.5, 1.5, (8, nx))
    HP = hp + rng.uniform(0.0, 0.1, (8, 6))
    return prob, d, X0, HP


def test_condensed_route_host_pieces():
    """the condensed route's host side (bqp.ocp.condensed_rhs with per-instance hp, trajectory
    and cost recovery) on an odd-dimension problem: the oracle's dense solve of the condensed QP
    equals the oracle's stage-wise Riccati IPM (oracle/ocp_ipm.py) on the same instance"""
    from bqp.ocp import condensed_rhs
    from oracle import dense_qp, ocp_ipm
    prob, d, X0, HP = odd_dims_problem()
    cd, f, b = condensed_rhs(prob, X0, HP)
    assert cd.n == prob.N * prob.nu + prob.np
    for i in range(len(X0)):
        qp = dict(H=cd.H, f=f[i], A=cd.A, b=b[i], Aeq=np.zeros((0, cd.n)), beq=np.zeros(0),
                  lb=np.full(cd.n, -np.inf), ub=np.full(cd.n, np.inf))
        z, fv, lam, info = dense_qp.solve(qp)
        u, th, x = cd.recover(z[None], X0[i:i + 1])
        r = ocp_ipm.solve(dict(d, hp=HP[i]), X0[i])
        assert r['exitflag'] == 1
        assert np.abs(u[0] - r['u']).max() < 1e-7
        assert np.abs(th[0] - r['theta']).max() < 1e-7
        assert np.abs(x[0] - r['x']).max() < 1e-7
