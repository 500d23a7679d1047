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
