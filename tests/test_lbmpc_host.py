"""Learning-based MPC on the CPU side: the oracle's restatement (oracle/lbmpc.py) pinned to the
reference's stored IPOPT solution of the hybrid LBMPC instance (examples/DSS_NMPC.m, y_OL), the
NW oracle's derivative, and the host shim's condensing of the nominal constraints."""
import numpy as np
import pytest

from conftest import golden


@pytest.fixture(scope='module')
def inst():
    return golden('lbmpc_instance.npz')


def _f4(mg, g):
    from oracle import lbmpc
    return lbmpc.f4_problem(mg, int(g['N']), g['data'], g['F_w_N'], g['h_w_N'], g['F_x_d'],
                            g['h_x_d'], float(g['delta']))


def test_nw_gradient_matches_finite_differences():
    from oracle import lbmpc
    td = golden('train_data.npz')['data'][:, :100]
    rng = np.random.default_rng(1)
    for _ in range(5):
        xi = td[:3, rng.integers(100)] + 0.05 * rng.standard_normal(3)
        g, dg = lbmpc.nw(xi, td)
        for c in range(3):
            e = np.zeros(3); e[c] = 1e-6
            fd = (lbmpc.nw(xi + e, td)[0] - lbmpc.nw(xi - e, td)[0]) / 2e-6
            assert np.abs(fd - dg[:, c]).max() < 1e-6 * max(1.0, np.abs(dg).max())


def test_f4_restatement_vs_ipopt(mg, inst):
    """hybrid_LBMPC_casadi.m at iteration 100 (N=100, 7x100 window): the restated NLP evaluated
    at IPOPT's y_OL, and the GN-SQP optimum vs y_OL.  IPOPT stopped at its own tolerance
    (constraint violation 9.9e-9, five near-active rows with slack <= 7e-7), so the pin is on
    the cost (<= 2e-6), the first move (<= 2e-5) and the strongly active set."""
    from oracle import lbmpc
    p = _f4(mg, inst)
    x0 = inst['lb'][:4] - mg['x_wp']
    y = inst['y_OL']
    zI = np.concatenate([y[404:504] - mg['u_wp'], y[504:]])
    # the nominal chain of y_OL is the reference's equality constraint (hybrid...m:283)
    assert np.abs(lbmpc.f4_to_y(p, x0, zI, mg['x_wp'], mg['u_wp']) - y).max() < 1e-12
    A, b = lbmpc.constraints(p, x0)
    assert (A @ zI - b).max() < 1e-8
    z, lam, info = lbmpc.sqp(p, x0)
    assert info['stat'] < 1e-8
    assert (A @ z - b).max() < 1e-10
    assert abs(lbmpc.cost(p, x0, z) - lbmpc.cost(p, x0, zI)) < 2e-6
    assert abs(z[0] - zI[0]) < 2e-5
    strong = np.flatnonzero(lam > 1e-3)
    assert np.all(b[strong] - A[strong] @ zI < 1e-6)


def test_shim_condensing_matches_restatement(mg, inst):
    import bqp
    from oracle import lbmpc
    g = inst
    N = 10
    td = golden('train_data.npz')['data'][:, :100]
    shim = bqp.LBMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                     mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                     g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], N=N)
    p = lbmpc.f3_problem(mg, N, td, g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'])
    for x0 in (np.array([-0.35, -0.4, 0, 0]), np.array([0.1, -0.2, 0.3, -1.0])):
        A, b = lbmpc.constraints(p, x0)
        assert np.allclose(shim.Ain, A, atol=1e-13)
        assert np.allclose(shim.b0 + shim.Bx @ x0, b, atol=1e-13)
    hy = bqp.HybridLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                         mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], g['F_w_N'],
                         g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'], mg['u_wp'], N=100)
    p4 = _f4(mg, g)
    x0 = g['lb'][:4] - mg['x_wp']
    A, b = lbmpc.constraints(p4, x0)
    assert np.allclose(hy.Ain, A, atol=1e-12)
    assert np.allclose(hy.b0 + hy.Bx @ x0, b, atol=1e-12)


def test_f3_sqp_converges(mg, inst):
    """config C1 (MG LBMPC N=10, window = train_data(:, 1:100)): KKT point, feasible."""
    from oracle import lbmpc
    td = golden('train_data.npz')['data'][:, :100]
    p = lbmpc.f3_problem(mg, 10, td, inst['F_w_N'], inst['h_w_N'], inst['F_x_d'], inst['h_x_d'])
    for x0 in (np.array([-0.35, -0.4, 0, 0]), np.array([-0.2, -0.1, 0.05, 0.1])):
        z, lam, info = lbmpc.sqp(p, x0)
        A, b = lbmpc.constraints(p, x0)
        assert info['stat'] < 1e-8 and (A @ z - b).max() < 1e-10 and lam.min() >= -1e-12
