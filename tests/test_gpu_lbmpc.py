"""GPU parity of the learning-based MPC path (bqp_nw_oracle, bqp_lbmpc_solve_batched through the
C ABI) against the oracle's restatement (oracle/lbmpc.py) and the reference's stored IPOPT
solution of the hybrid LBMPC instance (examples/DSS_NMPC.m)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


@pytest.fixture(scope='module')
def inst():
    return golden('lbmpc_instance.npz')


def test_nw_oracle_kernel(handle):
    """oracleL2NW.m: g and dg/dxi at 256 query points, shared and per-instance windows."""
    import bqp
    from oracle import lbmpc
    td = golden('train_data.npz')['data']
    rng = np.random.default_rng(7)
    b = 256
    xi = td[:3, rng.integers(0, 500, b)].T + 0.05 * rng.standard_normal((b, 3))
    g, dg = bqp.nw_oracle(td[:, :100], xi, handle=handle)
    for i in range(b):
        gr, dgr = lbmpc.nw(xi[i], td[:, :100])
        assert np.abs(g[i] - gr).max() <= 1e-13 * max(1.0, np.abs(gr).max())
        assert np.abs(dg[i] - dgr).max() <= 1e-12 * max(1.0, np.abs(dgr).max())
    W = np.stack([td[:, s:s + 100] for s in rng.integers(0, 400, b)])      # per-instance windows
    g2, _ = bqp.nw_oracle(W, xi, handle=handle)
    for i in range(0, b, 17):
        assert np.abs(g2[i] - lbmpc.nw(xi[i], W[i])[0]).max() <= 1e-13
    # the zero-initialised window of LBMPC_RunExample.m:80-81 (g = 0)
    g0, dg0 = bqp.nw_oracle(np.zeros((7, 1)), xi[:4], handle=handle)
    assert np.all(g0 == 0) and np.all(dg0 == 0)


def _lbmpc(mg, g, N):
    import bqp
    return bqp.LBMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                     mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                     g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], N=N)


def test_f3_lbmpc_c1_vs_restatement(mg, inst, handle):
    """config C1 (fmincon LBMPC, N=10, window train_data(:,1:100)): GPU SQP == oracle SQP."""
    from oracle import lbmpc
    td = golden('train_data.npz')['data'][:, :100]
    N = 10
    lb = _lbmpc(mg, inst, N)
    X0 = np.array([[-0.35, -0.4, 0, 0], [-0.2, -0.1, 0.05, 0.1], [0.0, 0.0, 0.0, 0.0],
                   [-0.1, 0.05, -0.02, 0.3]])
    r = lb.solve(X0, td, handle=handle)
    assert (r.exitflag == 1).all(), (r.exitflag, r.iterations)
    p = lbmpc.f3_problem(mg, N, td, inst['F_w_N'], inst['h_w_N'], inst['F_x_d'], inst['h_x_d'])
    for i, x0 in enumerate(X0):
        z, lam, info = lbmpc.sqp(p, x0)
        assert np.abs(r.z[i] - z).max() < 1e-7, np.abs(r.z[i] - z).max()
        assert abs(r.cost[i] - lbmpc.cost(p, x0, r.z[i])) < 1e-10 * max(1, abs(r.cost[i]))
        A, b = lbmpc.constraints(p, x0)
        assert (A @ r.z[i] - b).max() < 1e-9
        H, f = lbmpc.gn_model(p, x0, r.z[i])
        assert np.abs(f + A.T @ r.lam[i]).max() < 1e-6 * (1 + np.abs(f).max())


def test_f4_hybrid_lbmpc_vs_ipopt(mg, inst, handle):
    """hybrid_LBMPC_casadi.m iteration-100 instance (N=100): GPU == oracle SQP, and vs IPOPT's
    stored y_OL within IPOPT's own accuracy (see tests/test_lbmpc_host.py)."""
    import bqp
    from oracle import lbmpc
    g = inst
    hy = bqp.HybridLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                         mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], g['F_w_N'],
                         g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'], mg['u_wp'], N=100)
    xm = g['lb'][:4]
    r = hy.solve(xm, g['data'], handle=handle)
    assert r.exitflag[0] == 1, (r.exitflag, r.iterations)
    p = lbmpc.f4_problem(mg, 100, g['data'], g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], 0.01)
    x0 = xm - mg['x_wp']
    z, lam, info = lbmpc.sqp(p, x0)
    assert np.abs(r.z[0] - z).max() < 1e-6
    y = g['y_OL']
    zI = np.concatenate([y[404:504] - mg['u_wp'], y[504:]])
    assert abs(r.cost[0] - lbmpc.cost(p, x0, zI)) < 2e-6
    assert abs(r.u0[0, 0] - y[404]) < 2e-5
    assert np.abs(r.y_OL[0, :4] - y[:4]).max() < 1e-15


def test_batch_independence(mg, inst, handle):
    """a batch of 64 instances with per-instance windows == each solved alone"""
    td = golden('train_data.npz')['data']
    rng = np.random.default_rng(3)
    b = 64
    W = np.stack([td[:, s:s + 100] for s in rng.integers(0, 400, b)])
    X0 = np.column_stack([rng.uniform(-0.35, 0.0, b), rng.uniform(-0.4, 0.0, b),
                          0.01 * rng.standard_normal(b), 0.1 * rng.standard_normal(b)])
    lb = _lbmpc(mg, inst, 10)
    r = lb.solve(X0, W, handle=handle)
    assert (r.exitflag == 1).mean() > 0.9
    for i in range(0, b, 13):
        ri = lb.solve(X0[i:i + 1], W[i], handle=handle)
        assert ri.exitflag[0] == r.exitflag[i]
        assert ri.iterations[0] == r.iterations[i]
        # b_in = b0 + Bx x0 is formed by numpy on the host, whose matmul may round differently
        # for a (1, 4) and a (64, 4) operand: agreement to round-off, same iteration path
        assert np.abs(ri.z[0] - r.z[i]).max() < 1e-13
