"""GPU learned-model NLP closed loop (bqp.closed_loop_sqp -> bqp_closed_loop_sqp: the GN-SQP
kernels with the masked NW window, the RK4 plant kernel and get_data.m's window update per step)
against the reference's stored runs of examples/DMS_LBMPC_casadi.m (tests/golden/
dms_lbmpc_loops.npz) and against the oracle's restatement (oracle/lbmpc.py dms_lbmpc_loop)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _dms(mg, N=100):
    import bqp
    g = golden('lbmpc_instance.npz')
    return bqp.DMSLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                        mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], g['F_w_N'],
                        g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'], mg['u_wp'], N=N)


X_INIT = np.array([0.15, 1.2875, 1.1547, 0.0])


def test_dms_lbmpc_loop_vs_stored_q100(mg):
    """DMS_LBMPC_casadi.m as written (q = 100, 8 x q window): the GPU loop regenerates the stored
    plant trajectory DMS_tLBMPC_q100.mat"""
    import bqp
    st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC_q100']
    T = 40
    r = bqp.closed_loop_sqp(_dms(mg), X_INIT, T, learning=dict(q=100, mask=1))
    assert (r.exitflag == 1).all(), r.exitflag
    e = np.abs(r.X[0] - st[:T + 1])
    assert e[:4].max() < 5e-6, e[:4].max(axis=1)
    assert e[:, :2].max() < 1e-4, e[:, :2].max()


def test_dms_lbmpc_loop_vs_oracle(mg):
    """a batch of perturbed initial states: every instance's first moves equal the oracle's
    restatement of the loop (same algorithm, GN-SQP to a KKT point)"""
    import bqp
    from oracle import lbmpc
    sets = golden('lbmpc_instance.npz')
    rng = np.random.default_rng(11)
    B, T = 16, 3
    X0 = X_INIT + rng.uniform(-1, 1, (B, 4)) * np.array([0.02, 0.02, 0.0, 0.0])
    r = bqp.closed_loop_sqp(_dms(mg), X0, T, learning=dict(q=100, mask=1))
    assert (r.exitflag == 1).all(), r.exitflag
    for b in (0, 7):
        Xo, Uo, _, _ = lbmpc.dms_lbmpc_loop(mg, sets, 100, 100, T, x_init=X0[b])
        assert np.abs(r.U[b, :, 0] - Uo).max() < 1e-6, (b, r.U[b, :, 0] - Uo)
        assert np.abs(r.X[b] - Xo).max() < 1e-7


def test_dms_lbmpc_unmasked_window_vs_stored(mg):
    """the same cost with a 7-row window whose zero points count (mask = 0, q = 10) reproduces
    the stored DMS_tLBMPC.mat (its first learned move: x4 3.1073)"""
    import bqp
    st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC']
    T = 3
    r = bqp.closed_loop_sqp(_dms(mg), X_INIT, T, learning=dict(q=10, mask=0))
    assert (r.exitflag == 1).all(), r.exitflag
    assert np.abs(r.X[0] - st[:T + 1]).max() < 5e-6, np.abs(r.X[0] - st[:T + 1]).max(axis=1)
