"""CPU pin of the learned-model NLP closed loop examples/DMS_LBMPC_casadi.m against the
reference's stored runs (tests/golden/dms_lbmpc_loops.npz, oracle/make_dms_lbmpc_fixture.py):
the oracle's restatement (oracle/lbmpc.py: dms_problem / dms_lbmpc_loop - cost on the learned
states incl. the terminal term, 8 x q window with casadiL2NW.m's validity row, get_data.m)
reproduces the stored plant trajectory DMS_tLBMPC_q100.mat; the masked NW sums and their
derivative are checked against finite differences."""
import numpy as np

from conftest import golden


def test_masked_nw_derivative():
    from oracle import lbmpc
    rng = np.random.default_rng(5)
    data = np.zeros((8, 12))
    data[:3, :7] = rng.standard_normal((3, 7)) * 0.3
    data[3:7, :7] = rng.standard_normal((4, 7)) * 0.01
    data[7, :7] = 1.0
    xi = rng.standard_normal(3) * 0.2
    g, dg = lbmpc.nw_window(xi, data)
    # casadiL2NW.m literally: numerator over every point, normaliser over the valid ones
    k = np.exp(-np.sum((data[:3] - xi[:, None]) ** 2, axis=0) / 0.25)
    assert np.allclose(g, data[3:7] @ k / (1e-3 + k @ data[7]), rtol=1e-14, atol=1e-17)
    # the invalid points (Y = 0) leave g unchanged when dropped
    g7, _ = lbmpc.nw(xi, data[:7, :7])
    assert np.allclose(g, g7, rtol=1e-13, atol=1e-17)
    h = 1e-6
    for c in range(3):
        e = np.zeros(3); e[c] = h
        fd = (lbmpc.nw_window(xi + e, data)[0] - lbmpc.nw_window(xi - e, data)[0]) / (2 * h)
        assert np.allclose(dg[:, c], fd, rtol=1e-6, atol=1e-10)


def test_dms_lbmpc_loop_reproduces_stored_q100(mg):
    """the first three closed-loop states of DMS_tLBMPC_q100.mat: the learned correction enters
    at step 2 (x4 4.154 against 3.041 without learning, a 1.1 difference) and the restatement
    follows it to IPOPT's tolerance"""
    from oracle import lbmpc
    st = golden('dms_lbmpc_loops.npz')
    sets = golden('lbmpc_instance.npz')
    X, U, Z, IT = lbmpc.dms_lbmpc_loop(mg, sets, 100, 100, 3)
    ref = st['DMS_tLBMPC_q100'][:4]
    assert np.abs(X - ref).max() < 5e-6, np.abs(X - ref).max(axis=1)
    assert abs(X[2, 3] - 3.0406) > 1.0          # not the nominal (LMPC) move
