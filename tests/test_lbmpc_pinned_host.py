"""CPU: the F3 fixtures (oracle/make_lbmpc_fixtures.py) - the oracle's LBMPC restatement agrees
with fmincon's stored closed-loop moves (LBMPC_N{40,50}_sys_full.mat), and the window
reconstruction follows update_data.m (window sizes, the zero point leaving at solve 100)."""
import numpy as np
import pytest

from conftest import golden


@pytest.mark.parametrize('N', [40, 50])
def test_fixture_agreement(N):
    f = golden('lbmpc_N%d.npz' % N)
    assert f['early_err_vs_matlab'].max() < 5e-7
    assert np.median(f['late_err_vs_matlab']) < 1e-7 and f['late_err_vs_matlab'].max() < 2e-6
    for k in f['early_k']:
        w = f['window_%d' % k]
        assert w.shape == (7, k)
        assert np.all(w[:, 0] == 0)                      # the initial zero point
    assert f['late_windows'].shape[1:] == (7, 99) and np.all(f['late_k'] >= 100)
    assert np.all(f['late_windows'][:, :, 0] != 0)        # zero point dropped at solve 100


def test_solve1_is_the_qp(mg):
    """Solve 1 (zero window): the restated SQP reproduces fmincon's first move, g_NW = 0."""
    from oracle import lbmpc
    f = golden('lbmpc_N40.npz')
    g = golden('lbmpc_instance.npz')
    i = list(f['early_k']).index(1)
    p = lbmpc.f3_problem(mg, 40, f['window_1'], g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'])
    z, lam, info = lbmpc.sqp(p, f['early_dx'][i])
    assert abs(mg['K'].ravel() @ f['early_dx'][i] + z[0] - f['early_du_matlab'][i]) < 1e-7
    gz, _ = lbmpc.nw(np.array([0.1, -0.2, 0.3]), f['window_1'])
    assert np.all(gz == 0)
