"""GPU: the fmincon LBMPC path (form F3, ocpLBMPC.m:27-31, config C1's problem) pinned to the
reference's own stored closed loops LBMPC_N{40,50}_sys_full.mat (tests/golden/lbmpc_N*.npz,
oracle/make_lbmpc_fixtures.py): at each stored solve, the state, the data window rebuilt from
sysH by ocpLBMPC.m:12-19 / update_data.m:3-10 and fmincon's applied move du_k = sysH(5,k+1).

Solve 1 (zero window, g_NW = 0) is exactly a QP; the others are the learned-model NLP.  The GPU
SQP (bqp_lbmpc_solve_batched) must agree with the oracle's restated SQP (first move and theta
to 1e-8, the whole decision to 1e-6) and with
fmincon's move within the agreement the oracle itself reaches on that solve (+1e-7)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


def _lbmpc(mg, N):
    import bqp
    g = golden('lbmpc_instance.npz')
    return bqp.LBMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                     mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                     g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], N=N)


def _check(r, dx, du_m, z_or, err_or, K):
    assert (r.exitflag == 1).all(), (r.exitflag, r.iterations)
    du = dx @ K.ravel() + r.z[:, 0]
    # first move and theta to 1e-8; the last inputs are weakly determined (no running cost
    # on them, costLBMPC.m:30: only the terminal cost sees them), both SQPs stop at their own
    # tolerance there
    assert np.abs(r.z[:, 0] - z_or[:, 0]).max() < 1e-8
    assert np.abs(r.z[:, -1] - z_or[:, -1]).max() < 1e-8
    assert np.abs(r.z - z_or).max() < 1e-6, np.abs(r.z - z_or).max(axis=1)
    assert (np.abs(du - du_m) <= err_or + 1e-7).all(), np.abs(du - du_m) - err_or


@pytest.mark.parametrize('N', [40, 50])
def test_f3_early_solves_vs_fmincon(mg, handle, N):
    """solves with growing windows (one window size each): 1 (QP), 2, 3, 5, 10, 30, 60, 99"""
    f = golden('lbmpc_N%d.npz' % N)
    lb = _lbmpc(mg, N)
    for i, k in enumerate(f['early_k']):
        r = lb.solve(f['early_dx'][i:i + 1], f['window_%d' % k], handle=handle, max_iter=100)
        _check(r, f['early_dx'][i:i + 1], f['early_du_matlab'][i:i + 1],
               f['early_z_oracle'][i:i + 1], f['early_err_vs_matlab'][i:i + 1], mg['K'])


@pytest.mark.parametrize('N', [40, 50])
def test_f3_late_solves_batched(mg, handle, N):
    """32 solves past the window fill (99 points each) in ONE batched call, per-instance windows"""
    f = golden('lbmpc_N%d.npz' % N)
    lb = _lbmpc(mg, N)
    r = lb.solve(f['late_dx'], f['late_windows'], handle=handle, max_iter=100)
    _check(r, f['late_dx'], f['late_du_matlab'], f['late_z_oracle'], f['late_err_vs_matlab'],
           mg['K'])
