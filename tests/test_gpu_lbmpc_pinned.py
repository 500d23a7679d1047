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


def test_f3_fmincon_loop_end_to_end(mg):
    """examples/LBMPC_RunExample.m's loop regenerated on the GPU (bqp_closed_loop_sqp): per step
    the F3 SQP at the measured state (ocpLBMPC.m:27-31), u = K dx + c_0 + u_wp to the true plant
    (transitionTrue.m -> models/trueModel.m: MATLAB ode23, BQP_PLANT_MG_ODE23), then the window
    update of ocpLBMPC.m:12-19 / update_data.m with q = 100 - which keeps q - 1 = 99 points once
    full (the initial zero point leaves when the 100th sample arrives), i.e. the loop's ring with
    q = 99 and the validity row.  1000 steps from the stored x_init against the stored run
    LBMPC_N40_sys_full.mat (column k + 1: the state of step k and fmincon's move)."""
    import bqp
    from oracle.mg_model import mg_ode23
    H = golden('fmincon_runs.npz')['LBMPC_N40']
    xwp = np.asarray(mg['x_wp'], float); uwp = np.ravel(mg['u_wp'])[:1].astype(float)
    lb = _lbmpc(mg, 40)
    Xs = H[:4, 1:].T + xwp                          # states of steps 1..1000
    Us = H[4, 1:] + uwp
    T = len(Us)
    r = bqp.closed_loop_sqp(lb, Xs[:1], T, learning=dict(q=99, mask=1), plant='ode23',
                            x_eq=xwp, u_eq=uwp)
    assert (r.exitflag == 1).all()
    ep = max(np.abs(mg_ode23(0.01, r.X[0, k], r.U[0, k, 0]) - r.X[0, k + 1]).max()
             for k in range(0, T, 9))
    e = np.abs(r.X[0, :T] - Xs)
    eu = np.abs(r.U[0, :, 0] - Us)
    print('LBMPC N=40 fmincon loop on the GPU: plant kernel vs restatement %.2e; vs '
          'LBMPC_N40_sys_full.mat: slow states %.2e, all states %.2e (k >= 200: %.2e), moves '
          'median %.2e max %.2e; SQP iterations mean %.2f max %d'
          % (ep, e[:, :2].max(), e.max(), e[200:].max(), np.median(eu), eu.max(),
             r.iterations.mean(), r.iterations.max()))
    assert ep < 1e-13
    assert e[:, :2].max() < 5e-3


@pytest.mark.parametrize('polish', [0, 2, 3])
def test_f3_polish_modes_single_solve(mg, handle, polish):
    """the sub-problem polish of bqp_lbmpc_solve_batched per bqp_options.polish - 0 (the
    C default) and 2 polish 0 / -8 sub-problem exits before the SQP stalls (LB_POLISH_STALL = 6
    iterations) and every sub-problem after it, 3 polishes only after the stall - all reach the
    pinned optimum of the 32 late F3 solves (same bars as test_f3_late_solves_batched)"""
    f = golden('lbmpc_N40.npz')
    lb = _lbmpc(mg, 40)
    r = lb.solve(f['late_dx'], f['late_windows'], handle=handle, max_iter=100, polish=polish)
    _check(r, f['late_dx'], f['late_du_matlab'], f['late_z_oracle'], f['late_err_vs_matlab'],
           mg['K'])
