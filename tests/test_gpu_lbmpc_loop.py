"""GPU LBMPC closed loop with the learned model's data window (bqp_closed_loop_lbmpc,
SURVEY.md §8(f) row 2): the CasADi LBMPC run of the reference (examples/LBMPC_casadi.m, N=100,
500 steps, q = 100) regenerated on the GPU for a batch of initial states and compared with the
stored plant trajectory (tests/golden/lbmpc_loop.npz from tLBMPC.mat); the per-instance data
windows and learned predictions (update_data.m / get_data.m, casadiL2NW.m) against the oracle's
replay of the same closed-loop record."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _problem(mg):
    import bqp
    g = golden('lbmpc_instance.npz')
    return bqp.TrackingLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                             mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                             g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'],
                             mg['u_wp'], N=100)


def _ring_to_matlab(win, steps, q):
    """the kernel's ring (iteration it in point it mod q) -> get_data.m column order"""
    order = np.arange(q) if steps < q else (steps + 1 + np.arange(q)) % q
    return win[order].T


def test_lbmpc_loop_vs_stored(mg):
    import bqp
    from oracle import lbmpc
    lp = golden('lbmpc_loop.npz')
    xs = lp['xlo']
    T = len(xs) - 1
    tl = _problem(mg)
    X0 = xs[[0, 40, 120, 200, 300, 420, 460, 480]]
    r = bqp.closed_loop(tl, X0, T, delta=0.01, learning=dict(q=100, mask=1))
    assert (r.exitflag == 1).all()
    e = np.abs(r.X[0] - xs)
    print('LBMPC loop vs tLBMPC.mat: slow states max %.2e, all states k>=150 max %.2e'
          % (e[:, :2].max(), e[150:].max()))
    assert e[:, :2].max() < 1e-4
    assert e[150:].max() < 2e-4
    # data window and learned predictions: the oracle's replay of each instance's record
    for i in (0, 3, 7):
        XL, data = lbmpc.window_replay(r.X[i], r.U[i, :, 0], mg['A'], mg['B'], tl.x_eq, tl.u_eq, 100)
        assert np.abs(r.XL[i] - XL).max() < 1e-12 * max(1.0, np.abs(XL).max())
        assert np.abs(_ring_to_matlab(r.window[i], T, 100) - data).max() < 1e-13


@pytest.mark.parametrize('mask', [1, 0])
def test_window_wraps(mg, mask):
    """short horizon of the ring: q = 8 over 30 steps (wraps three times), both window kinds
    (validity row of get_data.m / every point counting, the 7-row window)"""
    import bqp
    from oracle import lbmpc
    lp = golden('lbmpc_loop.npz')
    tl = _problem(mg)
    X0 = lp['xlo'][[0, 10, 20, 30]]
    T, q = 30, 8
    r = bqp.closed_loop(tl, X0, T, delta=0.01, learning=dict(q=q, mask=mask))
    for i in range(len(X0)):
        XL, data = lbmpc.window_replay(r.X[i], r.U[i, :, 0], mg['A'], mg['B'], tl.x_eq, tl.u_eq,
                                       q, mask=bool(mask))
        assert np.abs(r.XL[i] - XL).max() < 1e-12 * max(1.0, np.abs(XL).max())
        assert np.abs(_ring_to_matlab(r.window[i], T, q) - data).max() < 1e-13
