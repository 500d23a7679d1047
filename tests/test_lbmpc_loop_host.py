"""CPU pin of the LBMPC closed loop (examples/LBMPC_casadi.m) against the reference's stored run
saved_data+plots/data/casadi/tLBMPC.mat (tests/golden/lbmpc_loop.npz): the loop of the C
restatement of the solver on the TrackingLBMPC problem (the DMS tracking cost with F_x_d and
the robust terminal set on x_1) and the RK4 plant reproduces the stored plant trajectory; the
data-window replay follows update_data.m / get_data.m."""
import numpy as np

from conftest import golden


def _problem(mg):
    import bqp
    g = golden('lbmpc_instance.npz')
    return bqp.TrackingLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                             mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                             g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'],
                             mg['u_wp'], N=100)


def test_lbmpc_casadi_loop_vs_stored(mg):
    from oracle import cpu_ref
    from oracle.mg_model import mg_rk4
    lp = golden('lbmpc_loop.npz')
    tl = _problem(mg)
    p = tl.prob
    ocp = dict(nx=4, nu=1, np=1, N=p.N, A=p.A, B=p.B, c=p.c, W=p.W, w=p.w, xlb=p.xlb, xub=p.xub,
               ulb=p.ulb, uub=p.uub, Fp=p.Fp, hp=p.hp, kp=p.poly_stage, const=0.0)
    xs = lp['xlo']
    x = xs[0].copy()
    X = [x]
    for k in range(len(xs) - 1):
        c = cpu_ref.solve(ocp, (x - tl.x_eq)[None])
        assert c['exitflag'][0] == 1
        x = mg_rk4(0.01, x, c['u'][0, 0, 0] + tl.u_eq[0])
        X.append(x)
    e = np.abs(np.array(X) - xs)
    # IPOPT's own tolerance and the chaotic throttle-rate state (tests/test_gpu_closed_loop.py):
    # slow states over the whole run, all states after the transient (measured 3.1e-6 / 6.9e-5)
    assert e[:, :2].max() < 1e-5, e[:, :2].max()
    assert e[150:].max() < 2e-4, e[150:].max()


def test_window_replay_follows_update_data():
    """window_replay against a literal list-based update_data.m (struct X, Y grown / shifted)"""
    from oracle import lbmpc
    rng = np.random.default_rng(3)
    T, q = 23, 8
    X = rng.standard_normal((T + 1, 4)) * 0.1
    U = rng.standard_normal(T) * 0.1
    A = np.eye(4) + 0.01 * rng.standard_normal((4, 4))
    B = rng.standard_normal(4) * 0.1
    XL, data = lbmpc.window_replay(X, U, A, B, np.zeros(4), np.zeros(1), q)
    Xs, Ys = [np.zeros(3)], [np.zeros(4)]                  # data.X = zeros(3,1), data.Y = zeros(4,1)
    for it in range(1, T + 1):
        t = it - 1
        nom = A @ X[t] + B * U[t]
        Dx = np.array(Xs).T; Dy = np.array(Ys).T
        k = np.exp(-np.sum((Dx - np.array([X[t, 0], X[t, 1], U[t]])[:, None]) ** 2, axis=0) / 0.25)
        assert np.allclose(XL[it], nom + Dy @ k / (1e-3 + k.sum()), rtol=1e-13, atol=1e-15)
        Xs.append(np.array([X[t, 0], X[t, 1], U[t]])); Ys.append(X[t + 1] - nom)
        if it >= q:                                          # update_data.m:9-10
            Xs.pop(0); Ys.pop(0)
    assert np.allclose(data[:3], np.array(Xs).T) and np.allclose(data[3:7], np.array(Ys).T)
