"""GPU learned-model NLP closed loop (bqp.closed_loop_sqp -> bqp_closed_loop_sqp: the GN-SQP
kernels with the masked NW window, the RK4 plant kernel and get_data.m's window update per step)
against the reference's stored runs of examples/DMS_LBMPC_casadi.m (tests/golden/
dms_lbmpc_loops.npz) and against the oracle's restatement of the loop (oracle/lbmpc.py
dms_lbmpc_loop, fixture tests/golden/dms_lbmpc_oracle.npz from oracle/make_dms_oracle_fixture.py).

Tolerances: the stored runs are IPOPT solutions (its default tol 1e-8 on the scaled NLP); the
throttle-rate state x4 = 1000 delta u amplifies a first-move difference tenfold.  The GN-SQP stops
at |d| <= tol (1 + |z|) with the KKT test, or once its step is below 1e-6 with the cost stagnant
(bqp_lbmpc.hip lbmpc_update_kernel), so first moves agree with the oracle's tighter stop
(|d| <= 1e-10) to ~1e-6."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _mpc(mg, cls='DMSLBMPC', N=100):
    import bqp
    g = golden('lbmpc_instance.npz')
    return getattr(bqp, cls)(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                             mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                             g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'],
                             mg['u_wp'], N=N)


X_INIT = np.array([0.15, 1.2875, 1.1547, 0.0])


def test_dms_lbmpc_loop_vs_stored_q100(mg):
    """DMS_LBMPC_casadi.m as written (q = 100, 8 x q window): the GPU loop regenerates the stored
    plant trajectory DMS_tLBMPC_q100.mat over its whole length (499 steps,
    DMS_LBMPC_casadi.m:81 mpciterations = 500) - the learned correction moves x4 at step 2 by 1.1
    away from the nominal (LMPC) loop.  The C restatement's loop (oracle/cpu_lbmpc.c) gives slow
    states 7.4e-8, all states 1.1e-4 in the transient (x4 = 1000 delta u amplifies the IPOPT
    tolerance of the stored moves), 3.6e-7 from step 200 on; the GPU loop is held to the same
    bars."""
    import bqp
    st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC_q100']
    T = len(st) - 1
    r = bqp.closed_loop_sqp(_mpc(mg), X_INIT, T, learning=dict(q=100, mask=1))
    assert (r.exitflag == 1).all(), r.exitflag
    e = np.abs(r.X[0] - st[:T + 1])
    print('DMS_tLBMPC_q100 over %d steps: slow %.2e, all %.2e, k >= 200 %.2e; SQP iterations mean '
          '%.2f max %d' % (T, e[:, :2].max(), e.max(), e[200:].max(), r.iterations.mean(),
                           r.iterations.max()))
    assert e[:, :2].max() < 1e-6, e[:, :2].max()
    assert e.max() < 5e-4, e.max(axis=1)
    assert e[200:].max() < 1e-5
    # the early steps, before the transient amplifies IPOPT's stopping tolerance (the round-3 bars
    # over 25 steps; C restatement: slow 1.4e-8, all 1.05e-5)
    assert e[:26, :2].max() < 1e-7, e[:26, :2].max()
    assert e[:26].max() < 3e-5, e[:26].max(axis=1)
    assert abs(r.X[0, 2, 3] - 3.0406) > 1.0
    # the logged learned one-step predictions: x_eq + A dx + B du + g with the window before the
    # update (DMS_LBMPC_casadi.m:199)
    from oracle import lbmpc
    XL, _ = lbmpc.window_replay(r.X[0], r.U[0, :, 0], mg['A'], mg['B'], mg['x_wp'], mg['u_wp'], 100)
    assert np.abs(r.XL[0] - XL).max() < 1e-12


def test_dms_lbmpc_loop_vs_oracle(mg):
    """16 initial states around x_init: every instance's closed loop equals the oracle's
    restatement of the loop (same GN-SQP; first moves to the SQP's stopping accuracy)"""
    import bqp
    o = golden('dms_lbmpc_oracle.npz')
    T = int(o['steps'])
    r = bqp.closed_loop_sqp(_mpc(mg), o['x0'], T, learning=dict(q=100, mask=1))
    assert (r.exitflag == 1).all(), r.exitflag
    du = np.abs(r.U[:, :, 0] - o['U'])
    assert du.max() < 2e-6, du.max(axis=0)
    assert np.median(du) < 5e-7
    assert np.abs(r.X - o['X'])[:, :, :2].max() < 1e-8


def test_hybrid_lbmpc_loop_vs_oracle(mg):
    """the hybrid cost (hybrid_LBMPC_casadi.m:250-311: terminal term on the nominal x_N) in the
    same loop with a 7-row window whose points all count (mask 0) vs the oracle's loop"""
    import bqp
    o = golden('dms_lbmpc_oracle.npz')
    T = int(o['steps'])
    r = bqp.closed_loop_sqp(_mpc(mg, 'HybridLBMPC'), X_INIT, T, learning=dict(q=100, mask=0))
    assert (r.exitflag == 1).all(), r.exitflag
    assert np.abs(r.U[0, :, 0] - o['hyb_U']).max() < 2e-6
    assert np.abs(r.X[0] - o['hyb_X']).max() < 2e-5


# every stored learned-model run of the reference and the window it was made with
# (tools/diag_learned_loops.py; the 8-row masked window does not depend on q until it wraps)
STORED = [('DMS_tLBMPC_q10', 100, 10, 1), ('DMS_tLBMPC_q50', 100, 50, 1),
          ('DMS_tLBMPC_q500', 100, 500, 0), ('DMS_tLBMPC', 100, 10, 0),
          ('DMS_N50_tLBMPC_q10', 50, 10, 1), ('DMS_N50_tLBMPC_q100', 50, 100, 1)]


@pytest.mark.parametrize('name,N,q,mask', STORED)
def test_stored_learned_loops(mg, name, N, q, mask):
    """DMS_LBMPC_casadi.m with the horizon and window of each stored run (mask 0: a 7-row window
    whose zero points count, the variant that made DMS_tLBMPC.mat and the q = 500 run) over the
    stored run's whole length (499 steps).  The C restatement's loop over the
    same runs (round 5): slow states <= 3.2e-7, all states <= 1.9e-4 (transient), <= 1.6e-6 from
    step 200 on"""
    import bqp
    st = golden('dms_lbmpc_loops.npz')[name]
    T = len(st) - 1
    r = bqp.closed_loop_sqp(_mpc(mg, N=N), X_INIT, T, learning=dict(q=q, mask=mask))
    assert (r.exitflag == 1).all(), r.exitflag
    e = np.abs(r.X[0] - st[:T + 1])
    print('%s over %d steps: slow %.2e, all %.2e, k >= 200 %.2e; SQP iterations mean %.2f max %d'
          % (name, T, e[:, :2].max(), e.max(), e[200:].max(), r.iterations.mean(), r.iterations.max()))
    assert e[:, :2].max() < 1e-6 and e.max() < 5e-4, e.max(axis=1)
    assert e[200:].max() < 1e-5
    # the first 25 steps at the round-3 bars (slow 1e-7, all 5e-5; C restatement over these runs:
    # slow <= 4.1e-8, all <= 3.13e-5 - the q = 500 run)
    assert e[:26, :2].max() < 1e-7 and e[:26].max() < 5e-5, e[:26].max(axis=1)


def test_dms_lbmpc_loop_vs_c_restatement(mg):
    """the GPU loop against the C restatement of the same algorithm (oracle/cpu_lbmpc.c, bench.py's
    CLL CPU baseline) on 32 perturbed initial states of the CLL bench workload, 6 steps"""
    import bqp
    from oracle import cpu_lbmpc
    rng = np.random.default_rng(11)
    X0 = X_INIT + rng.uniform(-1, 1, (32, 4)) * np.array([0.005, 0.005, 0.0, 0.0])
    T = 6
    r = bqp.closed_loop_sqp(_mpc(mg), X0, T, learning=dict(q=100, mask=1))
    Xc, Uc, itc, flc = cpu_lbmpc.loop(mg, dict(golden('lbmpc_instance.npz')), 100, 100, T, X0, threads=4)
    assert (r.exitflag == 1).all() and (flc == 1).all()
    e = np.abs(r.X - Xc)
    print('GPU loop vs C restatement: slow %.2e, all %.2e; SQP iterations GPU %.2f C %.2f'
          % (e[..., :2].max(), e.max(), r.iterations.mean(), itc.mean()))
    assert e[..., :2].max() < 1e-7
    assert e.max() < 1e-4


def test_indefinite_hessian_instance(mg):
    """the +-0.02 DMS instance whose exact Hessian is indefinite at its third
    closed-loop step (tests/golden/dms_indefinite.npz from oracle/make_indefinite_fixture.py): the
    GPU SQP shifts it by the smallest grid delta that makes it positive definite
    (lbmpc_hess_kernel) and ends every step within 20 SQP iterations at the oracle's first moves
    (1e-6); with the Gauss-Newton fallback this step ran into the 200-iteration limit"""
    import bqp
    f = golden('dms_indefinite.npz')
    r = bqp.closed_loop_sqp(_mpc(mg), f['x0'][None], 3, learning=dict(q=100, mask=1))
    print('indefinite instance: SQP iterations', r.iterations[0].tolist(), 'oracle',
          f['iterations'].tolist(), '|U - U_oracle|', np.abs(r.U[0, :, 0] - f['U']).tolist())
    assert (r.exitflag == 1).all(), r.exitflag
    assert r.iterations.max() <= 20
    assert np.abs(r.U[0, :, 0] - f['U']).max() < 1e-6


@pytest.mark.parametrize('polish,max_iter', [(0, 200), (1, 200), (-1, 200), (0, 3)])
def test_async_loop_equals_step_synchronous(mg, polish, max_iter):
    """bqp_closed_loop_sqp runs every instance at its own closed-loop step (round 5: the instances
    whose SQP has finished advance while the others iterate).  Per instance it performs the same
    operations in the same order as the step-synchronous loop (selected by BQP_LB_SYNC, which is
    not a tracing path: no host syncs or output beyond the step loop's own), so the trajectories,
    the learned predictions, the windows and the SQP iteration counts are equal bit for bit on 24
    perturbed instances over 6 steps - with the loop's default polish (3: only once an SQP
    stalls, then every converged sub-problem: the per-instance pol_it path), polish 1 (also every
    0 / -8 sub-problem exit), polish off (-1), and with max_iter = 3 so that the advance kernel also runs after SQP exits that
    did not converge"""
    import os
    import bqp
    rng = np.random.default_rng(11)
    X0 = X_INIT + rng.uniform(-1, 1, (24, 4)) * np.array([0.02, 0.02, 0.0, 0.0])
    T = 6
    kw = dict(learning=dict(q=100, mask=1), log_z=True, polish=polish, max_iter=max_iter)
    ra = bqp.closed_loop_sqp(_mpc(mg), X0, T, **kw)
    os.environ['BQP_LB_SYNC'] = '1'
    try:
        rs = bqp.closed_loop_sqp(_mpc(mg), X0, T, **kw)
    finally:
        del os.environ['BQP_LB_SYNC']
    print('polish %d max_iter %d: async vs synchronous loop: SQP iterations per step %s, max per '
          'step %s, flags %s' % (polish, max_iter, ra.iterations.sum(axis=0).tolist(),
                                 ra.iterations.max(axis=0).tolist(),
                                 np.unique(ra.exitflag, return_counts=True)))
    if max_iter == 3:
        assert (ra.exitflag != 1).any()          # some SQP exits at the iteration limit
    for k in ('X', 'U', 'XL', 'window', 'Z', 'iterations', 'exitflag'):
        assert np.array_equal(ra[k], rs[k]), k
