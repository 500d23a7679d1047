"""The C restatement of the learned-model NLP closed loop (oracle/cpu_lbmpc.c - bench.py's CLL
CPU baseline) against the reference's stored run of examples/DMS_LBMPC_casadi.m
(DMS_tLBMPC_q100.mat, tests/golden/dms_lbmpc_loops.npz) and the numpy restatement's loop
(tests/golden/dms_lbmpc_oracle.npz).  Same tolerances as the GPU loop tests
(tests/test_gpu_lbmpc_dms.py): IPOPT's stop on the stored run, the throttle-rate state x4
amplifying first-move differences."""
import numpy as np

from conftest import golden

X_INIT = np.array([0.15, 1.2875, 1.1547, 0.0])


def _loop(mg, x0, steps, **kw):
    from oracle import cpu_lbmpc
    return cpu_lbmpc.loop(mg, dict(golden('lbmpc_instance.npz')), 100, 100, steps, x0, **kw)


def test_cpu_loop_vs_stored_q100(mg):
    """the whole stored run (499 steps, DMS_LBMPC_casadi.m:81; ~20 s on one core): slow states
    7.4e-8, all states 1.1e-4 in the transient, 3.6e-7 from step 200 on (round 5; the same loop
    over every stored learned run: tests/test_gpu_lbmpc_dms.py)"""
    st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC_q100']
    T = len(st) - 1
    X, U, its, flags = _loop(mg, X_INIT[None], T, threads=1)
    assert (flags == 1).all()
    e = np.abs(X[0] - st[:T + 1])
    print('C loop vs DMS_tLBMPC_q100 over %d steps: slow %.2e, all %.2e, k >= 200 %.2e; SQP '
          'iterations mean %.2f max %d' % (T, e[:, :2].max(), e.max(), e[200:].max(), its.mean(),
                                           its.max()))
    assert e[:, :2].max() < 1e-6
    assert e.max() < 5e-4
    assert e[200:].max() < 1e-5
    # the first 25 steps (measured 1.4e-8 / 1.05e-5)
    assert e[:26, :2].max() < 1e-7 and e[:26].max() < 3e-5


def test_cpu_loop_vs_numpy_oracle(mg):
    o = golden('dms_lbmpc_oracle.npz')
    T = int(o['steps'])
    Xo, x0 = o['X'], o['x0']
    X, U, its, flags = _loop(mg, x0, T)
    assert (flags == 1).all()
    e = np.abs(X - Xo)
    print('C loop vs numpy oracle: slow %.2e, all %.2e' % (e[..., :2].max(), e.max()))
    assert e[..., :2].max() < 1e-7
    assert e.max() < 1e-4


def test_cpu_loop_threads_identical(mg):
    """OpenMP over instances: each instance's loop is sequential, so thread counts agree bit for bit"""
    rng = np.random.default_rng(5)
    x0 = X_INIT + rng.uniform(-1, 1, (6, 4)) * np.array([0.005, 0.005, 0.0, 0.0])
    a = _loop(mg, x0, 2, threads=1)
    b = _loop(mg, x0, 2, threads=3)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_cpu_loop_indefinite_hessian(mg):
    """the +-0.02 instance whose exact Hessian is indefinite at its third step
    (tests/golden/dms_indefinite.npz, oracle/make_indefinite_fixture.py).  With the smallest grid
    shift that makes it positive definite (hess_shift_k) the C restatement ends every step within
    20 SQP iterations at the oracle's first moves (the Gauss-Newton fallback took 200 there and
    stopped 6e-5 away)."""
    f = golden('dms_indefinite.npz')
    X, U, its, flags = _loop(mg, f['x0'][None], 3, threads=1)
    assert (flags == 1).all()
    assert its.max() <= 20, its
    assert np.abs(U[0] - f['U']).max() < 1e-6, np.abs(U[0] - f['U'])
