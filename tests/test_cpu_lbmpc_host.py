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
    st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC_q100']
    T = 25
    X, U, its, flags = _loop(mg, X_INIT[None], T)
    assert (flags == 1).all()
    e = np.abs(X[0] - st[:T + 1])
    print('C loop vs DMS_tLBMPC_q100: slow %.2e, all %.2e, SQP iterations %s'
          % (e[:, :2].max(), e.max(), its[0].tolist()))
    assert e[:, :2].max() < 1e-7
    assert e.max() < 1e-4


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
