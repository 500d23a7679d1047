"""Diagnostic (GPU): SQP iteration counts and exit flags of the DMS LBMPC closed loop
(bqp.closed_loop_sqp) for perturbed initial states against the oracle's loop
(oracle/lbmpc.py dms_lbmpc_loop), for a few (tol, max_iter) settings."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'learning-based-mpc_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import bqp  # noqa: E402
from conftest import golden  # noqa: E402
from oracle import lbmpc  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

mg = mg_problem()
g = golden('lbmpc_instance.npz')
dms = bqp.DMSLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                   mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], g['F_w_N'], g['h_w_N'],
                   g['F_x_d'], g['h_x_d'], mg['x_wp'], mg['u_wp'], N=100)
rng = np.random.default_rng(11)
B, T = 16, 3
X0 = np.array([0.15, 1.2875, 1.1547, 0.0]) + rng.uniform(-1, 1, (B, 4)) * np.array([0.02, 0.02, 0, 0])
t0 = time.time()
Uo = {b: lbmpc.dms_lbmpc_loop(mg, g, 100, 100, T, x_init=X0[b])[1] for b in (0, 8)}
print('oracle loops %.1f s' % (time.time() - t0), flush=True)
for tol, mi in ((1e-8, 200),):
    t0 = time.time()
    r = bqp.closed_loop_sqp(dms, X0, T, learning=dict(q=100, mask=1), tol=tol, max_iter=mi)
    print('tol %.0e max_iter %d: %.2f s' % (tol, mi, time.time() - t0))
    print('  flags', r.exitflag.tolist())
    print('  iterations', r.iterations.tolist())
    for b in (0, 8):
        print('  inst %d |U - U_oracle| per step' % b, np.abs(r.U[b, :, 0] - Uo[b]).tolist())
    sys.stdout.flush()
st = golden('dms_lbmpc_loops.npz')['DMS_tLBMPC_q100']
for tol in (1e-8,):
    r = bqp.closed_loop_sqp(dms, X0[:0].reshape(0, 4) if False else np.array([[0.15, 1.2875, 1.1547, 0.0]]),
                            25, learning=dict(q=100, mask=1), tol=tol, max_iter=500)
    e = np.abs(r.X[0] - st[:26])
    print('x_init, tol %.0e: flags %s' % (tol, r.exitflag[0].tolist()))
    print('  iterations', r.iterations[0].tolist())
    print('  |x - stored q100| slow states max %.2e, all states per step %s'
          % (e[:, :2].max(), np.array2string(e.max(axis=1), precision=2)))
