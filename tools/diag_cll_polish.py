"""Diagnostic (GPU): wall time of the CLL learned-model loop (bench.py --config CLL's workload, batch
256) with the QP sub-problems' polish launch on (default) and off, and the kernel time the
handle reports - whether the dense polish kernel costs anything when no sub-problem needs it."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'learning-based-mpc_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import bqp  # noqa: E402
from conftest import golden  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

mg = mg_problem()
g = golden('lbmpc_instance.npz')
dl = bqp.DMSLBMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                  mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], g['F_w_N'], g['h_w_N'],
                  g['F_x_d'], g['h_x_d'], mg['x_wp'], mg['u_wp'], N=100)
rng = np.random.default_rng(11)
x_init = np.array([0.15, 1.2875, 1.1547, 0.0])
X0 = x_init + rng.uniform(-1, 1, (256, 4)) * np.array([0.005, 0.005, 0.0, 0.0])
h = bqp.Handle(0)
bqp.closed_loop_sqp(dl, X0, 1, learning=dict(q=100, mask=1), handle=h)
for rep in range(2):
    for pol in (1, -1):
        t0 = time.perf_counter()
        r = bqp.closed_loop_sqp(dl, X0, 10, learning=dict(q=100, mask=1), handle=h, polish=pol)
        el = time.perf_counter() - t0
        print('polish %2d: %.1f ms per step, kernel %.1f ms, flags %s, SQP iterations mean %.2f'
              % (pol, 1e3 * el / 10, h.kernel_ms()[0] / 10, np.unique(r.exitflag).tolist(),
                 r.iterations.mean()), flush=True)
