"""Diagnostic: the condensed N=128 DMS instance that the dense workgroup kernel ends with -8
(tests/test_gpu_ocp.py::test_long_horizon_box_layouts) - exit flag and statistics against
max_iter, to find where the iterate turns non-finite."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'learning-based-mpc_amd'), os.path.join(ROOT, 'tests')]
import bqp  # noqa: E402
import conftest  # noqa: E402
from bqp.ocp import condensed_rhs  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

mg = mg_problem()
t = conftest.golden('term_set.npz')
g = conftest.golden('dms_DSS_tLMPC.npz')
X = g['x'][g['idx'][:8]]
tl = bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                      mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], t['F_w_N'],
                      t['h_w_N'], mg['x_wp'], mg['u_wp'], N=128)
cd, f, b = condensed_rhs(tl.prob, X - tl.x_eq)
for mi in list(range(1, 30)) + [40, 50, 80, 100, 150, 200]:
    x, fv, fl, out, lam = bqp.quadprog(cd.H, f[1:2], cd.A, b[1:2], options=dict(max_iter=mi))
    print(mi, int(fl[0]), int(out['iterations'][0]), '%.3e %.3e' % (out['firstorderopt'][0],
          out['constrviolation'][0]), 'finite' if np.isfinite(x).all() else 'NaN',
          'lam_max %.3e' % np.abs(lam['ineqlin']).max(), flush=True)
