"""Diagnostic: exit statistics of the fp32 structured solve on the C2 / C5 fixture states."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'learning-based-mpc_amd'), os.path.join(ROOT, 'tests')]
import bqp
from oracle.mg_model import mg_problem
mg = mg_problem()
ts = np.load(os.path.join(ROOT, 'tests/golden/term_set.npz'))
g = np.load(os.path.join(ROOT, 'tests/golden/lmpc_N20.npz'))
lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'], mg['PSI'],
              mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], ts['F_w_N'], ts['h_w_N'], N=20)
X = g['dx'][:1000]
for kw in (dict(), dict(tol_stat=1e-4), dict(tol_comp=1e-8), dict(tol_feas=1e-5)):
    r = lm.solve(X, precision=1, **kw)
    bad = r.exitflag != 1
    print(kw, 'flags', {int(f): int((r.exitflag == f).sum()) for f in np.unique(r.exitflag)},
          'iters', r.iterations.mean())
    if bad.any():
        i = np.flatnonzero(bad)[:5]
        print('   stat', r.firstorderopt[i], 'feas', r.constrviolation[i], 'mu', r.mu[i], 'it', r.iterations[i])
