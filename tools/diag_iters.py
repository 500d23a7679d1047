"""Diagnostic: instances whose GPU and C-port iteration counts differ (C2 fixture states)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'learning-based-mpc_amd')]
import bqp
from oracle import cpu_ref, qp_forms
from oracle.mg_model import mg_problem
mg = mg_problem()
ts = np.load(os.path.join(ROOT, 'tests/golden/term_set.npz'))
g = np.load(os.path.join(ROOT, 'tests/golden/lmpc_N20.npz'))
lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'], mg['PSI'],
              mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], ts['F_w_N'], ts['h_w_N'], N=20)
X = g['dx'][:256]
r = lm.solve(X)
c = cpu_ref.solve(qp_forms.lmpc_ocp(mg, 20, ts['F_w_N'], ts['h_w_N']), X)
d = r.iterations - c['iterations']
print('agree', np.mean(d == 0), 'hist', {int(k): int((d == k).sum()) for k in np.unique(d)})
for i in np.flatnonzero(d != 0)[:8]:
    print(i, 'gpu it', r.iterations[i], 'stat/feas/mu', r.firstorderopt[i], r.constrviolation[i], r.mu[i],
          '| cpu it', c['iterations'][i], 'kkt', c['kkt'][i], '| du', np.abs(r.u[i] - c['u'][i]).max())
