"""Diagnostic: GPU structured solve vs the C restatement (oracle/cpu_ipm.c) after a fixed number
of IPM iterations (max_iter = 0, 1, 2, ...) on the same C2 instances: locates the first
iteration at which the iterates part."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
import numpy as np
import bqp
from oracle import cpu_ref, qp_forms
from oracle.mg_model import mg_problem

mg = mg_problem()
ts = np.load(os.path.join(ROOT, 'tests/golden/term_set.npz'))
g = np.load(os.path.join(ROOT, 'tests/golden/lmpc_N20.npz'))
ocp = qp_forms.lmpc_ocp(mg, 20, ts['F_w_N'], ts['h_w_N'])
prob = bqp.OcpProblem(ocp['A'], ocp['B'], ocp['W'], 20, 1, w=ocp['w'], xlb=ocp['xlb'], xub=ocp['xub'],
                      ulb=ocp['ulb'], uub=ocp['uub'], Fp=ocp['Fp'], hp=ocp['hp'], poly_stage=ocp['kp'])
X0 = g['dx'][:16]
for mi in range(1, 7):
    r = bqp.solve_ocp(prob, X0, max_iter=mi)
    c = cpu_ref.solve(ocp, X0, max_iter=mi)
    dx = np.abs(r.x - c['x']).max(axis=(1, 2))
    du = np.abs(r.u - c['u']).max(axis=(1, 2))
    print('max_iter %d: |dx| max %.2e med %.2e  |du| max %.2e  it gpu %s cpu %s' %
          (mi, dx.max(), np.median(dx), du.max(), r.iterations[:6], c['iterations'][:6]))
    print('   gpu mu %s' % np.array2string(r.mu[:4], precision=3))
r = bqp.solve_ocp(prob, X0)
c = cpu_ref.solve(ocp, X0)
print('full: it gpu', r.iterations, '\n      it cpu', c['iterations'])
print('gpu stat/feas/mu', r.firstorderopt[:4], r.constrviolation[:4], r.mu[:4])
