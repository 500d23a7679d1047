"""Mixed-precision handoff sweep (C5 problem, N=100): for each fp32->fp64 switch point mu_sw
(BQP_MIXED_MU), the fp32-phase iterations, total iterations, first-move error vs z*, dual error
vs the oracle's lambda* (unique-multiplier instances), and the kernel time of a batch of 8192.
usage (GPU box): python tools/diag_mixed.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'learning-based-mpc_amd'), os.path.join(ROOT, 'tests')]

import bqp  # noqa: E402
import dual_map as dm  # noqa: E402
from oracle import dense_qp, qp_forms  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

G = os.path.join(ROOT, 'tests', 'golden')
mg = mg_problem()
ts = np.load(os.path.join(G, 'term_set.npz'))
g = np.load(os.path.join(G, 'dms_DSS_tLMPC.npz'))
N = int(g['N'])
tl = bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                      mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], ts['F_w_N'],
                      ts['h_w_N'], mg['x_wp'], mg['u_wp'], N=N)
h = bqp.Handle(0)
X8 = g['x'][g['idx'][:8]]
refs = []
for i in range(len(X8)):
    qp = qp_forms.dms_dense(mg, N, X8[i], ts['F_w_N'], ts['h_w_N'])
    refs.append((qp, dense_qp.solve(qp)))
XB = g['x'][np.arange(8192) % len(g['x'])]
XI = g['x'][g['idx']]


def lam_err(r):
    e = 0.0
    for i, (qp, (zs, fv, ls, info)) in enumerate(refs):
        lin, y = dm.f2_duals(N, r.lam_x[i], r.lam_u[i], r.lam_p[i], r.pi[i])
        if dm.licq(qp['A'], lin, ls['ineqlin']):
            sc = max(1.0, np.abs(ls['ineqlin']).max(), np.abs(ls['eqlin']).max())
            e = max(e, np.abs(lin - ls['ineqlin']).max() / sc, np.abs(y - ls['eqlin'][:4 * N]).max() / sc)
    return e


def timed(prec):
    tl.solve(XB, handle=h, precision=prec)
    t = []
    for _ in range(3):
        tl.solve(XB, handle=h, precision=prec)
        t.append(h.kernel_ms()[0])
    return min(t)


r64 = tl.solve(X8, handle=h, want_duals=True)
ri = tl.solve(XI, handle=h)
print('fp64: iterations %.2f  lam err %.2e  kernel %.2f ms' % (ri.iterations.mean(), lam_err(r64), timed(0)), flush=True)
for mu in ['1e-4', '1e-5', '1e-6', '1e-7', '1e-8', '1e-9']:
    os.environ['BQP_MIXED_MU'] = mu
    p1 = tl.solve(XI, handle=h, precision=1, tol_comp=float(mu))
    r = tl.solve(XI, handle=h, precision=2)
    rd = tl.solve(X8, handle=h, precision=2, want_duals=True)
    err = np.abs(r.u0[:, 0] - g['u_star']).max()
    print('mu_sw %s: fp32 its %.2f  total %.2f  flags ok %d/%d  du0 err %.2e  lam err %.2e  kernel %.2f ms'
          % (mu, p1.iterations.mean(), r.iterations.mean(), (r.exitflag == 1).sum(), len(r.exitflag), err,
             lam_err(rd), timed(2)), flush=True)
print('fp32 alone: kernel %.2f ms' % timed(1))
