"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Re-solves the exact optima stored in the F2 fixtures (tests/golden/dms_*.npz, written by
oracle/make_fixtures.py with the dense IPM + fp64 active-set polish of oracle/dense_qp.py) with
the LDP/NNLS solve and extended-precision polish of oracle/exact_qp.py, on the structured
restatement of DMS_tracking_LMPC_casadi.m:223-291 (oracle/qp_forms.dms_ocp, deviation
coordinates), and writes them back in the fixtures' absolute dense layout
y = [x_0 .. x_N; u_0 .. u_{N-1}; theta].  Round 3: the dense polish left DSS_tLMPC state 132's
first move 1.2e-8 from the optimum (its KKT solve on a 25-row active set in fp64); the exact
solve agrees with the structured IPM there to 1.2e-10.  The stored states, the IPOPT moves and
everything else in the files are unchanged; the dense values are kept as z_star_dense.

Adjudication of the stored IPOPT moves (DMS_tracking_LMPC_casadi*.m:163-172): with the first
move fixed to IPOPT's applied move (recovered from the RK4 plant) the rest of the QP is solved
exactly; `ipopt_excess` = J(IPOPT move) - J* (>= 0 for the strictly convex QP) and
`ipopt_fixed_feasible` record whether the gap to IPOPT is IPOPT stopping short (feasible, with a
cost excess) rather than a different problem.
Usage: python oracle/refine_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import exact_qp, qp_forms  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

GOLD = os.path.join(ROOT, 'tests', 'golden')


def refine(fname):
    path = os.path.join(GOLD, fname)
    g = dict(np.load(path))
    mg = mg_problem()
    ts = np.load(os.path.join(GOLD, 'term_set.npz'))
    N = int(g['N'])
    ocp = qp_forms.dms_ocp(mg, N, ts['F_w_N'], ts['h_w_N'])
    x_eq = np.asarray(mg['x_wp'], float).ravel()
    u_eq = float(np.atleast_1d(mg['u_wp'])[0])
    dense = g.get('z_star_dense', g['z_star'])
    Z = np.zeros_like(dense)
    for j, i in enumerate(g['idx']):
        r = exact_qp.solve_ocp(ocp, g['x'][i] - x_eq)
        assert r['status'] == 'optimal', (fname, i)
        Z[j, :(N + 1) * 4] = (r['x'] + x_eq).ravel()
        Z[j, (N + 1) * 4:(N + 1) * 4 + N] = r['u'].ravel() + u_eq
        Z[j, -1] = r['theta'][0]
    d = np.abs(Z - dense).max(axis=1)
    g['z_star_dense'] = dense
    g['z_star'] = Z
    g['u_star'] = Z[:, (N + 1) * 4]
    g['err_vs_ipopt'] = np.abs(g['u_star'] - g['u_ipopt'][g['idx']])
    from oracle.make_c2_fixture import fixed_move_qp
    exc = np.zeros(len(g['idx'])); ffe = np.zeros(len(g['idx']), bool)
    for j, i in enumerate(g['idx']):
        qp = exact_qp.condense_ocp(ocp, g['x'][i] - x_eq)
        r = exact_qp.solve(qp['H'], qp['f'], qp['A'], qp['b'])
        Hr, fr, Ar, br, c0 = fixed_move_qp(qp, g['u_ipopt'][i] - u_eq)
        rr = exact_qp.solve(Hr, fr, Ar, br)
        ffe[j] = rr['status'] == 'optimal'
        exc[j] = rr['fval'] + c0 - r['fval'] if ffe[j] else np.inf
    g['ipopt_excess'] = exc
    g['ipopt_fixed_feasible'] = ffe
    np.savez(path, **g)
    w = np.argsort(-g['err_vs_ipopt'])[:3]
    print('  largest IPOPT gaps: ' + ', '.join('state %d: |u* - u_ipopt| %.2e, cost excess %.2e (feasible %s)'
                                             % (g['idx'][k], g['err_vs_ipopt'][k], exc[k], ffe[k]) for k in w))
    print('%s: exact vs dense-polish z*: max %.2e (state %d), first move max %.2e'
          % (fname, d.max(), int(g['idx'][d.argmax()]),
             np.abs(Z[:, (N + 1) * 4] - dense[:, (N + 1) * 4]).max()))


def main():
    for f in ('dms_DSS_tLMPC.npz', 'dms_DMS_N50_tLMPC.npz', 'dms_DMS_tLMPC_K.npz', 'dms_tLMPC.npz'):
        refine(f)


if __name__ == '__main__':
    main()
