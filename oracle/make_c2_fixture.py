"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Golden fixture of config C2: the F1 QP (costLMPC.m / constraintsLMPC.m,
N = 20, terminal set term_set.mat) at ALL 1000 stored closed-loop states of
LMPC_N20_sys_full.mat, solved exactly by oracle/exact_qp.py (LDP/NNLS + extended-precision
active-set polish), and an adjudication of the stored fmincon moves (ocpLMPC.m:24) that
disagree with the exact optimum.

Adjudication: for every state the first move is fixed to fmincon's applied move
(sysH(5, k+1)) and the rest of the QP is solved exactly; the cost excess of fmincon's move over
the optimum (>= 0 for a strictly convex QP) and the feasibility of the fixed-move problem tell
which solver is wrong: an excess well above fmincon's own tolerance means fmincon stopped short
of the optimum at that state.

Writes tests/golden/lmpc_N20_all.npz:
    dx (1000, 4), du_matlab (1000,), z_star (1000, 21) = [u_0 .. u_19; theta] (u = K x + c,
    the applied deviation input), du_star (1000,), active_rows (1000,), fval_star (1000,),
    du_err (1000,) = |du_star - du_matlab|, excess (1000,) = J(fmincon move) - J*,
    fixed_feasible (1000,) bool, lam_max (1000,)
Usage: python oracle/make_c2_fixture.py
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


def fixed_move_qp(qp, u0):
    """the condensed QP with z_0 = u0 fixed: (H, f, A, b) over z_1.., and the constant part"""
    H, f, A, b = qp['H'], qp['f'], qp['A'], qp['b']
    Hr = H[1:, 1:]
    fr = f[1:] + H[1:, 0] * u0
    Ar = A[:, 1:]
    br = b - A[:, 0] * u0
    const = 0.5 * H[0, 0] * u0 * u0 + f[0] * u0
    return Hr, fr, Ar, br, const


def main():
    mg = mg_problem()
    ts = np.load(os.path.join(GOLD, 'term_set.npz'))
    g = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))
    dx, du_m = g['dx'], g['du_matlab']
    ocp = qp_forms.lmpc_ocp(mg, 20, ts['F_w_N'], ts['h_w_N'])
    n = len(dx)
    Z = np.zeros((n, 21)); fs = np.zeros(n); nact = np.zeros(n, int); lmx = np.zeros(n)
    exc = np.zeros(n); ffeas = np.zeros(n, bool)
    for i in range(n):
        qp = exact_qp.condense_ocp(ocp, dx[i])
        r = exact_qp.solve(qp['H'], qp['f'], qp['A'], qp['b'])
        assert r['status'] == 'optimal', i
        Z[i] = r['z']; fs[i] = r['fval']; nact[i] = len(r['active'])
        lmx[i] = r['lam'].max(initial=0.0)
        Hr, fr, Ar, br, c0 = fixed_move_qp(qp, du_m[i])
        rr = exact_qp.solve(Hr, fr, Ar, br)
        ffeas[i] = rr['status'] == 'optimal'
        exc[i] = (rr['fval'] + c0 - r['fval']) if ffeas[i] else np.inf
    du_err = np.abs(Z[:, 0] - du_m)
    np.savez_compressed(os.path.join(GOLD, 'lmpc_N20_all.npz'), dx=dx, du_matlab=du_m, z_star=Z,
                        du_star=Z[:, 0], active_rows=nact, fval_star=fs, du_err=du_err, excess=exc,
                        fixed_feasible=ffeas, lam_max=lmx)
    order = np.argsort(-du_err)
    print('C2 all 1000 states: |du* - du_fmincon| median %.2e, max %.2e' % (np.median(du_err), du_err.max()))
    for i in order[:5]:
        print('  state %4d: du err %.3e, cost excess of fmincon move %.3e (fixed-move QP feasible %s), '
              'active rows %d, lam max %.1f' % (i, du_err[i], exc[i], ffeas[i], nact[i], lmx[i]))


if __name__ == '__main__':
    main()
