"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Config C3 input data: the trackingMPC double-integrator design
(trackingMPC/RunExample.m:20-108, restated in oracle/mg_model.di_model) with its terminal set
(the MPIS restatement of compute_MPIS.m, oracle/mpis.py), and 1024 initial states drawn from
U([-5,5]^2) (seed 30) kept only if the N=30 problem is feasible for all four references of
RunExample.m:213-223 (x_s in {4.95, -5.5, 2, 0} e_1), checked with the C restatement.

    python -m oracle.make_di_fixture        # writes tests/golden/di_design.npz

The bench reads the .npz as plain data (no oracle import on the product path).
"""
import os
import sys

import numpy as np

from . import cpu_ref, mpis, qp_forms
from .mg_model import di_model

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')
N = 30
REFS = np.array([[4.95, 0.0], [-5.5, 0.0], [2.0, 0.0], [0.0, 0.0]])


def main():
    di = di_model()
    F_T, h_T = mpis.di_terminal_set(di)
    ocp = qp_forms.track_ocp(di, N, F_T, h_T)
    rng = np.random.default_rng(30)
    keep, kref = [], []
    while len(keep) < 1024:
        X = rng.uniform(-5, 5, size=(512, 2))
        ok = np.ones(len(X), bool)
        its = np.zeros((len(X), 4), np.int32)
        for j, xs in enumerate(REFS):
            w = np.repeat(qp_forms.track_w(di, N, xs)[0][None], len(X), axis=0)
            r = cpu_ref.solve(ocp, X, w=w)
            ok &= r['exitflag'] == 1
            its[:, j] = r['iterations']
        keep.extend(X[ok]); kref.extend(its[ok])
    x0 = np.array(keep[:1024]); kref = np.array(kref[:1024])
    np.savez(os.path.join(OUT, 'di_design.npz'), N=N, A=di['A'], B=di['B'], Q=di['Q'], R=di['R'],
             K=di['K'], P=di['P'], T=di['T'], LAMBDA=di['LAMBDA'], PSI=di['PSI'], F_x=di['F_x'],
             h_x=di['h_x'], F_u=di['F_u'], h_u=di['h_u'], F_T=F_T, h_T=h_T, x0=x0, xs=REFS,
             kref=kref)
    print('C3: %d feasible x0, terminal set %d rows, mean K_ref %.2f' % (len(x0), len(h_T), kref.mean()))


if __name__ == '__main__':
    sys.exit(main())
