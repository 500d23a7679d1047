"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Oracle closed loops for the GPU test of the learned-model NLP loop (tests/test_gpu_lbmpc_dms.py):
the restatement oracle/lbmpc.py dms_lbmpc_loop run on the CPU for
  * 16 initial states around x_init (x1, x2 perturbed by up to +-0.005, seed 11), 3 steps of
    DMS_LBMPC_casadi.m (8 x 100 window, learned terminal cost, warm start);
  * x_init, 3 steps of the hybrid cost (hybrid_LBMPC_casadi.m: nominal terminal term) with a
    7-row window of 100 points that all count (mask 0).
Writes tests/golden/dms_lbmpc_oracle.npz (plain arrays).  Usage:
    python -m oracle.make_dms_oracle_fixture [--procs 8]
"""
import argparse
import os
from multiprocessing import Pool

import numpy as np

from . import lbmpc
from .mg_model import mg_problem

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(os.path.dirname(HERE), 'tests', 'golden')
X_INIT = np.array([0.15, 1.2875, 1.1547, 0.0])
T = 3


def _sets():
    return dict(np.load(os.path.join(GOLD, 'lbmpc_instance.npz')))


def _run(args):
    x0, mask, term = args
    X, U, Z, IT = lbmpc.dms_lbmpc_loop(mg_problem(), _sets(), 100, 100, T, mask=mask,
                                       term_learned=term, x_init=x0)
    return X, U, IT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=8)
    a = ap.parse_args()
    rng = np.random.default_rng(11)
    X0 = X_INIT + rng.uniform(-1, 1, (16, 4)) * np.array([0.005, 0.005, 0.0, 0.0])
    jobs = [(x, True, True) for x in X0] + [(X_INIT, False, False)]
    with Pool(a.procs) as p:
        res = p.map(_run, jobs)
    out = dict(x0=X0, X=np.array([r[0] for r in res[:16]]), U=np.array([r[1] for r in res[:16]]),
               iterations=np.array([r[2] for r in res[:16]]),
               hyb_X=res[16][0], hyb_U=res[16][1], hyb_iterations=res[16][2], steps=T)
    np.savez_compressed(os.path.join(GOLD, 'dms_lbmpc_oracle.npz'), **out)
    print('iterations', out['iterations'].tolist(), 'hybrid', out['hyb_iterations'].tolist())


if __name__ == '__main__':
    main()
