"""TEST INFRASTRUCTURE ONLY: fixture of the regularised exact Hessian.

The +-0.02-perturbed DMS_LBMPC_casadi.m instance (seed 11, instance 0 of tools/diag_dms_gpu.py)
whose exact-Hessian SQP sub-problems are indefinite at its third closed-loop step: the oracle's
loop (oracle/lbmpc.py dms_lbmpc_loop, hessian 'exact' with hess_shift) over 3 steps - first moves,
SQP iterations per step - into tests/golden/dms_indefinite.npz.  Before the shift the oracle and
the GPU fell back to Gauss-Newton there and stopped at the 200-iteration limit with the
stationarity residual at 1.3e-4 (cost 39.69529784 against the optimum's 39.69527588)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]

from conftest import golden  # noqa: E402
from oracle import lbmpc  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402


def main():
    mg = mg_problem()
    g = golden('lbmpc_instance.npz')
    rng = np.random.default_rng(11)
    X0 = np.array([0.15, 1.2875, 1.1547, 0.0]) + rng.uniform(-1, 1, (16, 4)) * np.array([0.02, 0.02, 0, 0])
    X, U, Z, IT = lbmpc.dms_lbmpc_loop(mg, g, 100, 100, 3, x_init=X0[0])
    out = os.path.join(ROOT, 'tests', 'golden', 'dms_indefinite.npz')
    np.savez(out, x0=X0[0], X=X, U=U, iterations=np.asarray(IT))
    print('wrote', out, 'U', U, 'iterations', IT)


if __name__ == '__main__':
    main()
