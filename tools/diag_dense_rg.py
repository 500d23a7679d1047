"""Diagnostic: dense_ipm_kernel with the row state in registers (RG) against the workspace form
(BQP_DENSE_NO_RG=1) on the random QPs of tests/test_gpu_quadprog.py
(test_dense_rows_in_registers_equals_workspace_form): each form twice (run-to-run determinism),
exit flags, iteration counts, max |x - x'|, and the same with the polish off."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
import bqp

h = bqp.Handle(0)
for m in (300, 1024):
    n, B = 101, 4
    rng = np.random.default_rng(7 + m)
    M = rng.standard_normal((n, n))
    H = M @ M.T / n + np.eye(n)
    A = rng.standard_normal((m, n))
    f = rng.standard_normal((B, n))
    b = rng.uniform(0.2, 1.0, (B, m))
    lb, ub = -2.0 * np.ones(n), 2.0 * np.ones(n)
    for opts in (None, dict(polish=0)):
        res = {}
        for tag, env in (('rg', None), ('rg2', None), ('ws', '1'), ('ws2', '1')):
            if env: os.environ['BQP_DENSE_NO_RG'] = env
            try:
                res[tag] = bqp.quadprog(H, f, A, b, lb=lb, ub=ub, handle=h, options=opts)
            finally:
                os.environ.pop('BQP_DENSE_NO_RG', None)
        for tag in res:
            x, fv, fl, out, lam = res[tag]
            print('m %d opts %s %-4s flags %s it %s |x - x_rg| %.2e fval %s' % (
                m, opts, tag, fl, out['iterations'], np.abs(x - res['rg'][0]).max(), fv))
