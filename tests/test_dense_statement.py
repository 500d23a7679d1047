"""CPU: the dense IPM algorithm statement (oracle/dense_ipm.py, the algorithm of
csrc/bqp_dense.hip) against the ground-truth dense solver, and its quadprog exit flags on
instances with a known status (infeasible -2, unbounded -3, non-convex -6)."""
import numpy as np
import pytest

from status_cases import cases


@pytest.mark.parametrize('name,qp,flag', cases(), ids=[c[0] for c in cases()])
def test_statement_exitflags(name, qp, flag):
    from oracle import dense_ipm
    r = dense_ipm.solve(**qp)
    assert r['exitflag'] == flag, (name, r['exitflag'], r['iterations'])


def test_statement_matches_ground_truth():
    from oracle import dense_ipm, dense_qp, qp_forms
    rng = np.random.default_rng(3)
    for _ in range(12):
        n = int(rng.integers(2, 14))
        m = int(rng.integers(0, 30))
        M = rng.standard_normal((n, n))
        H = M @ M.T + 0.2 * np.eye(n)
        f = rng.standard_normal(n)
        A = rng.standard_normal((m, n))
        b = rng.uniform(0.5, 2.0, m)
        lb, ub = -2 * np.ones(n), 2 * np.ones(n)
        r = dense_ipm.solve(H, f, A, b, lb=lb, ub=ub)
        z, fv, lam, info = dense_qp.solve(qp_forms.dense_qp(H, f, A, b, lb=lb, ub=ub))
        assert r['exitflag'] == 1
        assert np.abs(r['x'] - z).max() < 1e-8
