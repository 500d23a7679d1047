"""The condensed route of bqp.solve_ocp (dimensions without a compiled structured kernel): host
condensing once per problem, the batch on the dense GPU kernels through the C ABI
(bqp_quadprog_batched).  Parity against the oracle's stage-wise Riccati IPM (oracle/ocp_ipm.py)
on an (nx, nu, np) = (3, 1, 1) problem with per-instance terminal-set right-hand sides, and
against the structured kernel on the C2 problem (route forced)."""
import numpy as np
import pytest

from conftest import golden
from test_condense import odd_dims_problem


@pytest.mark.gpu
def test_odd_dims_auto_route_vs_oracle():
    import bqp
    from oracle import ocp_ipm
    prob, d, X0, HP = odd_dims_problem()
    r = bqp.solve_ocp(prob, X0, hp=HP)
    assert (r.exitflag == 1).all(), r.exitflag
    assert r.x.shape == (len(X0), prob.N + 1, prob.nx) and r.u.shape == (len(X0), prob.N, prob.nu)
    for i in range(len(X0)):
        o = ocp_ipm.solve(dict(d, hp=HP[i]), X0[i])
        assert np.abs(r.u[i] - o['u']).max() < 1e-7
        assert np.abs(r.theta[i] - o['theta']).max() < 1e-7
        assert np.abs(r.x[i] - o['x']).max() < 1e-7
        assert r.iterations[i] >= 1
    with pytest.raises(Exception):
        bqp.solve_ocp(prob, X0, route='structured')


@pytest.mark.gpu
def test_forced_condensed_route_matches_structured(mg, term_set):
    """C2 (MG, F1 at N=20): route='condensed' gives the structured kernel's solution (both to
    the fixture's exact z*), and the same cost"""
    import bqp
    g = golden('lmpc_N20.npz')
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                  mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                  term_set[0], term_set[1], N=20)
    X0 = g['dx'][g['idx']]
    rs = bqp.solve_ocp(lm.prob, X0)
    rc = bqp.solve_ocp(lm.prob, X0, route='condensed')
    assert (rs.exitflag == 1).all() and (rc.exitflag == 1).all()
    assert np.abs(rc.u - rs.u).max() < 1e-7
    assert np.abs(rc.x - rs.x).max() < 1e-7
    assert np.abs(rc.fval - rs.fval).max() < 1e-7 * (1 + np.abs(rs.fval).max())
