"""GPU: quadprog exit flags of bqp_quadprog_batched (both dense kernels) on instances with a
known status - infeasible (-2), unbounded (-3), non-convex (-6) - against the algorithm
statement oracle/dense_ipm.py (same rules, same iterates), and the LBMPC SQP reporting an
infeasible sub-problem (-2) instead of running to its iteration limit."""
import numpy as np
import pytest

from conftest import golden
from status_cases import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


def _solve(qp, handle):
    import bqp
    return bqp.quadprog(qp['H'], qp['f'], qp.get('A'), qp.get('b'), qp.get('Aeq'), qp.get('beq'),
                        qp.get('lb'), qp.get('ub'), handle=handle)


@pytest.mark.parametrize('name,qp,flag', cases(), ids=[c[0] for c in cases()])
def test_exitflags_match_statement(name, qp, flag, handle):
    from oracle import dense_ipm
    x, fval, ef, out, lam = _solve(qp, handle)
    assert ef[0] == flag, (name, ef[0], out['iterations'][0])
    r = dense_ipm.solve(**qp)
    assert abs(int(out['iterations'][0]) - r['iterations']) <= 1
    if flag == 1:
        assert np.abs(x[0] - r['x']).max() < 1e-9 * max(1.0, np.abs(r['x']).max())


def _big(n, infeasible):
    """n > 32 variables: the workgroup kernel (dense_ipm_kernel)."""
    rng = np.random.default_rng(5)
    M = rng.standard_normal((n, n))
    H = M @ M.T + n * np.eye(n)
    f = rng.standard_normal(n)
    A = rng.standard_normal((20, n))
    b = rng.uniform(0.5, 2.0, 20)
    if infeasible:
        A = np.vstack([A, np.eye(n)[3], -np.eye(n)[3]])
        b = np.concatenate([b, [-1.0, -2.0]])
    return dict(H=H, f=f, A=A, b=b, lb=-3 * np.ones(n), ub=3 * np.ones(n))


@pytest.mark.parametrize('infeasible', [False, True])
def test_workgroup_kernel_flags(infeasible, handle):
    from oracle import dense_ipm
    qp = _big(40, infeasible)
    x, fval, ef, out, lam = _solve(qp, handle)
    r = dense_ipm.solve(**qp)
    assert ef[0] == r['exitflag'] == (-2 if infeasible else 1)
    if not infeasible:
        assert np.abs(x[0] - r['x']).max() < 1e-9


def test_batch_mixed_status(handle):
    """One batch holding feasible and infeasible instances (per-instance b): each instance gets
    its own flag, the feasible ones their optimum."""
    import bqp
    from oracle import dense_ipm
    qp = cases()[0][1]
    B = 8
    b = np.tile(qp['b'], (B, 1))
    A = np.vstack([qp['A'], np.eye(6)[0], -np.eye(6)[0]])
    bb = np.concatenate([b, np.tile([5.0, 5.0], (B, 1))], axis=1)
    bb[1::2, -1] = -6.0                 # x_1 >= 6 > 5: infeasible (also beyond ub = 2)
    x, fval, ef, out, lam = bqp.quadprog(qp['H'], qp['f'], A, bb, lb=qp['lb'], ub=qp['ub'],
                                         handle=handle)
    assert (ef[0::2] == 1).all() and (ef[1::2] == -2).all(), ef
    r = dense_ipm.solve(qp['H'], qp['f'], A, bb[0], lb=qp['lb'], ub=qp['ub'])
    assert np.abs(x[0] - r['x']).max() < 1e-9


def test_lbmpc_infeasible_subproblem(mg, handle):
    """x0 outside the LBMPC feasible set (the tightened box F_x_d on x_1 cannot be met):
    exitflag -2 from the QP sub-problem (bqp_lbmpc.hip update kernel), feasible x0 converge."""
    import bqp
    g = golden('lbmpc_instance.npz')
    td = golden('train_data.npz')['data'][:, :100]
    lb = bqp.LBMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                   mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                   g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], N=10)
    X0 = np.array([[3.0, 3.0, 0, 0], [-0.35, -0.4, 0, 0], [0.6, 0, 0, 0]])
    r = lb.solve(X0, td, handle=handle)
    assert r.exitflag[0] == -2 and r.exitflag[2] == -2, r.exitflag
    assert r.exitflag[1] == 1


@pytest.mark.parametrize('n', [20, 40])
def test_residual_recurrence_vs_exact_residuals(n, handle):
    """the dense kernels step the residuals by the (1 - alpha) recurrence and evaluate
    them exactly only at the start, after a short step (alpha < 0.5), every 8th iteration and to
    confirm convergence.  On a nearly singular H (eigenvalues 1 ... 1e-15: the factor of K runs
    into the pivot floor once the barrier terms dominate) the exit flag, iteration count and
    solution must match the path that evaluates them exactly every iteration
    (BQP_DENSE_RES_EVERY=1), and the algorithm statement oracle/dense_ipm.py.  n = 20: the one-wave
    kernel, n = 40: the workgroup kernel."""
    import os
    from oracle import dense_ipm
    rng = np.random.default_rng(17)
    M, _ = np.linalg.qr(rng.standard_normal((n, n)))
    H = (M * np.logspace(0, -15, n)) @ M.T
    H = 0.5 * (H + H.T)
    qp = dict(H=H, f=rng.standard_normal(n), A=rng.standard_normal((3 * n, n)),
              b=rng.uniform(0.5, 2.0, 3 * n), lb=-3 * np.ones(n), ub=3 * np.ones(n))
    x, fval, ef, out, lam = _solve(qp, handle)
    os.environ['BQP_DENSE_RES_EVERY'] = '1'
    try:
        xe, fe, efe, oute, lame = _solve(qp, handle)
    finally:
        del os.environ['BQP_DENSE_RES_EVERY']
    r = dense_ipm.solve(**qp)
    print('n %d: flags %d / %d (statement %d), iterations %d / %d (statement %d), |x - x_exact| %.2e'
          % (n, ef[0], efe[0], r['exitflag'], out['iterations'][0], oute['iterations'][0],
             r['iterations'], np.abs(x - xe).max()))
    assert ef[0] == efe[0] == r['exitflag'] == 1
    assert abs(int(out['iterations'][0]) - int(oute['iterations'][0])) <= 1
    assert abs(int(out['iterations'][0]) - r['iterations']) <= 1
    assert abs(fval[0] - fe[0]) <= 1e-10 * max(1.0, abs(fe[0]))
    assert np.abs(x - xe).max() < 1e-6
