"""GPU parity tests of the quadprog-compatible dense entry point (bqp_quadprog_batched) on the
reference's QPs in their own variable layout (oracle/qp_forms restates the MATLAB loops)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


def test_f1_dense_quadprog(mg, term_set, handle):
    """fmincon LMPC (F1) as a dense QP: 21 vars, 806 rows; batch of fixture states."""
    import bqp
    from oracle import qp_forms
    g = golden('lmpc_N20.npz')
    sel = np.arange(16)
    qps = [qp_forms.lmpc_dense(mg, 20, g['dx'][g['idx'][j]], *term_set) for j in sel]
    H = qps[0]['H']
    A = qps[0]['A']
    f = np.stack([q['f'] for q in qps])
    b = np.stack([q['b'] for q in qps])
    x, fval, flag, out, lam = bqp.quadprog(H, f, A, b, handle=handle)
    assert (flag == 1).all(), flag
    zs = g['z_star'][sel]
    assert np.abs(x - zs).max() / max(1, np.abs(zs).max()) < 1e-8
    # quadprog multiplier convention: H x + f + A'lam = 0, lam >= 0
    for i in range(len(sel)):
        r = H @ x[i] + f[i] + A.T @ lam['ineqlin'][i]
        assert np.abs(r).max() < 1e-6 * (1 + np.abs(f[i]).max())
    assert (lam['ineqlin'] >= -1e-12).all()


def test_f2_dense_with_equalities_and_fixed_vars(mg, term_set, handle):
    """DMS tracking LMPC (F2) at N=20 in quadprog form: equality dynamics, x_0 fixed by
    lb == ub (DMS_tracking_LMPC_casadi.m:161-162), 105 vars."""
    import bqp
    from oracle import dense_qp, qp_forms
    g = golden('dms_DMS_N50_tLMPC.npz')
    X = g['x'][g['idx'][:4]]
    qps = [qp_forms.dms_dense(mg, 20, x, *term_set) for x in X]
    q0 = qps[0]
    lb = np.stack([q['lb'] for q in qps]); ub = np.stack([q['ub'] for q in qps])
    x, fval, flag, out, lam = bqp.quadprog(q0['H'], q0['f'], q0['A'], q0['b'], q0['Aeq'],
                                           q0['beq'], lb, ub, handle=handle)
    assert (flag == 1).all(), flag
    for i, q in enumerate(qps):
        z, fv, _, _ = dense_qp.solve(q)
        assert np.abs(x[i] - z).max() / max(1, np.abs(z).max()) < 1e-7


def test_box_bounds_and_infeasible_free(handle):
    """Small random strictly convex QPs with bounds and inequalities vs the dense oracle."""
    import bqp
    from oracle import dense_qp, qp_forms
    rng = np.random.default_rng(7)
    n, m, B = 12, 30, 24
    M = rng.standard_normal((B, n, n))
    H = M @ np.swapaxes(M, 1, 2) + n * np.eye(n)
    f = rng.standard_normal((B, n))
    A = rng.standard_normal((B, m, n))
    b = rng.uniform(0.5, 2.0, (B, m))
    lb = -np.ones(n); ub = np.ones(n)
    x, fval, flag, out, lam = bqp.quadprog(H, f, A, b, lb=lb, ub=ub, handle=handle)
    assert (flag == 1).all()
    for i in range(B):
        z, fv, _, _ = dense_qp.solve(qp_forms.dense_qp(H[i], f[i], A[i], b[i], lb=lb, ub=ub))
        assert np.abs(x[i] - z).max() < 1e-8
        assert abs(fval[i] - fv) < 1e-8 * max(1, abs(fv))


def test_condensed_c2_batch_on_matrix_cores(mg, term_set, handle):
    """the C2 states through bqp.condense + bqp.quadprog (H, A shared; f, b per instance): the
    n = 21 instances run dense_wave_kernel<2> (MFMA factorisation); first moves within 1e-8 of
    z*, multipliers satisfy quadprog's stationarity"""
    import bqp
    from bqp.condense import Condensed
    g = golden('lmpc_N20.npz')
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                  mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                  term_set[0], term_set[1], N=20)
    cd = Condensed(lm.prob)
    X0 = g['dx'][g['idx']]
    f, b = cd.rhs(X0)
    x, fval, flag, out, lam = bqp.quadprog(cd.H, f, cd.A, b, handle=handle)
    assert (flag == 1).all()
    u, th, xs = cd.recover(x, X0)
    assert np.abs(u[:, 0, 0] - g['du_star']).max() < 1e-8
    for i in range(len(X0)):
        r = cd.H @ x[i] + f[i] + cd.A.T @ lam['ineqlin'][i]
        assert np.abs(r).max() < 1e-6 * (1 + np.abs(f[i]).max())


@pytest.mark.parametrize('n', [101, 108, 109, 122, 123, 130])
def test_dense_lds_layout_sizes(n, handle):
    """the workgroup kernel's LDS layouts around their budget edges: n <= 108 two
    global_load_lds A'DA buffers + the factor in LDS, 109 .. 122 one row tile + the factor in
    LDS, >= 123 the factor in the global workspace - each size must solve (not fail the launch)
    to the exact optimum (LDP/NNLS + active-set KKT solve, oracle/exact_qp.py)"""
    import bqp
    from oracle import exact_qp
    rng = np.random.default_rng(100 + n)
    m, B = 160, 4
    M = rng.standard_normal((n, n))
    H = M @ M.T / n + np.eye(n)
    A = rng.standard_normal((m, n))
    f = rng.standard_normal((B, n))
    b = rng.uniform(0.2, 1.0, (B, m))
    x, fval, flag, out, lam = bqp.quadprog(H, f, A, b, handle=handle)
    assert (flag == 1).all(), flag
    for i in range(B):
        z = exact_qp.solve(H, f[i], A, b[i])["z"]
        # the interior-point stop (stationarity 1e-8 relative, no polish after a converged exit)
        # leaves these 66-active-row random QPs within ~1e-8 of z*
        assert np.abs(x[i] - z).max() / max(1, np.abs(z).max()) < 5e-8


@pytest.mark.parametrize('m', [300, 1024])
def test_dense_rows_in_registers_equals_workspace_form(m, handle):
    """round 6: dense_ipm_kernel keeps the row state of A's rows in registers and the n-vectors in
    LDS when they fit (m <= 1024, n <= 106: the learned loop's sub-problem is n = 101, m = 1024);
    BQP_DENSE_NO_RG=1 selects the workspace form of the same iteration.  The two are compiled
    separately and are not bit-identical (a product with two uses, e.g. t lam in the residual
    pass, is fused into an FMA where the workspace form re-loads its operands and kept where the
    register form shares it), and on these degenerate random QPs (about a third of 1024 rows
    active) round-off moves the iteration count (tools/diag_dense_rg.py: 18 / 16 and 18 / 35
    iterations, each form deterministic run to run): both converge, to the same optimum (x within
    1e-8, f within 1e-9 relative), each run of the register form repeats bit for bit, KKT
    stationarity holds, and for m = 300 the result is the exact optimum (oracle/exact_qp.py)."""
    import os
    import bqp
    from oracle import exact_qp
    n, B = 101, 4
    rng = np.random.default_rng(7 + m)
    M = rng.standard_normal((n, n))
    H = M @ M.T / n + np.eye(n)
    A = rng.standard_normal((m, n))
    f = rng.standard_normal((B, n))
    b = rng.uniform(0.2, 1.0, (B, m))
    lb, ub = -2.0 * np.ones(n), 2.0 * np.ones(n)
    x, fval, flag, out, lam = bqp.quadprog(H, f, A, b, lb=lb, ub=ub, handle=handle)
    x2, fval2, flag2, out2, lam2 = bqp.quadprog(H, f, A, b, lb=lb, ub=ub, handle=handle)
    os.environ['BQP_DENSE_NO_RG'] = '1'
    try:
        xw, fw, flw, outw, lamw = bqp.quadprog(H, f, A, b, lb=lb, ub=ub, handle=handle)
    finally:
        del os.environ['BQP_DENSE_NO_RG']
    print('m %d: iterations %s / %s, max |dx| %.2e' % (m, out['iterations'], outw['iterations'], np.abs(x - xw).max()))
    assert np.array_equal(x, x2) and np.array_equal(out['iterations'], out2['iterations'])
    assert (flag == 1).all() and (flw == 1).all()
    assert np.abs(x - xw).max() < 1e-8 * max(1.0, np.abs(x).max())
    assert np.abs(fval - fw).max() < 1e-9 * max(1.0, np.abs(fw).max())
    for i in range(B):
        r = H @ x[i] + f[i] + A.T @ lam['ineqlin'][i] + lam['upper'][i] - lam['lower'][i]
        assert np.abs(r).max() < 1e-6 * (1 + np.abs(f[i]).max())
    if m == 300:
        A2 = np.vstack([A, np.eye(n), -np.eye(n)])
        z = exact_qp.solve(H, f[0], A2, np.concatenate([b[0], ub, -lb]))["z"]
        assert np.abs(x[0] - z).max() / max(1, np.abs(z).max()) < 5e-8


def test_nonsymmetric_h_uses_symmetric_part(handle):
    """MATLAB quadprog solves with (H + H')/2 when H is not symmetric; the host entry
    symmetrises its staging copy, so the result equals the solve with the symmetric part (to the
    same bits: the symmetrised copy is what the kernel reads) and the exact optimum of that QP"""
    import bqp
    from oracle import exact_qp
    rng = np.random.default_rng(71)
    for n, m in ((12, 30), (40, 120)):
        M = rng.standard_normal((n, n))
        Hs = M @ M.T / n + np.eye(n)
        S = rng.standard_normal((n, n))
        Hn = Hs + 0.3 * (S - S.T)                  # same symmetric part
        f = rng.standard_normal((3, n))
        A = rng.standard_normal((m, n))
        b = rng.uniform(0.2, 1.0, (3, m))
        xn, fn, flag_n, _, _ = bqp.quadprog(Hn, f, A, b, handle=handle)
        xs, fs, flag_s, _, _ = bqp.quadprog(0.5 * (Hn + Hn.T), f, A, b, handle=handle)
        assert (flag_n == 1).all() and (flag_s == 1).all()
        assert np.array_equal(xn, xs)
        for i in range(3):
            z = exact_qp.solve(Hs, f[i], A, b[i])['z']
            assert np.abs(xn[i] - z).max() / max(1, np.abs(z).max()) < 1e-8
