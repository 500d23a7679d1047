"""C emulation of the MATLAB drop-in: the MEX gateways
learning-based-mpc_amd/matlab/quadprog_gpu.c (dense, quadprog semantics) and ocp_gpu.c (the
structured fast path behind lmpc_solve_gpu.m / dms_tracking_solve_gpu.m) compiled against the
stub mex.h of tests/mex_stub/ and driven through tests/mexemu.py with arguments laid out as
MATLAB passes them.  CPU tests cover the argument checks (which run before the device is
taken); GPU tests solve through the gateways and compare with the exact optimum z* of the
fixtures and with the Python shims on the same library."""
import numpy as np
import pytest

from conftest import golden
from mexemu import Mex, MexError


def _has_gpu():
    try:
        import bqp
        bqp.Handle(0)
        return True
    except Exception:
        return False


@pytest.fixture(scope='module')
def qmex():
    return Mex('quadprog')


@pytest.fixture(scope='module')
def omex():
    return Mex('ocp')


def _lmpc(mg, ts, N=20):
    import bqp
    return bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                    mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                    ts[0], ts[1], N=N)


def _pstruct(m, prob, hp=None):
    """the stage-wise problem in ocp_gpu's MATLAB layout (column-major, stages last)"""
    return m.struct(dict(N=prob.N, nu=prob.nu, np=prob.np, A=prob.A, B=prob.B, c=prob.c,
                         W=np.moveaxis(prob.W, 0, -1), w=prob.w.T, xlb=prob.xlb.T, xub=prob.xub.T,
                         ulb=prob.ulb.T, uub=prob.uub.T, Fp=prob.Fp,
                         hp=prob.hp if hp is None else hp, poly_stage=prob.poly_stage))


# ------------------------------------------------------------------ CPU: argument checks
def test_gateways_export_mexfunction(qmex, omex):
    for m in (qmex, omex):
        assert hasattr(m.L, 'mexFunction') and hasattr(m.L, 'mexemu_call')


def test_quadprog_argument_errors(qmex):
    with pytest.raises(MexError) as e:
        qmex.call(1, qmex.mat(np.eye(2)))
    assert e.value.ident == 'bqp:args'
    with pytest.raises(MexError) as e:                       # H not n x n
        qmex.call(1, qmex.mat(np.eye(3)), qmex.mat(np.ones(2)))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # b neither m nor m x batch
        qmex.call(1, qmex.mat(np.eye(2)), qmex.mat(np.ones((2, 3))), qmex.mat(np.ones((4, 2))),
                  qmex.mat(np.ones(5)))
    assert e.value.ident == 'bqp:dims'
    lb = np.zeros((2, 3)); ub = np.ones((2, 3))
    lb[1, 2] = ub[1, 2] = 0.5                                # instance 3 fixes x2, the others do not
    with pytest.raises(MexError) as e:
        qmex.call(1, qmex.mat(np.eye(2)), qmex.mat(np.ones((2, 3))), qmex.mat(None), qmex.mat(None),
                  qmex.mat(None), qmex.mat(None), qmex.mat(lb), qmex.mat(ub))
    assert e.value.ident == 'bqp:fixed'
    with pytest.raises(MexError) as e:                       # f of a non-double class
        qmex.call(1, qmex.mat(np.eye(2)), qmex.string('ab'))
    assert e.value.ident == 'bqp:args'


def test_ocp_argument_errors(omex, mg, term_set):
    with pytest.raises(MexError) as e:                       # P must be a struct
        omex.call(1, omex.mat(np.eye(2)), omex.mat(np.ones((4, 1))))
    assert e.value.ident == 'bqp:args'
    prob = _lmpc(mg, term_set).prob
    with pytest.raises(MexError) as e:                       # x0 with the wrong number of rows
        omex.call(1, _pstruct(omex, prob), omex.mat(np.ones((3, 2))))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # hp neither shared nor per instance
        omex.call(1, _pstruct(omex, prob, hp=np.ones(len(prob.hp) + 1)), omex.mat(np.zeros((4, 2))))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # missing required field
        omex.call(1, omex.struct(dict(N=20, nu=1, np=1, A=prob.A)), omex.mat(np.zeros((4, 1))))
    assert e.value.ident == 'bqp:args'
    with pytest.raises(MexError) as e:                       # optional field of a non-double class
        omex.call(1, omex.struct(dict(N=20, nu=1, np=1, A=prob.A, B=prob.B,
                                      W=np.moveaxis(prob.W, 0, -1), w='abc')),
                  omex.mat(np.zeros((4, 1))))
    assert e.value.ident == 'bqp:args' and 'P.w' in str(e.value)
    with pytest.raises(MexError) as e:                       # x0 of a non-double class
        omex.call(1, _pstruct(omex, prob), omex.string('abcd'))
    assert e.value.ident == 'bqp:args'


def test_gateway_reports_missing_device(qmex):
    """a valid call on a machine without a gfx950 device ends in the gateway's bqp:gpu error
    (MATLAB error, not a crash)"""
    if _has_gpu():
        pytest.skip('a device is present')
    with pytest.raises(MexError) as e:
        qmex.call(1, qmex.mat(np.eye(2)), qmex.mat(np.ones(2)))
    assert e.value.ident == 'bqp:gpu'


# ------------------------------------------------------------------ GPU: solves
@pytest.mark.gpu
def test_quadprog_gateway_f1(qmex, mg, term_set):
    """fmincon LMPC (F1) in quadprog form through the MEX: 16 instances in one call (trailing
    batch dimension on f and b), x within 1e-8 of z*, lambda.ineqlin with quadprog's sign"""
    from oracle import qp_forms
    g = golden('lmpc_N20.npz')
    sel = np.arange(16)
    qps = [qp_forms.lmpc_dense(mg, 20, g['dx'][g['idx'][j]], *term_set) for j in sel]
    H, A = qps[0]['H'], qps[0]['A']
    f = np.stack([q['f'] for q in qps], axis=1)
    b = np.stack([q['b'] for q in qps], axis=1)
    x, fval, flag, out, lam = qmex.call(5, qmex.mat(H), qmex.mat(f), qmex.mat(A), qmex.mat(b))
    assert (flag == 1).all(), flag
    zs = g['z_star'][sel]
    assert np.abs(x.T - zs).max() / max(1, np.abs(zs).max()) < 1e-8
    for i in range(len(sel)):
        li = lam[i]['ineqlin'][:, 0]
        r = H @ x[:, i] + f[:, i] + A.T @ li
        assert np.abs(r).max() < 1e-6 * (1 + np.abs(f[:, i]).max())
        assert (li >= -1e-12).all()
        assert out[i]['iterations'][0, 0] >= 1
        assert abs(fval[0, i] - (0.5 * x[:, i] @ H @ x[:, i] + f[:, i] @ x[:, i])) < 1e-9 * (1 + abs(fval[0, i]))


@pytest.mark.gpu
def test_quadprog_gateway_fixed_variables(qmex):
    """lb == ub becomes an equality row inside the gateway; its multiplier comes back in
    lambda.lower / lambda.upper by sign, as quadprog reports it"""
    import bqp
    rng = np.random.default_rng(7)
    n, B = 6, 8
    M = rng.standard_normal((n, n))
    H = M @ M.T + n * np.eye(n)
    f = rng.standard_normal((n, B))
    A = rng.standard_normal((4, n))
    b = np.abs(rng.standard_normal((4, B))) + 0.1
    lb = -np.ones((n, B)); ub = np.ones((n, B))
    lb[2] = ub[2] = 0.3
    x, fval, flag, out, lam = qmex.call(5, qmex.mat(H), qmex.mat(f), qmex.mat(A), qmex.mat(b),
                                        qmex.mat(None), qmex.mat(None), qmex.mat(lb), qmex.mat(ub))
    xp, fp, flp, outp, lamp = bqp.quadprog(H, f.T, A, b.T, lb=lb.T, ub=ub.T)
    assert (flag == 1).all() and (flp == 1).all()
    assert np.abs(x.T - xp).max() < 1e-10
    assert np.abs(x[2] - 0.3).max() < 1e-12
    for i in range(B):
        r = (H @ x[:, i] + f[:, i] + A.T @ lam[i]['ineqlin'][:, 0] - lam[i]['lower'][:, 0]
             + lam[i]['upper'][:, 0])
        assert np.abs(r).max() < 1e-7


@pytest.mark.gpu
def test_ocp_gateway_lmpc(omex, mg, term_set):
    """the structured MEX on the C2 problem (F1, N=20): first moves within 1e-8 of z*, the
    same numbers as the Python shim on the same library, multipliers included"""
    g = golden('lmpc_N20.npz')
    lm = _lmpc(mg, term_set)
    prob = lm.prob
    X0 = g['dx'][g['idx']]
    X, U, th, fval, flag, out, lam = omex.call(7, _pstruct(omex, prob), omex.mat(X0.T))
    r = lm.solve(X0, want_duals=True)
    B = len(X0)
    assert (flag == 1).all()
    Xs = X.T.reshape(B, prob.N + 1, prob.nx)
    Us = U.T.reshape(B, prob.N, prob.nu)
    assert np.array_equal(Xs, r.x) and np.array_equal(Us, r.u) and np.array_equal(th.T, r.theta)
    c = Us - np.einsum('ij,bkj->bki', lm.K, Xs[:, :prob.N, :])
    opt = np.concatenate([c.reshape(B, -1), th.T], axis=1)
    zs = g['z_star']
    assert np.abs(opt - zs).max() / max(1, np.abs(zs).max()) < 1e-8
    for i in range(B):
        assert np.array_equal(lam[i]['lam_p'][:, 0], r.lam_p[i])
        assert np.array_equal(lam[i]['pi'][:, 0], r.pi[i].ravel())
        assert out[i]['iterations'][0, 0] == r.iterations[i]


@pytest.mark.gpu
def test_ocp_gateway_per_instance_and_options(omex, mg, term_set):
    """per-instance hp (a trailing batch dimension) and the options struct (precision 2 =
    mixed): same optimum as the shared-hp fp64 call"""
    g = golden('lmpc_N20.npz')
    prob = _lmpc(mg, term_set).prob
    X0 = g['dx'][g['idx'][:16]]
    ref = omex.call(5, _pstruct(omex, prob), omex.mat(X0.T))
    hpB = np.repeat(prob.hp[:, None], len(X0), axis=1)
    opt = omex.struct(dict(precision=2))
    X, U, th, fval, flag = omex.call(5, _pstruct(omex, prob, hp=hpB), omex.mat(X0.T), opt)
    assert (flag == 1).all()
    assert np.abs(U - ref[1]).max() < 1e-8
