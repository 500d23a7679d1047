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


# ------------------------------------------------------------------ LBMPC gateways
@pytest.fixture(scope='module')
def lmex():
    return Mex('lbmpc')


@pytest.fixture(scope='module')
def loopmex():
    return Mex('lbmpc_loop')


def _lbmpc_obj(mg, N, cls='LBMPC'):
    import bqp
    g = golden('lbmpc_instance.npz')
    if cls == 'LBMPC':
        return bqp.LBMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                         mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                         g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], N=N)
    return getattr(bqp, cls)(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                             mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                             g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], mg['x_wp'],
                             mg['u_wp'], N=N)


def _lbmpc_struct(m, lb, extra=None):
    """the model in lbmpc_gpu's MATLAB layout (the lbmpc_solve_gpu.m P struct)"""
    d = dict(N=lb.N, n_run=lb.n_run, term_learned=int(lb.term_learned), hessian=1, A=lb.A,
             B=lb.B, K=lb.K, Lq=lb.Lq, Lr=lb.Lr, Lp=lb.Lp, Lt=lb.Lt, LAMBDA=lb.LAMBDA, PSI=lb.PSI,
             xs=lb.xs, Ain=lb.Ain, bandwidth=lb.bandwidth, **{'lambda': lb.lam})
    d.update(extra or {})
    return m.struct(d)


def test_lbmpc_gateway_argument_errors(lmex, mg):
    lb = _lbmpc_obj(mg, 10)
    x0 = np.zeros((4, 2))
    win = np.zeros((7, 20))
    binm = np.repeat(lb.b0[:, None], 2, axis=1)
    with pytest.raises(MexError) as e:                       # P must be a struct
        lmex.call(1, lmex.mat(np.eye(2)), lmex.mat(x0), lmex.mat(win), lmex.mat(binm))
    assert e.value.ident == 'bqp:args'
    with pytest.raises(MexError) as e:                       # window with 6 rows
        lmex.call(1, _lbmpc_struct(lmex, lb), lmex.mat(x0), lmex.mat(np.zeros((6, 20))), lmex.mat(binm))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # bin not m x batch
        lmex.call(1, _lbmpc_struct(lmex, lb), lmex.mat(x0), lmex.mat(win), lmex.mat(binm[:, :1]))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # Ain with the wrong column count
        lmex.call(1, _lbmpc_struct(lmex, lb, dict(Ain=lb.Ain[:, 1:])), lmex.mat(x0), lmex.mat(win),
                  lmex.mat(binm))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # a weight factor of the wrong size
        lmex.call(1, _lbmpc_struct(lmex, lb, dict(Lq=np.eye(3))), lmex.mat(x0), lmex.mat(win),
                  lmex.mat(binm))
    assert e.value.ident == 'bqp:dims'


def test_lbmpc_loop_gateway_argument_errors(loopmex, mg):
    mpc = _lbmpc_obj(mg, 10, 'DMSLBMPC')
    P = dict(bin0=mpc.b0, Bx=mpc.Bx)
    L = dict(steps=2, delta=0.01, x_eq=mpc.x_eq, u_eq=mpc.u_eq, q=20, mask=1, warm=1)
    x0 = np.repeat(mpc.x_eq[:, None], 2, axis=1)
    with pytest.raises(MexError) as e:                       # L must be a struct
        loopmex.call(1, _lbmpc_struct(loopmex, mpc, P), loopmex.mat(np.eye(2)), loopmex.mat(x0))
    assert e.value.ident == 'bqp:args'
    with pytest.raises(MexError) as e:                       # L.q missing
        Lb = dict(L); del Lb['q']
        loopmex.call(1, _lbmpc_struct(loopmex, mpc, P), loopmex.struct(Lb), loopmex.mat(x0))
    assert e.value.ident == 'bqp:args'
    with pytest.raises(MexError) as e:                       # Bx of the wrong shape
        loopmex.call(1, _lbmpc_struct(loopmex, mpc, dict(bin0=mpc.b0, Bx=mpc.Bx[:, :3])),
                     loopmex.struct(L), loopmex.mat(x0))
    assert e.value.ident == 'bqp:dims'
    with pytest.raises(MexError) as e:                       # x_init with 3 rows
        loopmex.call(1, _lbmpc_struct(loopmex, mpc, P), loopmex.struct(L), loopmex.mat(x0[:3]))
    assert e.value.ident == 'bqp:dims'


@pytest.mark.gpu
def test_lbmpc_gateway_f3_late_solves(lmex, mg):
    """ocpLBMPC.m:31 through lbmpc_gpu: the 32 late solves of the stored fmincon closed loop
    LBMPC_N40_sys_full.mat (per-instance 7 x 99 windows in one call) - the same numbers as the
    Python shim bqp.LBMPC on the same library, first moves within 1e-8 of the restated SQP"""
    f = golden('lbmpc_N40.npz')
    lb = _lbmpc_obj(mg, 40)
    dx = f['late_dx']
    W = np.asarray(f['late_windows'])               # (batch, 7, q)
    B, _, q = W.shape
    binm = (lb.b0[None, :] + dx @ lb.Bx.T).T        # m x batch
    z, flag, lam, cost, its = lmex.call(5, _lbmpc_struct(lmex, lb, dict(q=q)), lmex.mat(dx.T),
                                        lmex.mat(np.moveaxis(W, 0, -1)), lmex.mat(binm),
                                        lmex.mat(None), lmex.struct(dict(max_iter=100, tol=1e-8)))
    r = lb.solve(dx, W, max_iter=100)
    assert (flag == 1).all() and (r.exitflag == 1).all()
    assert np.array_equal(z.T, r.z) and np.array_equal(lam.T, r.lam)
    assert np.array_equal(its[0], r.iterations)
    assert np.abs(z[0] - f['late_z_oracle'][:, 0]).max() < 1e-8


@pytest.mark.gpu
def test_lbmpc_loop_gateway_dms(loopmex, mg):
    """DMS_LBMPC_casadi.m:163-218 through lbmpc_loop_gpu (dms_lbmpc_loop_gpu.m): 6 closed-loop
    steps for two initial states - the same trajectories, learned predictions, windows and SQP
    solutions as bqp.closed_loop_sqp on the same library"""
    import bqp
    mpc = _lbmpc_obj(mg, 100, 'DMSLBMPC')
    X_INIT = np.array([[0.15, 1.2875, 1.1547, 0.0], [0.17, 1.30, 1.1547, 0.0]])
    T, q = 6, 100
    P = _lbmpc_struct(loopmex, mpc, dict(bin0=mpc.b0, Bx=mpc.Bx))
    L = loopmex.struct(dict(steps=T, delta=0.01, x_eq=mpc.x_eq, u_eq=mpc.u_eq, q=q, mask=1, warm=1))
    X, U, E, XL, I, Wn, Z = loopmex.call(7, P, L, loopmex.mat(X_INIT.T),
                                         loopmex.struct(dict(max_iter=200, tol=1e-8)))
    r = bqp.closed_loop_sqp(mpc, X_INIT, T, learning=dict(q=q, mask=1), log_z=True)
    b = len(X_INIT)
    assert (E == 1).all() and (r.exitflag == 1).all()
    assert np.array_equal(X.T.reshape(b, T + 1, 4), r.X)
    assert np.array_equal(U.T.reshape(b, T, 1), r.U)
    assert np.array_equal(XL.T.reshape(b, T + 1, 4), r.XL)
    assert np.array_equal(Wn.T.reshape(b, q, 8), r.window)
    assert np.array_equal(Z.T.reshape(b, T, -1), r.Z)
    assert np.array_equal(I.T, r.iterations)
