"""GPU: multiplier outputs of the structured solve (pi, lam_x, lam_u, lam_p) mapped onto the
rows of the reference's own QP forms (tests/dual_map.py) - F1 (costLMPC.m/constraintsLMPC.m,
N=20, the 64 states of lmpc_N20.npz) and F2 (DMS_tracking_LMPC_casadi.m, N=100 and N=50) -
checked against the full dense KKT conditions and against the ground truth lambda* of the
oracle's exact active-set solve wherever lambda* is unique (active rows linearly
independent; on the degenerate states any multiplier on the optimal face is valid, so only
the KKT conditions are checked there)."""
import numpy as np
import pytest

import dual_map as dm
from conftest import golden

pytestmark = pytest.mark.gpu

TOL_KKT = 1e-8      # dense stationarity, relative to 1 + |Hz + f|
TOL_LAM = 1e-7      # |lam - lam*|_inf / max(1, |lam*|_inf) where lam* is unique


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


def test_f1_duals_vs_oracle(mg, term_set, handle):
    import bqp
    from oracle import dense_qp, qp_forms
    g = golden('lmpc_N20.npz')
    N = 20
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                  mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                  term_set[0], term_set[1], N=N)
    X = g['dx'][g['idx']]
    r = lm.solve(X, handle=handle, want_duals=True)
    assert (r.exitflag == 1).all()
    n_unique = 0
    for i in range(len(X)):
        qp = qp_forms.lmpc_dense(mg, N, X[i], *term_set)
        lam = dm.f1_ineqlin(N, r.lam_x[i], r.lam_u[i], r.lam_p[i])
        st, comp, lmin, viol = dm.f1_kkt(qp, r.opt_var[i], lam)
        assert st < TOL_KKT and comp < 1e-9 and lmin > -1e-12 and viol < 1e-9, (i, st, comp, lmin, viol)
        zs, fv, ls, info = dense_qp.solve(qp)
        if dm.licq(qp['A'], lam, ls['ineqlin']):
            n_unique += 1
            err = np.abs(lam - ls['ineqlin']).max() / max(1.0, np.abs(ls['ineqlin']).max())
            assert err < TOL_LAM, (i, err)
    assert n_unique >= 60


@pytest.mark.parametrize('fname', ['dms_DSS_tLMPC.npz', 'dms_DMS_N50_tLMPC.npz'])
def test_f2_duals_vs_oracle(mg, term_set, handle, fname):
    import bqp
    from oracle import dense_qp, qp_forms
    g = golden(fname)
    N = int(g['N'])
    tl = bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                          mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                          term_set[0], term_set[1], mg['x_wp'], mg['u_wp'], N=N)
    X = g['x'][g['idx'][:8]]
    r = tl.solve(X, handle=handle, want_duals=True)
    assert (r.exitflag == 1).all()
    for i in range(len(X)):
        qp = qp_forms.dms_dense(mg, N, X[i], *term_set)
        lin, y = dm.f2_duals(N, r.lam_x[i], r.lam_u[i], r.lam_p[i], r.pi[i])
        st, comp, lmin, viol = dm.f2_kkt(qp, r.y_OL[i], lin, y, 4)
        assert st < TOL_KKT and comp < 1e-9 and lmin > -1e-12 and viol < 1e-9, (i, st, comp, lmin, viol)
        zs, fv, ls, info = dense_qp.solve(qp)
        if dm.licq(qp['A'], lin, ls['ineqlin']):
            sc = max(1.0, np.abs(ls['ineqlin']).max(), np.abs(ls['eqlin']).max())
            assert np.abs(lin - ls['ineqlin']).max() / sc < TOL_LAM
            assert np.abs(y - ls['eqlin'][:4 * N]).max() / sc < TOL_LAM
