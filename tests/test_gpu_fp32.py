"""fp32 instantiation of the structured solver (config C5, "fp32 vs fp64"): same problems, solver
arithmetic and LDS state in fp32, inputs/outputs fp64.  Accuracy is stated, not assumed: the
tests record how far the fp32 solution is from the exact fp64 optimum (z* of the fixtures)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def handle():
    import bqp
    return bqp.Handle(0)


def test_fp32_f2_n100(mg, term_set, handle):
    """C5 problem (MG DMS tracking LMPC, N=100, 616-row terminal set)"""
    import bqp
    g = golden('dms_DSS_tLMPC.npz')
    tl = bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                          mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                          term_set[0], term_set[1], mg['x_wp'], mg['u_wp'], N=100)
    X = g['x'][g['idx']]
    r64 = tl.solve(X, handle=handle)
    r32 = tl.solve(X, handle=handle, precision=1)
    assert (r64.exitflag == 1).all()
    ok = r32.exitflag == 1
    err = np.abs(r32.u0[:, 0] - g['u_star'])
    print('fp32 N=100: converged %d/%d, first-move error max %.2e median %.2e, iterations %.1f vs %.1f'
          % (ok.sum(), len(ok), err.max(), np.median(err), r32.iterations.mean(), r64.iterations.mean()))
    assert ok.mean() >= 0.9
    assert np.median(err[ok]) < 1e-3


def test_fp32_f1_n20(mg, term_set, handle):
    """C2 problem in fp32"""
    import bqp
    g = golden('lmpc_N20.npz')
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                  mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                  term_set[0], term_set[1], N=20)
    r = lm.solve(g['dx'][g['idx']], handle=handle, precision=1)
    err = np.abs(r.du0[:, 0] - g['du_star'])
    print('fp32 N=20: converged %d/%d, first-move error max %.2e median %.2e'
          % ((r.exitflag == 1).sum(), len(err), err.max(), np.median(err)))
    assert (r.exitflag == 1).mean() >= 0.9
    assert np.median(err) < 1e-3
