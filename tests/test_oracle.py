"""CPU tests: the oracle itself, pinned against the reference's stored MATLAB results."""
import numpy as np
import pytest

from conftest import golden


def test_mg_model_matches_matlab_dump(mg):
    """mgcmDLTI.m / matOCP.m restatement vs the R2019a workspace dump (DSS_NMPC.m:7-107)."""
    c = golden('mg_constants.npz')
    assert np.abs(mg['A'] - c['A']).max() < 1e-14
    assert np.abs(mg['B'].ravel() - c['B']).max() < 1e-14
    assert np.abs(mg['K'].ravel() - c['K']).max() < 1e-11
    assert np.abs(mg['P'] - c['P']).max() / np.abs(c['P']).max() < 1e-12
    assert np.abs(mg['LAMBDA'].ravel()[:3] - c['LAMBDA'][:3]).max() < 1e-13
    assert abs(mg['PSI'].item() - c['PSI'][0]) < 1e-13


def test_term_set_fixture(term_set):
    F, h = term_set
    assert F.shape == (616, 5) and h.shape == (616,)
    assert np.all(h == 1.0)


@pytest.mark.parametrize('N', [20, 40, 50])
def test_f1_oracle_matches_fmincon(N):
    """Exact QP optimum of the restated costLMPC/constraintsLMPC vs fmincon's stored move."""
    g = golden('lmpc_N%d.npz' % N)
    err = g['err_vs_matlab']
    # fmincon (sqp, default tolerances) agrees to ~1e-7; a few degenerate steps to ~1e-6.
    assert np.median(err) < 1e-7
    assert err.max() < 1e-6


def test_f1_oracle_recompute(mg, term_set):
    from oracle import dense_qp, qp_forms
    g = golden('lmpc_N20.npz')
    for j in range(3):
        i = g['idx'][j]
        qp = qp_forms.lmpc_dense(mg, 20, g['dx'][i], *term_set)
        z, fval, lam, info = dense_qp.solve(qp)
        assert np.abs(z - g['z_star'][j]).max() < 1e-9
        k = info['kkt']
        assert k['stationarity'] < 1e-9 and k['primal_ineq'] < 1e-12


def test_f2_oracle_matches_ipopt():
    g = golden('dms_DSS_tLMPC.npz')
    assert np.median(g['err_vs_ipopt']) < 1e-8
    assert g['err_vs_ipopt'].max() < 1e-5
    assert g['rk4_residual'].max() < 1e-13
    g = golden('dms_DMS_N50_tLMPC.npz')
    assert np.median(g['err_vs_ipopt']) < 1e-6


def test_structured_form_equals_reference_loops(mg, term_set):
    """lmpc_ocp (stage-wise description) has the same optimum as lmpc_dense (reference loops)."""
    from oracle import dense_qp, qp_forms
    g = golden('lmpc_N20.npz')
    ocp = qp_forms.lmpc_ocp(mg, 20, *term_set)
    for j in (0, 5):
        dx = g['dx'][g['idx'][j]]
        z2, f2, _, _ = dense_qp.solve(qp_forms.ocp_to_dense(ocp, dx))
        u0 = z2[21 * 4]
        assert abs(u0 - g['du_star'][j]) < 1e-9


def test_numpy_spec_ipm(mg, term_set):
    from oracle import ocp_ipm, qp_forms
    g = golden('lmpc_N20.npz')
    ocp = qp_forms.lmpc_ocp(mg, 20, *term_set)
    for j in range(4):
        r = ocp_ipm.solve(ocp, g['dx'][g['idx'][j]])
        assert r['exitflag'] == 1
        assert abs(r['u'][0, 0] - g['du_star'][j]) < 1e-8


def test_cpu_port_matches_spec_and_golden(mg, term_set):
    """C port (oracle/cpu_ipm.c) == numpy spec to round-off, == z* to 1e-8."""
    from oracle import cpu_ref, ocp_ipm, qp_forms
    g = golden('lmpc_N20.npz')
    ocp = qp_forms.lmpc_ocp(mg, 20, *term_set)
    X0 = g['dx'][g['idx']]
    r = cpu_ref.solve(ocp, X0)
    assert (r['exitflag'] == 1).all()
    assert np.abs(r['u'][:, 0, 0] - g['du_star']).max() < 1e-8
    K = mg['K'].ravel()
    c = r['u'][:, :, 0] - r['x'][:, :20, :] @ K
    zs = g['z_star']
    assert np.abs(c - zs[:, :20]).max() / max(1.0, np.abs(zs).max()) < 1e-8
    for j in range(2):
        rn = ocp_ipm.solve(ocp, X0[j])
        assert rn['iterations'] == r['iterations'][j]
        assert np.abs(rn['x'] - r['x'][j]).max() < 1e-11


def test_cpu_port_f2_n100(mg, term_set):
    from oracle import cpu_ref, qp_forms
    g = golden('dms_DSS_tLMPC.npz')
    ocp = qp_forms.dms_ocp(mg, 100, *term_set)
    sel = np.arange(6)
    X0 = g['x'][g['idx'][sel]] - mg['x_wp']
    r = cpu_ref.solve(ocp, X0)
    assert (r['exitflag'] == 1).all()
    u0 = r['u'][:, 0, 0] + mg['u_wp']
    assert np.abs(u0 - g['u_star'][sel]).max() < 1e-8


def test_lbmpc_instance_fixture():
    g = golden('lbmpc_instance.npz')
    assert g['y_OL'].shape == (505,)
    assert g['data'].shape == (7, 100)
    assert g['F_w_N'].shape == (16, 5)


@pytest.mark.parametrize('name', ['LMPC_N20', 'LMPC_N40', 'LMPC_N50', 'LBMPC_N40', 'LBMPC_N50'])
def test_ode23_plant_reproduces_stored_transitions(mg, name):
    """the ode23 restatement (oracle/mg_model.py mg_ode23, models/trueModel.m:14/48) against every
    transition of the reference's stored fmincon runs: x_{k+1} = ode23(x_k, u_k) to round-off"""
    from oracle.mg_model import mg_ode23
    H = golden('fmincon_runs.npz')[name]
    xwp = np.asarray(mg['x_wp'], float); uwp = float(np.ravel(mg['u_wp'])[0])
    if name.startswith('LMPC'):       # column k+1: state after step k, move of step k
        pairs = [(H[:4, k], H[4, k + 1], H[:4, k + 1]) for k in range(H.shape[1] - 1)]
    else:                             # column k+1: state of step k and its move
        pairs = [(H[:4, k], H[4, k], H[:4, k + 1]) for k in range(1, H.shape[1] - 1)]
    err = max(np.abs(mg_ode23(0.01, x + xwp, u + uwp) - (xn + xwp)).max() for x, u, xn in pairs)
    assert err < 5e-15, err
