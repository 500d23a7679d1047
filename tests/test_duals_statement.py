"""CPU: the dual mapping of tests/dual_map.py on the algorithm statement (oracle/ocp_ipm.py, the
iterates the GPU kernel reproduces): full dense KKT of F1 / F2 and agreement with the ground
truth lambda* where it is unique - the same checks test_gpu_duals.py runs on the GPU output."""
import numpy as np

import dual_map as dm
from conftest import golden


def test_statement_duals_f1(mg, term_set):
    from oracle import dense_qp, ocp_ipm, qp_forms
    g = golden('lmpc_N20.npz')
    N = 20
    ocp = qp_forms.lmpc_ocp(mg, N, *term_set)
    for j in (8, 9, 11, 17, 50, 63):
        dx = g['dx'][g['idx'][j]]
        r = ocp_ipm.solve(ocp, dx)
        lx, lu, lp, pi = dm.from_statement(r, N, 4, 1)
        lam = dm.f1_ineqlin(N, lx, lu, lp)
        qp = qp_forms.lmpc_dense(mg, N, dx, *term_set)
        c = r['u'][:, 0] - r['x'][:N] @ mg['K'].ravel()
        z = np.concatenate([c, r['theta']])
        st, comp, lmin, viol = dm.f1_kkt(qp, z, lam)
        assert st < 1e-10 and comp < 1e-10 and lmin > -1e-12 and viol < 1e-9
        zs, fv, ls, info = dense_qp.solve(qp)
        if dm.licq(qp['A'], lam, ls['ineqlin']):
            assert np.abs(lam - ls['ineqlin']).max() / max(1, np.abs(ls['ineqlin']).max()) < 1e-7
        else:
            assert j == 9          # the degenerate state of this set (3 active rows, rank 2)


def test_statement_duals_f2(mg, term_set):
    from oracle import dense_qp, ocp_ipm, qp_forms
    g = golden('dms_DMS_N50_tLMPC.npz')
    N = int(g['N'])
    ocp = qp_forms.dms_ocp(mg, N, *term_set)
    x = g['x'][g['idx'][0]]
    r = ocp_ipm.solve(ocp, x - mg['x_wp'].ravel())
    lx, lu, lp, pi = dm.from_statement(r, N, 4, 1)
    lin, y = dm.f2_duals(N, lx, lu, lp, pi)
    qp = qp_forms.dms_dense(mg, N, x, *term_set)
    z = np.concatenate([(r['x'] + mg['x_wp'].ravel()).ravel(),
                        (r['u'] + np.atleast_1d(mg['u_wp'])).ravel(), r['theta']])
    st, comp, lmin, viol = dm.f2_kkt(qp, z, lin, y, 4)
    assert st < 1e-10 and comp < 1e-10 and lmin > -1e-12 and viol < 1e-9
