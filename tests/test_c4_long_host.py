"""CPU: the C restatement (oracle/cpu_ipm.c, the kernel's algorithm incl. the active-set polish)
on the whole C4 generator (65 536 perturbed nominalModel.m:28 models solved at ocpLMPC.m:24) at
the long horizons N = 80 and N = 100 (the round-3 polish left -8 exits on
strictly feasible models there).  Every model must end 1 or -2, equal to the exact LDP/NNLS
classification (tests/golden/c4_exact_N{80,100}.npz, oracle/make_c4_fixture.py --N), and the
polished / sampled models must sit at z* (first move and theta within 1e-8)."""
import numpy as np
import pytest

from conftest import golden


@pytest.mark.parametrize('N', [80, 100])
def test_c4_generator_long_horizon_restatement(N):
    from oracle import cpu_ref, qp_forms
    from oracle.make_c4_fixture import c4_models
    from oracle.mg_model import mg_problem
    ex = golden('c4_exact_N%d.npz' % N)
    ts = golden('term_set.npz')
    ocp = qp_forms.lmpc_ocp(mg_problem(), N, ts['F_w_N'], ts['h_w_N'])
    A, B, X = c4_models()
    c = cpu_ref.solve(ocp, X, A=A, B=B)
    f = c['exitflag']
    hist = {int(k): int((f == k).sum()) for k in np.unique(f)}
    print('C4 N=%d restatement: %s, polished %d' % (N, hist, int(c['polished'].sum())))
    assert set(hist) <= {1, -2}, hist
    assert np.array_equal(f == 1, ex['feasible'])
    zi = ex['z_idx']
    z = np.concatenate([c['u'].reshape(len(X), -1), c['theta']], axis=1)[zi]
    err = np.abs(z - ex['z_star'])
    assert err[:, 0].max() < 1e-8 and err[:, -1].max() < 1e-8, (err[:, 0].max(), err[:, -1].max())
