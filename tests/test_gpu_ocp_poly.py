"""Per-instance polytope blocks (bqp_ocp_data.sFp != 0): each instance of a batch carries its own
terminal-set matrix - e.g. sets rebuilt per learned / perturbed model (getCONSPOLY.m:28-69,
compute_MPIS.m for config C4's models).  The instance's table lives in its own LDS slot."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _lmpc(mg, ts):
    import bqp
    return bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                    mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                    ts[0], ts[1], N=20)


def test_per_instance_sets_vs_c_restatement(mg, term_set):
    """64 instances, each with its own perturbed 616-row set: GPU vs the C restatement solving
    each instance with its own set"""
    from oracle import cpu_ref, qp_forms
    g = golden('lmpc_N20.npz')
    lm = _lmpc(mg, term_set)
    prob = lm.prob
    rng = np.random.default_rng(11)
    X0 = g['dx'][g['idx']]
    B = len(X0)
    Fp = prob.Fp[None] * (1.0 + 1e-3 * rng.standard_normal((B,) + prob.Fp.shape))
    r = lm.solve(X0, Fp=Fp)
    ocp = qp_forms.lmpc_ocp(mg, 20, *term_set)
    flags = []
    for i in range(B):
        oi = dict(ocp)
        oi['Fp'] = Fp[i]
        c = cpu_ref.solve(oi, X0[i:i + 1])
        flags.append(c['exitflag'][0])
        if c['exitflag'][0] == 1:
            assert np.abs(r.u[i] - c['u'][0]).max() < 1e-8, i
            assert np.abs(r.x[i] - c['x'][0]).max() < 1e-8, i
    assert np.array_equal(r.exitflag, np.array(flags))
    assert (r.exitflag == 1).mean() > 0.9


def test_per_instance_sets_same_polytope(mg, term_set):
    """rows permuted and scaled per instance (F_i = D_i P_i F, h_i = D_i P_i h): the same set,
    so the optimum of the shared-set solve"""
    g = golden('lmpc_N20.npz')
    lm = _lmpc(mg, term_set)
    prob = lm.prob
    rng = np.random.default_rng(5)
    X0 = g['dx'][g['idx'][:32]]
    B = len(X0)
    Fp = np.empty((B,) + prob.Fp.shape)
    hp = np.empty((B, len(prob.hp)))
    for i in range(B):
        perm = rng.permutation(len(prob.hp))
        d = rng.uniform(0.5, 2.0, len(prob.hp))
        Fp[i] = d[:, None] * prob.Fp[perm]
        hp[i] = d * prob.hp[perm]
    r = lm.solve(X0, Fp=Fp, hp=hp)
    r0 = lm.solve(X0)
    assert (r.exitflag == 1).all()
    assert np.abs(r.opt_var - r0.opt_var).max() < 1e-8
