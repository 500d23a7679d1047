"""bqp.sets (the product's per-model terminal sets, compute_MPIS.m / RunExample.m:77-108): for the
nominal double integrator the same polytope as the oracle's restatement and as the C3 fixture's
22-row set (mutual containment by LP: every row of one is implied by the other)."""
import numpy as np
from scipy.optimize import linprog

from conftest import golden


def _contains(F_out, h_out, F_in, h_in):
    """{F_in w <= h_in} subset of {F_out w <= h_out}"""
    for r, b in zip(F_out, h_out):
        res = linprog(-r, A_ub=F_in, b_ub=h_in, bounds=[(None, None)] * F_in.shape[1], method='highs')
        if res.status != 0 or -res.fun > b + 1e-7:
            return False
    return True


def test_di_terminal_set_matches_oracle_and_fixture(di):
    from bqp import sets
    from oracle import mpis
    g = golden('di_design.npz')
    F, h = sets.tracking_terminal_set(di['A'], di['B'], di['K'], di['LAMBDA'], di['PSI'],
                                      di['F_x'], di['h_x'], di['F_u'], di['h_u'])
    Fo, ho = mpis.di_terminal_set(di)
    for Fr, hr in ((Fo, ho), (g['F_T'], g['h_T'])):
        assert _contains(F, h, Fr, hr) and _contains(Fr, hr, F, h)
    assert len(h) == len(g['h_T'])


def test_pack_sets_pads_inactive_rows():
    from bqp import sets
    s1 = (np.array([[1.0, 0, 2.0]]), np.array([1.0]))
    s2 = (np.array([[0, 1.0, 0], [1.0, 1.0, 1.0]]), np.array([1.0, 2.0]))
    Fp, hp = sets.pack_sets([s1, s2], nx=2, nu=2)
    assert Fp.shape == (2, 2, 5) and hp.shape == (2, 2)
    assert np.array_equal(Fp[0, 0], [1.0, 0, 0, 0, 2.0]) and (Fp[0, 1] == 0).all() and hp[0, 1] == 1.0
    assert np.array_equal(Fp[1, 1], [1.0, 1.0, 0, 0, 1.0]) and hp[1, 1] == 2.0


def test_tracking_design_matches_oracle(di):
    """bqp.design (RunExample.m:42-60) on the nominal double integrator = the oracle's restatement"""
    from bqp import design
    d = design.tracking_design(di['A'], di['B'], di['C'], di['Q'], di['R'])
    for k in ('K', 'P', 'T', 'LAMBDA', 'PSI'):
        assert np.abs(d[k] - di[k]).max() < 1e-12, k
