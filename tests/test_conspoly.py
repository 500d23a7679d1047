"""Restated constraint-set construction (getCONSPOLY.m / pdiff.m) vs the sets stored in the
reference's workspace dump (DSS_NMPC.m), compared as sets of rows (MPT3 fixes no row order)."""
import numpy as np

from conftest import golden


def _match(F, h, Fr, hr, tol):
    """every row of (Fr, hr) appears in (F, h), and vice versa"""
    A = np.hstack([F, h[:, None]]); B = np.hstack([Fr, hr[:, None]])
    assert A.shape == B.shape, (A.shape, B.shape)
    for row in B:
        d = np.abs(A - row).max(axis=1)
        assert d.min() < tol, (row, d.min())
    for row in A:
        assert np.abs(B - row).max(axis=1).min() < tol


def test_getconspoly_matches_workspace_dump(mg):
    from oracle.conspoly import mg_conspoly
    g = golden('lbmpc_instance.npz')
    s = mg_conspoly(mg)
    _match(s['F_x_d'], s['h_x_d'], g['F_x_d'], g['h_x_d'], 1e-12)
    _match(s['F_x'], s['h_x'], g['F_x'], g['h_x'], 1e-12)
    # the 16-row robust terminal set (measured agreement 1.3e-12)
    _match(s['F_w_N'], s['h_w_N'], g['F_w_N'], g['h_w_N'], 1e-10)
