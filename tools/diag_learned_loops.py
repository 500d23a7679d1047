"""Diagnostic (CPU, test infrastructure): can any restatement of examples/DMS_LBMPC_casadi.m
reproduce the reference's stored learned-model closed loops
saved_data+plots/data/casadi/DMS_tLBMPC_q{10,50,100,500}.mat / DMS_tLBMPC.mat?

Those files hold only the plant trajectory `xlo` (4 x 500/501; the 501-column files repeat x_init
in their first two columns).  The script (DMS_LBMPC_casadi.m:163-218) solves per step the NLP

    min  delta sum_{k=0}^{N-1} |xl_k - x_eq - LAMBDA th|_Q^2 + |u_k - u_eq - PSI th|_R^2
         + |xl_N - x_eq - LAMBDA th|_P^2 + |LAMBDA th|_T^2                        (:223-247)
    s.t. xl_{k+1} = x_eq + A dxl_k + B du_k + casadiL2NW(dxl_k, du_k, data)      (:268, learned)
         x_{k+1}  = x_eq + A dx_k + B du_k                                       (:269, nominal)
         F_x_d dx_1 <= h_x_d, F_w_N [dx_1; th] <= h_w_N, F_x dx_k <= h_x, F_u du_k <= h_u

i.e. the F4 form of oracle/lbmpc.py with the terminal cost on the LEARNED state and the masked
8-row window of casadiL2NW.m (numerator not masked, denominator lambda + sum v_j k_j), then
applies u_0 to the RK4 plant and appends [dx1; dx2; du; Y; 1] by get_data.m.  Every variant
below is solved to a KKT point by the oracle's Gauss-Newton SQP (dense_qp sub-problems), cold
(z = 0) and warm (the script's shifted guess), and its second closed-loop state is compared
with the stored runs.  Usage:

    python tools/diag_learned_loops.py [--steps 3] > profiles/r03_learned/diag.log

The reference directory is read for the stored .mat files (this runs in the build container,
never on the GPU box)."""
import argparse
import os
import sys

import numpy as np
import scipy.io as sio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import lbmpc  # noqa: E402
from oracle.mg_model import mg_rk4  # noqa: E402

REF = '/root/reference/matlab/LBMPC/saved_data+plots/data/casadi'
_nw_plain = lbmpc.nw


def nw_window(mask_num=False):
    """casadiL2NW.m on an 8 x q window [X; Y; v]: g = sum Y_i k_i / (lam + sum v_j k_j)
    (mask_num: numerator weighted by v too); returns g and dg/dxi like oracle.lbmpc.nw"""
    def f(xi, data):
        X, Y, v = data[:3], data[3:7], data[7]
        d = X - xi[:, None]
        k = np.exp(-(d * d).sum(0) / lbmpc.H_BW ** 2)
        kn = k * v if mask_num else k
        den = lbmpc.LAM_NW + k @ v
        sy = Y @ kn
        dk = (k[None, :] * d) * (2.0 / lbmpc.H_BW ** 2)
        dkn = dk * v[None, :] if mask_num else dk
        dsy = Y @ dkn.T
        ds = dk @ v
        return sy / den, dsy / den - np.outer(sy, ds) / den ** 2
    return f


def load_stored():
    out = {}
    for name in ('DMS_tLBMPC_q10', 'DMS_tLBMPC_q50', 'DMS_tLBMPC_q100', 'DMS_tLBMPC_q500',
                 'DMS_tLBMPC', 'DMS_N50_tLBMPC_q10', 'DMS_N50_tLBMPC_q100', 'DSS_tLMPC'):
        p = os.path.join(REF, name + '.mat')
        d = sio.loadmat(p)
        xs = (d['xlo'] if 'xlo' in d else d['xl']).T
        if np.allclose(xs[0], xs[1]):          # 501-column files: x_init twice
            xs = xs[1:]
        out[name] = xs
    return out


def closed_loop(mg, sets, N, q, steps, variant, warm):
    """variant: dict(window='masked'|'plain'|'none', term_learned, mask_num)"""
    x_eq, u_eq = mg['x_wp'], float(mg['u_wp'])
    A, B = mg['A'], mg['B'].reshape(4)
    data = np.zeros((8, q))
    if variant['window'] == 'masked':
        data[7, 0] = 1.0                        # DMS_LBMPC_casadi.m:160-161
    lbmpc.nw = nw_window(variant.get('mask_num', False)) if variant['window'] == 'masked' else _nw_plain
    x = np.array([0.15, 1.2875, 1.1547, 0.0])  # x_init (:99)
    X = [x.copy()]
    z = None
    info = []
    for it in range(1, steps + 1):
        dwin = data if variant['window'] == 'masked' else data[:7]
        if variant['window'] == 'none':
            dwin = np.zeros((7, 1))
        p = lbmpc.f4_problem(mg, N, dwin, sets['F_w_N'], sets['h_w_N'], sets['F_x_d'], sets['h_x_d'])
        p['term_learned'] = variant['term_learned']
        z0 = z if (warm and z is not None) else None
        z, lam, inf = lbmpc.sqp(p, x - x_eq, z0=z0, max_iter=200)
        du = z[0]
        info.append((inf['iterations'], inf['stat'], du + u_eq))
        xn = mg_rk4(0.01, x, du + u_eq)
        dx = x - x_eq
        nom = A @ dx + B * du
        col = np.concatenate([[dx[0], dx[1], du], (xn - x_eq) - nom, [1.0]])
        if it < q:                              # get_data.m
            data[:, it] = col
        else:
            data = np.hstack([data[:, 1:], col[:, None]])
        if warm:                                # :209-213 shifted guess, Kstabil = 0 tail
            z = np.concatenate([z[1:N], [0.0], z[N:]])
        x = xn
        X.append(x.copy())
    return np.array(X), info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    from conftest import golden
    from oracle.mg_model import mg_problem
    mg = mg_problem()
    sets = golden('lbmpc_instance.npz')
    stored = load_stored()
    np.set_printoptions(precision=6, suppress=True, linewidth=140)
    print('stored plant states x_1, x_2 (after the first and second applied moves):')
    for k, v in stored.items():
        print('  %-22s x1 %s   x2 %s' % (k, v[1], v[2]))
    variants = [
        ('DMS_LBMPC as written (masked window, learned terminal)', dict(window='masked', term_learned=True)),
        ('masked window, nominal terminal (hybrid F4 cost)', dict(window='masked', term_learned=False)),
        ('masked numerator and denominator', dict(window='masked', term_learned=True, mask_num=True)),
        ('7-row window, zero columns counted (no validity row)', dict(window='plain', term_learned=True)),
        ('no learning (nominal model, = DSS tracking LMPC)', dict(window='none', term_learned=True)),
    ]
    for N, qs in ((100, (100, 10)), (50, (100,))):
        for q in qs:
            for name, var in variants:
                if var['window'] != 'plain' and q != qs[0]:
                    continue                    # the masked window does not depend on q early on
                for warm in (False, True):
                    X, info = closed_loop(mg, sets, N, q, args.steps, var, warm)
                    ref = 'DMS_tLBMPC_q%d' % q if N == 100 else 'DMS_N50_tLBMPC_q%d' % q
                    d = np.abs(X[:args.steps + 1] - stored[ref][:args.steps + 1]).max(axis=1)
                    print('\nN=%d q=%d %s, %s start' % (N, q, name, 'warm' if warm else 'cold'))
                    for it, (nit, st, u) in enumerate(info, 1):
                        print('  step %d: SQP it %3d stat %.1e u %.8f -> x %s  |x - %s| %.2e'
                              % (it, nit, st, u, X[it], ref, d[it]))
    lbmpc.nw = _nw_plain


if __name__ == '__main__':
    main()
