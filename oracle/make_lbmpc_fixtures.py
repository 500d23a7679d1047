"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Golden fixtures pinning the fmincon LBMPC path (form F3, ``functions/ocpLBMPC.m``) to the
reference's stored closed loops ``saved_data+plots/data/LBMPC_N{40,50}_sys_full.mat``.  Runs
only in the build container (reads /root/reference); writes plain numeric .npz data.

    python -m oracle.make_lbmpc_fixtures        # writes tests/golden/lbmpc_N{40,50}.npz

Reconstruction of each stored solve (ocpLBMPC.m:10-31 with update_data.m:3-10):
* sysH(:, k+1) = [dx_k; du_k]: the state the k-th solve used and the move it applied
  (the first column is [dx_init; 0] and the `x = x_k1` lag makes column 2 repeat dx_init);
* the data window of solve k (k >= 2) holds, after the initial zero point, the transitions
  j = 1..k-1:  X_j = [dx_j(1:2); du_j],  Y_j = dx_{j+1} - (A dx_j + B du_j)  (ocpLBMPC.m:13-14);
  update_data appends while k < q = 100 and afterwards drops the oldest column, so from k = 100
  on the window holds 99 points (the zero point leaves first);
* solve 1 uses the zero window alone: g_NW = 0 and F3 is exactly the LMPC QP with the
  LBMPC sets (the 16-row robust terminal set and F_x_d at x_1).
The oracle's F3 restatement (oracle/lbmpc.py: costLBMPC.m / constraintsLBMPC.m, GN-SQP) is
solved at the selected solves and its first move du = K dx + c_0 compared with fmincon's
stored du_k; the per-solve agreement is stored with the fixture (err_vs_matlab).
"""
import os
import sys

import numpy as np
import scipy.io as sio

from . import lbmpc
from .make_fixtures import DATA, OUT
from .mg_model import mg_problem

Q_WIN = 100                       # ocpLBMPC.m:18


def windows(sysH, A, B):
    """data window (7 x q) of every solve k = 1..K (list index k - 1)."""
    K = sysH.shape[1] - 1
    ds = lambda k: sysH[:4, k]     # dx_k (1-based solve k) = sysH(1:4, k+1)
    da = lambda k: sysH[4, k]
    X = [np.zeros(3)]
    Y = [np.zeros(4)]
    out = [np.vstack([np.array(X).T, np.array(Y).T])]
    for k in range(2, K + 1):
        j = k - 1
        Xj = np.array([ds(j)[0], ds(j)[1], da(j)])
        Yj = ds(j + 1) - (A @ ds(j) + B * da(j))
        if k < Q_WIN:
            X.append(Xj); Y.append(Yj)
        else:
            X = X[1:] + [Xj]; Y = Y[1:] + [Yj]
        out.append(np.vstack([np.array(X).T, np.array(Y).T]))
    return out


def main():
    mg = mg_problem()
    g = np.load(os.path.join(OUT, 'lbmpc_instance.npz'))
    A, B = mg['A'], mg['B'].ravel()
    rng = np.random.default_rng(40)
    for N in (40, 50):
        sysH = sio.loadmat(DATA + '/LBMPC_N%d_sys_full.mat' % N)['sysH']
        W = windows(sysH, A, B)
        early = [1, 2, 3, 5, 10, 30, 60, 99]                         # one window size each
        late = np.sort(rng.choice(np.arange(100, 1000), 32, replace=False))   # q = 99
        res = {}
        for name, ks in (('early', early), ('late', list(late))):
            dx, du, z, it, err = [], [], [], [], []
            kept = []
            for k in ks:
                x0 = sysH[:4, k]
                p = lbmpc.f3_problem(mg, N, W[k - 1], g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'])
                try:
                    with np.errstate(all='ignore'):
                        zk, lam, info = lbmpc.sqp(p, x0, max_iter=200)
                except np.linalg.LinAlgError:
                    zk = np.full(N + 1, np.nan)
                if not np.all(np.isfinite(zk)):
                    # the restated SQP breaks down at this solve (its dense QP sub-problem
                    # diverges): not a pinned instance
                    print('  N=%d solve %d: oracle SQP failed, skipped' % (N, k))
                    continue
                kept.append(k)
                d = float(mg['K'].ravel() @ x0 + zk[0])
                dx.append(x0); du.append(sysH[4, k]); z.append(zk); it.append(info['iterations'])
                err.append(abs(d - sysH[4, k]))
            ks = kept
            res[name + '_k'] = np.array(ks)
            res[name + '_dx'] = np.array(dx)
            res[name + '_du_matlab'] = np.array(du)
            res[name + '_z_oracle'] = np.array(z)
            res[name + '_sqp_iters'] = np.array(it)
            res[name + '_err_vs_matlab'] = np.array(err)
            print('F3 N=%d %s: oracle vs fmincon first move median %.2e max %.2e' %
                  (N, name, np.median(err), np.max(err)))
        for k in res['early_k']:
            res['window_%d' % k] = W[k - 1]
        res['late_windows'] = np.stack([W[k - 1] for k in res['late_k']])
        np.savez(os.path.join(OUT, 'lbmpc_N%d.npz' % N), N=N, **res)


if __name__ == '__main__':
    sys.exit(main())
