"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Generates the committed golden fixtures under ``tests/golden/`` from the reference's stored
results.  Runs ONLY in the build container (it reads ``/root/reference``, which does not exist
on the GPU box); the fixtures it writes are plain numeric ``.npz`` data (inputs + expected
outputs), never reference source.

    python -m oracle.make_fixtures            # rewrites tests/golden/*.npz

Sources (all MAT v5 read with scipy.io.loadmat, or numeric literals of the workspace dump):

* ``saved_data+plots/data/term_set.mat``            -> term_set.npz (F_w_N 616x5, h_w_N)
* ``examples/DSS_NMPC.m`` (R2019a workspace dump)   -> mg_constants.npz (A,B,K,P,LAMBDA,PSI,
  Mtheta) and lbmpc_instance.npz (16-row robust terminal set, F_x_d/h_x_d, data window 7x100,
  lb/ub, IPOPT optimum y_OL; hybrid LBMPC N=100)
* ``saved_data+plots/data/LMPC_N{20,40,50}_{sys,art}_full.mat`` -> lmpc_N*.npz: the 1000 stored
  closed-loop states dx_k with MATLAB fmincon's first move du_k = sysH(5,k+1) and theta via
  art_refH (ocpLMPC.m:25-38), plus exact oracle solutions z* for a subset.
* ``data/casadi/{DSS_tLMPC,DMS_tLMPC_K,tLMPC}.mat`` (N=100) and ``DMS_N50_tLMPC.mat`` (N=50)
  -> dms_N*.npz: states and IPOPT's applied input recovered by inverting the RK4 plant step
  (DMS_tracking_LMPC_casadi.m:184,297-304), plus oracle solutions for a subset.
* ``data/casadi/train_data.mat`` -> train_data.npz (LBMPC data window, 7x500).
"""
import os
import re
import sys

import numpy as np
import scipy.io as sio
from scipy.optimize import brentq

from . import dense_qp, qp_forms
from .mg_model import mg_problem, mg_rk4

REF = '/root/reference/matlab/LBMPC'
DATA = REF + '/saved_data+plots/data'
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')


def parse_matlab_literal(text, name):
    """Numeric literal ``name = [ ... ];`` of an auto-generated MATLAB workspace dump."""
    m = re.search(r'^%s = ' % re.escape(name), text, re.M)
    if m is None:
        raise KeyError(name)
    rest = text[m.end():]
    j = rest.index(';') if '[' not in rest[:rest.index(';') + 1] else None
    if j is not None:
        body = rest[:j]
    else:
        i0 = rest.index('[')
        depth = 0
        for i in range(i0, len(rest)):
            if rest[i] == '[':
                depth += 1
            elif rest[i] == ']':
                depth -= 1
                if depth == 0:
                    body = rest[i0 + 1:i]
                    break
    body = body.replace('...', ' ')
    rows = [r for r in body.split(';') if r.strip()]
    conv = lambda s: float(s.replace('Inf', 'inf').replace('NaN', 'nan'))
    mat = [[conv(v) for v in r.split()] for r in rows]
    width = max(len(r) for r in mat)
    if width == 1:
        return np.array([r[0] for r in mat])
    return np.array(mat)


def dump_constants():
    text = open(REF + '/examples/DSS_NMPC.m').read()
    g = lambda n: parse_matlab_literal(text, n)
    consts = dict(A=g('A'), B=g('B'), K=g('Kstabil'), P=g('P'), LAMBDA=g('LAMBDA'),
                  PSI=np.atleast_1d(float(re.search(r'^PSI = ([^;]+);', text, re.M).group(1))),
                  Mtheta=g('Mtheta'), Klqr=g('Klqr'))
    inst = dict(F_w_N=g('F_w_N'), h_w_N=g('h_w_N'), F_x=g('F_x'), h_x=g('h_x'),
                F_x_d=g('F_x_d'), h_x_d=g('h_x_d'), data=g('data'), lb=g('lb'), ub=g('ub'),
                y_OL=g('y_OL'), x_init=g('x_init'), solve_times=g('solve_times'),
                N=np.array(100), q=np.array(100), delta=np.array(0.01))
    return consts, inst


def write_design(consts, inst):
    """mg_design.npz: the MG LMPC design data exactly as MATLAB held it (DSS_NMPC.m dump:
    A, B, Kstabil, P, LAMBDA, PSI, F_x, h_x, F_u, h_u; Q = I, R = 1, T = 1000 from matOCP.m:27-31;
    working point from LMPC_RunExample.m:48-52).  Used by bench.py / smoke() as problem data."""
    text = open(REF + '/examples/DSS_NMPC.m').read()
    d = dict(A=consts['A'], B=consts['B'].reshape(4, 1), K=consts['K'].reshape(1, 4),
             P=consts['P'], LAMBDA=consts['LAMBDA'].reshape(4, 1), PSI=consts['PSI'].reshape(1, 1),
             Q=np.eye(4), R=np.eye(1), T=np.array(1000.0), F_x=inst['F_x'], h_x=inst['h_x'],
             F_u=parse_matlab_literal(text, 'F_u').reshape(2, 1),
             h_u=parse_matlab_literal(text, 'h_u'),
             x_wp=parse_matlab_literal(text, 'x_wp'), u_wp=np.array(1.1547))
    np.savez(os.path.join(OUT, 'mg_design.npz'), **d)


def invert_rk4(x, xn, delta=0.01):
    """Applied input u with RK4(x,u) = xn (1-D root find on the x4 component)."""
    f = lambda u: mg_rk4(delta, x, u)[3] - xn[3]
    u = brentq(f, -50.0, 50.0, xtol=1e-15, rtol=1e-15, maxiter=500)
    res = np.abs(mg_rk4(delta, x, u) - xn).max()
    return u, res


def solve_subset(build, states, idx):
    zs, its, kkts = [], [], []
    for i in idx:
        qp = build(states[i])
        z, fval, lam, info = dense_qp.solve(qp)
        zs.append(z)
        its.append(info['iterations'])
        k = info['kkt']
        kkts.append([k['stationarity'], k['primal_eq'], k['primal_ineq'], k['complementarity']])
    return np.array(zs), np.array(its), np.array(kkts)


def main():
    os.makedirs(OUT, exist_ok=True)
    consts, inst = dump_constants()
    np.savez(os.path.join(OUT, 'mg_constants.npz'), **consts)
    write_design(consts, inst)
    np.savez(os.path.join(OUT, 'lbmpc_instance.npz'), **inst)
    ts = sio.loadmat(DATA + '/term_set.mat')
    F_T = ts['F_w_N'].astype(float)
    h_T = ts['h_w_N'].astype(float).ravel()
    np.savez(os.path.join(OUT, 'term_set.npz'), F_w_N=F_T, h_w_N=h_T)
    td = sio.loadmat(DATA + '/casadi/train_data.mat')['data']
    np.savez(os.path.join(OUT, 'train_data.npz'), data=td)
    mg = mg_problem()
    rng = np.random.default_rng(20)
    # ---- F1: fmincon LMPC -----------------------------------------------------------------
    for N, nsub in ((20, 64), (40, 16), (50, 16)):
        sysH = sio.loadmat(DATA + '/LMPC_N%d_sys_full.mat' % N)['sysH']
        art = sio.loadmat(DATA + '/LMPC_N%d_art_full.mat' % N)['art_refH'].ravel()
        dx = sysH[:4, :1000].T.copy()                    # state at step k
        du = sysH[4, 1:1001].copy()                      # fmincon move applied at step k
        art_k = art[1:1001].copy()                       # Mtheta(1)*theta at step k
        idx = np.sort(np.concatenate([np.arange(8), rng.choice(np.arange(8, 1000), nsub - 8, replace=False)]))
        zs, its, kkt = solve_subset(lambda x: qp_forms.lmpc_dense(mg, N, x, F_T, h_T), dx, idx)
        du_or = zs[:, 0] + dx[idx] @ mg['K'].ravel()
        np.savez(os.path.join(OUT, 'lmpc_N%d.npz' % N), N=N, dx=dx, du_matlab=du, art_matlab=art_k,
                 idx=idx, z_star=zs, du_star=du_or, dense_iters=its, kkt=kkt,
                 err_vs_matlab=np.abs(du_or - du[idx]))
        print('F1 N=%d: oracle vs fmincon first move: median %.2e max %.2e' %
              (N, np.median(np.abs(du_or - du[idx])), np.abs(du_or - du[idx]).max()))
    f2_fixtures(mg, F_T, h_T, rng)
    # ---- F4 instance (hybrid LBMPC N=100) -------------------------------------------------
    print('lbmpc instance: y_OL', inst['y_OL'].shape, 'data', inst['data'].shape)


def f2_fixtures(mg, F_T, h_T, rng, only=None):
    # ---- F2: DMS/DSS tracking LMPC (IPOPT) ----------------------------------------------------
    # tLMPC.mat: the 600-step N = 100 tracking-LMPC run (same x_init, DSS/DMS form)
    for fname, N, nsub in (('DSS_tLMPC', 100, 64), ('DMS_tLMPC_K', 100, 8), ('DMS_N50_tLMPC', 50, 16),
                           ('tLMPC', 100, 16)):
        if only and fname not in only:
            continue
        xl = sio.loadmat(DATA + '/casadi/%s.mat' % fname)['xl']
        T = xl.shape[1] - 1
        u = np.zeros(T); res = np.zeros(T)
        for k in range(T):
            u[k], res[k] = invert_rk4(xl[:, k], xl[:, k + 1])
        idx = np.sort(np.concatenate([np.arange(4), rng.choice(np.arange(4, T), nsub - 4, replace=False)]))
        X = xl[:, :T].T.copy()
        zs, its, kkt = solve_subset(lambda x: qp_forms.dms_dense(mg, N, x, F_T, h_T), X, idx)
        u_or = zs[:, (N + 1) * 4]
        err = np.abs(u_or - u[idx])
        np.savez(os.path.join(OUT, 'dms_%s.npz' % fname), N=N, x=X, u_ipopt=u, rk4_residual=res,
                 idx=idx, z_star=zs, u_star=u_or, dense_iters=its, kkt=kkt, err_vs_ipopt=err)
        print('F2 %s N=%d: oracle vs IPOPT first move: median %.2e max %.2e (rk4 inv res %.1e)' %
              (fname, N, np.median(err), err.max(), res.max()))


if __name__ == '__main__':
    if len(sys.argv) > 1:
        # python -m oracle.make_fixtures tLMPC ...: only those F2 fixtures (then re-solve their
        # optima exactly with python oracle/refine_fixtures.py)
        ts = sio.loadmat(DATA + '/term_set.mat')
        f2_fixtures(mg_problem(), ts['F_w_N'].astype(float), ts['h_w_N'].astype(float).ravel(),
                    np.random.default_rng(21), only=sys.argv[1:])
    else:
        sys.exit(main())
