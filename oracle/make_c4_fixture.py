"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Golden fixture of config C4 (65 536 perturbed Moore-Greitzer models, N = 20):
the perturbed nominalModel.m:28 solved at the call site ocpLMPC.m:24, i.e. the F1 QP of
costLMPC.m / constraintsLMPC.m with A_i = A + 0.01 E_i |A|, B_i = B + 0.01 e_i |B| (seed 4) and
x0 cycled from the 1000 stored closed-loop states of LMPC_N20_sys_full.mat.

For every model the exact LDP/NNLS solve of oracle/exact_qp.py classifies the QP (feasible /
primal infeasible); the feasible ones get z* = [u_0 .. u_19; theta], the infeasible ones the LP
margin max s: C z + s <= b (< 0).  Committed as tests/golden/c4_exact.npz:
    feasible   (65536,) bool
    z_idx      (K,) indices of the models whose optimum is stored: the round-2 reproducers
               (20712, 11001, 6264, 2008, 7019) and a seeded sample of 4096 feasible models
    z_star     (K, 21)
    margin_inf (n_infeasible,)  LP margin of the infeasible models (row-normalised)
Usage: python oracle/make_c4_fixture.py [--procs 8]

Long horizons (the C4 generator at N = 80 and N = 100, where the round-3
polish left -8 exits on strictly feasible models): ``--N 80`` / ``--N 100`` writes
tests/golden/c4_exact_N{80,100}.npz with the same fields; z_idx there holds every model the C
restatement polishes (oracle/cpu_ipm.c, the instances that need the active-set polish) plus a
seeded sample of 512 feasible models.

``--mixed``: the 512-model sample of tests/test_gpu_mixed.py (the same generator drawn for 512
models, x0 = the first 512 stored C2 states) at N = 80, exact classification and z* of every
feasible model -> tests/golden/c4_mixed_N80.npz.  Its model 28 is the strictly feasible QP (LP
margin 0.115) on which the round-3 restatement ended -8.
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import exact_qp, qp_forms  # noqa: E402
from oracle.mg_model import mg_problem  # noqa: E402

GOLD = os.path.join(ROOT, 'tests', 'golden')
TOTAL = 65536


def c4_models(total=TOTAL):
    """the C4 generator (seed 4): per-model A (total, 4, 4), B (total, 4, 1),
    x0 (total, 4); identical to bench.py workload('C4')"""
    mg = mg_problem()
    rng = np.random.default_rng(4)
    E = rng.standard_normal((total, 4, 4))
    e = rng.standard_normal((total, 4, 1))
    A = mg['A'] + 0.01 * E * np.abs(mg['A'])
    B = mg['B'].reshape(4, 1) + 0.01 * e * np.abs(mg['B'].reshape(4, 1))
    dx = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))['dx']
    X = dx[np.arange(total) % 1000]
    return A, B, X


_W = {}


def _init(N=20):
    ts = np.load(os.path.join(GOLD, 'term_set.npz'))
    _W['ocp'] = qp_forms.lmpc_ocp(mg_problem(), N, ts['F_w_N'], ts['h_w_N'])
    _W['A'], _W['B'], _W['X'] = c4_models()


def _one(i):
    ocp = _W['ocp']
    qp = exact_qp.condense_ocp(ocp, _W['X'][i], A=_W['A'][i], B=_W['B'][i])
    r = exact_qp.solve(qp['H'], qp['f'], qp['A'], qp['b'])
    if r['status'] == 'optimal':
        return True, r['z'], 0.0
    return False, None, exact_qp.lp_margin(qp['A'], qp['b'])


def mixed_models(n=512):
    """tests/test_gpu_mixed.py's sample: the C4 generator drawn for n models"""
    mg = mg_problem()
    rng = np.random.default_rng(4)
    E = rng.standard_normal((n, 4, 4))
    e = rng.standard_normal((n, 4, 1))
    A = mg['A'] + 0.01 * E * np.abs(mg['A'])
    B = mg['B'].reshape(4, 1) + 0.01 * e * np.abs(mg['B'].reshape(4, 1))
    X = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))['dx'][:n]
    return A, B, X


def _one_mixed(i):
    ocp = _W['ocp']
    qp = exact_qp.condense_ocp(ocp, _W['X'][i], A=_W['A'][i], B=_W['B'][i])
    r = exact_qp.solve(qp['H'], qp['f'], qp['A'], qp['b'])
    return (True, r['z'], exact_qp.lp_margin(qp['A'], qp['b'])) if r['status'] == 'optimal' else (False, None, 0.0)


def _init_mixed(N):
    ts = np.load(os.path.join(GOLD, 'term_set.npz'))
    _W['ocp'] = qp_forms.lmpc_ocp(mg_problem(), N, ts['F_w_N'], ts['h_w_N'])
    _W['A'], _W['B'], _W['X'] = mixed_models()


def main_mixed(procs):
    from multiprocessing import Pool
    with Pool(procs, initializer=_init_mixed, initargs=(80,)) as pool:
        res = pool.map(_one_mixed, range(512), chunksize=8)
    feas = np.array([r[0] for r in res])
    zi = np.flatnonzero(feas)
    Z = np.array([res[i][1] for i in zi])
    marg = np.array([r[2] for r in res])
    np.savez_compressed(os.path.join(GOLD, 'c4_mixed_N80.npz'), feasible=feas, z_idx=zi, z_star=Z,
                        margin=marg, N=80)
    print('C4 mixed sample N=80: %d feasible, %d infeasible; model 28 LP margin %.3f'
          % (feas.sum(), (~feas).sum(), marg[28]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=8)
    ap.add_argument('--N', type=int, default=20)
    ap.add_argument('--mixed', action='store_true')
    args = ap.parse_args()
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    if args.mixed:
        return main_mixed(args.procs)
    from multiprocessing import Pool
    with Pool(args.procs, initializer=_init, initargs=(args.N,)) as pool:
        res = pool.map(_one, range(TOTAL), chunksize=128)
    feas = np.array([r[0] for r in res])
    marg = np.array([r[2] for r in res if not r[0]])
    if args.N != 20:
        from oracle import cpu_ref
        _init(args.N)
        c = cpu_ref.solve(_W['ocp'], _W['X'], A=_W['A'], B=_W['B'])
        rng = np.random.default_rng(44 + args.N)
        pol = np.flatnonzero(c['polished'] != 0)
        pool_ = np.setdiff1d(np.flatnonzero(feas), pol)
        zi = np.sort(np.concatenate([pol[feas[pol]], rng.choice(pool_, 512, replace=False)]))
        Z = np.array([res[i][1] for i in zi])
        out = os.path.join(GOLD, 'c4_exact_N%d.npz' % args.N)
        np.savez_compressed(out, feasible=feas, z_idx=zi, z_star=Z, margin_inf=marg, N=args.N)
        print('C4 N=%d: %d feasible, %d infeasible (LP margin max %.3e); %d polished by the C '
              'restatement' % (args.N, feas.sum(), (~feas).sum(), marg.max(), len(pol)))
        return
    named = np.array([20712, 11001, 6264, 2008, 7019])
    rng = np.random.default_rng(44)
    pool_ = np.setdiff1d(np.flatnonzero(feas), named)
    zi = np.concatenate([named, np.sort(rng.choice(pool_, 4096, replace=False))])
    Z = np.array([res[i][1] for i in zi])
    np.savez_compressed(os.path.join(GOLD, 'c4_exact.npz'), feasible=feas, z_idx=zi, z_star=Z,
                        margin_inf=marg)
    print('C4: %d feasible, %d infeasible (LP margin max %.3e)' % (feas.sum(), (~feas).sum(), marg.max()))


if __name__ == '__main__':
    main()
