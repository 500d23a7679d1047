"""GPU check of config C4 (65 536 perturbed MG models, N = 20): exit-flag histogram of the GPU
solve, agreement with the C restatement (oracle/cpu_ipm.c), polish counts.

    python tools/c4_check.py [--batch B] [--no-polish]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=65536)
    ap.add_argument('--config', default='C4')
    ap.add_argument('--no-polish', action='store_true')
    args = ap.parse_args()
    import bench
    import bqp
    from oracle import cpu_ref
    wl = bench.workload(args.config, args.batch, 0, 1)
    prob = wl['prob']
    h = bqp.Handle(0)
    t0 = time.time()
    kw = {}
    if wl['A'] is not None:
        kw = dict(A=wl['A'], B=wl['B'])
    if wl['w'] is not None:
        kw['w'] = wl['w']
    r = bqp.solve_ocp(prob, wl['X'], handle=h, polish=not args.no_polish, **kw)
    t1 = time.time()
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or len(os.sched_getaffinity(0))
    c = cpu_ref.solve(bench.ocp_dict(prob), wl['X'], threads=threads, polish=not args.no_polish, **kw)
    t2 = time.time()
    fg, fc = r.exitflag, c['exitflag']
    hist = lambda f: {int(k): int((f == k).sum()) for k in np.unique(f)}
    both = (fg == 1) & (fc == 1)
    du = np.abs(r.u - c['u']).reshape(len(fg), -1).max(axis=1)
    print('%s batch %d: GPU flags %s (%.1fs host call), C flags %s (%.1fs)'
          % (args.config, len(fg), hist(fg), t1 - t0, hist(fc), t2 - t1))
    print('flag mismatches %d; |u_gpu - u_c| max over converged %.3e (>1e-8: %d)'
          % (int((fg != fc).sum()), du[both].max() if both.any() else 0.0, int((du[both] > 1e-8).sum())))
    print('polished GPU %d  C %d; iterations GPU mean %.3f  C mean %.3f'
          % (int(r.polished.sum()), int(c['polished'].sum()), r.iterations.mean(), c['iterations'].mean()))
    bad = np.flatnonzero(fg != fc)[:20]
    for i in bad:
        print('  mismatch', i, 'gpu', fg[i], 'c', fc[i], 'it', r.iterations[i], c['iterations'][i])
    return 0 if (fg != fc).sum() == 0 else 1


if __name__ == '__main__':
    sys.exit(main())
