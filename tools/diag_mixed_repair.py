"""Diagnostic: why did the mixed mode's repair differ from the fp64 solve's at
max_iter = 2 (gpurun_out/r05_f3: u mismatch; r05_f1: 5 instances unpolished)?

Runs the C5 problem (F2, N = 100) on the first 64 stored states with max_iter in {1, 2, 4}:
  * the fp64 path three times and the mixed path three times, with an unrelated C2 batch solved in
    between (other data left in LDS / workspaces), and reports run-to-run bitwise equality of each;
  * per instance: fp64 vs mixed (u, x, theta, exitflag, polished, iterations) and which instances
    the mixed mode's phase 3 redid (the per-instance phase flags of the handoff);
  * the C restatement (oracle/cpu_ipm.c) at the same max_iter with the polish, as the referee.
Writes one JSON summary to stdout."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import numpy as np  # noqa: E402


def main():
    import bqp
    from conftest import golden
    from oracle import cpu_ref, qp_forms
    from oracle.mg_model import mg_problem
    mg = mg_problem()
    ts = golden('term_set.npz')
    g = golden('dms_DSS_tLMPC.npz')
    tl = bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                          mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], ts['F_w_N'],
                          ts['h_w_N'], mg['x_wp'], mg['u_wp'], N=100)
    lm = bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'], mg['LAMBDA'],
                  mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'], ts['F_w_N'], ts['h_w_N'], N=20)
    dx20 = golden('lmpc_N20.npz')['dx']
    h = bqp.Handle(0)
    X = g['x'][g['idx'][:64]]
    out = {}

    def same(a, b):
        return bool(np.array_equal(a.u, b.u) and np.array_equal(a.x, b.x) and
                    np.array_equal(a.theta, b.theta) and np.array_equal(a.exitflag, b.exitflag) and
                    np.array_equal(a.polished, b.polished))

    for mi in (1, 2, 4):
        r64, rmx = [], []
        for rep in range(3):
            lm.solve(dx20[:1024 - 24 * rep], handle=h)          # unrelated launch in between
            r64.append(tl.solve(X, handle=h, max_iter=mi))
            lm.solve(dx20[:512 + 7 * rep], handle=h)
            rmx.append(tl.solve(X, handle=h, precision=2, max_iter=mi))
        a, b = r64[0], rmx[0]
        diff = [i for i in range(len(X)) if not (np.array_equal(a.u[i], b.u[i]) and
                                                  np.array_equal(a.x[i], b.x[i]) and
                                                  a.exitflag[i] == b.exitflag[i] and
                                                  a.polished[i] == b.polished[i])]
        # referee: the C restatement, same iteration limit, polish after 0 / -8 exits
        prob = tl.prob
        ocp = dict(nx=prob.nx, nu=prob.nu, np=prob.np, N=prob.N, A=prob.A, B=prob.B, c=prob.c,
                   W=prob.W, w=prob.w, xlb=prob.xlb, xub=prob.xub, ulb=prob.ulb, uub=prob.uub,
                   Fp=prob.Fp, hp=prob.hp, kp=prob.poly_stage)
        c = cpu_ref.solve(ocp, X - tl.x_eq, max_iter=mi, threads=4)
        rec = {
            'fp64_runs_equal': [same(r64[0], r) for r in r64[1:]],
            'mixed_runs_equal': [same(rmx[0], r) for r in rmx[1:]],
            'fp64_flags': np.unique(a.exitflag, return_counts=True)[1].tolist(),
            'fp64_flag_values': np.unique(a.exitflag).tolist(),
            'fp64_polished': int(a.polished.sum()), 'mixed_polished': int(b.polished.sum()),
            'mixed_flag_values': np.unique(b.exitflag).tolist(),
            'differ_fp64_vs_mixed': diff,
            'diff_detail': [dict(i=i, flag64=int(a.exitflag[i]), flagmx=int(b.exitflag[i]),
                                 pol64=int(a.polished[i]), polmx=int(b.polished[i]),
                                 it64=int(a.iterations[i]), itmx=int(b.iterations[i]),
                                 du=float(np.abs(a.u[i] - b.u[i]).max()))
                            for i in diff[:16]],
            'cpu_flags_equal_fp64': bool(np.array_equal(c['exitflag'], a.exitflag)),
            'cpu_polished_equal_fp64': bool(np.array_equal(c['polished'], a.polished)),
            'cpu_vs_fp64_u_max': float(np.abs(c['u'] - a.u).max()),
            'cpu_vs_mixed_u_max': float(np.abs(c['u'] - b.u).max()),
            'cpu_polished': int(c['polished'].sum()),
        }
        out['max_iter_%d' % mi] = rec
        print(json.dumps({'max_iter': mi, **rec}), flush=True)


if __name__ == '__main__':
    main()
