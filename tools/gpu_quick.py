"""Quick GPU sanity run: F1 N=20 fixtures through libbqp vs C port and oracle z*."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
import numpy as np
import bqp
from oracle import qp_forms as qf, cpu_ref
from oracle.mg_model import mg_problem
mg = mg_problem()
ts = np.load(os.path.join(ROOT, 'tests/golden/term_set.npz'))
g = np.load(os.path.join(ROOT, 'tests/golden/lmpc_N20.npz'))
N = 20
ocp = qf.lmpc_ocp(mg, N, ts['F_w_N'], ts['h_w_N'])
prob = bqp.OcpProblem(ocp['A'], ocp['B'], ocp['W'], N, 1, w=ocp['w'], xlb=ocp['xlb'], xub=ocp['xub'],
                      ulb=ocp['ulb'], uub=ocp['uub'], Fp=ocp['Fp'], hp=ocp['hp'], poly_stage=ocp['kp'])
X0 = g['dx'][g['idx']]
r = bqp.solve_ocp(prob, X0)
c = cpu_ref.solve(ocp, X0)
print('exitflag', np.unique(r.exitflag, return_counts=True), 'iters gpu', r.iterations[:16], 'cpu', c['iterations'][:16])
print('gpu vs cpu x', np.abs(r.x - c['x']).max(), 'u', np.abs(r.u - c['u']).max())
print('gpu du0 vs z*', np.abs(r.u[:, 0, 0] - g['du_star']).max())
for B in (1024, 65536):
    Xb = g['dx'][np.arange(B) % 1000]
    r = bqp.solve_ocp(prob, Xb)
    h = bqp.ocp._default_handle()
    t0 = time.time(); r = bqp.solve_ocp(prob, Xb); t1 = time.time()
    ms, _ = h.kernel_ms()
    print('batch', B, 'kernel ms', ms, 'QP/s', B / (ms * 1e-3), 'wall', t1 - t0, 'conv', (r.exitflag == 1).mean(), 'mean it', r.iterations.mean())
