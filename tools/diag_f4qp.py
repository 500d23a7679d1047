import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'learning-based-mpc_amd'); sys.path.insert(0, 'tests')
import bqp
from oracle import lbmpc
from oracle.mg_model import mg_problem
mg = mg_problem()
g = np.load('tests/golden/lbmpc_instance.npz')
p = lbmpc.f4_problem(mg, 100, g['data'], g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'], 0.01)
x0 = g['lb'][:4] - mg['x_wp']
A, b = lbmpc.constraints(p, x0)
z = np.zeros(101)
H, f = lbmpc.gn_model(p, x0, z)
print('cond H', np.linalg.cond(H), 'viol at 0', (A@z-b).max())
for opts in [dict(), dict(tol_stat=1e-10, tol_feas=1e-10, tol_comp=1e-16, max_iter=100), dict(max_iter=200)]:
    x, fv, fl, out, lam = bqp.quadprog(H, f, A, b - A @ z, options=opts)
    d_ref = lbmpc.dense_qp.solve(dict(H=H, f=f, A=A, b=b - A @ z, Aeq=np.zeros((0, 101)), beq=np.zeros(0), lb=np.full(101, -np.inf), ub=np.full(101, np.inf)))[0] if not opts else None
    print(opts, fl, out, None if d_ref is None else np.abs(x[0]-d_ref).max())
