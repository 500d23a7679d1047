"""Diagnostic: per-phase cycle shares of the structured kernel (build: make -C learning-based-mpc_amd stamps).
Runs the C2 workload through libbqp_stamps.so and prints the mean cycles per phase per instance."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
import numpy as np
import bqp
from bqp import _lib

_lib.LIB_PATH = os.path.join(ROOT, 'learning-based-mpc_amd', 'build', 'stamps', 'libbqp_stamps.so')
lib = _lib.load()
lib.bqp_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _lib._PD]
import bench
lm = bench.build_problem()
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'lmpc_N20.npz'))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
X = g['dx'][np.arange(B) % 1000]
h = bqp.Handle(0)
r = bqp.solve_ocp(lm.prob, X, handle=h)
r = bqp.solve_ocp(lm.prob, X, handle=h)
ms, _ = h.kernel_ms()
st = np.zeros((B, 16))
_lib.check(lib.bqp_debug_stamps(h.value, 20, 6, 616, _lib.ptr(st)), 'stamps')
names = ['residuals', 'factor:recip+Dx', 'factor:F\'DF', 'factor:riccati', 'solve:q+F\'e',
         'solve:prepass', 'solve:backward', 'solve:post-bwd', 'solve:forward', 'solve:post-fwd',
         'step_len', 'comp_after', 'row update', 'stage update', 'loop top', 'factor tail']
tot = st.sum(axis=1).mean()
print('batch %d kernel %.3f ms, mean iterations %.2f, cycles/instance (stamped) %.0f' % (B, ms, r.iterations.mean(), tot))
for i, n in enumerate(names):
    if st[:, i].mean() > 0:
        print('%-18s %10.0f cyc  %5.1f %%  per-iter %8.0f' % (n, st[:, i].mean(), 100 * st[:, i].mean() / tot, st[:, i].mean() / r.iterations.mean()))
