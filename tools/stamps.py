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
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'lmpc_N20.npz'))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
lm = bench.workload('C2', B, 0, 1)['prob']
X = g['dx'][np.arange(B) % 1000]
h = bqp.Handle(0)
r = bqp.solve_ocp(lm, X, handle=h)
r = bqp.solve_ocp(lm, X, handle=h)
st = np.zeros((B, 32))
_lib.check(lib.bqp_debug_stamps(h.value, 20, 6, 616, _lib.ptr(st)), 'stamps')
# STAMP(id) closes phase id; the phase names follow the barrier schedule of bqp_ocp.hip
stage = ['wait B0 + residual combine', 'combine', 'wait B1', 'decide + factor', 'wait B2',
         'solve pred (post-fwd)', 'wait B3,B4', 'solve corr (post-fwd)', 'wait B5,B6', 'update + partials',
         'solves: rhs + pre-pass', 'solves: backward sweep', 'solves: post-backward',
         'solves: theta + forward sweep', 'solves: post-forward']
row = ['wait B0', 'row residuals', 'rhs pred', 'wait B1,B2', 'wait B3',
       'pred pass/sigma/rhs corr', 'wait B4,B5', 'ratio corr + box apply', 'wait B6 + poly apply/lam side']
ms, _ = h.kernel_ms()
it = r.iterations.mean()
print('batch %d kernel %.3f ms, mean iterations %.2f' % (B, ms, it))
for role, names, base in (('stage wave', stage, 0), ('row wave', row, 16)):
    tot = st[:, base:base + 16].sum(axis=1).mean()
    print('%s: cycles/instance (stamped loop) %.0f' % (role, tot))
    for i, n in enumerate(names):
        v = st[:, base + i].mean()
        if v > 0:
            print('  %-28s %10.0f cyc  %5.1f %%  per-iter %8.0f' % (n, v, 100 * v / tot, v / it))
