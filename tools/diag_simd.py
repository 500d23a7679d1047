"""Diagnostic (stamps build): which SIMD each wave of a workgroup runs on (slot 15 of the stamps)."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'learning-based-mpc_amd')]
import bqp
from bqp import _lib
_lib.LIB_PATH = os.path.join(ROOT, 'learning-based-mpc_amd', 'build', 'stamps', 'libbqp_stamps.so')
lib = _lib.load()
lib.bqp_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _lib._PD]
import bench
B = 64
lm = bench.workload('C2', B, 0, 1)['prob']
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'lmpc_N20.npz'))
h = bqp.Handle(0)
bqp.solve_ocp(lm, g['dx'][:B], handle=h)
st = np.zeros((B, 32))
_lib.check(lib.bqp_debug_stamps(h.value, 20, 6, 616, _lib.ptr(st)), 'stamps')
for wg in range(3):
    print('WG', wg, 'stage-wave SIMDs', st[4 * wg:4 * wg + 4, 15].astype(int), 'row-wave SIMDs', st[4 * wg:4 * wg + 4, 31].astype(int))
# per-instance B0 waits (slot 0 stage, 16 row) vs iterations, full C2 batch
B = 1024
X = g['dx'][np.arange(B) % 1000]
r = bqp.solve_ocp(lm, X, handle=h)
st = np.zeros((B, 32))
_lib.check(lib.bqp_debug_stamps(h.value, 20, 6, 616, _lib.ptr(st)), 'stamps')
it = r.iterations.astype(float)
tot = st[:, 1:10].sum(1) + st[:, 0]
print('iterations', np.unique(it, return_counts=True))
for name, col in (('stage B0 wait', 0), ('row B0 wait', 16), ('stage total', None)):
    v = (st[:, col] if col is not None else tot) / it
    print('%-14s per-iter: min %.0f median %.0f max %.0f' % (name, v.min(), np.median(v), v.max()))
# by slot within the workgroup
for sl in range(4):
    v = st[sl::4, 0] / it[sl::4]
    print('slot', sl, 'stage B0 wait per-iter median %.0f' % np.median(v))
wg_it = it.reshape(-1, 4)
print('workgroups with mixed iteration counts: %d of %d' % ((wg_it.max(1) != wg_it.min(1)).sum(), len(wg_it)))
