"""Diagnostic: per-phase cycle shares of the structured kernel (build: make -C learning-based-mpc_amd stamps).
Runs the C2 workload through libbqp_stamps.so and prints the mean cycles per phase per instance.

    python tools/stamps.py [BATCH] [--json OUT.json]

--json writes the summary bench.py reports as roofline.latency (stage-wave busy fraction and
cycles per iteration), tagged with the sha1 of csrc/bqp_ocp.hip so that bench can tell whether
the stamps were taken on the kernel source it runs."""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))
import numpy as np
import bqp
from bqp import _lib

_lib.LIB_PATH = os.environ.get('BQP_STAMPS_LIB') or os.path.join(ROOT, 'learning-based-mpc_amd', 'build', 'stamps',
                                                                 'libbqp_stamps.so')
lib = _lib.load()
lib.bqp_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _lib._PD]
import bench
pos = [a for a in sys.argv[1:] if not a.startswith('--')]
jout = sys.argv[sys.argv.index('--json') + 1] if '--json' in sys.argv else None
cfg = sys.argv[sys.argv.index('--config') + 1] if '--config' in sys.argv else 'C2'
for o in (jout, cfg):
    if o in pos:
        pos.remove(o)
B = int(pos[0]) if pos else {'C2': 1024, 'C3': 4096}[cfg]
# the config's bench workload (C2: MG N = 20, 616-row terminal set; C3: DI N = 30, 22 rows,
# per-instance linear terms)
wl = bench.workload(cfg, B, 0, 1)
lm, X = wl['prob'], wl['X']
h = bqp.Handle(0)
kw = {} if wl['w'] is None else dict(w=wl['w'])
r = bqp.solve_ocp(lm, X, handle=h, **kw)
r = bqp.solve_ocp(lm, X, handle=h, **kw)
st = np.zeros((B, 32))
_lib.check(lib.bqp_debug_stamps(h.value, lm.N, lm.nx + lm.nu + lm.np, lm.mp, _lib.ptr(st)), 'stamps')
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
if jout:
    src = os.path.join(ROOT, 'learning-based-mpc_amd', 'csrc', 'bqp_ocp.hip')
    waits = [i for i, n in enumerate(stage) if n.startswith('wait')]
    sw = st[:, 0:16].sum(axis=1).mean()
    busy = sw - sum(st[:, i].mean() for i in waits)
    res = {'config': cfg, 'batch': B, 'kernel_ms_stamp_build': ms, 'iterations_mean': float(it),
           'stage_wave_cycles_per_instance': float(sw),
           'stage_wave_busy_frac': float(busy / sw),
           'stage_wave_cycles_per_iter': float(busy / it),
           'phases_stage_per_iter': {n: float(st[:, i].mean() / it) for i, n in enumerate(stage)},
           'phases_row_per_iter': {n: float(st[:, 16 + i].mean() / it) for i, n in enumerate(row)},
           'source_sha1': hashlib.sha1(open(src, 'rb').read()).hexdigest(),
           'note': 's_memtime stamps of the diagnostic build (make stamps); busy = all stage-wave '
                   'phases except the barrier waits'}
    json.dump(res, open(jout, 'w'), indent=1)
    print('wrote', jout)
