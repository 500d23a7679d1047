"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

ctypes binding of ``oracle/_build/libcpu_lbmpc.so`` (``oracle/cpu_lbmpc.c``: the C restatement
of bqp_closed_loop_sqp's learned-model NLP closed loop, DMS_LBMPC_casadi.m:157-218) - bench.py's
CLL CPU baseline and a cross-check of the GPU loop (tests/test_cpu_lbmpc_host.py).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'libcpu_lbmpc.so')
_P = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int)


class CllProb(C.Structure):
    _fields_ = ([(k, C.c_int) for k in ('N', 'q', 'max_iter', 'nd', 'nT', 'nFx', 'nFu')] +
                [('A', C.c_double * 16), ('B', C.c_double * 4), ('Q', C.c_double * 16),
                 ('R', C.c_double), ('P', C.c_double * 16), ('T', C.c_double * 16),
                 ('LAM', C.c_double * 4), ('PSI', C.c_double), ('xeq', C.c_double * 4),
                 ('ueq', C.c_double)] +
                [(k, C.c_double) for k in ('w_run', 'dt_plant', 'bw', 'lam_nw', 'tol')] +
                [('hessian', C.c_int)] +
                [(k, _P) for k in ('Fxd', 'hxd', 'FT', 'hT', 'Fx', 'hx', 'Fu', 'hu')])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(['make', '-s', '-C', HERE], check=True)
        _lib = C.CDLL(LIB)
        _lib.cll_loop.restype = C.c_int
        _lib.cll_loop.argtypes = [C.POINTER(CllProb), C.c_int, C.c_int, _P, C.c_int, _P, _P, _I, _I,
                                  C.c_int]
    return _lib


def _arr(a):
    return np.ascontiguousarray(np.asarray(a, float))


def loop(mg, sets, N, q, steps, x_init, mask=True, hessian=True, max_iter=200, tol=1e-8,
         delta=0.01, threads=1):
    """Closed loops of DMS_LBMPC_casadi.m from x_init (batch, 4) absolute.  mg: oracle.mg_model
    mg_problem(); sets: F_w_N, h_w_N, F_x_d, h_x_d.  Returns X (batch, steps+1, 4), U (batch,
    steps), iterations and exit flags (batch, steps)."""
    x_init = _arr(np.atleast_2d(x_init))
    b = x_init.shape[0]
    keep = {k: _arr(v) for k, v in dict(Fxd=sets['F_x_d'], hxd=np.ravel(sets['h_x_d']),
                                         FT=sets['F_w_N'], hT=np.ravel(sets['h_w_N']),
                                         Fx=mg['F_x'], hx=np.ravel(mg['h_x']),
                                         Fu=np.ravel(mg['F_u']), hu=np.ravel(mg['h_u'])).items()}
    p = CllProb()
    p.N, p.q, p.max_iter = N, q, max_iter
    p.nd, p.nT = keep['Fxd'].shape[0], keep['FT'].shape[0]
    p.nFx, p.nFu = keep['Fx'].shape[0], keep['Fu'].shape[0]
    assert keep['FT'].shape[1] == 5 and keep['Fxd'].shape[1] == 4 and keep['Fx'].shape[1] == 4
    for k, v in (('A', mg['A']), ('B', mg['B']), ('Q', mg['Q']), ('P', mg['P']),
                 ('T', float(mg['Tscalar']) * np.eye(4)), ('LAM', mg['LAMBDA']), ('xeq', mg['x_wp'])):
        getattr(p, k)[:] = list(np.ravel(np.asarray(v, float)))
    p.R = float(np.ravel(mg['R'])[0]); p.PSI = float(np.ravel(mg['PSI'])[0])
    p.ueq = float(np.ravel(mg['u_wp'])[0])
    p.w_run, p.dt_plant, p.bw, p.lam_nw, p.tol = delta, 0.01, 0.5, 1e-3, tol
    p.hessian = int(bool(hessian))
    for k, v in keep.items():
        setattr(p, k, v.ctypes.data_as(_P))
    X = np.zeros((b, steps + 1, 4)); U = np.zeros((b, steps))
    its = np.zeros((b, steps), np.int32); flags = np.zeros((b, steps), np.int32)
    rc = lib().cll_loop(C.byref(p), int(bool(mask)), b, x_init.ctypes.data_as(_P), steps,
                        X.ctypes.data_as(_P), U.ctypes.data_as(_P), its.ctypes.data_as(_I),
                        flags.ctypes.data_as(_I), int(threads))
    if rc:
        raise RuntimeError('cll_loop failed (%d)' % rc)
    return X, U, its, flags
