"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

ctypes binding of ``oracle/_build/libcpu_ipm.so`` (the C restatement of the structured IPM,
``oracle/cpu_ipm.c``) — used by tests as the iterate-level cross-check of the GPU kernel and by
bench.py as the timed CPU baseline.  The struct layouts mirror include/bqp.h.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'libcpu_ipm.so')


class OcpDims(C.Structure):
    _fields_ = [('nx', C.c_int), ('nu', C.c_int), ('np', C.c_int), ('N', C.c_int),
                ('n_poly', C.c_int), ('poly_stage', C.c_int)]


_P = C.POINTER(C.c_double)


class OcpData(C.Structure):
    _fields_ = [(n, _P) for n in ('A', 'B', 'c', 'W', 'w', 'xlb', 'xub', 'ulb', 'uub', 'Fp', 'hp', 'x0')] + \
               [(n, C.c_int64) for n in ('sA', 'sB', 'sc', 'sW', 'sw', 'sxb', 'sub', 'sFp', 'shp', 'sx0')]


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.cpu_ocp_solve.restype = C.c_int
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_P)


def pack_ocp(ocp, x0, w=None, hp=None, A=None, B=None):
    """Column-major API arrays + strides for a structured OCP (oracle/qp_forms *_ocp dict).
    x0: (batch, nx); w: (batch, N+1, nv) or None; hp: (batch, mp) or None;
    A/B: (batch, nx, nx)/(batch, nx, nu) per-instance models or None (shared)."""
    nx, nu, p, N = ocp['nx'], ocp['nu'], ocp['np'], ocp['N']
    nv = nx + nu + p
    x0 = np.ascontiguousarray(np.atleast_2d(x0), dtype=np.float64)
    batch = x0.shape[0]
    keep = []

    def arr(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        keep.append(a)
        return a

    Aa = arr(ocp['A'].T) if A is None else arr(np.transpose(A, (0, 2, 1)))
    Ba = arr(ocp['B'].T) if B is None else arr(np.transpose(B, (0, 2, 1)))
    Wa = arr(np.transpose(ocp['W'], (0, 2, 1)))
    wa = arr(ocp['w']) if w is None else arr(w)
    Fa = arr(ocp['Fp'].T)
    ha = arr(ocp['hp']) if hp is None else arr(hp)
    xlb = arr(ocp['xlb']); xub = arr(ocp['xub'])
    ulb = arr(ocp['ulb']); uub = arr(ocp['uub'])
    c = arr(ocp['c'])
    dims = OcpDims(nx, nu, p, N, ocp['Fp'].shape[0], ocp['kp'])
    d = OcpData(A=_ptr(Aa), B=_ptr(Ba), c=_ptr(c), W=_ptr(Wa), w=_ptr(wa), xlb=_ptr(xlb),
                xub=_ptr(xub), ulb=_ptr(ulb), uub=_ptr(uub), Fp=_ptr(Fa), hp=_ptr(ha),
                x0=_ptr(x0),
                sA=0 if A is None else nx * nx, sB=0 if B is None else nx * nu, sc=0, sW=0,
                sw=0 if w is None else (N + 1) * nv, sxb=0, sub=0, sFp=0,
                shp=0 if hp is None else ocp['Fp'].shape[0], sx0=nx)
    keep.append(x0)
    return dims, d, batch, keep


def solve(ocp, x0, w=None, hp=None, A=None, B=None, max_iter=50, tol_stat=1e-8,
          tol_feas=1e-10, tol_comp=1e-14, tau=0.995, threads=0, polish=1):
    """polish: 1 (True, default) after 0 / -8 exits, 2 also with weakly active rows, 0 (False)
    off - the bqp_options.polish levels of the GPU solver; the result's 'polished' marks the
    instances whose answer is the active-set polish."""
    dims, d, batch, keep = pack_ocp(ocp, x0, w, hp, A, B)
    nx, nu, p, N = ocp['nx'], ocp['nu'], ocp['np'], ocp['N']
    x = np.zeros((batch, N + 1, nx)); u = np.zeros((batch, N, nu)); th = np.zeros((batch, p))
    flag = np.zeros(batch, np.int32); it = np.zeros(batch, np.int32); k3 = np.zeros((batch, 3))
    pol = np.zeros(batch, np.int32)
    rc = lib().cpu_ocp_solve(C.byref(dims), C.c_int(batch), C.byref(d), C.c_int(max_iter),
                             C.c_double(tol_stat), C.c_double(tol_feas), C.c_double(tol_comp),
                             C.c_double(tau), C.c_int(threads), _ptr(x), _ptr(u), _ptr(th),
                             flag.ctypes.data_as(C.POINTER(C.c_int)),
                             it.ctypes.data_as(C.POINTER(C.c_int)), _ptr(k3), C.c_int(int(polish)),
                             pol.ctypes.data_as(C.POINTER(C.c_int)))
    if rc != 0:
        raise RuntimeError('cpu_ocp_solve failed: %d' % rc)
    return dict(x=x, u=u, theta=th, exitflag=flag, iterations=it, kkt=k3, polished=pol)
