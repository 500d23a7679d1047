"""ctypes binding of libbqp.so (include/bqp.h).  The HIP library is mandatory: importing the
solver on a machine without the built library raises, there is no CPU fallback."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BQP_LIB: another build of the library, for A/B timing diagnostics (tools/gpu_r03_ab.sh)
LIB_PATH = os.environ.get('BQP_LIB') or os.path.join(_HERE, 'libbqp.so')

BQP_OK = 0
BQP_E_ARG = -1
BQP_E_HIP = -2
BQP_E_NODEV = -3
BQP_E_UNSUPPORTED = -4
_ERR = {BQP_E_ARG: 'invalid argument', BQP_E_HIP: 'HIP runtime error',
        BQP_E_NODEV: 'no usable gfx950 device', BQP_E_UNSUPPORTED: 'unsupported dimensions'}

_PD = C.POINTER(C.c_double)
_PI = C.POINTER(C.c_int)


class Options(C.Structure):
    _fields_ = [('max_iter', C.c_int), ('tol_stat', C.c_double), ('tol_feas', C.c_double),
                ('tol_comp', C.c_double), ('tau', C.c_double), ('precision', C.c_int),
                ('want_duals', C.c_int), ('polish', C.c_int)]


class Output(C.Structure):
    _fields_ = [('iterations', C.c_int), ('constrviolation', C.c_double),
                ('firstorderopt', C.c_double), ('mu', C.c_double), ('kkt', C.c_double * 4),
                ('polished', C.c_int)]


class OcpDims(C.Structure):
    _fields_ = [('nx', C.c_int), ('nu', C.c_int), ('np', C.c_int), ('N', C.c_int),
                ('n_poly', C.c_int), ('poly_stage', C.c_int)]


class OcpData(C.Structure):
    _fields_ = [(n, _PD) for n in ('A', 'B', 'c', 'W', 'w', 'xlb', 'xub', 'ulb', 'uub', 'Fp', 'hp', 'x0')] + \
               [(n, C.c_int64) for n in ('sA', 'sB', 'sc', 'sW', 'sw', 'sxb', 'sub', 'sFp', 'shp', 'sx0')]


class OcpDuals(C.Structure):
    _fields_ = [('pi', _PD), ('lam_x', _PD), ('lam_u', _PD), ('lam_p', _PD)]


class Dims(C.Structure):
    _fields_ = [('n', C.c_int), ('m', C.c_int), ('me', C.c_int)]


class Strides(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ('sH', 'sf', 'sA', 'sb', 'sAeq', 'sbeq', 'slb', 'sub')]


class LbmpcDims(C.Structure):
    _fields_ = [(n, C.c_int) for n in ('nx', 'nu', 'np', 'N', 'n_run', 'term_learned', 'q', 'm', 'mask',
                                       'hessian')]


class SqpLoop(C.Structure):
    _fields_ = [('bin0', _PD), ('Bx', _PD), ('warm', C.c_int), ('Z', _PD), ('iterations', _PI)]


class LbmpcData(C.Structure):
    _fields_ = [(n, _PD) for n in ('A', 'B', 'K', 'Lq', 'Lr', 'Lp', 'Lt', 'LAMBDA', 'PSI', 'xs')] + \
               [('data', _PD), ('sdata', C.c_int64), ('x0', _PD), ('sx0', C.c_int64),
                ('Ain', _PD), ('bin', _PD), ('sbin', C.c_int64),
                ('bandwidth', C.c_double), ('lambda_', C.c_double)]


EXPORTS = ['bqp_create', 'bqp_destroy', 'bqp_default_options', 'bqp_version', 'bqp_build_source_sha1',
           'bqp_solve_ocp_batched', 'bqp_solve_ocp_batched_device', 'bqp_quadprog_batched',
           'bqp_quadprog_batched_device', 'bqp_last_kernel_ms', 'bqp_nw_oracle',
           'bqp_nw_oracle_device', 'bqp_lbmpc_solve_batched', 'bqp_lbmpc_solve_batched_device',
           'bqp_closed_loop_ocp', 'bqp_closed_loop_ocp_device', 'bqp_closed_loop_lbmpc',
           'bqp_closed_loop_lbmpc_device', 'bqp_closed_loop_sqp', 'bqp_closed_loop_sqp_device',
           'bqp_debug_mixed_flags']

_lib = None


class BqpError(RuntimeError):
    pass


def load():
    """Load libbqp.so; raises BqpError (loudly) if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BqpError('libbqp.so not built (%s); run `make -C learning-based-mpc_amd` or '
                       '__graft_entry__.build()' % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    lib.bqp_version.restype = C.c_char_p
    lib.bqp_build_source_sha1.restype = C.c_char_p
    lib.bqp_create.argtypes = [C.POINTER(C.c_void_p), C.c_int]
    lib.bqp_destroy.argtypes = [C.c_void_p]
    lib.bqp_default_options.argtypes = [C.POINTER(Options)]
    lib.bqp_default_options.restype = None
    lib.bqp_solve_ocp_batched.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int,
                                          C.POINTER(OcpData), C.POINTER(Options), _PD, _PD,
                                          _PD, _PD, _PI, C.POINTER(Output), C.POINTER(OcpDuals)]
    lib.bqp_solve_ocp_batched_device.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int,
                                                 C.POINTER(OcpData), C.POINTER(Options), _PD,
                                                 _PD, _PD, _PD, _PI, C.c_void_p,
                                                 C.POINTER(OcpDuals), C.c_void_p]
    lib.bqp_quadprog_batched.argtypes = [C.c_void_p, C.POINTER(Dims), C.c_int, C.POINTER(Strides)] + \
        [_PD] * 9 + [C.POINTER(Options), _PD, _PD, _PI, _PD, _PD, _PD, _PD, C.POINTER(Output)]
    lib.bqp_quadprog_batched_device.argtypes = [C.c_void_p, C.POINTER(Dims), C.c_int, C.POINTER(Strides)] + \
        [_PD] * 8 + [C.POINTER(Options), _PD, _PD, _PI, _PD, _PD, _PD, _PD, C.c_void_p, C.c_void_p]
    lib.bqp_last_kernel_ms.argtypes = [C.c_void_p, _PD, _PI]
    lib.bqp_debug_mixed_flags.argtypes = [C.c_void_p, C.c_int, _PI]
    lib.bqp_nw_oracle.argtypes = [C.c_void_p, C.c_int, C.c_int, _PD, C.c_int64, _PD, _PD, _PD,
                                  C.c_double, C.c_double]
    lib.bqp_nw_oracle_device.argtypes = [C.c_void_p, C.c_int, C.c_int, _PD, C.c_int64, _PD, _PD,
                                         _PD, C.c_double, C.c_double, C.c_void_p]
    lib.bqp_lbmpc_solve_batched.argtypes = [C.c_void_p, C.POINTER(LbmpcDims), C.c_int,
                                            C.POINTER(LbmpcData), C.POINTER(Options), _PD, _PD,
                                            _PD, _PI, _PI]
    lib.bqp_lbmpc_solve_batched_device.argtypes = [C.c_void_p, C.POINTER(LbmpcDims), C.c_int,
                                                   C.POINTER(LbmpcData), C.POINTER(Options), _PD,
                                                   _PD, _PD, _PI, _PI, C.c_void_p]
    lib.bqp_closed_loop_ocp.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int, C.POINTER(OcpData),
                                        C.POINTER(Options), C.c_void_p, _PD, _PD, _PD, _PI]
    lib.bqp_closed_loop_ocp_device.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int,
                                               C.POINTER(OcpData), C.POINTER(Options), C.c_void_p,
                                               _PD, _PD, _PD, _PI, C.c_void_p]
    lib.bqp_closed_loop_lbmpc.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int,
                                          C.POINTER(OcpData), C.POINTER(Options), C.c_void_p,
                                          C.c_void_p, _PD, _PD, _PD, _PI]
    lib.bqp_closed_loop_lbmpc_device.argtypes = [C.c_void_p, C.POINTER(OcpDims), C.c_int,
                                                 C.POINTER(OcpData), C.POINTER(Options),
                                                 C.c_void_p, C.c_void_p, _PD, _PD, _PD, _PI,
                                                 C.c_void_p]
    lib.bqp_closed_loop_sqp.argtypes = [C.c_void_p, C.POINTER(LbmpcDims), C.c_int,
                                        C.POINTER(LbmpcData), C.POINTER(SqpLoop), C.POINTER(Options),
                                        C.c_void_p, C.c_void_p, _PD, _PD, _PD, _PI]
    lib.bqp_closed_loop_sqp_device.argtypes = [C.c_void_p, C.POINTER(LbmpcDims), C.c_int,
                                               C.POINTER(LbmpcData), C.POINTER(SqpLoop),
                                               C.POINTER(Options), C.c_void_p, C.c_void_p, _PD,
                                               _PD, _PD, _PI, C.c_void_p]
    _lib = lib
    return lib


def ocp_dims_supported(nx, nu, np_, N, mp):
    """the structured kernels' compiled set (csrc/bqp_api.cpp: ocp_supported, N + 1 <= 128,
    at most 1024 polytope rows): outside it bqp_solve_ocp_batched answers BQP_E_UNSUPPORTED by
    design"""
    return ((nx, nu, np_) in ((4, 1, 1), (2, 2, 2))) and N + 1 <= 128 and mp <= 1024


def check(rc, what):
    if rc != BQP_OK:
        raise BqpError('%s failed: %s (%d)' % (what, _ERR.get(rc, 'error'), rc))


def ptr(a):
    import numpy as np
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags['C_CONTIGUOUS']
    return a.ctypes.data_as(_PD)


def iptr(a):
    return None if a is None else a.ctypes.data_as(_PI)


def dptr(t):
    """Device pointer of a torch tensor (float64)."""
    if t is None:
        return None
    return C.cast(C.c_void_p(t.data_ptr()), _PD)


class Handle:
    """Owns a bqp_handle (one per host thread / stream)."""

    def __init__(self, device=-1):
        lib = load()
        h = C.c_void_p()
        check(lib.bqp_create(C.byref(h), C.c_int(device)), 'bqp_create')
        self._h = h
        self._lib = lib

    @property
    def value(self):
        return self._h

    def kernel_ms(self):
        ms = C.c_double(0.0)
        n = C.c_int(0)
        check(self._lib.bqp_last_kernel_ms(self._h, C.byref(ms), C.byref(n)), 'bqp_last_kernel_ms')
        return ms.value, n.value

    def mixed_flags(self, batch):
        """per instance of the last mixed-precision solve on this handle: the fp32 phase's exit
        flag, 2 where the retry launch solved it again from the fp64 start (bqp_debug_mixed_flags)"""
        import numpy as np
        out = np.zeros(batch, np.int32)
        check(self._lib.bqp_debug_mixed_flags(self._h, int(batch), out.ctypes.data_as(_PI)),
              'bqp_debug_mixed_flags')
        return out

    def close(self):
        if self._h:
            self._lib.bqp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def options(max_iter=50, tol_stat=1e-8, tol_feas=1e-10, tol_comp=1e-14, tau=0.995,
            want_duals=0, precision=0, polish=1):
    """precision: 0 fp64, 1 fp32 (structured solver; see include/bqp.h).  polish takes the C
    encoding of bqp_options.polish: 0 (the C default) or 1 after 0 / -8 exits, 2 also with weakly
    active rows, -1 off; the booleans True / False name 1 / -1."""
    o = Options()
    load().bqp_default_options(C.byref(o))
    o.max_iter, o.tol_stat, o.tol_feas, o.tol_comp, o.tau = max_iter, tol_stat, tol_feas, tol_comp, tau
    o.want_duals = want_duals
    o.precision = precision
    o.polish = (1 if polish else -1) if isinstance(polish, bool) else int(polish)
    return o
