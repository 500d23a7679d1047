"""ctypes driver of the C-emulated MEX gateways (learning-based-mpc_amd/build/libmexemu_*.so:
matlab/<name>_gpu.c compiled against tests/mex_stub/mex.h).  Arguments go in as MATLAB would
pass them (column-major doubles, structs); outputs come back as numpy arrays / lists of dicts.
Test infrastructure only."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, 'learning-based-mpc_amd', 'build')


class MexError(Exception):
    def __init__(self, ident, msg):
        super().__init__('%s: %s' % (ident, msg))
        self.ident = ident


class Mex:
    def __init__(self, name):
        path = os.path.join(BUILD, 'libmexemu_%s.so' % name)
        if not os.path.exists(path):
            raise FileNotFoundError('%s missing: run __graft_entry__.build()' % path)
        L = self.L = C.CDLL(path)
        vp = C.c_void_p
        L.mxCreateDoubleMatrix.restype = vp
        L.mxCreateDoubleMatrix.argtypes = [C.c_size_t, C.c_size_t, C.c_int]
        L.mxCreateStructMatrix.restype = vp
        L.mxCreateStructMatrix.argtypes = [C.c_size_t, C.c_size_t, C.c_int, C.POINTER(C.c_char_p)]
        L.mxSetField.argtypes = [vp, C.c_size_t, C.c_char_p, vp]
        L.mxGetField.restype = vp
        L.mxGetField.argtypes = [vp, C.c_size_t, C.c_char_p]
        L.mxGetDoubles.restype = C.POINTER(C.c_double)
        L.mxGetDoubles.argtypes = [vp]
        L.mxGetM.restype = C.c_size_t
        L.mxGetM.argtypes = [vp]
        L.mxGetN.restype = C.c_size_t
        L.mxGetN.argtypes = [vp]
        L.mxIsStruct.argtypes = [vp]
        L.mxDestroyArray.argtypes = [vp]
        L.mexemu_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp), C.c_char_p, C.c_char_p]
        L.mexemu_nfields.argtypes = [vp]
        L.mexemu_field_name.restype = C.c_char_p
        L.mexemu_field_name.argtypes = [vp, C.c_int]
        L.mexemu_is_char.argtypes = [vp]
        L.mxCreateString.restype = vp
        L.mxCreateString.argtypes = [C.c_char_p]
        self.live = []

    # ---- inputs ----
    def mat(self, a):
        """numpy -> mxArray: 1-D -> column vector; (m, n) -> m x n; (..., B) trailing batch axis
        flattened into the columns as MATLAB's column-major storage does"""
        if a is None:
            return self.L.mxCreateDoubleMatrix(0, 0, 0)
        a = np.asarray(a, dtype=np.float64)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        if a.ndim == 1:
            a = a.reshape(-1, 1)
        m = a.shape[0]
        flat = a.reshape(m, -1, order='F') if a.ndim > 2 else a
        flat = np.asfortranarray(flat)
        p = self.L.mxCreateDoubleMatrix(m, flat.shape[1], 0)
        C.memmove(self.L.mxGetDoubles(p), flat.ctypes.data, flat.nbytes)
        return p

    def string(self, text):
        """a char array (a non-double class, for the gateways' class checks)"""
        return self.L.mxCreateString(text.encode())

    def struct(self, d):
        names = (C.c_char_p * len(d))(*[k.encode() for k in d])
        s = self.L.mxCreateStructMatrix(1, 1, len(d), names)
        for k, v in d.items():
            self.L.mxSetField(s, 0, k.encode(), self.string(v) if isinstance(v, str) else self.mat(v))
        return s

    # ---- outputs ----
    def value(self, p):
        if not p:
            return None
        if self.L.mxIsStruct(p):
            n = self.L.mxGetM(p) * self.L.mxGetN(p)
            names = [self.L.mexemu_field_name(p, i).decode() for i in range(self.L.mexemu_nfields(p))]
            return [{k: self.value(self.L.mxGetField(p, i, k.encode())) for k in names} for i in range(n)]
        if self.L.mexemu_is_char(p):
            return '<char>'
        m, n = self.L.mxGetM(p), self.L.mxGetN(p)
        if m * n == 0:
            return np.zeros((m, n))
        buf = np.ctypeslib.as_array(self.L.mxGetDoubles(p), shape=(m * n,)).copy()
        return buf.reshape((m, n), order='F')

    def call(self, nlhs, *args):
        """[out1, ...] = gateway(args...); raises MexError for mexErrMsgIdAndTxt"""
        prhs = (C.c_void_p * max(1, len(args)))(*[a if isinstance(a, int) else a.value
                                                   for a in args])
        plhs = (C.c_void_p * max(1, nlhs))()
        eid = C.create_string_buffer(256)
        emsg = C.create_string_buffer(1024)
        rc = self.L.mexemu_call(nlhs, plhs, len(args), prhs, eid, emsg)
        for a in args:
            self.L.mxDestroyArray(a)
        if rc:
            raise MexError(eid.value.decode(), emsg.value.decode())
        outs = [self.value(plhs[i]) for i in range(nlhs)]
        for i in range(nlhs):
            if plhs[i]:
                self.L.mxDestroyArray(plhs[i])
        return outs
