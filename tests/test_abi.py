"""CPU tests of the drop-in boundary: libbqp.so loads and exports every symbol of include/bqp.h;
API errors are reported without a GPU (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT


def header_functions():
    txt = open(os.path.join(ROOT, 'include', 'bqp.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char\*)\s+(bqp_\w+)\s*\(', txt, re.M)))


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ('bqp_quadprog_batched', 'bqp_solve_ocp_batched', 'bqp_create', 'bqp_destroy',
              'bqp_quadprog_batched_device', 'bqp_solve_ocp_batched_device'):
        assert f in fns


def test_library_exports_all_symbols():
    import bqp
    lib = bqp.load()
    for f in header_functions():
        assert hasattr(lib, f), f
    from bqp._lib import EXPORTS
    assert set(EXPORTS) == set(header_functions())


def test_version_and_defaults():
    import bqp
    lib = bqp.load()
    assert b'gfx950' in lib.bqp_version()
    o = bqp.options()
    assert o.max_iter == 50 and o.tau == 0.995


def test_create_without_gpu_fails_loudly():
    """No silent CPU fallback: with no device bqp_create returns BQP_E_NODEV."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    import bqp
    with pytest.raises(bqp.BqpError):
        bqp.Handle()


def test_argument_validation_null_handle():
    import bqp
    from bqp import _lib
    lib = bqp.load()
    dims = _lib.OcpDims(4, 1, 1, 20, 0, 20)
    rc = lib.bqp_solve_ocp_batched(None, C.byref(dims), 1, None, None, None, None, None, None,
                                   None, None, None)
    assert rc == _lib.BQP_E_ARG


def source_sha1():
    """SHA-1 over csrc/* in name order, then include/bqp.h (the Makefile's SRC_ALL)"""
    import glob
    import hashlib
    h = hashlib.sha1()
    pkg = os.path.join(ROOT, 'learning-based-mpc_amd')
    for f in sorted(glob.glob(os.path.join(pkg, 'csrc', '*'))) + [os.path.join(ROOT, 'include', 'bqp.h')]:
        h.update(open(f, 'rb').read())
    return h.hexdigest()


def test_library_built_from_this_tree():
    """the prebuilt libbqp.so that travels to the GPU box (the round-end GPU tests load it without
    building) was compiled from the sources in this tree"""
    if os.environ.get('BQP_LIB'):
        pytest.skip('BQP_LIB points at a diagnostic build')
    import bqp
    lib = bqp.load()
    assert lib.bqp_build_source_sha1().decode() == source_sha1()
