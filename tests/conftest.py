import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'learning-based-mpc_amd')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libbqp.so on the GPU)')


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope='session')
def mg():
    from oracle.mg_model import mg_problem
    return mg_problem()


@pytest.fixture(scope='session')
def term_set():
    t = golden('term_set.npz')
    return t['F_w_N'], t['h_w_N']


@pytest.fixture(scope='session')
def di():
    from oracle.mg_model import di_model
    return di_model()
