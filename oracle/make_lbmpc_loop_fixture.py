"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Golden fixture of the CasADi LBMPC closed loop (examples/LBMPC_casadi.m, N = 100, 500 steps
from x_init = [0.15; 1.2875; 1.1547; 0], RK4 Moore-Greitzer plant, data window q = 100): the
stored plant trajectory saved_data+plots/data/casadi/tLBMPC.mat (`xlo`, 4 x 500) plus the sets
of the run (getCONSPOLY.m: F_x_d 8x4 and the 16-row robust terminal set, as pinned to the
DSS_NMPC.m workspace in tests/golden/lbmpc_instance.npz).  Runs only in the build container
(reads /root/reference); writes plain numeric .npz data.

    python -m oracle.make_lbmpc_loop_fixture     # writes tests/golden/lbmpc_loop.npz
"""
import os

import numpy as np
import scipy.io as sio

from .make_fixtures import DATA, OUT


def main():
    xlo = sio.loadmat(os.path.join(DATA, 'casadi', 'tLBMPC.mat'))['xlo'].T   # (500, 4)
    np.savez_compressed(os.path.join(OUT, 'lbmpc_loop.npz'), xlo=xlo, x_init=xlo[0],
                        N=100, q=100, delta=0.01,
                        source='LBMPC_casadi.m closed loop, saved_data+plots/data/casadi/tLBMPC.mat')
    print('lbmpc_loop.npz: %d states' % len(xlo))


if __name__ == '__main__':
    main()
