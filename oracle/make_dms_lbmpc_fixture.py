"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Golden fixture of the learned-model NLP closed loops of examples/DMS_LBMPC_casadi.m (N = 100 or
50, 500 steps from x_init = [0.15; 1.2875; 1.1547; 0], RK4 Moore-Greitzer plant): the stored plant
trajectories saved_data+plots/data/casadi/DMS_tLBMPC_q{10,50,100,500}.mat, DMS_tLBMPC.mat and
DMS_N50_tLBMPC_q{10,100}.mat (`xlo`, 4 x 500 or 4 x 501 - the 501-column files hold x_init
twice; stored here from x_init on, 500 states each).  Which script variant produced which file is
established by tools/diag_learned_loops.py (profiles/r03_learned/): the q10/q50/q100 runs (N = 100
and N = 50) are DMS_LBMPC_casadi.m as written (8 x q window with validity row, cost on the learned
states); DMS_tLBMPC.mat (q = 10) and DMS_tLBMPC_q500.mat the same cost with a 7-row window whose
zero points count.  Runs only in
the build container (reads /root/reference); writes plain numeric .npz data.

    python -m oracle.make_dms_lbmpc_fixture     # writes tests/golden/dms_lbmpc_loops.npz
"""
import os

import numpy as np
import scipy.io as sio

from .make_fixtures import DATA, OUT

FILES = ('DMS_tLBMPC_q10', 'DMS_tLBMPC_q50', 'DMS_tLBMPC_q100', 'DMS_tLBMPC_q500', 'DMS_tLBMPC',
         'DMS_N50_tLBMPC_q10', 'DMS_N50_tLBMPC_q100')


def main():
    out = {}
    for name in FILES:
        xs = sio.loadmat(os.path.join(DATA, 'casadi', name + '.mat'))['xlo'].T
        if np.array_equal(xs[0], xs[1]):
            xs = xs[1:]
        out[name] = xs[:500]
    np.savez_compressed(os.path.join(OUT, 'dms_lbmpc_loops.npz'), **out)
    print('dms_lbmpc_loops.npz:', {k: v.shape for k, v in out.items()})


if __name__ == '__main__':
    main()
