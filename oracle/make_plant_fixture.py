"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Writes tests/golden/fmincon_runs.npz: the plant records sysH (5 x 1001, [x - x_wp; u - u_wp]) of
the reference's stored fmincon closed loops (saved_data+plots/data/LMPC_N{20,40,50}_sys_full.mat,
LBMPC_N{40,50}_sys_full.mat; functions/ocpLMPC.m:33-36 / ocpLBMPC.m:36-39 write them).  Column
layout: LMPC - column k + 1 holds the state after step k and the move of step k; LBMPC - column
k + 1 holds the state of step k and its move (the state is logged before the plant step).
They pin the ode23 plant (oracle/mg_model.py mg_ode23, csrc/bqp_plant.hip) transition by
transition and are the end-to-end reference of the GPU LMPC loop (tests/test_gpu_closed_loop.py).
Usage: python oracle/make_plant_fixture.py"""
import os

import numpy as np
import scipy.io as sio

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = '/root/reference/matlab/LBMPC/saved_data+plots/data'


def main():
    out = {}
    for name in ('LMPC_N20', 'LMPC_N40', 'LMPC_N50', 'LBMPC_N40', 'LBMPC_N50'):
        out[name] = sio.loadmat(os.path.join(DATA, '%s_sys_full.mat' % name))['sysH'].astype(float)
    np.savez_compressed(os.path.join(HERE, '..', 'tests', 'golden', 'fmincon_runs.npz'), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == '__main__':
    main()
