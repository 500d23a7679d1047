"""bqp — batched MPC QP solver for AMD MI355X (gfx950).

Drop-in replacement for the per-step QP solve of bevanda/Learning-Based-MPC (fmincon / CasADi
IPOPT call sites, see include/bqp.h).  All arithmetic runs in the HIP kernels of libbqp.so;
this package only marshals arrays across the C ABI.
"""
from ._lib import BqpError, Handle, load, options  # noqa: F401
from .ocp import OcpProblem, solve_ocp  # noqa: F401
from .mpc import LMPC, TrackingLBMPC, TrackingLMPC, TrackingMPC  # noqa: F401
from .quadprog import quadprog  # noqa: F401
from .lbmpc import LBMPC, DMSLBMPC, HybridLBMPC, nw_oracle  # noqa: F401
from .loop import closed_loop, closed_loop_sqp  # noqa: F401
from . import condense, design, sets  # noqa: F401

__version__ = '0.1.0'
