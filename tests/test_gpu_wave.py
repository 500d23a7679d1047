"""Device check of the wave helpers in csrc/bqp_wave.h: the transposed multi-value sum (wsum_t,
DPP pair exchanges + gfx950 v_permlane16/32_swap) that the row wave uses for F'lam, F'DF, the
complementarity sum and the corrector Fp'e terms.  Lane l must hold the wave total of value l & 31."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'learning-based-mpc_amd', 'build', 'wsum_t_check')


def test_wsum_t_device():
    assert os.path.exists(EXE), 'build first: make -C learning-based-mpc_amd'
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count('max err') == 4
