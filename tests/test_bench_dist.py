"""CPU rehearsal of bench.py's multi-GPU path (gloo, world size 2): `bench.py --gpus 2` starts
its own ranks through torch.distributed.run (as the driver's `--gpus N` call does without a
launcher), shards the workload, times with barrier + max over ranks and all-gathers the first
moves and exit flags.  A stub solver stands in for the GPU solve (--dry-run); the gathered
rows must equal the unsharded run and rank 0 must report n_gpus = 2."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(*args):
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    env.setdefault('OMP_NUM_THREADS', '1')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + list(args),
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize('cfg,batch,scaling', [('C4', '96', 'strong'), ('C2', '40', 'weak')])
def test_two_rank_dry_run(cfg, batch, scaling):
    r = _run('--gpus', '2', '--config', cfg, '--dry-run', '--batch', batch, '--steps', '2',
             '--warmup', '1')
    assert r['n_gpus'] == 2
    assert r['scaling'] == scaling
    assert r['config']['parallelism'] == 'dp2'
    c = r['check']
    assert c['gather_matches_unsharded'] is True
    assert c['gathered_rows'] == (96 if cfg == 'C4' else 80)
    assert r['value'] > 0


@pytest.mark.timeout(120)
def test_single_rank_dry_run():
    r = _run('--config', 'C4', '--dry-run', '--batch', '16', '--steps', '1', '--warmup', '0')
    assert r['n_gpus'] == 1 and r['check']['gather_matches_unsharded'] is True
