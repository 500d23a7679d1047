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


@pytest.mark.timeout(300)
@pytest.mark.parametrize('cfg', ['CL', 'CLL'])
def test_closed_loop_two_rank_dry_run(cfg):
    """bench.py --config CL|CLL --gpus 2: both ranks run the closed loops of
    their shard, and one all-gather per trajectory array (X, U, exit flags, and XL for CLL)
    assembles the whole job's trajectories - equal to the unsharded run of the same instances;
    the instance numbering does not depend on the world size."""
    r = _run('--gpus', '2', '--config', cfg, '--dry-run', '--batch', '6', '--steps', '4',
             '--warmup', '1')
    assert r['n_gpus'] == 2 and r['scaling'] == 'weak'
    assert r['config']['parallelism'] == 'dp2'
    c = r['check']
    assert c['gather_matches_unsharded'] is True
    assert c['x0_independent_of_world'] is True
    assert c['gathered_instances'] == 12
    # X (12, 5, 4) + U (12, 4, 1) doubles + flags (12, 4) int32 [+ XL (12, 5, 4)]
    want = 12 * 5 * 4 * 8 + 12 * 4 * 8 + 12 * 4 * 4 + (12 * 5 * 4 * 8 if cfg == 'CLL' else 0)
    assert c['gathered_bytes'] == want


def _gather_worker(rank, world, port, q):
    import sys
    import numpy as np
    import torch
    for p in (ROOT, os.path.join(ROOT, 'learning-based-mpc_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    from bqp import dist as bd
    dist.init_process_group('gloo', rank=rank, world_size=world)
    total = 11                                   # uneven shards 3 / 4 / 4
    a, b = bd.shard(total, rank, world)
    full = np.arange(total * 5 * 3 * 2, dtype=np.float64).reshape(total, 5, 3, 2)
    out = {}
    for dt in (torch.float64, torch.int32):
        t = torch.from_numpy(full[a:b]).to(dt)
        out[str(dt)] = bd.gather_rows(t, total, world).numpy()
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gather_rows_trailing_shape_three_ranks():
    """bqp.dist.gather_rows with an arbitrary trailing shape (trajectory blocks) and unequal
    shards over three gloo ranks."""
    import socket
    import numpy as np
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    full = np.arange(11 * 5 * 3 * 2, dtype=np.float64).reshape(11, 5, 3, 2)
    assert np.array_equal(out['torch.float64'], full)
    assert np.array_equal(out['torch.int32'], full.astype(np.int32))
