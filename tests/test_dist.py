"""Multi-rank path on CPU (gloo, world size 2): contiguous sharding of a C4-style Monte-Carlo
batch (per-instance perturbed (A, B)), each rank solving only its shard, one all-gather of the
results - equal to the unsharded solve.  The per-rank solver here is the C restatement
(oracle/cpu_ipm.c, test infrastructure); on the GPU box the same host logic drives libbqp."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle.mg_model import mg_problem
    from oracle import qp_forms
    mg = mg_problem()
    ts = np.load(os.path.join(GOLDEN, 'term_set.npz'))
    g = np.load(os.path.join(GOLDEN, 'lmpc_N20.npz'))
    total = 13                                     # odd: shards of unequal size
    rng = np.random.default_rng(4)
    A = mg['A'] + 0.01 * rng.standard_normal((total, 4, 4)) * np.abs(mg['A'])
    B = mg['B'] + 0.01 * rng.standard_normal((total, 4, 1)) * np.abs(mg['B'])
    X0 = g['dx'][:total]
    ocp = qp_forms.lmpc_ocp(mg, 20, ts['F_w_N'], ts['h_w_N'])
    return ocp, X0, A, B


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    from bqp import dist as bd
    from oracle import cpu_ref
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ocp, X0, A, B = _batch()
    total = X0.shape[0]
    a, b = bd.shard(total, rank, world)
    r = cpu_ref.solve(ocp, X0[a:b], A=A[a:b], B=B[a:b], threads=1)
    u = bd.gather_rows(torch.from_numpy(np.ascontiguousarray(r['u'])), total, world)
    f = bd.gather_rows(torch.from_numpy(r['exitflag'].astype(np.int32)), total, world)
    t = bd.max_over_ranks(float(rank + 1), torch.device('cpu'), world)
    if rank == 0:
        q.put((u.numpy(), f.numpy(), t))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partition():
    from bqp import dist as bd
    for total in (1, 7, 1024, 65536):
        for world in (1, 2, 3, 8):
            sl = [bd.shard(total, r, world) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == total
            assert all(sl[r][1] == sl[r + 1][0] for r in range(world - 1))
            assert max(b - a for a, b in sl) - min(b - a for a, b in sl) <= 1
            for i in range(0, total, max(1, total // 37)):
                r = bd.owner(i, total, world)
                assert sl[r][0] <= i < sl[r][1]


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_unsharded():
    from oracle import cpu_ref
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    u, f, t = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ocp, X0, A, B = _batch()
    ref = cpu_ref.solve(ocp, X0, A=A, B=B, threads=1)
    assert t == 2.0
    assert np.array_equal(f, ref['exitflag'].astype(np.int32))
    assert np.array_equal(u, ref['u'])
