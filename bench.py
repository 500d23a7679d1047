"""Benchmark: batched Moore-Greitzer N=20 MPC QP solves on MI355X (BASELINE.json configs[1]).

One "step" = one batched solve of the config-C2 workload: 1024 independent F1 LMPC QPs
(costLMPC.m / constraintsLMPC.m; 21 decision variables, 806 inequality rows incl. the 616-row
terminal set) at the 1000 stored closed-loop states of LMPC_N20_sys_full.mat cycled to 1024,
fp64, inputs resident in HBM, through bqp_solve_ocp_batched_device (one kernel launch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

N > 1: launched by torch.distributed.run, one rank per GPU; each rank solves its own batch
(weak scaling, no collective in the timed region); results are gathered once after timing
(RCCL all-gather) and checked on rank 0.

Prints ONE JSON line (rank 0) with value = QP-steps/s over all ranks, the roofline of the solve
kernel (algorithmic FP64 flops / kernel time, hipEvents on the launch stream) and the CPU
baseline (oracle/cpu_ipm.c, the same algorithm in C, OpenMP over host cores, bounded sample).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
HBM_PEAK_GBS = 8000.0


def flops_per_iter(N, ns, nu, nx, m_T):
    """algorithmic FP64 work of one IPM iteration (FMA = 2 flops)."""
    m_s = 2 * nx + 2 * nu
    return N * (4 * ns ** 3 + 10 * ns ** 2 + 6 * ns ** 2 * nu + 4 * ns * nu ** 2 + 12 * ns * nu
                + 8 * m_s) + m_T * (ns ** 2 + 9 * ns + 12)


def build_problem():
    """MG LMPC design data exactly as MATLAB held it (tests/golden/mg_design.npz, from the
    R2019a workspace dump) + the 616-row terminal set (term_set.mat)."""
    import bqp
    d = np.load(os.path.join(ROOT, 'tests', 'golden', 'mg_design.npz'))
    ts = np.load(os.path.join(ROOT, 'tests', 'golden', 'term_set.npz'))
    lm = bqp.LMPC(d['A'], d['B'], d['K'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                  d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], ts['F_w_N'], ts['h_w_N'], N=20)
    return lm


def cpu_baseline(prob, X_unique, threads):
    """CPU leg: the C restatement of the same IPM (oracle/cpu_ipm.c), fp64, timed on the host
    cores (single-core and all-core samples); also returns its per-instance iteration counts,
    the K_ref of the algorithmic-flop count."""
    from oracle import cpu_ref
    ocp = dict(nx=prob.nx, nu=prob.nu, np=prob.np, N=prob.N, A=prob.A, B=prob.B, c=prob.c,
               W=prob.W, w=prob.w, xlb=prob.xlb, xub=prob.xub, ulb=prob.ulb, uub=prob.uub,
               Fp=prob.Fp, hp=prob.hp, kp=prob.poly_stage)
    cpu_ref.lib()
    s1 = X_unique[:256]
    t0 = time.perf_counter(); cpu_ref.solve(ocp, s1, threads=1); t1 = time.perf_counter()
    single = len(s1) / (t1 - t0)
    reps = max(1, int(np.ceil(single * threads * 1.0 / len(X_unique))))
    sa = np.tile(X_unique, (reps, 1))
    t0 = time.perf_counter(); ra = cpu_ref.solve(ocp, sa, threads=threads); t1 = time.perf_counter()
    allc = len(sa) / (t1 - t0)
    kref = ra['iterations'][:len(X_unique)]
    return dict(value=round(allc, 1), unit='QP-steps/s', cores=threads, kind='port',
                single_core=round(single, 1),
                sample='%d C2 QPs all-core + %d single-core; oracle/cpu_ipm.c (same IPM, fp64, '
                       '-O3 -march=native, OpenMP)' % (len(sa), len(s1))), kref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=1024)
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import bqp
    from bqp import _lib

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('nccl')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    lm = build_problem()
    prob = lm.prob
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'lmpc_N20.npz'))
    B = args.batch
    X = g['dx'][(np.arange(B) + rank * B) % 1000]

    # ---- resident device inputs / outputs (torch is only the allocator) ------------------
    from bqp.ocp import pack
    dims, hdata, batch, keep = pack(prob, X)
    N, nx, nu, npar, mp = prob.N, prob.nx, prob.nu, prob.np, prob.mp

    def dt(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    from bqp.ocp import _cm
    dA, dB = dt(_cm(prob.A)), dt(_cm(prob.B))
    dW, dw, dc = dt(_cm(prob.W)), dt(prob.w), dt(prob.c)
    dxlb, dxub, dulb, duub = dt(prob.xlb), dt(prob.xub), dt(prob.ulb), dt(prob.uub)
    dF, dh, dx0 = dt(_cm(prob.Fp)), dt(prob.hp), dt(X)
    P = _lib.dptr
    data = _lib.OcpData(A=P(dA), B=P(dB), c=P(dc), W=P(dW), w=P(dw), xlb=P(dxlb), xub=P(dxub),
                        ulb=P(dulb), uub=P(duub), Fp=P(dF), hp=P(dh), x0=P(dx0),
                        sA=0, sB=0, sc=0, sW=0, sw=0, sxb=0, sub=0, sFp=0, shp=0, sx0=nx)
    ox = torch.empty((B, N + 1, nx), dtype=torch.float64, device=dev)
    ou = torch.empty((B, N, nu), dtype=torch.float64, device=dev)
    ot = torch.empty((B, npar), dtype=torch.float64, device=dev)
    of = torch.empty((B,), dtype=torch.float64, device=dev)
    oe = torch.empty((B,), dtype=torch.int32, device=dev)
    lib = bqp.load()
    h = bqp.Handle(local)
    opt = _lib.options()
    stream = torch.cuda.current_stream(dev)

    def step():
        rc = lib.bqp_solve_ocp_batched_device(
            h.value, C.byref(dims), B, C.byref(data), C.byref(opt), P(ox), P(ou), P(ot), P(of),
            C.cast(C.c_void_p(oe.data_ptr()), C.POINTER(C.c_int)), None, None,
            C.c_void_p(stream.cuda_stream))
        _lib.check(rc, 'bqp_solve_ocp_batched_device')

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # kernel-only timing: hipEvents on the launch stream, separate pass (one event pair / step)
    for _ in range(min(args.steps, 20)):
        step()
        ms, _ = h.kernel_ms()
        kms.append(ms)
    kernel_ms = float(np.mean(kms))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # one RCCL all-gather of the first moves + status after timing (result collection)
        u0 = ou[:, 0, :].contiguous()
        gath = [torch.empty_like(u0) for _ in range(world)]
        dist.all_gather(gath, u0)
        fl = [torch.empty_like(oe) for _ in range(world)]
        dist.all_gather(fl, oe)
    flags = oe.cpu().numpy()
    u0 = ou[:, 0, 0].cpu().numpy()
    # correctness on the bench batch vs fixture optima (instances present in the fixture)
    sel = g['idx']
    pos = {int(i): j for j, i in enumerate(sel)}
    err = max([abs(u0[b] - g['du_star'][pos[int(((b + rank * B) % 1000))]])
               for b in range(B) if int((b + rank * B) % 1000) in pos] or [0.0])

    if rank == 0:
        total = world * B * args.steps
        value = total / elapsed
        ms_per_step = 1e3 * elapsed / args.steps
        threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)
        cpu, kref_u = cpu_baseline(prob, g['dx'][:1000], threads)
        # algorithmic flops per launch: sum over the batch of K_ref x F_iter
        kref = kref_u[(np.arange(B) + rank * B) % 1000].astype(float)
        F_it = flops_per_iter(20, 5, 1, 4, 616)
        flops_launch = float((kref * F_it).sum())
        achieved = flops_launch / (kernel_ms * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(ROOT, 'profiles', 'pmc_latest.json')
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get('hbm_bytes_per_launch')
            except Exception:
                traffic = None
        if args.no_cpu:
            cpu = None
        line = {
            'metric': 'QP-steps/s (whole node) at N=20 Moore-Greitzer; KKT-residual vs MATLAB ref',
            'value': round(value, 1), 'unit': 'QP-steps/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic: the 1000 stored closed-loop states of LMPC_N20_sys_full.mat cycled',
            'config': {'workload': 'C2: MG LMPC (F1) N=20, 616-row terminal set, batch %d per GPU, fp64' % B,
                       'batch_per_gpu': B, 'horizon': 20, 'parallelism': 'dp%d' % world},
            'roofline': {'bound': 'mfma', 'achieved': round(achieved, 4),
                         'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(achieved / FP64_PEAK_TFLOPS, 5), 'traffic': traffic,
                         'kernel_ms': round(kernel_ms, 4),
                         'flops_per_launch': flops_launch,
                         'note': 'FP64 vector ALU roof (MI355X FP64 matrix peak is the same 78.6 TF/s); '
                                 'algorithmic flops = K_ref x F_iter (SURVEY.md 8(d))'},
            'cpu_baseline': cpu,
            'check': {'converged_frac': float((flags == 1).mean()),
                      'max_abs_du0_vs_exact': float(err),
                      'mean_iterations_ref': float(kref.mean())},
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
