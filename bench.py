"""Benchmark: batched MPC QP solves on MI355X (BASELINE.json configs).

Default (the driver's bench line) = config C2, BASELINE.json configs[1]: one "step" = one
batched solve of 1024 independent F1 LMPC QPs per GPU (costLMPC.m / constraintsLMPC.m; 21
decision variables, 806 inequality rows incl. the 616-row terminal set) at the 1000 stored
closed-loop states of LMPC_N20_sys_full.mat cycled to 1024, fp64, inputs resident in HBM,
through bqp_solve_ocp_batched_device (one solve-kernel launch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5] [--batch B]

Other configs - measured the same way, reported in DESIGN.md:
  C3  trackingMPC double integrator (F5), N=30, 22-row terminal set, 4096 per GPU (1024 x0 x 4
      references), per-instance linear terms;
  C4  learned-model Monte-Carlo: 65 536 perturbed (A, B) MG models in total, N=20, sharded
      contiguously over the ranks (strong scaling), per-instance models;
  C5  long-horizon MG DMS tracking LMPC (F2), N=100, 8192 per GPU, fp64 (no fp32 path yet).

N > 1: one rank per GPU.  Without a launcher (`python bench.py --gpus N`) this script starts
torch.distributed.run itself as a child process before touching the GPU; each rank solves its
own shard (no collective in the timed region); the first moves and exit flags are all-gathered
once after timing (RCCL over xGMI) - bqp.dist.  `--dry-run` rehearses the same multi-rank code
on CPU (gloo, stub solver; tests/test_bench_dist.py).

Prints ONE JSON line (rank 0): value = QP-steps/s over all ranks; roofline of the solve kernel
(algorithmic FP64 flops / kernel time from hipEvents on the launch stream; HBM traffic from the
committed rocprofv3 PMC summary profiles/pmc_latest.json); the CPU baseline (oracle/cpu_ipm.c,
the same algorithm in C, OpenMP over host cores, bounded sample).
"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'learning-based-mpc_amd'))

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
METRIC = 'QP-steps/s (whole node) at N=20 Moore-Greitzer; KKT-residual vs MATLAB ref'
GOLD = os.path.join(ROOT, 'tests', 'golden')


def flops_per_iter(N, ns, nu, nx, m_T):
    """algorithmic FP64 work of one IPM iteration (FMA = 2 flops)."""
    m_s = 2 * nx + 2 * nu
    return N * (4 * ns ** 3 + 10 * ns ** 2 + 6 * ns ** 2 * nu + 4 * ns * nu ** 2 + 12 * ns * nu
                + 8 * m_s) + m_T * (ns ** 2 + 9 * ns + 12)


# ------------------------------------------------------------------------------------------
# workloads: (problem, per-instance inputs of this rank, K_ref source)
# ------------------------------------------------------------------------------------------
def _mg_design():
    d = np.load(os.path.join(GOLD, 'mg_design.npz'))
    ts = np.load(os.path.join(GOLD, 'term_set.npz'))
    return d, ts


def workload(cfg, batch, rank, world):
    """Returns dict(prob, X (b, nx), A, B, w (per-instance or None), uniq (index of each
    instance into the K_ref sample), sample (x0/A/B/w of the unique instances), total,
    scaling, text)."""
    import bqp
    from bqp import dist as bd
    if cfg in ('C2', 'C4'):
        d, ts = _mg_design()
        lm = bqp.LMPC(d['A'], d['B'], d['K'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                      d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], ts['F_w_N'], ts['h_w_N'], N=20)
        dx = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))['dx']
        if cfg == 'C2':
            B = batch or 1024
            gi = (np.arange(B) + rank * B) % 1000
            return dict(prob=lm.prob, X=dx[gi], A=None, B=None, w=None, uniq=gi,
                        sample=dict(X=dx[:1000]), total=B * world, scaling='weak', gidx=gi,
                        text='C2: MG LMPC (F1) N=20, 616-row terminal set, batch %d per GPU, fp64' % B,
                        data='synthetic: the 1000 stored closed-loop states of LMPC_N20_sys_full.mat cycled')
        total = batch or 65536
        a, b = bd.shard(total, rank, world)
        rng = np.random.default_rng(4)                 # SURVEY 8(d) C4 generator, seed 4
        E = rng.standard_normal((total, 4, 4))
        e = rng.standard_normal((total, 4, 1))
        A = d['A'] + 0.01 * E[a:b] * np.abs(d['A'])
        Bm = d['B'].reshape(4, 1) + 0.01 * e[a:b] * np.abs(d['B'].reshape(4, 1))
        gi = np.arange(a, b)
        ns = b - a                                     # K_ref of every instance of the shard
        return dict(prob=lm.prob, X=dx[gi % 1000], A=A, B=Bm, w=None, uniq=np.arange(b - a) % ns,
                    sample=dict(X=dx[gi[:ns] % 1000], A=A[:ns], B=Bm[:ns]), total=total,
                    scaling='strong', gidx=gi,
                    text='C4: MG LMPC (F1) N=20, %d perturbed (A,B) models in total, sharded over %d GPU(s), fp64'
                         % (total, world),
                    data='synthetic: A_i = A + 0.01 E_i|A|, B_i = B + 0.01 e_i|B| (seed 4), x0 cycled from C2')
    if cfg == 'C3':
        g = np.load(os.path.join(GOLD, 'di_design.npz'))
        N = int(g['N'])
        tm = bqp.TrackingMPC(g['A'], g['B'], g['Q'], g['R'], g['P'], g['T'], g['LAMBDA'], g['PSI'],
                             g['F_x'], g['h_x'], g['F_u'], g['h_u'], g['F_T'], g['h_T'], N=N)
        B = batch or 4096
        nu_ = len(g['x0']) * len(g['xs'])
        gi = (np.arange(B) + rank * B) % nu_
        X = g['x0'][gi // len(g['xs'])]
        XS = g['xs'][gi % len(g['xs'])]
        w, _ = tm.linear_terms(XS)
        allx = g['x0'][np.arange(nu_) // len(g['xs'])]
        allw, _ = tm.linear_terms(g['xs'][np.arange(nu_) % len(g['xs'])])
        return dict(prob=tm.prob, X=X, A=None, B=None, w=w, uniq=gi, sample=dict(X=allx, w=allw),
                    total=B * world, scaling='weak', gidx=gi,
                    text='C3: trackingMPC DI (F5) N=%d, %d-row terminal set, batch %d per GPU, fp64'
                         % (N, len(g['h_T']), B),
                    data='synthetic: 1024 feasible x0 ~ U([-5,5]^2) (seed 30) x 4 references '
                         '(RunExample.m:213-223), tests/golden/di_design.npz')
    if cfg == 'C5':
        d, ts = _mg_design()
        g = np.load(os.path.join(GOLD, 'dms_DSS_tLMPC.npz'))
        N = int(g['N'])
        tl = bqp.TrackingLMPC(d['A'], d['B'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                              d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], ts['F_w_N'],
                              ts['h_w_N'], d['x_wp'], d['u_wp'], N=N)
        B = batch or 8192
        nx_ = len(g['x'])
        gi = (np.arange(B) + rank * B) % nx_
        X = g['x'] - tl.x_eq
        return dict(prob=tl.prob, X=X[gi], A=None, B=None, w=None, uniq=gi, sample=dict(X=X),
                    total=B * world, scaling='weak', gidx=gi,
                    text='C5: MG DMS tracking LMPC (F2) N=%d, 616-row terminal set, batch %d per GPU, fp64'
                         % (N, B),
                    data='synthetic: the 499 stored closed-loop states of DSS_tLMPC.mat cycled')
    raise ValueError(cfg)


def ocp_dict(prob):
    return dict(nx=prob.nx, nu=prob.nu, np=prob.np, N=prob.N, A=prob.A, B=prob.B, c=prob.c,
                W=prob.W, w=prob.w, xlb=prob.xlb, xub=prob.xub, ulb=prob.ulb, uub=prob.uub,
                Fp=prob.Fp, hp=prob.hp, kp=prob.poly_stage)


def host_cpu_quota():
    """CPUs the cgroup lets this process use (cgroup v2 cpu.max / v1 cfs quota), or None when
    unlimited: on the GPU box the affinity mask shows the whole machine (256 CPUs) while the
    job's quota is its per-GPU share, so threads beyond the quota only contend."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            return float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def sweep_points(share):
    """thread counts of the CPU-baseline sweep: 1, 16, 64, 128 and every core of the affinity
    mask, plus the per-GPU share the box sets (OMP_NUM_THREADS)"""
    present = len(os.sched_getaffinity(0))
    pts = sorted({t for t in (1, 16, 64, 128, present, share) if 1 <= t <= present})
    return pts, present


def thread_sweep(rate, share, unit, what):
    """CPU baseline over a thread sweep: rate(nthr, eff) -> (units/s, sample size) where eff is
    the parallelism the work should be sized for (min(nthr, cgroup quota)).  value = the best
    point, cores = its thread count; every point is reported."""
    pts, present = sweep_points(share)
    quota = host_cpu_quota()
    sweep = {}
    for t in pts:
        eff = t if quota is None else max(1, min(t, int(round(quota))))
        sweep[t] = rate(t, eff)
    best = max(pts, key=lambda t: sweep[t][0])
    note = ('every core of the affinity mask (%d) is available' % present if quota is None else
            'the cgroup CPU quota of this job is %.1f CPUs of the %d in the affinity mask: thread '
            'counts above it time-share the quota (contention), so the all-mask point is not '
            'an all-core figure' % (quota, present))
    return dict(value=round(sweep[best][0], 2), unit=unit, cores=best, kind='port',
                sweep={str(t): round(v[0], 2) for t, v in sweep.items()},
                single_core=round(sweep[1][0], 2),
                share_value=round(sweep[share][0], 2) if share in sweep else None,
                share_cores=share, cores_present=present, cpu_quota=quota,
                cores_note='value = the best point of the thread sweep (threads = cores); ' + note,
                sample=what % {'pts': '/'.join(str(t) for t in pts),
                               'n': ', '.join('%d@%d' % (v[1], t) for t, v in sweep.items())})


def cpu_reference(prob, sample, threads, timed):
    """CPU leg: the C restatement of the same IPM (oracle/cpu_ipm.c), fp64.  Returns the
    per-instance iteration counts of the sample (K_ref of the algorithmic flop count, SURVEY.md
    8(d)) and, if timed, the throughput over a thread sweep on a bounded sample."""
    from oracle import cpu_ref
    ocp = ocp_dict(prob)
    cpu_ref.lib()
    X = sample['X']
    kw = {k: sample[k] for k in ('A', 'B', 'w') if k in sample}
    r = cpu_ref.solve(ocp, X, threads=threads, **kw)
    kref = r['iterations'].astype(float)
    if not timed:
        return None, kref
    n1 = min(256, len(X))
    kw1 = {k: v[:n1] for k, v in kw.items()}
    t0 = time.perf_counter(); cpu_ref.solve(ocp, X[:n1], threads=1, **kw1); t1 = time.perf_counter()
    single = n1 / (t1 - t0)

    def rate(nthr, eff):
        # about one second of work on the parallelism the box grants (at least 64 QPs per thread)
        want = max(64 * nthr, int(single * eff * 1.0))
        reps = max(1, int(np.ceil(want / len(X))))
        kwa = {k: np.concatenate([v] * reps) for k, v in kw.items()}
        Xa = np.concatenate([X] * reps)
        t0 = time.perf_counter(); cpu_ref.solve(ocp, Xa, threads=nthr, **kwa); t1 = time.perf_counter()
        return len(Xa) / (t1 - t0), len(Xa)

    return thread_sweep(rate, threads, 'QP-steps/s',
                        'thread sweep %(pts)s over the same workload (QPs@threads: %(n)s); '
                        'oracle/cpu_ipm.c (same IPM, fp64, -O3 -march=native, OpenMP, per-thread '
                        'workspaces)'), kref


def cll_cpu_baseline(g, X0, threads):
    """CPU leg of the CLL line: oracle/cpu_lbmpc.c, the C restatement of the same closed loop
    (exact-Hessian SQP, dense IPM + polish, RK4 plant, window update; fp64, -O3 -march=native,
    OpenMP over instances) - 3 steps from the first instances' states, over a thread sweep."""
    from oracle import cpu_lbmpc                  # CPU leg only
    from oracle.mg_model import mg_problem
    mg = mg_problem()
    cpu_lbmpc.lib()

    def rate(nthr, eff):
        ninst = max(4 * eff, nthr)
        xi = X0[np.arange(ninst) % len(X0)]
        t0 = time.perf_counter()
        cpu_lbmpc.loop(mg, dict(g), 100, 100, 3, xi, threads=nthr)
        return 3 * ninst / (time.perf_counter() - t0), ninst

    return thread_sweep(rate, threads, 'instance-steps/s',
                        'thread sweep %(pts)s, 3 closed-loop steps per instance (instances@threads: '
                        '%(n)s); oracle/cpu_lbmpc.c (same algorithm, fp64, -O3 -march=native, OpenMP)')


def free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """bench.py --gpus N without a torch.distributed launcher: start N ranks (one process per
    GPU) through torch.distributed.run as a child process - before this process touches the
    GPU - and exit with its status.  Rank 0 of the children prints the JSON line."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.call(cmd, env=env)


class GpuSolver:
    """One batched structured solve per step through bqp_solve_ocp_batched_device (inputs and
    outputs resident in HBM, caller stream).  streams > 1: consecutive steps go to `streams`
    HIP streams in turn, each with its own handle (workspace) and output buffers, so a step's
    workgroups start on the CUs the previous step's workgroups have left - a launch lasts as long
    as its slowest instance (one instance per SIMD at batch 1024), and its other CUs would idle
    until then.  Every step still solves the whole batch and writes every output."""

    def __init__(self, wl, local, precision, polish=True, streams=1):
        import torch
        import bqp
        from bqp import _lib
        from bqp.ocp import _cm
        self.torch, self._lib = torch, _lib
        prob, X = wl['prob'], wl['X']
        self.B = B = X.shape[0]
        N, nx, nu, npar, mp = prob.N, prob.nx, prob.nu, prob.np, prob.mp
        nv = nx + nu + npar
        dev = self.dev = torch.device('cuda', local)

        def dt(a):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)

        self.keep = [dt(_cm(prob.A) if wl['A'] is None else _cm(wl['A'])),
                     dt(_cm(prob.B) if wl['B'] is None else _cm(wl['B'])),
                     dt(prob.w if wl['w'] is None else wl['w']), dt(_cm(prob.W)), dt(prob.c),
                     dt(prob.xlb), dt(prob.xub), dt(prob.ulb), dt(prob.uub), dt(_cm(prob.Fp)),
                     dt(prob.hp), dt(X)]
        dA, dB, dw, dW, dc, dxlb, dxub, dulb, duub, dF, dh, dx0 = self.keep
        P = _lib.dptr
        self.data = _lib.OcpData(A=P(dA), B=P(dB), c=P(dc), W=P(dW), w=P(dw), xlb=P(dxlb),
                                 xub=P(dxub), ulb=P(dulb), uub=P(duub), Fp=P(dF), hp=P(dh),
                                 x0=P(dx0), sA=0 if wl['A'] is None else nx * nx,
                                 sB=0 if wl['B'] is None else nx * nu, sc=0, sW=0,
                                 sw=0 if wl['w'] is None else (N + 1) * nv, sxb=0, sub=0,
                                 sFp=0, shp=0, sx0=nx)
        self.dims = _lib.OcpDims(nx, nu, npar, N, mp, prob.poly_stage)
        self.lib = bqp.load()
        self.opt = _lib.options(precision={'fp64': 0, 'fp32': 1, 'mixed': 2}[precision], polish=polish)
        self.S = max(1, int(streams))
        self.active = self.S                 # streams the steps rotate over (<= S)
        self.sets = []
        for i in range(self.S):
            self.sets.append(dict(
                ox=torch.empty((B, N + 1, nx), dtype=torch.float64, device=dev),
                ou=torch.empty((B, N, nu), dtype=torch.float64, device=dev),
                ot=torch.empty((B, npar), dtype=torch.float64, device=dev),
                of=torch.empty((B,), dtype=torch.float64, device=dev),
                oe=torch.empty((B,), dtype=torch.int32, device=dev),
                oo=torch.empty((B * C.sizeof(_lib.Output),), dtype=torch.uint8, device=dev),
                h=bqp.Handle(local),
                stream=torch.cuda.current_stream(dev) if i == 0 else torch.cuda.Stream(dev)))
        self.k = 0
        self.last = 0

    def next_stream(self):
        """the stream the next step() launches on"""
        return self.sets[self.k % self.active]['stream']

    def step(self, with_out=False):
        P = self._lib.dptr
        i = 0 if with_out else self.k % self.active
        self.k += 0 if with_out else 1
        st = self.sets[i]
        rc = self.lib.bqp_solve_ocp_batched_device(
            st['h'].value, C.byref(self.dims), self.B, C.byref(self.data), C.byref(self.opt),
            P(st['ox']), P(st['ou']), P(st['ot']), P(st['of']),
            C.cast(C.c_void_p(st['oe'].data_ptr()), C.POINTER(C.c_int)),
            C.c_void_p(st['oo'].data_ptr()) if with_out else None, None,
            C.c_void_p(st['stream'].cuda_stream))
        self._lib.check(rc, 'bqp_solve_ocp_batched_device')
        self.last = i

    def sync(self):
        self.torch.cuda.synchronize()

    def kernel_ms(self):
        return self.sets[self.last]['h'].kernel_ms()[0]

    def first_moves(self):
        st = self.sets[0]
        return st['ou'][:, 0, :].contiguous(), st['oe']

    def outputs(self):
        """per-instance exit statistics (bqp_output) of a step(with_out=True)"""
        raw = self.sets[0]['oo'].cpu().numpy().tobytes()
        out = (self._lib.Output * self.B).from_buffer_copy(raw)
        return dict(iterations=np.array([o.iterations for o in out]),
                    kkt=np.array([list(o.kkt) for o in out]),
                    polished=np.array([o.polished for o in out]))


class StubSolver:
    """CPU dry run of the multi-rank harness (bench.py --dry-run, gloo): a deterministic stand-in
    for the solve (first move = a fixed function of the instance's x0 / A / B), so the sharding,
    timing barrier, max-over-ranks and all-gather code of this file runs without a GPU and its
    gathered rows can be compared with the unsharded run."""

    def __init__(self, wl):
        import torch
        self.torch = torch
        self.B = wl['X'].shape[0]
        self.wl = wl

    @staticmethod
    def moves(wl):
        X = np.asarray(wl['X'], float)
        u = X.sum(axis=1) + 0.5 * X[:, 0] ** 2
        if wl['A'] is not None:
            u = u + np.trace(wl['A'], axis1=1, axis2=2) + wl['B'].reshape(len(X), -1).sum(axis=1)
        return u.reshape(-1, 1), (np.floor(np.abs(u) * 7) % 3 - 1).astype(np.int32)

    def step(self, with_out=False):
        self.u, self.e = self.moves(self.wl)

    def sync(self):
        pass

    def kernel_ms(self):
        return None

    def first_moves(self):
        return self.torch.from_numpy(self.u), self.torch.from_numpy(self.e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='C2', choices=['C1', 'C2', 'C2H', 'C2D', 'C3', 'C4', 'C5', 'CL', 'CLL'])
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (C4: total)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--precision', default='fp64', choices=['fp64', 'fp32', 'mixed'],
                    help='structured solver arithmetic (C5 compares both)')
    ap.add_argument('--no-polish', action='store_true',
                    help='interior-point iterates only (bqp_options.polish = -1)')
    ap.add_argument('--no-two-groups', action='store_true',
                    help='skip the two-group pass of check.value_two_groups (profiling runs: every '
                         'launch of the command then runs alone)')
    ap.add_argument('--dry-run', action='store_true',
                    help='CPU/gloo rehearsal of the multi-rank path with a stub solver (tests)')
    ap.add_argument('--streams', type=int, default=None,
                    help='structured configs: consecutive steps on this many HIP streams in turn '
                         '(independent plant groups: a launch lasts as long as its slowest '
                         'instance, and the other group\'s workgroups start on the CUs it has '
                         'left).  Default 1: one batch per control step, the BASELINE config; the '
                         'two-group rate is reported in check.value_two_groups.  CL / CLL: the '
                         'rank\'s instances in this many concurrent groups (default 2; the same '
                         'instances, split)')
    args = ap.parse_args()
    if args.streams is None:
        args.streams = 2 if args.config in ('CL', 'CLL') else 1
    if args.config in ('C1', 'C2H', 'C2D'):
        return bench_aux(args)
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return launch_ranks(args)
    if args.config in ('CL', 'CLL'):
        return bench_loop(args)

    import torch
    import torch.distributed as dist
    from bqp import dist as bd

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('gloo' if args.dry_run else 'nccl')
    if args.dry_run:
        dev = torch.device('cpu')
    else:
        torch.cuda.set_device(local)
        dev = torch.device('cuda', local)

    wl = workload(args.config, args.batch, rank, world)
    prob, B = wl['prob'], wl['X'].shape[0]
    N, nx, nu, npar, mp = prob.N, prob.nx, prob.nu, prob.np, prob.mp
    # two stream sets at least: the line's value is the --streams rate, check.value_two_groups the
    # rate of two independent plant groups (consecutive steps on two streams)
    solver = StubSolver(wl) if args.dry_run else GpuSolver(wl, local, args.precision, not args.no_polish,
                                                           max(2, args.streams))
    if not args.dry_run:
        solver.active = max(1, args.streams)

    for _ in range(args.warmup):
        solver.step()
    solver.sync()
    if world > 1:
        dist.barrier()
    solver.sync()
    # launch durations over the timed region: an event pair around every step on the stream it
    # is launched on (the steps overlap on --streams streams, so a launch's duration includes the
    # time its workgroups wait for the CUs the other stream's launch still holds)
    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if args.dry_run:
            solver.step()
            continue
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        st = solver.next_stream()
        e0.record(st)
        solver.step()
        e1.record(st)
        evs.append((e0, e1))
    solver.sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = bd.max_over_ranks(t1 - t0, dev, world)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else None
    # two independent plant groups (reported beside the value, never as it):
    # the same steps with consecutive steps on two streams
    two_groups = None
    if not args.dry_run and solver.active == 1 and not args.no_two_groups:
        solver.active = 2
        for _ in range(2):
            solver.step()
        solver.sync()
        if world > 1:
            dist.barrier()
        solver.sync()
        tg0 = time.perf_counter()
        for _ in range(args.steps):
            solver.step()
        solver.sync()
        if world > 1:
            dist.barrier()
        two_groups = bd.max_over_ranks(time.perf_counter() - tg0, dev, world)
        solver.active = 1
    # one launch alone (separate pass, host-synchronised per step): the isolated launch time
    kernel_ms_alone = None
    if not args.dry_run:
        kms = []
        for _ in range(min(args.steps, 20)):
            solver.step()
            kms.append(solver.kernel_ms())
        kernel_ms_alone = float(np.mean(kms))
    # one all-gather of the first moves + status after timing (result collection, bqp.dist)
    total_rows = wl['total'] if wl['scaling'] == 'strong' else B * world
    u0_loc, fl_loc = solver.first_moves()
    u0_all = bd.gather_rows(u0_loc, total_rows, world).cpu().numpy()
    fl_all = bd.gather_rows(fl_loc, total_rows, world).cpu().numpy()
    flags = fl_loc.cpu().numpy()
    u0 = u0_loc[:, 0].cpu().numpy()

    check = {'converged_frac': float((flags == 1).mean()),
             'converged_frac_all_ranks': float((fl_all == 1).mean()),
             'infeasible_count_all_ranks': int((fl_all == -2).sum()),
             # every exit flag of the whole job (quadprog meanings: 1 converged, 0 iteration
             # limit, -2 primal infeasible, -8 numerical failure)
             'exitflag_hist_all_ranks': {str(int(k)): int((fl_all == k).sum()) for k in np.unique(fl_all)},
             'gathered_rows': int(u0_all.shape[0])}
    if args.dry_run and rank == 0:
        # the gathered rows must equal the unsharded run of the same workload
        full = workload(args.config, args.batch if wl['scaling'] == 'strong' else B * world, 0, 1)
        uf, ef = StubSolver.moves(full)
        check['gather_matches_unsharded'] = bool(np.array_equal(u0_all, uf) and
                                                 np.array_equal(fl_all, ef))
    if not args.dry_run:
        # KKT residuals of this batch at exit (bqp_output: stationarity, primal eq, primal
        # ineq, complementarity mu) and the first move against MATLAB's stored moves and the
        # exact optima of the fixtures
        solver.step(with_out=True)
        solver.sync()
        o = solver.outputs()
        conv = flags == 1
        kk = o['kkt'][conv] if conv.any() else np.zeros((1, 4))
        check.update(kkt_stationarity_max=float(kk[:, 0].max()),
                     kkt_primal_eq_max=float(kk[:, 1].max()),
                     kkt_primal_ineq_max=float(kk[:, 2].max()),
                     kkt_mu_max=float(kk[:, 3].max()),
                     iterations_mean=float(o['iterations'].mean()),
                     iterations_max=int(o['iterations'].max()),
                     polished_count=int(o['polished'].sum()))
        if args.config == 'C2':
            g = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))
            pos = {int(i): j for j, i in enumerate(g['idx'])}
            gi = wl['gidx']
            err = [abs(u0[b] - g['du_star'][pos[int(gi[b])]]) for b in range(B) if int(gi[b]) in pos]
            check['max_abs_du0_vs_exact'] = float(max(err or [0.0]))
            # fmincon's stored applied moves (LMPC_N20_sys_full.mat, tolerance ~1e-6 of fmincon)
            dm = np.abs(u0 - g['du_matlab'][gi])
            check['du0_vs_matlab_median'] = float(np.median(dm))
            check['du0_vs_matlab_max'] = float(dm.max())
        if args.config == 'C5':
            g5 = np.load(os.path.join(GOLD, 'dms_DSS_tLMPC.npz'))
            pos = {int(i): j for j, i in enumerate(g5['idx'])}
            u_eq = float(np.atleast_1d(_mg_design()[0]['u_wp'])[0])
            err = [abs(u0[b] + u_eq - g5['u_star'][pos[int(wl['gidx'][b])]])
                   for b in range(B) if int(wl['gidx'][b]) in pos]
            check['max_abs_u0_vs_exact'] = float(max(err or [0.0]))

    if rank == 0:
        value = wl['total'] / (elapsed / args.steps) if wl['scaling'] == 'strong' \
            else world * B * args.steps / elapsed
        if args.config == 'C4' and 'converged_frac_all_ranks' in check:
            # C4: only the converged instances count as QP-steps; the primal-infeasible models
            # (exitflag -2, found in fewer iterations) are reported in `check`, not in `value`
            check['value_all_instances'] = round(value, 1)
            value *= check['converged_frac_all_ranks']
        ms_per_step = 1e3 * elapsed / args.steps
        if two_groups is not None:
            v2 = wl['total'] / (two_groups / args.steps) if wl['scaling'] == 'strong' \
                else world * B * args.steps / two_groups
            if args.config == 'C4' and 'converged_frac_all_ranks' in check:
                v2 *= check['converged_frac_all_ranks']
            check['value_two_groups'] = round(v2, 1)
            check['ms_per_step_two_groups'] = round(1e3 * two_groups / args.steps, 4)
        roof, cpu = None, None
        if not args.dry_run:
            present = len(os.sched_getaffinity(0))
            threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or present
            # the CPU baseline is timed at N=1 only (the multi-GPU lines carry K_ref, not a timing)
            cpu, kref_u = cpu_reference(prob, wl['sample'], threads, not args.no_cpu and world == 1)
            # algorithmic flops per launch: sum over the batch of K_ref x F_iter;
            # instances the reference solver does not converge on (infeasible) count with their
            # own iteration count
            kref = kref_u[wl['uniq']]
            F_it = flops_per_iter(N, nx + npar, nu, nx, mp)
            flops_launch = float((kref * F_it).sum())
            achieved = flops_launch / (kernel_ms * 1e-3) / 1e12
            # HBM bytes per launch of this config's kernel: rocprofv3 PMC passes of the same
            # bench command (tools/gpu_r03_prof.sh -> tools/pmc_summary.py --config)
            traffic, traffic_src = None, None
            tag = args.config + ('' if args.precision == 'fp64' else '_' + args.precision)
            pmc = os.path.join(ROOT, 'profiles', 'pmc_%s.json' % tag)
            if os.path.exists(pmc):
                try:
                    pj = json.load(open(pmc))
                    traffic, traffic_src = pj.get('hbm_bytes_per_launch'), pj.get('source')
                except Exception:
                    traffic = None
            check['mean_iterations_ref'] = float(kref.mean())
            # the device rate over the timed region (flops per step / ms per step)
            achieved_pipe = flops_launch / (ms_per_step * 1e-3) / 1e12
            # achieved / frac: flops per launch / the mean launch duration over the timed region
            # (hipEvents around each step on its stream: the solve launch and the repair launch
            # that follows it; at config.streams = 1, the default, every launch runs alone, so
            # this is the launch's own duration and rocprofv3's kernel average reproduces it)
            roof = {'bound': 'fp64_valu', 'achieved': round(achieved, 4),
                    'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                    'frac': round(achieved / FP64_PEAK_TFLOPS, 5), 'traffic': traffic,
                    'kernel_ms': round(kernel_ms, 4), 'flops_per_launch': flops_launch,
                    'kernel_ms_alone': round(kernel_ms_alone, 4),
                    'achieved_per_step': round(achieved_pipe, 4),
                    'frac_per_step': round(achieved_pipe / FP64_PEAK_TFLOPS, 5),
                    'frac_per_launch_alone': round(flops_launch / (kernel_ms_alone * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 5),
                    'traffic_source': traffic_src,
                    'note': 'bound: FP64 VALU issue plus the latency of the sequential N-stage '
                            'Riccati chain (roofline.latency); 78.6 TF/s is the FP64 vector peak '
                            '(= the FP64 MFMA peak) of MI355X; this kernel issues no MFMA (5x5 '
                            'stage blocks, DESIGN.md 4); algorithmic flops = K_ref x F_iter (SURVEY.md 8(d)); '
                            'traffic = HBM bytes per launch from rocprofv3 FETCH_SIZE/WRITE_SIZE '
                            'passes of this config (traffic_source); achieved = flops per launch / '
                            'kernel_ms, the mean duration of a step\'s launches over the timed steps '
                            '(hipEvents on the launch stream; one stream, so each launch runs alone); '
                            'achieved_per_step = flops per launch / ms_per_step, the device rate over '
                            'the timed region; kernel_ms_alone = one launch by itself '
                            '(host-synchronised pass)'}
            st_json = os.path.join(ROOT, 'profiles', 'stamps_%s.json' % args.config)
            if args.precision == 'fp64' and os.path.exists(st_json):
                # latency roof: at batch 1024 one instance runs per SIMD, so the
                # kernel time is one instance's dependency chain; the stage wave (Riccati factor,
                # two sweeps, update) works this fraction of the instance's cycles and waits on
                # the row wave for the rest (s_memtime stamps of the diagnostic build,
                # tools/stamps.py --json); current_source says whether they were taken on the
                # kernel source this bench runs
                try:
                    sj = json.load(open(st_json))
                    src = os.path.join(ROOT, 'learning-based-mpc_amd', 'csrc', 'bqp_ocp.hip')
                    roof['latency'] = {
                        'stage_wave_busy_frac': round(sj['stage_wave_busy_frac'], 4),
                        'stage_wave_cycles_per_iter': round(sj['stage_wave_cycles_per_iter']),
                        'current_source': sj.get('source_sha1') == hashlib.sha1(open(src, 'rb').read()).hexdigest(),
                        'source': os.path.relpath(st_json, ROOT)}
                except Exception:
                    pass
        line = {
            'metric': METRIC,
            'value': round(value, 1), 'unit': 'QP-steps/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
            'higher_is_better': True, 'scaling': wl['scaling'], 'vs_baseline': None,
            'dtype': {'fp64': 'f64', 'fp32': 'f32', 'mixed': 'f32+f64'}[args.precision],
            'data': wl['data'] + (' [CPU dry run: stub solver, gloo]' if args.dry_run else ''),
            'config': {'workload': wl['text'], 'batch_per_gpu': B, 'horizon': N,
                       'parallelism': 'dp%d' % world, 'streams': args.streams},
            'roofline': roof,
            'cpu_baseline': cpu,
            'check': check,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def cll_subproblem_roofline(dl, X0, h):
    """roofline of the learned-model loop's dominant kernel (dense_ipm_kernel, 83 % of the loop
    in round 3): the loop's QP sub-problem shape - n = N nu + np = 101 variables, the m = 1024
    condensed nominal rows Ain of DMS_LBMPC_casadi.m:262-276 shared by the batch - at the first
    SQP iterate of every instance (zero window: the learned rollout is the nominal one, so the
    sub-problem is this QP exactly), one batched launch.  Algorithmic flops per IPM iteration
    (DESIGN.md 4): K = H + A'DA (lower triangle) n(n+1)m, Cholesky n^3/3, row products and A'v
    (A z, A dz twice, A'lam, A'w twice) 12 n m, triangular solves 8 n^2; x the iterations each
    instance takes."""
    import bqp
    n, m_, p, N = dl.n, dl.m, dl.p, dl.N
    nz = dl.nz
    B = len(X0)
    dX = X0 - dl.x_eq
    # nominal rollout x_k = Mx_k dx0 + Sx_k z (K = 0), u_k = e_k z
    Et = np.zeros((p, nz)); Et[:, N * m_:] = np.eye(p)
    H = np.zeros((nz, nz)); F = np.zeros((nz, n))            # f = F dx0
    Mx, Sx = np.eye(n), np.zeros((n, nz))
    for k in range(N + 1):
        Ex = dl.Lq @ (Sx - dl.LAMBDA @ Et)
        if k < dl.n_run:
            Eu = np.zeros((m_, nz)); Eu[:, k * m_:(k + 1) * m_] = np.eye(m_)
            Ur = dl.Lr @ (Eu - dl.PSI @ Et)
            H += 2 * (Ex.T @ Ex + Ur.T @ Ur); F += 2 * Ex.T @ (dl.Lq @ Mx)
        if k == N:
            Ep = dl.Lp @ (Sx - dl.LAMBDA @ Et)
            Lt = dl.Lt @ (dl.LAMBDA @ Et)
            H += 2 * (Ep.T @ Ep + Lt.T @ Lt); F += 2 * Ep.T @ (dl.Lp @ Mx)
        if k < N:
            Eu = np.zeros((m_, nz)); Eu[:, k * m_:(k + 1) * m_] = np.eye(m_)
            Sx = dl.A @ Sx + dl.B @ Eu
            Mx = dl.A @ Mx
    H = 0.5 * (H + H.T)
    f = dX @ F.T
    b = dl.b0[None, :] + dX @ dl.Bx.T
    A = dl.Ain
    mr = A.shape[0]
    bqp.quadprog(H, f[:2], A, b[:2], handle=h)              # warm-up (module load, workspaces)
    x, fv, flag, out, lam = bqp.quadprog(H, f, A, b, handle=h)
    kms, nl = h.kernel_ms()
    its = out['iterations'].astype(float)
    F_it = nz * (nz + 1) * mr + nz ** 3 / 3.0 + 12.0 * nz * mr + 8.0 * nz * nz
    # the work the kernel forms: A'DA only on the 16 x 16 output tiles of the
    # lower block triangle that a 32-row tile's rows reach (1 + last nonzero column of each row;
    # the skipped products are exact zeros), 2 x 16 x 16 x 32 flops per reached tile and row tile;
    # the row products A v / A'v over each row's nonzero columns
    hr = np.array([(np.flatnonzero(A[r])[-1] + 1) if A[r].any() else 0 for r in range(mr)])
    reach = [int(np.ceil(hr[t:t + 32].max() / 16.0)) for t in range(0, mr, 32)]
    ada_nz = sum(R * (R + 1) / 2 for R in reach) * 2.0 * 16 * 16 * 32
    F_it_nz = ada_nz + nz ** 3 / 3.0 + 12.0 * float(hr.sum()) + 8.0 * nz * nz
    # HBM bytes per launch and MFMA busy fraction of the same kernel in the loop (rocprofv3 PMC
    # passes of bench.py --config CLL, tools/gpu_r04_prof.sh -> profiles/pmc_CLL.json)
    traffic = tsrc = mfma = None
    pj = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'pmc_CLL.json')
    if os.path.exists(pj):
        pm = json.load(open(pj))
        traffic, tsrc, mfma = pm['hbm_bytes_per_launch'], pm['source'], round(pm['mfma_busy_frac_est'], 4)
    flops = float(its.sum() * F_it_nz)
    flops_dense = float(its.sum() * F_it)
    ach = flops / (kms * 1e-3) / 1e12
    ach_d = flops_dense / (kms * 1e-3) / 1e12
    return dict(bound='fp64_mfma', achieved=round(ach, 4), peak=FP64_PEAK_TFLOPS, unit='TFLOP/s',
                frac=round(ach / FP64_PEAK_TFLOPS, 5), traffic=traffic, kernel_ms=round(kms, 4),
                flops_per_launch=flops, flops_per_launch_dense_count=flops_dense,
                frac_dense_count=round(ach_d / FP64_PEAK_TFLOPS, 5),
                ada_tiles_formed_frac=round(ada_nz / (nz * (nz + 1) * mr), 4),
                launches=nl, traffic_source=tsrc, mfma_busy_frac=mfma,
                note='dense_ipm_kernel on the loop sub-problem shape (n = %d, m = %d, batch %d, '
                     'mean %.1f IPM iterations, exit flags %s): K = H + A\'DA on the fp64 matrix '
                     'cores; frac counts the work the kernel forms (A\'DA on the reached tiles, '
                     'row products over the nonzero columns), frac_dense_count the dense n(n+1)m '
                     'A\'DA; kernel_ms covers the solve and the polish launch' %
                     (nz, mr, B, its.mean(), dict(zip(*[v.tolist() for v in np.unique(flag, return_counts=True)]))))


def loop_workload(cfg, batch, rank, world):
    """Closed-loop configs: the instances of the whole job are numbered
    globally and rank r runs its contiguous shard [r B, (r + 1) B) (weak scaling: B per GPU), so
    the trajectories a rank produces do not depend on the number of ranks.
    CL  the DSS tracking LMPC loop (DMS_tracking_LMPC_casadi.m:153-189, N = 100, RK4 plant) from
        the stored DSS_tLMPC.mat states cycled;
    CLL the learned-model NLP loop (DMS_LBMPC_casadi.m:163-218, N = 100, q = 100) from x_init
        (:99) and seeded perturbations of it (+-0.005 in x1, x2)."""
    import bqp
    d, ts = _mg_design()
    B = batch or (256 if cfg == 'CLL' else 1024)
    gi = np.arange(rank * B, (rank + 1) * B)
    if cfg == 'CL':
        gl = np.load(os.path.join(GOLD, 'dms_DSS_tLMPC.npz'))
        mpc = bqp.TrackingLMPC(d['A'], d['B'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                               d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], ts['F_w_N'],
                               ts['h_w_N'], d['x_wp'], d['u_wp'], N=100)
        X0 = gl['x'][gi % len(gl['x'])]
        return dict(mpc=mpc, X0=X0, gidx=gi, B=B,
                    text='CL: DSS tracking LMPC closed loop (N=100, RK4 plant), batch %d per GPU' % B,
                    data='initial states = stored DSS_tLMPC.mat states cycled',
                    metric='closed-loop MPC steps/s (DSS tracking LMPC N=100, RK4 plant)')
    g = np.load(os.path.join(GOLD, 'lbmpc_instance.npz'))
    mpc = bqp.DMSLBMPC(d['A'], d['B'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                       d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], g['F_w_N'], g['h_w_N'],
                       g['F_x_d'], g['h_x_d'], d['x_wp'], d['u_wp'], N=100)
    x_init = np.array([0.15, 1.2875, 1.1547, 0.0])
    # perturbation of global instance i: row i of a seed-11 stream (independent of world size)
    P = np.random.default_rng(11).uniform(-1, 1, ((rank + 1) * B, 4))[gi]
    X0 = x_init + P * np.array([0.005, 0.005, 0.0, 0.0])
    if rank == 0:
        X0[0] = x_init                                     # DMS_LBMPC_casadi.m:99
    return dict(mpc=mpc, X0=X0, gidx=gi, B=B, g=g,
                text='CLL: DMS LBMPC closed loop (N=100, q=100), batch %d per GPU' % B,
                data='x_init of DMS_LBMPC_casadi.m and seeded perturbations (+-0.005 in x1, x2)',
                metric='learned-model NLP closed-loop steps/s (DMS_LBMPC_casadi.m, N=100, q=100)')


class LoopRunner:
    """One rank's closed loops on its GPU (bqp.closed_loop / bqp.closed_loop_sqp).  With
    streams > 1 the rank's instances are split into that many contiguous groups, each run by its
    own host thread on its own handle (HIP stream, workspace): the groups' launches overlap, so the
    CUs that one group's latency-bound kernels leave idle (the learned rollouts use one wave per
    instance) run the other group's dense sub-problems.  The instances are independent, so every
    group's trajectories are the ones the whole batch in one call gives."""

    def __init__(self, cfg, wl, local, streams=1):
        import torch
        import bqp
        self.bqp, self.cfg, self.wl, self.torch = bqp, cfg, wl, torch
        self.local = local
        self.streams = max(1, min(int(streams), len(wl['X0'])))
        self.hs = [bqp.Handle(local) for _ in range(self.streams)]
        self.h = self.hs[0]
        # each group launches on its own torch stream (the loop's _device entry points run on the
        # caller's current stream); the trajectories come back as tensors in this GPU's HBM
        dev = torch.device('cuda', local)
        self.ss = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(self.streams - 1)]

    def _one(self, X0, steps, h, s):
        b = self.bqp
        with self.torch.cuda.stream(s):
            if self.cfg == 'CL':
                return b.closed_loop(self.wl['mpc'], X0, steps, handle=h, device=self.local)
            return b.closed_loop_sqp(self.wl['mpc'], X0, steps, learning=dict(q=100, mask=1), handle=h,
                                     device=self.local)

    def run(self, steps):
        X0 = self.wl['X0']
        if self.streams == 1:
            return self._one(X0, steps, self.h, self.ss[0])
        import threading
        parts = np.array_split(np.arange(len(X0)), self.streams)
        res = [None] * self.streams
        err = []

        def work(i):
            try:
                res[i] = self._one(X0[parts[i]], steps, self.hs[i], self.ss[i])
            except Exception as e:               # re-raised on the main thread
                err.append(e)
        th = [threading.Thread(target=work, args=(i,)) for i in range(self.streams)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise err[0]
        out = dict(res[0])
        for k, v in res[0].items():
            if isinstance(v, np.ndarray):
                out[k] = np.concatenate([r[k] for r in res])
            elif isinstance(v, self.torch.Tensor):
                out[k] = self.torch.cat([r[k] for r in res])
        return out

    def kernel_ms(self):
        return self.h.kernel_ms()[0]


class StubLoop:
    """CPU dry run of the multi-rank closed-loop harness (--dry-run, gloo): a deterministic stand-in
    for the loop (x+ = 0.9 x + 0.01 sin(sum x) + u, u = -0.1 sum x), so the per-rank shards, the
    timing and the trajectory all-gather run without a GPU and can be compared with the unsharded
    run."""

    def __init__(self, cfg, wl):
        self.cfg, self.wl = cfg, wl

    @staticmethod
    def simulate(X0, steps, learned):
        b, n = X0.shape
        X = np.zeros((b, steps + 1, n)); U = np.zeros((b, steps, 1))
        X[:, 0] = X0
        for k in range(steps):
            u = -0.1 * X[:, k].sum(axis=1)
            U[:, k, 0] = u
            X[:, k + 1] = 0.9 * X[:, k] + 0.01 * np.sin(X[:, k].sum(axis=1))[:, None] + u[:, None]
        fl = (np.floor(np.abs(U[:, :, 0]) * 1e3) % 2).astype(np.int32)
        r = dict(X=X, U=U, exitflag=fl)
        if learned:
            r['XL'] = X + 1e-3
        return r

    def run(self, steps):
        return self.simulate(self.wl['X0'], steps, self.cfg == 'CLL')

    def kernel_ms(self):
        return None


def bench_loop(args):
    """CL / CLL on N ranks (north_star: "an RCCL all-gather over xGMI only to
    collect trajectories"): each rank runs the closed loops of its shard for --steps steps (one
    call: solve + plant + window per step on its GPU, no communication), timed between barriers
    with the max over ranks; then one all-gather per trajectory array - X (B, steps+1, 4), U
    (B, steps, 1), the exit flags (B, steps) and for CLL the learned predictions XL - assembles the
    whole job's trajectories on every rank (bqp.dist.gather_rows; RCCL on the GPU box, gloo in the
    dry run).  value = instance-steps/s of all ranks."""
    import torch
    import torch.distributed as dist
    from bqp import dist as bd
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('gloo' if args.dry_run else 'nccl')
    if args.dry_run:
        dev = torch.device('cpu')
    else:
        torch.cuda.set_device(local)
        dev = torch.device('cuda', local)
    wl = loop_workload(args.config, args.batch, rank, world)
    B = wl['B']
    runner = StubLoop(args.config, wl) if args.dry_run else LoopRunner(args.config, wl, local, args.streams)
    if args.warmup > 0:
        runner.run(1)                                   # module load, workspaces
    if not args.dry_run:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    r = runner.run(args.steps)
    if not args.dry_run:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = bd.max_over_ranks(time.perf_counter() - t0, dev, world)
    kms = runner.kernel_ms()
    # trajectory collection: one all-gather per array after the timed region
    total = B * world
    names = ['X', 'U', 'exitflag'] + (['XL'] if args.config == 'CLL' else [])
    tg0 = time.perf_counter()
    gathered = {}
    nbytes = 0
    # (the GPU loop's trajectories are already tensors in this rank's HBM: bqp.closed_loop*(...,
    # device=...), so the all-gather reads them there - no host round trip before the collective)
    dev_resident = all(isinstance(r[k], torch.Tensor) for k in names)
    for k in names:
        t = r[k] if isinstance(r[k], torch.Tensor) else torch.from_numpy(np.ascontiguousarray(r[k])).to(dev)
        gathered[k] = bd.gather_rows(t, total, world)
    if not args.dry_run:
        torch.cuda.synchronize()
    t_gather = bd.max_over_ranks(time.perf_counter() - tg0, dev, world)
    gathered = {k: v.cpu().numpy() for k, v in gathered.items()}
    nbytes = sum(v.nbytes for v in gathered.values())
    fl = gathered['exitflag']
    check = dict(converged_frac_all_ranks=float((fl == 1).mean()),
                 gathered_instances=int(gathered['X'].shape[0]),
                 gathered_bytes=int(nbytes), gather_s=round(t_gather, 4),
                 gather_from_device=bool(dev_resident))
    if 'iterations' in r and r.get('iterations') is not None:
        its = r['iterations']
        its = its.cpu().numpy() if isinstance(its, torch.Tensor) else its
        check.update(sqp_iterations_mean=float(np.mean(its)), sqp_iterations_max=int(np.max(its)))
    if args.dry_run and rank == 0:
        full = loop_workload(args.config, B * world, 0, 1)
        # the stub's per-instance result depends only on the instance's own x0, so the unsharded
        # run of the same global instances must equal the gathered shards
        X0_all = np.concatenate([loop_workload(args.config, B, q, world)['X0'] for q in range(world)])
        ref = StubLoop.simulate(X0_all, args.steps, args.config == 'CLL')
        check['gather_matches_unsharded'] = bool(all(np.array_equal(gathered[k], ref[k]) for k in names))
        check['x0_independent_of_world'] = bool(np.array_equal(full['X0'], X0_all))
    line = None
    if rank == 0:
        cpu, roof = None, None
        if args.config == 'CLL' and not args.dry_run:
            g = wl['g']
            X0 = wl['X0']
            st = np.load(os.path.join(GOLD, 'dms_lbmpc_loops.npz'))['DMS_tLBMPC_q100']
            e0 = np.abs(gathered['X'][0] - st[:args.steps + 1])
            check.update(x_init_vs_stored_q100_slow_max=float(e0[:, :2].max()),
                         x_init_vs_stored_q100_all_max=float(e0.max()))
            roof = cll_subproblem_roofline(wl['mpc'], X0, runner.h)
            if not args.no_cpu and world == 1:
                present = len(os.sched_getaffinity(0))
                cpu = cll_cpu_baseline(g, X0, int(os.environ.get('OMP_NUM_THREADS', '0')) or present)
        elif args.config == 'CL' and not args.dry_run and not args.no_cpu and world == 1:
            from oracle import cpu_ref, qp_forms          # CPU leg only
            from oracle.mg_model import mg_problem, mg_rk4
            mgp = mg_problem()
            _, ts = _mg_design()
            ocp = qp_forms.dms_ocp(mgp, 100, ts['F_w_N'], ts['h_w_N'])
            c0 = time.perf_counter()
            x = wl['X0'][:16].copy()
            for k in range(10):
                c = cpu_ref.solve(ocp, x - mgp['x_wp'], threads=1)
                u = c['u'][:, 0, 0] + mgp['u_wp']
                x = np.array([mg_rk4(0.01, x[i], u[i]) for i in range(len(x))])
            cpu = dict(value=round(16 * 10 / (time.perf_counter() - c0), 1), unit='instance-steps/s',
                       cores=1, kind='port', sample='16 instances x 10 steps, oracle/cpu_ipm.c + numpy RK4')
        line = dict(metric=wl['metric'], value=round(total * args.steps / elapsed, 1),
                    unit='instance-steps/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
                    ms_per_step=round(1e3 * elapsed / args.steps, 4), higher_is_better=True,
                    scaling='weak', vs_baseline=None, dtype='f64',
                    data=wl['data'] + (' [CPU dry run: stub loop, gloo]' if args.dry_run else ''),
                    config={'workload': wl['text'] + ', %d steps' % args.steps, 'batch_per_gpu': B,
                            'horizon': 100, 'parallelism': 'dp%d' % world,
                            'streams': 1 if args.dry_run else runner.streams},
                    roofline=roof, kernel_ms=None if kms is None else round(kms, 4),
                    cpu_baseline=cpu, check=check)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def bench_aux(args):
    """Single-GPU measurements of the SURVEY.md §8(f) paths (not the driver's bench line):
    C1  LBMPC (fmincon form F3, costLBMPC.m / constraintsLBMPC.m), N=10, NW window
        train_data(:, 1:100), Gauss-Newton SQP on the GPU (bqp_lbmpc_solve_batched); one step =
        one batched SQP solve (default batch 1 = the reference's single-instance config);
    C2H / C2D  the C2 workload through the host-pointer entry point / in quadprog form.
    The CPU leg of C1 is the numpy restatement (oracle/lbmpc.py, interpreted), on a bounded
    sample.  The closed-loop configs CL / CLL run on N ranks: bench_loop."""
    import time as _t
    import torch
    import bqp
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    d, ts = _mg_design()
    h = bqp.Handle(0)
    if args.config == 'C2H':
        # the C2 workload through the HOST-pointer entry point: PCIe-inclusive rate (inputs
        # copied in, trajectories copied out every call) - reported in DESIGN.md, never `value`
        wl = workload('C2', args.batch, 0, 1)
        for _ in range(args.warmup):
            bqp.solve_ocp(wl['prob'], wl['X'], handle=h)
        t0 = _t.perf_counter()
        for _ in range(args.steps):
            r = bqp.solve_ocp(wl['prob'], wl['X'], handle=h)
        el = _t.perf_counter() - t0
        B = wl['X'].shape[0]
        line = dict(metric='QP-steps/s, host-pointer API (PCIe-inclusive)', value=round(B * args.steps / el, 1),
                    unit='QP-steps/s', n_gpus=1, steps=args.steps, warmup=args.warmup,
                    ms_per_step=round(1e3 * el / args.steps, 4), higher_is_better=True, scaling='weak',
                    vs_baseline=None, dtype='f64', data=wl['data'],
                    config={'workload': wl['text'] + ', host buffers', 'batch_per_gpu': B, 'horizon': 20,
                            'parallelism': 'dp1'},
                    roofline=None, kernel_ms=round(h.kernel_ms()[0], 4), cpu_baseline=None,
                    check=dict(converged_frac=float((r.exitflag == 1).mean())))
    elif args.config == 'C2D':
        # the C2 problem in fmincon's own form F1 (21 variables, 806 rows) through the dense
        # quadprog entry point on device buffers: H and A shared, f and b per instance; the
        # K = H + A'DA factorisation runs on the fp64 matrix cores (dense_wave_kernel<2>)
        from bqp import _lib
        from bqp.condense import Condensed
        wl = workload('C2', args.batch, 0, 1)
        cd = Condensed(wl['prob'])
        B = wl['X'].shape[0]
        f, b = cd.rhs(wl['X'])
        n, m = cd.n, cd.m

        def dt(a_):
            return torch.from_numpy(np.ascontiguousarray(a_, dtype=np.float64)).to(dev)
        dH, dA, df, db = dt(cd.H.T), dt(cd.A.T), dt(f), dt(b)      # column-major H, A
        ox = torch.empty((B, n), dtype=torch.float64, device=dev)
        ofv = torch.empty((B,), dtype=torch.float64, device=dev)
        oe = torch.empty((B,), dtype=torch.int32, device=dev)
        lam = torch.empty((B, m), dtype=torch.float64, device=dev)
        lib = bqp.load()
        dims = _lib.Dims(n, m, 0)
        strides = _lib.Strides(0, n, 0, m, 0, 0, 0, 0)
        opt = _lib.options()
        P = _lib.dptr
        stream = torch.cuda.current_stream(dev)

        def step():
            rc = lib.bqp_quadprog_batched_device(
                h.value, C.byref(dims), B, C.byref(strides), P(dH), P(df), P(dA), P(db), None, None,
                None, None, C.byref(opt), P(ox), P(ofv),
                C.cast(C.c_void_p(oe.data_ptr()), C.POINTER(C.c_int)), P(lam), None, None, None,
                None, C.c_void_p(stream.cuda_stream))
            _lib.check(rc, 'bqp_quadprog_batched_device')
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = _t.perf_counter()
        kms = []
        for _ in range(args.steps):
            step()
            kms.append(h.kernel_ms()[0])
        torch.cuda.synchronize()
        el = _t.perf_counter() - t0
        Z = ox.cpu().numpy()
        u, th, x = cd.recover(Z, wl['X'])
        g2 = np.load(os.path.join(GOLD, 'lmpc_N20.npz'))
        du_star = g2['du_star']
        sel = np.flatnonzero(np.isin(wl['gidx'], g2['idx']))
        pos = {int(v): i for i, v in enumerate(g2['idx'])}
        err = max(abs(u[i, 0, 0] - du_star[pos[int(wl['gidx'][i])]]) for i in sel) if len(sel) else None
        kms_mean = float(np.mean(kms))
        flops_iter = m * n * n + n ** 3 / 3.0 + 8.0 * m * n          # A'DA (MFMA), Cholesky, mat-vecs
        its = None
        try:
            out = (_lib.Output * B)()
            rc = lib.bqp_quadprog_batched(h.value, C.byref(dims), B, C.byref(strides),
                                          _lib.ptr(np.ascontiguousarray(cd.H.T)), _lib.ptr(f),
                                          _lib.ptr(np.ascontiguousarray(cd.A.T)), _lib.ptr(b),
                                          None, None, None, None, None, C.byref(opt),
                                          _lib.ptr(np.zeros((B, n))), None,
                                          _lib.iptr(np.zeros(B, np.int32)), None, None, None, None,
                                          out)
            its = float(np.mean([o.iterations for o in out])) if rc == 0 else None
        except Exception:
            its = None
        ach = B * (its or 0) * flops_iter / (kms_mean * 1e-3) / 1e12
        line = dict(metric='dense quadprog QP-steps/s (F1, N=20: 21 vars, 806 rows)',
                    value=round(B * args.steps / el, 1), unit='QP-steps/s', n_gpus=1, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(1e3 * el / args.steps, 4),
                    higher_is_better=True, scaling='weak', vs_baseline=None, dtype='f64',
                    data=wl['data'],
                    config={'workload': 'C2 problem in quadprog form F1 (bqp.condense), batch %d' % B,
                            'batch_per_gpu': B, 'horizon': 20, 'parallelism': 'dp1'},
                    roofline=dict(bound='fp64_mfma', achieved=round(ach, 4), peak=78.6,
                                  unit='TFLOP/s', frac=round(ach / 78.6, 5), kernel_ms=round(kms_mean, 4),
                                  note='per-iteration flops m n^2 + n^3/3 + 8 m n x the kernel\'s own mean '
                                       'iteration count (no CPU K_ref for this form)'),
                    cpu_baseline=None,
                    check=dict(converged_frac=float((oe.cpu().numpy() == 1).mean()),
                               iterations_mean=its,
                               max_abs_du0_vs_exact=None if err is None else float(err)))
    elif args.config == 'C1':
        g = np.load(os.path.join(GOLD, 'lbmpc_instance.npz'))
        td = np.load(os.path.join(GOLD, 'train_data.npz'))['data'][:, :100]
        lb = bqp.LBMPC(d['A'], d['B'], d['K'], d['Q'], d['R'], d['P'], float(d['T']), d['LAMBDA'],
                       d['PSI'], d['F_x'], d['h_x'], d['F_u'], d['h_u'], g['F_w_N'], g['h_w_N'],
                       g['F_x_d'], g['h_x_d'], N=10)
        B = args.batch or 1
        rng = np.random.default_rng(1)
        X0 = np.column_stack([rng.uniform(-0.35, 0.0, B), rng.uniform(-0.4, 0.0, B),
                              0.01 * rng.standard_normal(B), 0.1 * rng.standard_normal(B)])
        X0[0] = [-0.35, -0.4, 0.0, 0.0]                      # LBMPC_RunExample.m:41-44
        for _ in range(args.warmup):
            r = lb.solve(X0, td, handle=h)
        t0 = _t.perf_counter()
        kms = []
        for _ in range(args.steps):
            r = lb.solve(X0, td, handle=h)
            kms.append(h.kernel_ms()[0])
        el = _t.perf_counter() - t0
        # CPU leg: the oracle's numpy SQP (interpreted) on the first instances
        from oracle import lbmpc as olb               # CPU leg only
        from oracle.mg_model import mg_problem
        p = olb.f3_problem(mg_problem(), 10, td, g['F_w_N'], g['h_w_N'], g['F_x_d'], g['h_x_d'])
        ns = min(B, 8)
        c0 = _t.perf_counter()
        for i in range(ns):
            olb.sqp(p, X0[i])
        cpu = ns / (_t.perf_counter() - c0)
        line = dict(metric='LBMPC SQP solves/s (F3, N=10)', value=round(B * args.steps / el, 2),
                    unit='SQP-solves/s', n_gpus=1, steps=args.steps, warmup=args.warmup,
                    ms_per_step=round(1e3 * el / args.steps, 4), higher_is_better=True,
                    scaling='weak', vs_baseline=None, dtype='f64',
                    data='x0 = LBMPC_RunExample.m dx_init (+ seeded random states), window train_data(:,1:100)',
                    config={'workload': 'C1: MG LBMPC (F3) N=10, batch %d' % B, 'batch_per_gpu': B,
                            'horizon': 10, 'parallelism': 'dp1'},
                    roofline=None, kernel_ms=round(float(np.mean(kms)), 4),
                    cpu_baseline=dict(value=round(cpu, 2), unit='SQP-solves/s', cores=1,
                                      kind='port', sample='%d solves of oracle/lbmpc.py (numpy)' % ns),
                    check=dict(converged_frac=float((r.exitflag == 1).mean()),
                               mean_sqp_iterations=float(r.iterations.mean())))
    print(json.dumps(line))


if __name__ == '__main__':
    sys.exit(main() or 0)
