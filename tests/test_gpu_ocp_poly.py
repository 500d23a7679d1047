"""Per-instance polytope blocks (bqp_ocp_data.sFp != 0): each instance of a batch carries its own
terminal-set matrix - e.g. sets rebuilt per learned / perturbed model (getCONSPOLY.m:28-69,
compute_MPIS.m for config C4's models).  The instance's table lives in its own LDS slot."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _lmpc(mg, ts):
    import bqp
    return bqp.LMPC(mg['A'], mg['B'], mg['K'], mg['Q'], mg['R'], mg['P'], mg['Tscalar'],
                    mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'], mg['F_u'], mg['h_u'],
                    ts[0], ts[1], N=20)


def test_per_instance_sets_vs_c_restatement(mg, term_set):
    """64 instances, each with its own perturbed 616-row set: GPU vs the C restatement solving
    each instance with its own set"""
    from oracle import cpu_ref, qp_forms
    g = golden('lmpc_N20.npz')
    lm = _lmpc(mg, term_set)
    prob = lm.prob
    rng = np.random.default_rng(11)
    X0 = g['dx'][g['idx']]
    B = len(X0)
    Fp = prob.Fp[None] * (1.0 + 1e-3 * rng.standard_normal((B,) + prob.Fp.shape))
    r = lm.solve(X0, Fp=Fp)
    ocp = qp_forms.lmpc_ocp(mg, 20, *term_set)
    flags = []
    for i in range(B):
        oi = dict(ocp)
        oi['Fp'] = Fp[i]
        c = cpu_ref.solve(oi, X0[i:i + 1])
        flags.append(c['exitflag'][0])
        if c['exitflag'][0] == 1:
            assert np.abs(r.u[i] - c['u'][0]).max() < 1e-8, i
            assert np.abs(r.x[i] - c['x'][0]).max() < 1e-8, i
    assert np.array_equal(r.exitflag, np.array(flags))
    assert (r.exitflag == 1).mean() > 0.9


def test_per_instance_sets_same_polytope(mg, term_set):
    """rows permuted and scaled per instance (F_i = D_i P_i F, h_i = D_i P_i h): the same set,
    so the optimum of the shared-set solve"""
    g = golden('lmpc_N20.npz')
    lm = _lmpc(mg, term_set)
    prob = lm.prob
    rng = np.random.default_rng(5)
    X0 = g['dx'][g['idx'][:32]]
    B = len(X0)
    Fp = np.empty((B,) + prob.Fp.shape)
    hp = np.empty((B, len(prob.hp)))
    for i in range(B):
        perm = rng.permutation(len(prob.hp))
        d = rng.uniform(0.5, 2.0, len(prob.hp))
        Fp[i] = d[:, None] * prob.Fp[perm]
        hp[i] = d * prob.hp[perm]
    r = lm.solve(X0, Fp=Fp, hp=hp)
    r0 = lm.solve(X0)
    assert (r.exitflag == 1).all()
    assert np.abs(r.opt_var - r0.opt_var).max() < 1e-8


def test_terminal_sets_rebuilt_per_model(di):
    """per-model terminal sets (bqp.sets, compute_MPIS.m / RunExample.m:77-108 per model): each
    instance's set is rebuilt from its own state constraints - here tightened by a per-model
    margin, as a learned-uncertainty bound would tighten them (the sets differ in shape and row
    count and are padded with 0 <= 1) - and one batched solve takes the per-instance polytopes
    and right-hand sides; vs the C restatement solving each instance with its own set"""
    import bqp
    from bqp import sets
    from oracle import cpu_ref
    g = golden('di_design.npz')
    N = int(g['N'])
    rng = np.random.default_rng(12)
    M = 24
    scale = rng.uniform(0.6, 1.0, M)
    ts = [sets.tracking_terminal_set(di['A'], di['B'], di['K'], di['LAMBDA'], di['PSI'],
                                     di['F_x'], scale[i] * di['h_x'], di['F_u'], di['h_u'])
          for i in range(M)]
    rows = max(len(h) for _, h in ts)
    Fp, hp = sets.pack_sets(ts, nx=2, nu=2, rows=rows)
    assert len({round(float(h.sum()), 9) for _, h in ts}) > 1      # the sets really differ
    F0 = np.zeros((rows, 4)); F0[:len(g['h_T'])] = g['F_T']
    h0 = np.ones(rows); h0[:len(g['h_T'])] = g['h_T']
    tm = bqp.TrackingMPC(di['A'], di['B'], di['Q'], di['R'], di['P'], di['T'], di['LAMBDA'],
                         di['PSI'], di['F_x'], di['h_x'], di['F_u'], di['h_u'], F0, h0, N=N)
    X = g['x0'][rng.choice(len(g['x0']), M, replace=False)] * 0.5
    XS = g['xs'][rng.integers(0, len(g['xs']), M)] * 0.5
    r = tm.solve(X, XS, Fp=Fp, hp=hp)
    p = tm.prob
    w, _ = tm.linear_terms(XS)
    ok = 0
    for i in range(M):
        ocp = dict(nx=2, nu=2, np=2, N=N, A=p.A, B=p.B, c=p.c, W=p.W, w=p.w, xlb=p.xlb,
                   xub=p.xub, ulb=p.ulb, uub=p.uub, Fp=Fp[i], hp=hp[i], kp=p.poly_stage)
        c = cpu_ref.solve(ocp, X[i:i + 1], w=w[i:i + 1])
        assert r.exitflag[i] == c['exitflag'][0], i
        if c['exitflag'][0] == 1:
            ok += 1
            assert np.abs(r.u[i] - c['u'][0]).max() < 1e-8, i
    assert ok >= M // 2


@pytest.mark.parametrize('N', [20, 100])
def test_per_instance_stage_costs(mg, term_set, N):
    """per-instance stage costs (bqp_ocp_data.sW != 0; e.g. a model's own weights or steady-state
    parametrisation): a batch whose instances carry different input weights R_i gives, instance
    by instance, the solve of that instance's own problem with shared costs (short horizons: the
    table in the LDS slot; N = 100: read from L2 by the long-horizon layout)"""
    import bqp
    g = golden('dms_DSS_tLMPC.npz')
    X = g['x'][g['idx'][:12]]
    rs = np.array([0.25, 0.5, 1.0, 2.0, 4.0, 8.0] * 2)

    def tl(r):
        return bqp.TrackingLMPC(mg['A'], mg['B'], mg['Q'], r * np.atleast_2d(mg['R']), mg['P'],
                                mg['Tscalar'], mg['LAMBDA'], mg['PSI'], mg['F_x'], mg['h_x'],
                                mg['F_u'], mg['h_u'], term_set[0], term_set[1], mg['x_wp'],
                                mg['u_wp'], N=N)
    probs = [tl(r) for r in rs]
    W = np.stack([p.prob.W for p in probs])
    rb = probs[0].solve(X, W=W)
    assert (rb.exitflag == 1).all()
    for i, p in enumerate(probs):
        ri = p.solve(X[i:i + 1])
        assert ri.exitflag[0] == 1
        assert np.abs(rb.u[i] - ri.u[0]).max() < 1e-12 * max(1.0, np.abs(ri.u[0]).max())
        assert np.abs(rb.x[i] - ri.x[0]).max() < 1e-12 * max(1.0, np.abs(ri.x[0]).max())
    # the weights matter: with the shared costs of instance 0 the other instances move differently
    r0 = probs[0].solve(X)
    assert np.abs(rb.u[rs != rs[0], 0, 0] - r0.u[rs != rs[0], 0, 0]).min() > 1e-9


def test_c4_per_model_design_end_to_end(di):
    """config C4's use end to end on the tracking MPC: perturbed models (A_i, B_i), each with its
    own LQR gain, steady-state parametrisation and terminal weights (bqp.design,
    RunExample.m:42-60), its own stage costs (sW != 0) and its own terminal set (bqp.sets) - one
    batched GPU solve vs the C restatement solving each instance's own problem"""
    import bqp
    from bqp import design, sets
    from oracle import cpu_ref
    g = golden('di_design.npz')
    N = int(g['N'])
    rng = np.random.default_rng(21)
    M = 16
    A = di['A'][None] + 0.01 * rng.standard_normal((M, 2, 2)) * np.abs(di['A'])[None]
    Bm = di['B'][None] + 0.01 * rng.standard_normal((M, 2, 2)) * np.abs(di['B'])[None]
    probs, tsets = [], []
    for i in range(M):
        d = design.tracking_design(A[i], Bm[i], di['C'], di['Q'], di['R'])
        F_T, h_T = sets.tracking_terminal_set(A[i], Bm[i], d['K'], d['LAMBDA'], d['PSI'],
                                              di['F_x'], di['h_x'], di['F_u'], di['h_u'])
        tsets.append((F_T, h_T))
        probs.append(bqp.TrackingMPC(A[i], Bm[i], di['Q'], di['R'], d['P'], d['T'], d['LAMBDA'],
                                     d['PSI'], di['F_x'], di['h_x'], di['F_u'], di['h_u'], F_T,
                                     h_T, N=N))
    rows = max(len(h) for _, h in tsets)
    Fp, hp = sets.pack_sets(tsets, nx=2, nu=2, rows=rows)
    F0 = np.zeros((rows, 4)); F0[:len(tsets[0][1])] = tsets[0][0]
    h0 = np.ones(rows); h0[:len(tsets[0][1])] = tsets[0][1]
    d0 = design.tracking_design(A[0], Bm[0], di['C'], di['Q'], di['R'])
    base = bqp.TrackingMPC(A[0], Bm[0], di['Q'], di['R'], d0['P'], d0['T'], d0['LAMBDA'], d0['PSI'],
                           di['F_x'], di['h_x'], di['F_u'], di['h_u'], F0, h0, N=N)
    X = g['x0'][rng.choice(len(g['x0']), M, replace=False)] * 0.5
    XS = g['xs'][rng.integers(0, len(g['xs']), M)] * 0.5
    # per-model linear terms follow each model's own T and LAMBDA
    w = np.stack([p.linear_terms(XS[i:i + 1])[0][0] for i, p in enumerate(probs)])
    W = np.stack([p.prob.W for p in probs])
    r = bqp.solve_ocp(base.prob, X, w=w, A=A, B=Bm, W=W, Fp=Fp, hp=hp)
    ok = 0
    for i, p in enumerate(probs):
        q = p.prob
        ocp = dict(nx=2, nu=2, np=2, N=N, A=q.A, B=q.B, c=q.c, W=q.W, w=q.w, xlb=q.xlb, xub=q.xub,
                   ulb=q.ulb, uub=q.uub, Fp=q.Fp, hp=q.hp, kp=q.poly_stage)
        c = cpu_ref.solve(ocp, X[i:i + 1], w=w[i:i + 1])
        assert r.exitflag[i] == c['exitflag'][0], i
        if c['exitflag'][0] == 1:
            ok += 1
            assert np.abs(r.u[i] - c['u'][0]).max() < 1e-8, i
    assert ok >= M // 2
