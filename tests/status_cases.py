"""Dense QP instances with known quadprog exit flags (shared by the CPU statement test and the
GPU status test).  Each case: (name, dict(H, f, A, b, Aeq, beq, lb, ub), expected exitflag)."""
import numpy as np


def cases():
    rng = np.random.default_rng(11)
    out = []
    n = 6
    M = rng.standard_normal((n, n))
    H = M @ M.T + 0.5 * np.eye(n)
    f = rng.standard_normal(n)
    A = rng.standard_normal((10, n))
    b = rng.uniform(0.5, 2.0, 10)
    out.append(('feasible', dict(H=H, f=f, A=A, b=b, lb=-2 * np.ones(n), ub=2 * np.ones(n)), 1))
    # contradictory rows x_1 <= -1, -x_1 <= -1.5  (x_1 >= 1.5)
    Ai = np.vstack([A, np.eye(n)[0], -np.eye(n)[0]])
    bi = np.concatenate([b, [-1.0, -1.5]])
    out.append(('infeasible rows', dict(H=H, f=f, A=Ai, b=bi), -2))
    # bounds vs a row: 0 <= x <= 1, x_1 + x_2 <= -5
    out.append(('infeasible bounds', dict(H=np.eye(2), f=np.ones(2), A=np.array([[1.0, 1.0]]),
                                          b=np.array([-5.0]), lb=np.zeros(2), ub=np.ones(2)), -2))
    # unbounded: no curvature on x_2, f_2 < 0, nothing bounds x_2 from above
    out.append(('unbounded', dict(H=np.diag([1.0, 0.0]), f=np.array([0.0, -1.0]),
                                  A=np.array([[1.0, 0.0]]), b=np.array([1.0])), -3))
    out.append(('unbounded LP', dict(H=np.zeros((3, 3)), f=np.array([1.0, -1.0, 0.0]),
                                     lb=np.zeros(3)), -3))
    # bounded LP
    out.append(('bounded LP', dict(H=np.zeros((2, 2)), f=np.array([1.0, 1.0]), lb=np.zeros(2),
                                   ub=np.ones(2)), 1))
    # non-convex
    out.append(('non-convex', dict(H=np.diag([1.0, -1.0]), f=np.zeros(2), lb=-np.ones(2),
                                   ub=np.ones(2)), -6))
    Hn = M @ M.T - 3.0 * np.eye(n)
    out.append(('non-convex dense', dict(H=Hn, f=f, A=A, b=b), -6))
    # with equality rows (block kernel on the GPU): feasible and infeasible
    Aeq = rng.standard_normal((2, n))
    beq = 0.1 * rng.standard_normal(2)
    out.append(('feasible eq', dict(H=H, f=f, A=A, b=b, Aeq=Aeq, beq=beq, lb=-2 * np.ones(n),
                                    ub=2 * np.ones(n)), 1))
    out.append(('infeasible eq', dict(H=H, f=f, Aeq=np.array([np.eye(n)[0]]), beq=np.array([5.0]),
                                      lb=-np.ones(n), ub=np.ones(n)), -2))
    return out
