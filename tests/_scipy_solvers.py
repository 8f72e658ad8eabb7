"""Independent CPU solvers for the exact-FTL comparator (exact_ftl.py:83-105, which the
reference solves with cvxpy, absent here): scipy SLSQP on the l2 SOCP's epigraph, scipy
HiGHS on the l1 / linf LPs.  Shared by the CPU checks of the closed forms and the GPU
checks of the general solver."""
import numpy as np
from scipy.optimize import linprog, minimize


def socp_solve(z, y):
    """min_x 0.5*sum|z_i.x - y_i| s.t. ||x||_2 <= 1 (exact_ftl.py:83-105), via SLSQP on
    (x, s): min 0.5*sum s, s >= z x - y, s >= y - z x, 1 - ||x||^2 >= 0."""
    T, d = z.shape
    x0 = np.zeros(d + T)
    x0[d:] = np.abs(y) + 1.0
    cons = [{"type": "ineq", "fun": lambda v: v[d:] - (z @ v[:d] - y),
             "jac": lambda v: np.hstack([-z, np.eye(T)])},
            {"type": "ineq", "fun": lambda v: v[d:] + (z @ v[:d] - y),
             "jac": lambda v: np.hstack([z, np.eye(T)])},
            {"type": "ineq", "fun": lambda v: np.array([1.0 - v[:d] @ v[:d]]),
             "jac": lambda v: np.hstack([-2.0 * v[:d], np.zeros(T)])[None]}]
    res = minimize(lambda v: 0.5 * v[d:].sum(), x0, jac=lambda v: np.r_[np.zeros(d), 0.5 * np.ones(T)],
                   constraints=cons, method="SLSQP", options={"maxiter": 1000, "ftol": 1e-10})
    x = res.x[:d] / max(1.0, np.linalg.norm(res.x[:d]))     # feasible point
    f = 0.5 * np.abs(z @ x - y).sum()                       # its true objective
    return x, f


def objective(z, y, x):
    return 0.5 * np.abs(z @ x - y).sum()


def lp_solve(z, y, norm):
    """min_x 0.5*sum|z_i.x - y_i| s.t. ||x||_norm <= 1 (exact_ftl.py:83-105 'l1' / 'linf')
    as an LP over (u, v, s) with x = u - v, u, v >= 0, s >= |z x - y| (HiGHS)."""
    T, d = z.shape
    c = np.r_[np.zeros(2 * d), 0.5 * np.ones(T)]
    A = np.block([[z, -z, -np.eye(T)], [-z, z, -np.eye(T)]])
    b = np.r_[y, -y]
    if norm == "l1":
        A = np.vstack([A, np.r_[np.ones(2 * d), np.zeros(T)]])
        b = np.r_[b, 1.0]
        bounds = [(0, None)] * (2 * d + T)
    else:
        bounds = [(0, 1)] * (2 * d) + [(0, None)] * T
    res = linprog(c, A_ub=A, b_ub=b, bounds=bounds, method="highs")
    assert res.status == 0
    return res.x[:d] - res.x[d:2 * d], res.fun
