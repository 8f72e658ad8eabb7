"""The exact-FTL comparator (exact_ftl.py:62-193 solves it with cvxpy, absent here):
validate the closed form the engine uses against an INDEPENDENT solver (scipy SLSQP on
the SOCP epigraph).  Parity with the reference's cvxpy path is unpinned; this pins the
mathematics.  CPU only."""
import numpy as np
import pytest
from scipy.optimize import minimize

from oracle import oracle as O


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


@pytest.mark.parametrize("seed,T,d", [(0, 30, 3), (1, 40, 5), (2, 25, 8), (3, 60, 2)])
def test_closed_form_is_the_socp_minimiser(seed, T, d):
    z, y = O.gT_sample(seed, T, 0, d)          # rows clipped to the ball, labels ±1
    cum, comp, act, in_regime = O.ftl_exact_closed_form(z, y)
    assert in_regime
    x_s, f_s = socp_solve(z, y)
    # optimality: no point the independent solver finds is better, and it gets within 1e-5
    assert comp <= f_s + 1e-9
    assert f_s - comp < 1e-5
    assert np.allclose(act, x_s, atol=1e-2)
    # and random feasible points never beat it
    rng = np.random.default_rng(seed)
    for _ in range(200):
        x = rng.standard_normal(d)
        x /= max(1.0, np.linalg.norm(x)) * rng.uniform(1.0, 3.0)
        assert comp <= objective(z, y, x) + 1e-12
    S = (y[:, None] * z).sum(axis=0)
    assert comp == pytest.approx(0.5 * (T - np.linalg.norm(S)), abs=1e-12)


def test_prefix_actions_are_prefix_minimisers():
    z, y = O.gT_sample(7, 40, 1, 4)
    for t in (1, 5, 17, 39):
        _, _, act_t, _ = O.ftl_exact_closed_form(z[:t], y[:t])
        x_s, f_s = socp_solve(z[:t], y[:t])
        assert objective(z[:t], y[:t], act_t) <= f_s + 1e-9, t


def test_regime_flag():
    z, y = O.gT_sample(1, 20, 0, 3)
    assert O.ftl_exact_closed_form(z, y)[3]
    assert not O.ftl_exact_closed_form(2.0 * z, y)[3]         # rows outside the ball
    assert not O.ftl_exact_closed_form(z, 0.5 * y)[3]         # labels not ±1
