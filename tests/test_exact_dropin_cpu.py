"""CPU checks of the exact_ftl drop-in surface (no GPU calls): the exact names
exact_ftl_driver.py:23-30 imports resolve from this package, and ExactFTLNoClip /
compute_prefix_actions keep the reference's argument checks (exact_ftl.py:62-193,
:280-303)."""
import numpy as np
import pytest


def test_exact_ftl_driver_imports_resolve():
    # exact_ftl_driver.py:23-30, with the package in place of the reference's modules
    from online_convex_optimization_amd.algorithms import _rng  # noqa: F401
    from online_convex_optimization_amd.exact_ftl import (  # noqa: F401
        ExactFTLNoClip,
        compute_prefix_actions,
        replay_exact_ftl,
        run_ftrl,
    )
    from online_convex_optimization_amd.sequence_generation import (  # noqa: F401
        CASES,
        REPLICATES_BY_TITLE,
        RUNS_BY_TITLE,
    )
    assert set(CASES) >= set(RUNS_BY_TITLE)


def test_solver_object_surface_and_buffers():
    from online_convex_optimization_amd.exact_ftl import ExactFTLNoClip
    s = ExactFTLNoClip(d=5, T_max=7, norm="l2", solver="ECOS", solver_opts={"max_iters": 5})
    assert (s.d, s.T_max, s.norm, s.solver, s.solver_opts) == (5, 7, "l2", "ECOS",
                                                                {"max_iters": 5})
    z = np.arange(35, dtype=np.float64).reshape(7, 5) / 100.0
    y = np.ones(7)
    s._set_prefix(z, y, 4)
    assert s._last_length == 4 and np.array_equal(s._Z_buf[:4], z[:4])
    assert s._w_buf.tolist() == [1, 1, 1, 1, 0, 0, 0]
    s._set_prefix(z, y, 2)  # shrinking clears the tail, as exact_ftl.py:160-165
    assert not s._Z_buf[2:].any() and s._w_buf.tolist() == [1, 1, 0, 0, 0, 0, 0]
    s.reset_buffers()
    assert s._last_length == 0 and not s._Z_buf.any() and not s._w_buf.any()
    with pytest.raises(ValueError):
        s._set_prefix(z, y, 8)
    with pytest.raises(ValueError):
        s.solve_prefix(np.zeros((3, 4)), np.ones(3))
    with pytest.raises(ValueError):
        s.solve_prefix(np.zeros((8, 5)), np.ones(8))
    s._last_length = 7
    with pytest.raises(ValueError):
        s.append_row(z[0], 1.0)


def test_solver_norms():
    from online_convex_optimization_amd.exact_ftl import ExactFTLNoClip
    with pytest.raises(ValueError):
        ExactFTLNoClip(3, 4, norm="l3")
    for norm in ("l1", "linf"):  # LPs in the reference: closed forms in their regime
        assert ExactFTLNoClip(3, 4, norm=norm).norm == norm


def test_compute_prefix_actions_argument_checks():
    from online_convex_optimization_amd.exact_ftl import ExactFTLNoClip, compute_prefix_actions
    z = np.zeros((6, 5))
    y = np.ones(6)
    with pytest.raises(ValueError, match="dimension"):
        compute_prefix_actions(ExactFTLNoClip(4, 10), z, y)
    with pytest.raises(ValueError, match="T_max"):
        compute_prefix_actions(ExactFTLNoClip(5, 5), z, y)


def test_compute_prefix_actions_drives_foreign_solvers_row_by_row():
    """A solver object that is not ours (e.g. a caller's cvxpy solver) is driven through
    reset_buffers/append_row exactly as exact_ftl.py:296-301 does; no GPU involved."""
    from online_convex_optimization_amd.exact_ftl import compute_prefix_actions

    class Recorder:
        d, T_max = 2, 5

        def __init__(self):
            self.calls = []

        def reset_buffers(self):
            self.calls.append("reset")

        def append_row(self, z_row, y_val):
            self.calls.append((tuple(z_row), y_val))
            return np.array([len(self.calls), -1.0])

    z = np.array([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], dtype=np.float32)
    rec = Recorder()
    a = compute_prefix_actions(rec, z, [1, -1, 1])
    assert rec.calls == ["reset", ((1.0, 2.0), 1.0), ((3.0, 4.0), -1.0), ((5.0, 6.0), 1.0)]
    assert a.shape == (4, 2) and a[0].tolist() == [0.0, 0.0] and a[3].tolist() == [4.0, -1.0]
