"""ctypes binding of libocx.so (include/ocx.h) — the reference-side FFI stub.

This is exactly the binding a maintainer of the reference would add next to
``fast_algorithms.py`` (INTEGRATION.md shows it in that setting).  There is no
CPU fallback: if ``libocx.so`` is missing or no HIP device is usable, every call
raises.  Build the library with ``python -m online_convex_optimization_amd._build``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCX_LIB", os.path.join(_HERE, "libocx.so"))

c_dp = ctypes.POINTER(ctypes.c_double)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_double = ctypes.c_double
c_vp = ctypes.c_void_p
c_fp = ctypes.POINTER(ctypes.c_float)


class OCXError(RuntimeError):
    """A libocx call failed (bad argument, HIP error, unsupported shape)."""


class Layout(ctypes.Structure):
    """Mirror of ``ocx_layout`` (include/ocx.h)."""
    _fields_ = [("B", c_i64), ("T", c_i64), ("d", c_i64), ("P", ctypes.c_int32),
                ("C", ctypes.c_int32), ("S", ctypes.c_int32), ("chain", ctypes.c_int32),
                ("Dp", c_i64), ("G", c_i64), ("z_elems", c_i64), ("y_elems", c_i64)]

    def __repr__(self):
        return (f"Layout(B={self.B}, T={self.T}, d={self.d}, P={self.P}, C={self.C}, "
                f"S={self.S}, Dp={self.Dp}, G={self.G}, chain={self.chain})")


# name → (restype, argtypes); every symbol declared in include/ocx.h
SIGNATURES = {
    "ocx_version": (c_int, []),
    "ocx_last_error": (c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "ocx_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "ocx_release_buffers": (c_int, [c_int]),
    "ocx_layout_init": (c_int, [c_i64, c_i64, c_i64, c_int, ctypes.POINTER(Layout)]),
    "ocx_simulate_alg_batch": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_int, c_double, c_dp,
                                       c_dp, c_dp, c_dp, c_dp, c_int, c_int]),
    "ocx_simulate_smart_batch": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_dp, c_double, c_dp,
                                         c_i64p, c_int, c_int]),
    "ocx_ftl_exact_batch": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_int, c_dp, c_dp, c_dp,
                                    ctypes.POINTER(ctypes.c_int32), c_int, c_int]),
    "ocx_dev_ftl_exact": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                  c_vp]),
    "ocx_ftl_prefix_actions_batch": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_int, c_dp,
                                             ctypes.POINTER(ctypes.c_int32), c_int, c_int]),
    "ocx_dev_ftl_prefix_actions": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_vp, c_vp,
                                           c_vp]),
    "ocx_ftrl_vs_exact_batch": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_double, c_dp, c_dp,
                                        c_dp, c_dp, c_dp, ctypes.POINTER(ctypes.c_int32), c_int,
                                        c_int]),
    "ocx_ftrl_vs_exact_batch_ex": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_double, c_dp, c_dp,
                                           c_dp, c_dp, c_dp, ctypes.POINTER(ctypes.c_int32),
                                           c_int, c_int, c_int]),
    "ocx_dev_ftrl_vs_exact": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_double, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ocx_replay_batch": (c_int, [c_dp, c_dp, c_dp, c_i64, c_i64, c_i64, c_dp, c_dp, c_int]),
    "ocx_gT_regrets": (c_int, [c_u64, c_i64, c_i64, c_i64, c_i64, c_double, c_dp, c_int, c_int]),
    "ocx_gT_regrets_dev": (c_int, [c_u64, c_i64, c_i64, c_i64, c_i64, c_double, c_vp, c_int,
                                   c_int]),
    "ocx_gT_max": (c_int, [c_u64, c_i64, c_i64, c_i64, c_i64, c_double, c_int, c_int, c_dp]),
    "ocx_dev_pack": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ocx_dev_gen_gT": (c_int, [ctypes.POINTER(Layout), c_u64, c_i64, c_vp, c_vp, c_vp]),
    "ocx_dev_gen_family": (c_int, [ctypes.POINTER(Layout), c_int, c_vp, c_vp, c_double, c_i64,
                                   c_vp, c_vp, c_vp]),
    "ocx_dev_simulate_alg": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_double, c_vp,
                                     c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ocx_dev_simulate_smart": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_vp, c_double, c_vp,
                                       c_vp, c_vp]),
    "ocx_dev_simulate_smart_ex": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_vp, c_double,
                                          c_vp, c_vp, c_int, c_vp, c_vp]),
    "ocx_dev_replay": (c_int, [ctypes.POINTER(Layout), ctypes.POINTER(Layout), c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp]),
    "ocx_dev_max_regret": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "ocx_dev_gen_simulate": (c_int, [ctypes.POINTER(Layout), c_u64, c_i64, c_i64, c_vp, c_vp,
                                     c_double, c_vp, c_vp, ctypes.c_uint32, c_i64, c_vp]),
    "ocx_dev_simulate_alg_ex": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_double, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "ocx_dev_ftrl_vs_exact_ex": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_double, c_vp, c_vp,
                                         c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "ocx_gT_sweep": (c_int, [c_i64p, c_int, c_i64, c_u64, c_i64, c_double, c_int, c_dp, c_dp]),
    "ocx_gT_sweep_devices": (c_int, [c_i64p, c_int, c_i64, c_u64, c_i64, c_double,
                                     ctypes.POINTER(c_int), c_int, c_int, c_dp, c_dp]),
    "ocx_comparator_loss_blas_batch": (c_int, [c_dp, c_dp, c_dp, c_i64, c_i64, c_i64, c_dp, c_int]),
    "ocx_twin32_batch": (c_int, [c_fp, c_fp, c_i64, c_i64, c_i64, c_int, c_double, c_dp, c_fp,
                                 c_dp, c_fp, c_i64p, c_int]),
    "ocx_dev_twin32": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_double, c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp]),
    "ocx_twin32_gT_regrets": (c_int, [c_u64, c_i64, c_i64, c_i64, c_i64, c_double, c_fp, c_int]),
    "ocx_exact_ball_solve": (c_int, [c_dp, c_dp, c_i64, c_i64, c_i64, c_int, c_int, c_dp, c_dp,
                                     c_dp, c_dp, ctypes.POINTER(ctypes.c_int32), c_int]),
    "ocx_dev_exact_ball_solve": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_int, c_vp, c_vp,
                                         c_vp, c_vp, c_vp, c_vp]),
    "ocx_dev_exact_ball_solve_tiled": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_int, c_int,
                                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
}
# include/ocx_testing.h: test-only entry points (bound like the others, never called by the
# package itself)
TEST_SIGNATURES = {
    "ocx_test_gT_regrets_unclean": (c_int, [c_u64, c_i64, c_i64, c_i64, c_i64, c_double, c_dp,
                                            c_int, c_int, c_i64]),
    "ocx_test_alg_pipe_chunked": (c_int, [ctypes.POINTER(Layout), c_vp, c_vp, c_double, c_i64,
                                          c_vp, c_vp, c_vp]),
    "ocx_test_trailing_batches": (c_i64, []),
}
OCX_VERSION = 400  # include/ocx.h OCX_VERSION: the ABI these signatures describe
OCX_ALG_CLIPPED_ROWS = 1
OCX_EXACT_BALL_MAX_D = 256  # include/ocx.h
OCX_ALG_CLOSED_COMPARATOR = 2
OCX_ALG_TREE_SUMS = 4
OCX_SMART_CLOSED_PREFIX = 8
OCX_GENSIM_SEQUENTIAL = 1
OCX_GENSIM_TWO_PASS = 2

_lib = None
_lock = threading.Lock()


def _share_torch_hip_runtime() -> None:
    """Load PyTorch's HIP runtime first when PyTorch is installed.

    torch ships its own libamdhip64 (soname libamdhip64.so.7, NEEDED as the
    unversioned libamdhip64.so).  libocx NEEDs libamdhip64.so.7: if torch is loaded
    first, the dynamic loader binds libocx to torch's runtime and the process has ONE
    HIP runtime, so device pointers and streams from torch tensors are valid in
    libocx.  Loading libocx first would pull /opt/rocm's runtime and torch would then
    load a second one and see no GPU."""
    if os.environ.get("OCX_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load():
    """Load libocx.so (raises OCXError if it is missing: no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _share_torch_hip_runtime()
            if not os.path.exists(LIB_PATH):
                raise OCXError(f"libocx.so not found at {LIB_PATH}: the HIP extension is not "
                               "built (python -m online_convex_optimization_amd._build)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in {**SIGNATURES, **TEST_SIGNATURES}.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.ocx_version() != OCX_VERSION:
                raise OCXError(f"{LIB_PATH} implements ABI version {lib.ocx_version()}, this "
                               f"binding expects {OCX_VERSION}: rebuild the library")
            _lib = lib
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(4096)
    load().ocx_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        kind = {-1: "invalid argument", -2: "HIP error", -3: "unsupported"}.get(rc, str(rc))
        msg = f"{what}: {kind}: {last_error()}"
        if rc == -1:
            raise ValueError(msg)
        raise OCXError(msg)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def device_count() -> int:
    n = c_int(0)
    call("ocx_device_count", ctypes.byref(n))
    return int(n.value)


def release_buffers(device: int = 0) -> None:
    """Free the HBM the library caches on `device` between calls (ocx_release_buffers)."""
    call("ocx_release_buffers", int(device))


def layout(B: int, T: int, d: int, lanes_per_seq: int = 0) -> Layout:
    L = Layout()
    call("ocx_layout_init", int(B), int(T), int(d), int(lanes_per_seq), ctypes.byref(L))
    return L


def ptr(a):
    """ctypes double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(c_dp)
