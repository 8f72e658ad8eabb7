"""Build libocx.so (the HIP kernels + C ABI) in-tree for gfx950.

    python -m online_convex_optimization_amd._build [--force] [-j N]

Each ``csrc/*.hip`` is compiled by hipcc to an object under ``build/`` and linked
into ``online_convex_optimization_amd/libocx.so``.  ``-ffp-contract=off`` is part of
the numerical contract (no FMA contraction → the reference's operation order).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "ocx")
LIB = os.path.join(PKG, "libocx.so")
ARCH = os.environ.get("OCX_OFFLOAD_ARCH", "gfx950")

SOURCES = ["ocx_sim.hip", "ocx_alg_pipe.hip", "ocx_smart_wave.hip", "ocx_smart_closed.hip", "ocx_ftrl_exact.hip", "ocx_gen.hip",
           "ocx_gen_wave.hip", "ocx_stream.hip", "ocx_twin32.hip", "ocx_comp_blas.hip",
           "ocx_exact_ball.hip", "ocx_exact_wide.hip", "ocx_exact_big.hip", "ocx_pipeline.hip", "ocx_capi.hip"]
HEADERS = ["../../include/ocx_testing.h", "ocx_internal.h", "ocx_rng.h", "ocx_sim_kernels.h", "zig_tables.h",
           "ocx_device_math.h", "ocx_dispatch.h", "ocx_exact_src.h"]

CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-fno-fast-math", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X engine cannot be built")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, jobs: int = 4, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "ocx.h")]
    objs, todo = [], []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _stale(o, [s, *hdrs, __file__]):
            todo.append([hipcc, *CFLAGS, "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed ({' '.join(cmd)}):\n{r.stderr[-6000:]}")
        return r.stderr

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for err in ex.map(run, todo):
            if err.strip() and verbose:
                print(err)
    if force or todo or _stale(LIB, objs):
        run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB])
    return LIB


def build_variant(name: str, defines, jobs: int = 4, source="ocx_sim.hip",
                  out_dir: str = None) -> str:
    """Tuning variant: one source (or a list of sources) recompiled with -D overrides, linked
    with the other objects into <out_dir, default tune_build>/libocx_<name>.so (never loaded by
    the product path; select it with OCX_LIB)."""
    hipcc = _hipcc()
    out_dir = out_dir or os.path.join(ROOT, "tune_build")
    os.makedirs(out_dir, exist_ok=True)
    build(jobs=jobs)  # the shared objects of the other sources
    srcs = [source] if isinstance(source, str) else list(source)
    lib = os.path.join(out_dir, f"libocx_{name}.so")
    dflags = [f"-D{d}" for d in defines]
    deps = [os.path.join(CSRC, s) for s in srcs] + [os.path.join(CSRC, h) for h in HEADERS]
    if _stale(lib, deps):
        objs = []
        for sname in srcs:
            obj = os.path.join(out_dir, f"{sname.replace('.hip', '')}_{name}.o")
            subprocess.run([hipcc, *CFLAGS, *dflags, "-c", os.path.join(CSRC, sname), "-o", obj],
                           check=True)
            objs.append(obj)
        others = [os.path.join(BUILD, s.replace(".hip", ".o")) for s in SOURCES if s not in srcs]
        subprocess.run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, *others, "-o", lib],
                       check=True)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=4)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=a.v))
    sys.exit(0)
