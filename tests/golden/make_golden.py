"""Generate the golden fixtures by running the REFERENCE itself (build container only).

Usage (needs /root/reference, which never travels to the GPU box)::

    python tests/golden/make_golden.py [--ref /root/reference] [--skip-gT-kat]

numba and cvxpy are absent here, so the reference is imported with two stubs that
live in a temporary directory outside both repositories:

* ``numba.njit`` = identity decorator.  The @njit bodies then run as plain Python
  over ``np.float64`` scalars, which is the same IEEE operation sequence numba's
  default (non-fastmath) mode compiles to; this reproduces the published
  ``empirical_g_T_fast.png`` values exactly (checked below against BASELINE.md).
* ``cvxpy`` = empty module, so ``exact_ftl.py`` imports; only its paths that take a
  caller-supplied comparator (``run_ftrl(..., comparator_action=)``,
  ``replay_exact_ftl``) are exercised.  The SOCP comparator stays unpinned.

Outputs (small, committed): ``golden_inputs.npz`` (explicit z/y/actions arrays)
and ``golden.json`` (every expected float as ``float.hex``).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

PUBLISHED_GT = [6.034165981694009, 8.297032923590692, 10.446825985542404, 12.032218781087039,
                13.383600324774818, 14.946774913365687, 15.951320592930585, 17.196625822976216,
                18.087283038366593, 19.088517830594924]


def _install_stubs() -> str:
    d = tempfile.mkdtemp(prefix="ocx_ref_stubs_")
    os.makedirs(os.path.join(d, "numba"))
    os.makedirs(os.path.join(d, "cvxpy"))
    with open(os.path.join(d, "numba", "__init__.py"), "w") as f:
        f.write("def njit(*args, **kwargs):\n"
                "    if len(args) == 1 and callable(args[0]) and not kwargs:\n"
                "        return args[0]\n"
                "    return lambda f: f\n")
    with open(os.path.join(d, "cvxpy", "__init__.py"), "w") as f:
        f.write("# stub: the exact SOCP comparator is not exercised\n")
    return d


def H(x: float) -> str:
    return float(x).hex()


def clipped_normal(gen, T, d):
    z = gen.standard_normal((T, d))
    n = np.linalg.norm(z, axis=1, keepdims=True)
    return z / np.maximum(n, 1.0)


def explicit_inputs():
    """Deterministic explicit inputs (stored verbatim in golden_inputs.npz)."""
    g = np.random.default_rng(20251128)
    cases = {}

    def pm1(T):
        return np.where(g.random(T) < 0.5, -1.0, 1.0)

    for (T, d) in [(0, 3), (1, 1), (7, 2), (50, 5), (1000, 5), (200, 16), (300, 64), (64, 100),
                   (20, 1024), (500, 2), (129, 33)]:
        cases[f"rand_T{T}_d{d}"] = (clipped_normal(g, T, d), pm1(T))
    # unclipped rows and real-valued labels: exercises every branch of the projection
    cases["unclipped_T100_d8"] = (2.0 * g.standard_normal((100, 8)), g.standard_normal(100))
    # rows of zeros → q == 0 exactly
    z = clipped_normal(g, 30, 4)
    z[::3] = 0.0
    cases["zero_rows_T30_d4"] = (z, pm1(30))
    # float32 inputs as the drivers pass them (simulate_alg casts to float64)
    z32 = clipped_normal(g, 100, 5).astype(np.float32)
    cases["f32_T100_d5"] = (z32, pm1(100).astype(np.float32))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--skip-gT-kat", action="store_true")
    args = ap.parse_args()

    sys.path.insert(0, args.ref)
    sys.path.insert(0, _install_stubs())
    import fast_algorithms as fa  # noqa: E402  (the reference)
    import exact_ftl as ef  # noqa: E402
    import sequence_generation as sg  # noqa: E402

    out = {"meta": {"numpy": np.__version__, "reference": args.ref,
                    "generator": "tests/golden/make_golden.py"}}
    npz = {}

    # ---------------- explicit inputs: simulate_alg / SMART / exact_ftl --------------
    cases = explicit_inputs()
    rec = {}
    g = np.random.default_rng(7)
    for name, (z, y) in cases.items():
        T, d = z.shape
        npz[f"{name}__z"] = z
        npz[f"{name}__y"] = y
        r = {"T": T, "d": d, "alg": {}, "smart": {}}
        for flag, eta0 in [(0, math.sqrt(2)), (0, 1.0), (0, 0.1), (1, math.sqrt(2)), (7, 1.0)]:
            r["alg"][f"{flag}_{H(eta0)}"] = H(fa.simulate_alg(z, y, flag, eta0))
        for th in [math.sqrt(2 * max(T, 0)), 0.0, -1.0, 3.0, 1e9]:
            r["smart"][H(th)] = H(fa.simulate_SMART_like(z, y, th, math.sqrt(2)))
        r["smart_default"] = H(fa.simulate_SMART(z, y))
        # exact_ftl: FTRL loop with a caller-supplied comparator; replay of given actions
        if T > 0:
            a = g.standard_normal(d)
            a /= max(1.0, np.linalg.norm(a))
            acts = g.standard_normal((T + 1, d)) / math.sqrt(d)
            npz[f"{name}__comparator"] = a
            npz[f"{name}__actions"] = acts
            rr = ef.run_ftrl(z, y, eta0=1.0, comparator_action=a)
            r["run_ftrl"] = {"cum_loss": H(rr.cum_loss), "regret": H(rr.regret),
                             "comp_loss": H(rr.comp_loss), "x_last": [H(v) for v in rr.x_last]}
            rr2 = ef.run_ftrl(z, y, eta0=math.sqrt(2), comparator_action=a)
            r["run_ftrl_sqrt2"] = {"cum_loss": H(rr2.cum_loss), "regret": H(rr2.regret),
                                   "comp_loss": H(rr2.comp_loss)}
            rp = ef.replay_exact_ftl(z, y, acts)
            r["replay"] = {"cum_loss": H(rp.cum_loss), "regret": H(rp.regret),
                           "comp_loss": H(rp.comp_loss)}
        rec[name] = r
    out["explicit"] = rec

    # ---------------- seeded g(T) sequences via the reference's _rng + simulate_alg -----
    seeded = []
    for base_seed in (0, 3):
        for T in (1, 2, 3, 10, 57, 100, 1000):
            for run in range(6):
                gen = fa._rng(base_seed, T, run)
                z = gen.standard_normal((T, 5)).astype(np.float64, copy=False)
                norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float64, copy=False)
                z *= (1.0 / np.maximum(norms, 1.0))
                y = gen.choice([-1.0, 1.0], size=T).astype(np.float64, copy=False)
                seeded.append({"base_seed": base_seed, "T": T, "run": run, "d": 5,
                               "regret": H(fa.simulate_alg(z, y, 0, math.sqrt(2))),
                               "z_sum": H(float(z.sum())), "y_sum": H(float(y.sum()))})
    out["seeded_gT"] = seeded
    # small direct calls of the reference's sweep
    gsmall = fa.empirical_worst_case_thresholds(np.array([5, 40, 300]), runs=7, base_seed=11)
    out["gT_small"] = {"T_grid": [5, 40, 300], "runs": 7, "base_seed": 11,
                       "g": {str(k): H(v) for k, v in gsmall.items()}}

    # ---------------- deterministic families (exact-tie KAT) ---------------------------
    fam = {}
    T_grid = list(range(100, 1100, 100))
    g_pub = dict(zip(T_grid, PUBLISHED_GT))
    for title, builder in (("Label flips", sg.flip_sequence),
                           ("Switching leaders", sg.switching_two_leaders_sequence)):
        rows = {}
        for T in T_grid:
            z, y, _ = builder(T)
            rows[str(T)] = {
                "FTRL": H(fa.simulate_alg(z, y, 0, math.sqrt(2))),
                "FTL": H(fa.simulate_alg(z, y, 1, math.sqrt(2))),
                "SMART": H(fa.simulate_SMART(z, y)),
                "EMP": H(fa.simulate_empirical_g_SMART(z, y, g_pub[T])),
            }
        fam[title] = rows
    out["families"] = fam

    # ---------------- random families: the reference's own stream builders -------------
    streams = []
    for title, builder in (("Random i.i.d. (separable)",
                            lambda rs: sg.make_random_iid_stream(d=5, run_seed=rs)),
                           ("Massart noise 10%",
                            lambda rs: sg.make_noisy_iid_stream(p=0.10, d=5, run_seed=rs))):
        for run_seed in (2025, 4050):
            sampler = builder(run_seed)
            for T in (100, 1000):
                for rep in (0, 1):
                    z, y, u = sampler(T, rep=rep)
                    key = f"{title}|{run_seed}|{T}|{rep}"
                    if T == 100 and rep == 0:
                        npz[f"stream__{key}__z"] = z
                        npz[f"stream__{key}__y"] = y
                    streams.append({
                        "title": title, "run_seed": run_seed, "T": T, "rep": rep,
                        "z_sum": H(float(z.astype(np.float64).sum())),
                        "y_sum": H(float(y.astype(np.float64).sum())),
                        "u": [H(float(v)) for v in u],
                        "FTRL": H(fa.simulate_alg(z, y, 0, math.sqrt(2))),
                        "FTL": H(fa.simulate_alg(z, y, 1, math.sqrt(2))),
                        "SMART": H(fa.simulate_SMART(z, y)),
                        "EMP": H(fa.simulate_empirical_g_SMART(z, y, g_pub[T] if T in g_pub
                                                               else 10.0)),
                    })
    out["streams"] = streams

    # ---------------- fast_driver.evaluate_stream_with_stats (reduced sizes) ------------
    import fast_driver as fd  # the reference driver (matplotlib/tqdm import only)
    drv = {"T_grid": [100, 200], "g_emp": {"100": H(PUBLISHED_GT[0]), "200": H(PUBLISHED_GT[1])},
           "cases": {}}
    g_small = {100: PUBLISHED_GT[0], 200: PUBLISHED_GT[1]}
    for title, builder in sg.CASES.items():
        runs = 3 if title.startswith(("Random", "Massart")) else 1
        reps = 2 if runs > 1 else 1
        st = fd.evaluate_stream_with_stats(builder, np.array([100, 200]), g_small, runs=runs,
                                           replicates=reps, base_seed=0, stream_name=title)
        drv["cases"][title] = {"runs": runs, "replicates": reps,
                               "stats": {k: [[H(v) for v in m], [H(v) for v in c]]
                                         for k, (m, c) in st.items()}}
    out["driver"] = drv

    # ---------------- published end-to-end KAT: g(T), runs=1000, d=5 --------------------
    if not args.skip_gT_kat:
        t0 = time.time()
        gk = fa.empirical_worst_case_thresholds(np.arange(100, 1100, 100, dtype=int), runs=1000)
        vals = [gk[T] for T in T_grid]
        assert vals == PUBLISHED_GT, (vals, PUBLISHED_GT)
        out["gT_published"] = {"T_grid": T_grid, "runs": 1000, "base_seed": 0,
                               "g": [H(v) for v in vals], "seconds": time.time() - t0}

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "golden_inputs.npz"), **npz)
    print("wrote golden.json / golden_inputs.npz",
          os.path.getsize(os.path.join(HERE, "golden_inputs.npz")), "bytes")


if __name__ == "__main__":
    main()
