"""Secondary measurements on one MI355X (one JSON line each; not the bench contract).

  gen      generator throughput (d=64 g(T) rows) at several batch sizes
  sweep    configs[3]-style g(T) sweep per T, generation included (runs scaled down)
  driver   fast_driver.main() on device (g(T) runs=1000 + the four cases, full sizes)
  smart    SMART kernel throughput (d=5, T=1000, 768 sequences)
  config1  configs[1] (65 536 x 1e3 x 16) per lanes_per_seq layout
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sync():
    import torch
    torch.cuda.synchronize()


def gen(args):
    import torch
    from online_convex_optimization_amd import engine
    for B, T in ((32768, 10000), (131072, 2000), (262144, 1000)):
        db = engine.DeviceBatch(B, T, 64, lanes_per_seq=1)
        db.generate_gT(0, 0)
        sync()
        t0 = time.perf_counter()
        db.generate_gT(0, 0)
        sync()
        tg = time.perf_counter() - t0
        t0 = time.perf_counter()
        db.simulate_alg()
        sync()
        ts = time.perf_counter() - t0
        print(json.dumps({"what": "gen", "B": B, "T": T, "d": 64, "gen_s": tg,
                          "normals_per_s": B * T * 64 / tg, "gen_timesteps_per_s": B * T / tg,
                          "sim_s": ts, "gen+sim_timesteps_per_s": B * T / (tg + ts)}), flush=True)
        del db
        torch.cuda.empty_cache()


def gen1(args):
    """One generation config, for PMC passes (rocprofv3 --pmc ... -- python tools/perf_extra.py gen1)."""
    from online_convex_optimization_amd import engine
    db = engine.DeviceBatch(65536, 2000, 64, lanes_per_seq=1)
    for _ in range(2):
        db.generate_gT(0, 0)
        sync()
    t0 = time.perf_counter()
    db.generate_gT(0, 0)
    sync()
    tg = time.perf_counter() - t0
    print(json.dumps({"what": "gen1", "B": 65536, "T": 2000, "d": 64, "gen_s": tg,
                      "normals_per_s": 65536 * 2000 * 64 / tg}), flush=True)


def sweep(args):
    from online_convex_optimization_amd import engine
    cases = ((100, 1000000), (1000, 1000000), (10000, 131072), (100000, 131072))
    if args.Ts:
        keep = {int(v) for v in args.Ts.split(",")}
        cases = tuple(c for c in cases if c[0] in keep)
    for T, runs in cases:
        engine.gT_regrets(T, runs, d=64, lanes_per_seq=args.lanes)  # warm (incl. HBM buffers)
        t0 = time.perf_counter()
        regs = engine.gT_regrets(T, runs, d=64, lanes_per_seq=args.lanes)
        dt = time.perf_counter() - t0
        # what empirical_worst_case_thresholds needs per T: g(T) only, reduced on device
        engine.gT_max(T, runs, d=64, lanes_per_seq=args.lanes)
        t0 = time.perf_counter()
        g = engine.gT_max(T, runs, d=64, lanes_per_seq=args.lanes)
        dm = time.perf_counter() - t0
        assert g == engine.max_regret(regs)
        print(json.dumps({"what": "gT_sweep", "T": T, "runs": runs, "d": 64, "lanes": args.lanes,
                          "seconds": dt, "timesteps_per_s": T * runs / dt,
                          "frac_1040B": T * runs / dt * 1040 / 8e12,
                          "gmax_seconds": dm, "gmax_timesteps_per_s": T * runs / dm,
                          "gmax_frac_1040B": T * runs / dm * 1040 / 8e12,
                          "g": engine.max_regret(regs)}), flush=True)


def driver(args):
    from online_convex_optimization_amd import drivers
    t0 = time.perf_counter()
    g_emp, stats = drivers.fast_driver_main()
    dt = time.perf_counter() - t0
    out = {"what": "fast_driver_main", "seconds": dt,
           "g_emp": [g_emp[T] for T in range(100, 1100, 100)],
           "T1000": {title: {k: float(st[k][0][-1]) for k in st} for title, st in stats.items()}}
    print(json.dumps(out), flush=True)


def config3(args):
    """configs[2]: exact_ftl vs fast FTRL, d=64, T=1e4, 1e5 trials on one GPU: per trial
    FTRL's regret against the exact comparator and against its own FTL comparator, and
    exact FTL's regret, generation included (resident batches of 32768).  Two variants:
    "fused" (ocx_dev_ftrl_vs_exact: both loops in one pass, comparators in a second) and
    "separate" (exact FTL kernel, then FTRL twice); their regrets must agree bit for bit."""
    import torch
    from online_convex_optimization_amd import engine
    T, d, trials, Bb = 10000, 64, 100000, 32768
    engine.release_buffers()  # the sweeps' cached HBM, if run in the same process
    db = engine.DeviceBatch(Bb, T, d, lanes_per_seq=1)
    results = {}
    for variant in ("fused", "separate", "fused", "fused_best"):
        lanes = 128 if variant == "fused_best" else 1  # best: closed-form comparators
        sync()
        t0 = time.perf_counter()
        out = []
        for r0 in range(0, trials, Bb):
            B = min(Bb, trials - r0)
            if B != db.L.B or lanes != (1 if db.exact else 128):
                del db
                db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes)
            db.generate_gT(0, r0)
            if variant.startswith("fused"):
                cf = torch.zeros(B, dtype=torch.float64, device=db.device)
                regime = db.ftrl_vs_exact(math.sqrt(2), comp_ftl=cf)
                exact = db.cum - db.comp
                fast = db.cum - cf
                ftl_exact = db.cum_exact - db.comp
            else:
                act = torch.zeros((B, d), dtype=torch.float64, device=db.device)
                regime = db.ftl_exact(cmp_action=act)
                ftl_exact = (db.cum - db.comp).clone()
                exact = db.simulate_alg(0, math.sqrt(2), comparator=act).clone()
                fast = db.simulate_alg(0, math.sqrt(2)).clone()
            assert bool(regime[:B].all())
            out.append(torch.stack([exact[:B], fast[:B], ftl_exact[:B]]).cpu().numpy())
        sync()
        dt = time.perf_counter() - t0
        res = np.concatenate(out, axis=1)
        results[variant] = res
        dd = res[0] - res[1]
        print(json.dumps({"what": "config3_exact_vs_fast", "variant": variant, "trials": trials,
                          "T": T, "d": d, "seconds": dt, "trial_steps_per_s": trials * T / dt,
                          "mean_regret_exact_minus_fast": float(dd.mean()),
                          "max_abs_diff": float(np.abs(dd).max()),
                          "mean_regret_ftl_exact": float(res[2].mean())}), flush=True)
    rb, rf = results["fused_best"], results["fused"]
    print(json.dumps({"what": "config3_fused_equals_separate",
                      "bitexact": bool(np.array_equal(results["fused"], results["separate"])),
                      "best_vs_exact_max_rel": float((np.abs(rb - rf) / np.maximum(1.0, np.abs(rf))).max())}),
          flush=True)


def config4(args):
    """configs[4]: g(T) adversary at d=1024, T=1e4 (runs scaled down), generation included,
    exact and butterfly sums, at two HBM budgets (resident vs streamed batches)."""
    from online_convex_optimization_amd import engine
    T, d = 10000, 1024
    cases = [(8192, 128, None, None), (8192, 1, None, None), (32768, 128, None, None)]
    for runs, lanes, budget, minres in cases:
        if budget:
            os.environ["OCX_HBM_BUDGET_GB"] = budget
        else:
            os.environ.pop("OCX_HBM_BUDGET_GB", None)
        if minres:
            os.environ["OCX_MIN_RESIDENT"] = minres
        else:
            os.environ.pop("OCX_MIN_RESIDENT", None)
        # warm with the same shape: the first call grows the HBM buffers and loads kernels
        engine.gT_regrets(T, runs, d=d, lanes_per_seq=lanes)
        t0 = time.perf_counter()
        regs = engine.gT_regrets(T, runs, d=d, lanes_per_seq=lanes)
        dt = time.perf_counter() - t0
        print(json.dumps({"what": "config4_gT", "T": T, "runs": runs, "d": d, "lanes": lanes,
                          "hbm_budget_gb": budget, "min_resident": minres, "seconds": dt,
                          "timesteps_per_s": T * runs / dt, "g": engine.max_regret(regs)}),
              flush=True)
    os.environ.pop("OCX_HBM_BUDGET_GB", None)
    os.environ.pop("OCX_MIN_RESIDENT", None)


def sweep_budget(args):
    """HBM budget for resident g(T) batches (OCX_HBM_BUDGET_GB): few-wave, latency-bound
    batches (T=1e5 at d=64, T=1e4 at d=1024) run faster the more sequences a batch holds."""
    from online_convex_optimization_amd import engine
    cases = [(100000, 64, 32768, b) for b in ("192", "220", "240", "255")]
    cases += [(10000, 1024, 8192, b) for b in ("192", "240")]
    for T, d, runs, budget in cases:
        os.environ["OCX_HBM_BUDGET_GB"] = budget
        try:
            engine.release_buffers()
            engine.gT_regrets(T, runs, d=d, lanes_per_seq=1)
            t0 = time.perf_counter()
            regs = engine.gT_regrets(T, runs, d=d, lanes_per_seq=1)
            dt = time.perf_counter() - t0
            out = {"seconds": dt, "timesteps_per_s": T * runs / dt, "g": engine.max_regret(regs)}
        except Exception as e:  # an over-large budget fails allocation: report it
            out = {"error": str(e)[:200]}
        print(json.dumps({"what": "gT_budget", "T": T, "runs": runs, "d": d,
                          "hbm_budget_gb": budget, **out}), flush=True)
    os.environ.pop("OCX_HBM_BUDGET_GB", None)
    engine.release_buffers()


def prof_long(args):
    """One call each of configs[4] (d=1024, T=1e4, 8192 runs, exact) and a T=1e5, d=64
    sweep point (16384 runs), for rocprofv3 --kernel-trace --stats."""
    from online_convex_optimization_amd import engine
    for T, d, runs in ((10000, 1024, 8192), (100000, 64, 16384)):
        t0 = time.perf_counter()
        regs = engine.gT_regrets(T, runs, d=d, lanes_per_seq=1)
        dt = time.perf_counter() - t0
        print(json.dumps({"what": "prof_long", "T": T, "d": d, "runs": runs, "seconds": dt,
                          "timesteps_per_s": T * runs / dt, "g": engine.max_regret(regs)}),
              flush=True)


def exact_driver(args):
    from online_convex_optimization_amd import drivers
    t0 = time.perf_counter()
    g, stats = drivers.exact_ftl_driver_main()
    dt = time.perf_counter() - t0
    print(json.dumps({"what": "exact_ftl_driver_main", "seconds": dt,
                      "g_emp": [g[T] for T in range(100, 1100, 100)],
                      "T1000": {t: {k: float(v[0][-1]) for k, v in st.items()}
                                for t, st in stats.items()}}), flush=True)


def config1(args):
    """configs[1]: batched FTRL, 65 536 sequences, d=16, T=1e3 (g(T) adversary at d=16),
    per layout: kernel time from HIP events, fraction of 8 TB/s for one and two passes over z,
    generation time, and regrets against the exact layout."""
    import torch
    from online_convex_optimization_amd import engine
    B, T, d = 65536, 1000, args.d
    ref = None
    for lanes in [int(v) for v in args.lanes_list.split(",")]:
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes)
        st = torch.cuda.current_stream()
        db.generate_gT(0, 0)
        sync()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(st)
        db.generate_gT(0, 0)
        ev[1].record(st)
        db.simulate_alg()
        ev[2].record(st)
        sync()
        res = []
        for closed in (True, False):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            db.simulate_alg(closed_comparator=closed)
            e0.record(st)
            for _ in range(10):
                db.simulate_alg(closed_comparator=closed)
            e1.record(st)
            sync()
            res.append(e0.elapsed_time(e1) / 10)
        r = db.regret[:B].cpu().numpy()
        if ref is None and db.exact:
            ref = r.copy()
        err = None if ref is None else float(np.max(np.abs(r - ref) / np.maximum(1, np.abs(ref))))
        one, two = B * T * (8 * d + 8), 2 * B * T * (8 * d + 8)
        print(json.dumps({"what": "config1", "d": d, "lanes": lanes, "layout": [db.L.P, db.L.C, db.L.chain],
                          "exact": bool(db.exact), "gen_ms": ev[0].elapsed_time(ev[1]),
                          "ftrl_ms_default": ev[1].elapsed_time(ev[2]),
                          "ftrl_ms_closed": res[0], "ftrl_ms_two_pass": res[1],
                          "frac_closed": one / (res[0] * 1e-3) / 8e12,
                          "frac_two_pass": two / (res[1] * 1e-3) / 8e12,
                          "timesteps_per_s_closed": B * T / (res[0] * 1e-3),
                          "max_rel_vs_exact": err}), flush=True)
        del db
        engine.release_buffers()
        torch.cuda.empty_cache()


def smart(args):
    """SMART on the driver's batch shape (768 iid sequences, d=5, T=1000) and a large
    batch, through both kernels (OCX_SMART_KERNEL=lanes|wave)."""
    import os
    from online_convex_optimization_amd import engine
    for B, T, d in ((768, 1000, 5), (32768, 1000, 5), (768, 1000, 64)):
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=1)
        if d == 5:
            n = B // 16
            db.generate_family("iid", 2025 * (1 + np.repeat(np.arange(n), 16)),
                               13 + np.tile(np.arange(16), n))
        else:
            db.generate_gT(0, 0)
        for kern in ("lanes", "wave"):
            os.environ["OCX_SMART_KERNEL"] = kern
            r0 = db.simulate_smart(math.sqrt(2 * T)).clone()
            sync()
            t0 = time.perf_counter()
            r = db.simulate_smart(math.sqrt(2 * T))
            sync()
            dt = time.perf_counter() - t0
            print(json.dumps({"what": "smart", "kernel": kern, "B": B, "T": T, "d": d,
                              "seconds": dt, "timesteps_per_s": B * T / dt,
                              "same_as_first": bool((r == r0).all())}), flush=True)
        os.environ.pop("OCX_SMART_KERNEL", None)
        del db


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=128, help="lanes_per_seq of the sweeps")
    ap.add_argument("--Ts", default="", help="sweep: only these horizons (comma list)")
    ap.add_argument("--d", type=int, default=16, help="config1: the dimension")
    ap.add_argument("--lanes-list", default="128,1,0,2,4,-2,-4", help="config1: layouts to time")
    ap.add_argument("what", nargs="+", choices=["gen", "gen1", "sweep", "driver", "smart", "config1", "config3", "exact_driver", "config4", "sweep_budget", "prof_long"])
    a = ap.parse_args()
    for w in a.what:
        globals()[w](a)
        # hand everything back before the next item: the sweeps size their resident batches
        # by the free HBM, which torch's cache and the engine's buffers would otherwise hold
        import torch
        from online_convex_optimization_amd import engine
        engine.release_buffers()
        torch.cuda.empty_cache()
