"""Per-kernel times of one resident g(T) batch: generator, FTRL (closed-form comparator)
and FTRL two-pass, for (B, T, d, lanes) cases given as BxTxDxL.  One JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from online_convex_optimization_amd import engine
    for case in sys.argv[1].split(","):
        B, T, d, lanes = (int(v) for v in case.split("x"))
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes)
        res = {"B": B, "T": T, "d": d, "lanes": lanes, "P": int(db.L.P), "C": int(db.L.C),
               "chain": int(db.L.chain), "waves": int(db.L.G)}
        fns = [("gen_ms", lambda: db.generate_gT(0, 0)),
               ("sim_closed_ms", lambda: db.simulate_alg(closed_comparator=True)),
               ("sim_two_pass_ms", lambda: db.simulate_alg(closed_comparator=False))]
        if os.environ.get("PROBE_EXACT"):  # the fused FTRL + exact FTL kernel (configs[2])
            cf = torch.zeros(B, dtype=torch.float64, device=db.device)
            fns += [("fe_closed_ms", lambda: db.ftrl_vs_exact(comp_ftl=cf, closed_comparator=True)),
                    ("fe_two_pass_ms", lambda: db.ftrl_vs_exact(comp_ftl=cf, closed_comparator=False))]
        for name, fn in fns:
            fn()
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
            for _ in range(2):
                fn()
            e[1].record()
            torch.cuda.synchronize()
            res[name] = e[0].elapsed_time(e[1]) / 2
        bpp = B * T * (8 * d + 8)
        res["sim_closed_frac"] = bpp / (res["sim_closed_ms"] * 1e-3) / 8e12
        res["sim_two_pass_frac"] = 2 * bpp / (res["sim_two_pass_ms"] * 1e-3) / 8e12
        res["e2e_timesteps_per_s"] = B * T / ((res["gen_ms"] + res["sim_closed_ms"]) * 1e-3)
        print(json.dumps(res), flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
