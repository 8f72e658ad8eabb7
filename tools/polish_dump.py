import numpy as np, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from online_convex_optimization_amd import engine as eng
out = {}
for norm, code in (("linf", 2), ("l1", 1), ("l2", 0)):
    d = 33
    B, T = 2, 3 * d + 20
    rng = np.random.default_rng(1000 + d + code)
    z = 3.0 * rng.standard_normal((B, T, d)); y = rng.standard_normal((B, T))
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    for k, v in res.items(): out[f"{norm}_{k}"] = v
    out[f"{norm}_z"] = z; out[f"{norm}_y"] = y
# the LP case d=8 real linf clip
rng = np.random.default_rng(11 * 8)
z = rng.standard_normal((3, 40, 8)); z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True)); y = rng.standard_normal((3, 40))
res = eng.exact_ball_solve(z, y, norm="linf", all_prefixes=True)
for k, v in res.items(): out[f"c8_{k}"] = v
out["c8_z"] = z; out["c8_y"] = y
np.savez(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "polish_dump.npz"), **out)
print("ok")
