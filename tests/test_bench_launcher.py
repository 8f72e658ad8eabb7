"""bench.py --gpus N (CPU): the launcher starts N ranks itself when no launcher is around
it, and refuses a --gpus that does not match the ranks or devices it would run on."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "bench_rank_stub.py")
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    # at most one visible GPU, whatever box runs this: the refusals below must not turn into
    # a real multi-GPU bench
    env.update(HIP_VISIBLE_DEVICES="0", ROCR_VISIBLE_DEVICES="0", CUDA_VISIBLE_DEVICES="0")
    env.update(kw)
    return env


def test_launcher_spawns_two_gloo_ranks():
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, ['--gpus', '2', '--dist-backend', 'gloo', "
            "'--B', '6', '--T', '200', '--d', '8', '--cpu-seconds', '0.2'], "
            "script=%r))" % (ROOT, STUB))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=180, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["world_size"] == 2
    ranks = out["ranks"]
    assert sorted(r["rank"] for r in ranks) == [0, 1]
    assert sorted(r["local_rank"] for r in ranks) == [0, 1]
    assert len({r["pid"] for r in ranks}) == 2
    assert all(r["dist_on"] for r in ranks)
    # the CPU leg and the parity check at world size 2 (rank 0, bench.cpu_leg)
    cpu, par = out["cpu_baseline"], out["parity"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] == 1
    assert cpu["value_all_cores"] > 0 and cpu["kind"] == "port"
    assert par is not None and par["n_checked"] >= 1 and par["bitexact"]
    assert par["within_tolerance"]


def test_gpus_must_match_world_size():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True,
                       timeout=180, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "WORLD_SIZE=1" in p.stderr


def test_gpus_beyond_visible_devices_fails():
    # at most one GPU visible (_env): an RCCL run over 2 ranks must refuse, not share device 0
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True,
                       timeout=180, env=_env())
    assert p.returncode == 2
    assert "GPUs visible" in p.stderr
