"""GPU: generation overlapped with FTRL (ocx_dev_gen_simulate, csrc/ocx_pipeline.hip).

The pipelined path runs the same generator and FTRL arithmetic as the sequential
generate-then-simulate loop (fast_algorithms.py:230-247 over resident batches), split into
sub-batches on two streams: its regrets and g(T) must be bit-identical to that loop's, and
the sampled sequences within the closed-form bar of the oracle."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.test_gpu_parity import close_closed

pytestmark = pytest.mark.gpu
SQ2 = math.sqrt(2)


@pytest.fixture(scope="module")
def eng():
    from online_convex_optimization_amd import _lib, engine
    assert _lib.device_count() >= 1
    return engine


@pytest.mark.parametrize("B,T,d,lanes,sub", [(3000, 300, 64, 8, 512), (2048, 257, 64, 16, 0),
                                             (1000, 64, 64, 128, 0), (36000, 40, 64, 128, 0),
                                             (3000, 300, 16, 8, 512), (20000, 77, 16, 8, 0),
                                             (2500, 129, 32, 8, 1024), (17000, 50, 32, 8, 0)])
def test_pipelined_equals_sequential(eng, B, T, d, lanes, sub):
    """d = 64 in the lean pipelined FTRL layouts; d = 16 / 32 (round 6) in the g(T) layouts of
    8 lanes (2 / 4 coordinates each), whose FTRL side is the plain kernel over group ranges."""
    import torch
    nb = 3
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=lanes)
    out = {}
    for mode in (False, True):
        g = torch.zeros(1, dtype=torch.float64, device=db.device)
        db.regret.zero_()
        db.generate_simulate(base_seed=9, run0=5, nbatch=nb, gmax=g, pipelined=mode,
                             sub_seqs=sub)
        torch.cuda.synchronize()
        out[mode] = (db.regret[:B].cpu().numpy().copy(), float(g.item()))
    assert np.array_equal(out[True][0], out[False][0])
    assert out[True][1] == out[False][1]
    # the last batch's regrets are those of runs 5 + 2B ..; g(T) over all 3 batches
    allr = eng.gT_regrets(T, nb * B, base_seed=9, d=d, run0=5, lanes_per_seq=lanes)
    assert close_closed(out[True][0], allr[2 * B:], T)
    assert out[True][1] == eng.max_regret(allr) or close_closed(out[True][1], eng.max_regret(allr), T)
    for b in (0, B - 1):
        z, y = O.gT_sample(9, T, 5 + 2 * B + b, d)
        assert close_closed(out[True][0][b], O.simulate_alg(z, y, 0, SQ2), T), b


@pytest.mark.parametrize("T,d,runs", [(120, 16, 40000), (60, 32, 33000)])
def test_gT_small_d_pipeline_equals_sequential(eng, monkeypatch, T, d, runs):
    """engine.gT_regrets / gT_max at d = 16 / 32 (configs[1]'s g(T) layouts) through the sub-batch
    pipeline (round 6) equal the sequential loop (OCX_PIPELINE=0) bit for bit, and sampled
    sequences are within the closed-form bar of the oracle."""
    out = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("OCX_PIPELINE", pipe)
        out[pipe] = (eng.gT_regrets(T, runs, base_seed=12, d=d, run0=3),
                     eng.gT_max(T, runs, base_seed=12, d=d, run0=3))
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][1] == out["0"][1] == eng.max_regret(out["0"][0])
    for r in (0, runs // 3, runs - 1):
        z, y = O.gT_sample(12, T, 3 + r, d)
        assert close_closed(out["1"][0][r], O.simulate_alg(z, y, 0, SQ2), T), r


def test_pipelined_exact_layout_two_pass(eng):
    """A bit-exact layout is not pipelined (sequential fallback) and keeps the reference's
    streamed comparator: bit-identical to the oracle."""
    import torch
    B, T, d = 70, 120, 64
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=1)
    g = torch.zeros(1, dtype=torch.float64, device=db.device)
    db.generate_simulate(base_seed=2, run0=0, nbatch=2, gmax=g)
    torch.cuda.synchronize()
    reg = db.regret[:B].cpu().numpy()
    for b in (0, 33, B - 1):
        z, y = O.gT_sample(2, T, B + b, d)
        assert reg[b] == O.simulate_alg(z, y, 0, SQ2), b
    ref = max(0.0, max(O.simulate_alg(*O.gT_sample(2, T, r, d), 0, SQ2) for r in range(2 * B)))
    assert float(g.item()) == ref


@pytest.mark.parametrize("streams", ["1", "2"])
def test_pipelined_stream_counts(eng, streams, monkeypatch):
    """One or two streams per side (OCX_PIPE_GEN_STREAMS / OCX_PIPE_SIM_STREAMS): the sub-batches
    only reorder, so regrets and g(T) are the sequential loop's bit for bit."""
    import torch
    B, T, d = 3000, 150, 64
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=8)
    out = {}
    for mode in (False, True):
        if mode:
            monkeypatch.setenv("OCX_PIPE_GEN_STREAMS", streams)
            monkeypatch.setenv("OCX_PIPE_SIM_STREAMS", streams)
        g = torch.zeros(1, dtype=torch.float64, device=db.device)
        db.generate_simulate(base_seed=4, run0=1, nbatch=3, gmax=g, pipelined=mode, sub_seqs=256)
        torch.cuda.synchronize()
        out[mode] = (db.regret[:B].cpu().numpy().copy(), float(g.item()))
    assert np.array_equal(out[True][0], out[False][0])
    assert out[True][1] == out[False][1]


def test_generation_in_rounds_is_bit_identical(eng, monkeypatch):
    """ocx_launch_gen_gT takes generator rounds over two streams for d = 64 batches of four or
    more rounds: the tiles equal the single launch's (OCX_GEN_ROUNDS=0) bit for bit."""
    import torch
    B, T, d = 16384, 40, 64
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=eng.LANES_BEST)
    tiles = {}
    for rounds in ("0", "1"):
        monkeypatch.setenv("OCX_GEN_ROUNDS", rounds)
        db.z.fill_(float("nan"))
        db.y.fill_(float("nan"))
        db.generate_gT(base_seed=6, run0=3)
        torch.cuda.synchronize()
        tiles[rounds] = (db.z.view(torch.int64).clone(), db.y.view(torch.int64).clone())
    assert torch.equal(tiles["0"][0], tiles["1"][0]) and torch.equal(tiles["0"][1], tiles["1"][1])
    for b in (0, 4097, B - 1):  # sequences of the first, second and last rounds vs NumPy
        z, y = O.gT_sample(6, T, 3 + b, d)
        zz, yy = db.rows_of(torch.tensor([b], device=db.device))
        assert np.array_equal(zz[0].cpu().numpy(), z) and np.array_equal(yy[0].cpu().numpy(), y), b


def test_pipeline_captures_into_a_graph(eng):
    """ocx_dev_gen_simulate allocates nothing and never synchronises.  Under HIP graph capture
    on the HIP 7.0 runtime torch ships, which segfaults ending the capture of any three-stream
    fork / join (tools/capture_repro.hip, tools/capture_torch_repro.py), it keeps
    to the capturing stream (ocx_stream_fork_ok); on ROCm 7.2's runtime the overlapped
    pipeline itself captures (the reproducer's stages 2-3).  Either way a captured graph
    replays with regrets and g(T) equal to the eager, overlapped call's, bit for bit."""
    import torch
    B, T, d = 3000, 120, 64
    s = torch.cuda.Stream()
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=8, stream=s)
    ge = torch.zeros(1, dtype=torch.float64, device=db.device)
    with torch.cuda.stream(s):
        db.generate_simulate(base_seed=7, run0=0, nbatch=2, gmax=ge, sub_seqs=512)  # eager
    torch.cuda.synchronize()
    ref, gref = db.regret[:B].clone(), float(ge.item())
    gm = torch.zeros(1, dtype=torch.float64, device=db.device)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        db.generate_simulate(base_seed=7, run0=0, nbatch=2, gmax=gm, sub_seqs=512)
    torch.cuda.synchronize()
    for _ in range(2):
        db.regret.zero_()
        gm.zero_()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(db.regret[:B], ref) and float(gm.item()) == gref


# ---- the trailing pipeline (ocx_run_gen_sim_trailing): capacity-limited resident batches
# of ocx_gT_regrets / ocx_gT_max, batch k+1 generated chunk by chunk behind the chunked FTRL
# pass over batch k in one z buffer.  A small OCX_HBM_BUDGET_GB makes the batches capacity-
# limited at test sizes; OCX_TRAILING=0 is the sequential generate-then-simulate loop.

def _capacity_limited(monkeypatch, gb):
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", str(gb))
    monkeypatch.setenv("OCX_MIN_RESIDENT", "16")


@pytest.mark.parametrize("T,d,runs,gb,chunks", [(2000, 64, 1000, 0.35, "8"), (700, 64, 900, 0.06, "3"),
                                                (300, 64, 500, 0.02, "2"), (200, 64, 9000, 0.5, "2")])
def test_trailing_equals_sequential(eng, monkeypatch, T, d, runs, gb, chunks):
    """Regrets (host and device-resident) and g(T) of the trailing path equal the sequential
    loop's bit for bit, over several batches and a smaller last one, and sampled sequences are
    within the closed-form bar of the oracle.  The first three cases' batches (< 4 096 runs)
    take the 16 x 4 layout, the last one's (4 500 runs) 8 x 8; each call is checked to have
    gone through the trailing pipeline (ocx_test_trailing_batches)."""
    import torch
    from online_convex_optimization_amd import _lib
    _capacity_limited(monkeypatch, gb)
    monkeypatch.setenv("OCX_TRAIL_CHUNKS", chunks)
    out = {}
    for trail in ("0", "1"):
        monkeypatch.setenv("OCX_TRAILING", trail)
        n0 = _lib.load().ocx_test_trailing_batches()
        reg = eng.gT_regrets(T, runs, base_seed=3, d=d, run0=11, lanes_per_seq=eng.LANES_BEST)
        gm = eng.gT_max(T, runs, base_seed=3, d=d, run0=11, lanes_per_seq=eng.LANES_BEST)
        dev = eng.gT_regrets_device(T, runs, base_seed=3, d=d, run0=11,
                                    lanes_per_seq=eng.LANES_BEST)
        torch.cuda.synchronize()
        ran = _lib.load().ocx_test_trailing_batches() - n0
        # three calls, two or more batches each through the trailing path (none without it)
        assert (ran >= 6) if trail == "1" else (ran == 0), (trail, ran)
        out[trail] = (reg, gm, dev.cpu().numpy())
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][1] == out["0"][1] == eng.max_regret(out["0"][0])
    assert np.array_equal(out["1"][2], out["0"][0])
    for r in (0, runs // 2, runs - 1):
        z, y = O.gT_sample(3, T, 11 + r, d)
        assert close_closed(out["1"][0][r], O.simulate_alg(z, y, 0, SQ2), T), r


def test_trailing_rerun_of_flagged_batches(eng, monkeypatch):
    """A batch the trailing path flags (a sequence the closed form cannot certify: NaN regret)
    runs again whole; the test hook flags every second batch, and the regrets stay the
    sequential loop's bit for bit."""
    from online_convex_optimization_amd import _lib
    _capacity_limited(monkeypatch, 0.12)
    T, d, runs = 1000, 64, 600
    monkeypatch.setenv("OCX_TRAILING", "0")
    ref = eng.gT_regrets(T, runs, base_seed=5, d=d, lanes_per_seq=eng.LANES_BEST)
    monkeypatch.setenv("OCX_TRAILING", "1")
    got = np.zeros(runs)
    _lib.call("ocx_test_gT_regrets_unclean", 5, T, 0, runs, d, SQ2, _lib.ptr(got),
              eng.LANES_BEST, 0, 2)
    assert np.array_equal(got, ref)


def test_trailing_full_size_t1e5(eng):
    """configs[3]'s T = 1e5 point at its full per-batch size (d = 64, the default HBM budget:
    ≈4 500 runs per batch, 3 batches, the last smaller): the trailing path's regrets for
    sequences of the first, middle and last batch within the closed-form bar of the oracle,
    and g(T) equal to the max of the regrets the same call returns."""
    import torch
    T, d, runs = 100000, 64, 9800
    reg = eng.gT_regrets(T, runs, base_seed=0, d=d, lanes_per_seq=eng.LANES_BEST)
    gm = eng.gT_max(T, runs, base_seed=0, d=d, lanes_per_seq=eng.LANES_BEST)
    assert gm == eng.max_regret(reg)
    picks = [0, runs // 2, runs - 1]
    zs, ys = zip(*(O.gT_sample(0, T, r, d) for r in picks))
    ref = O.simulate_alg_batch(np.stack(zs), np.stack(ys), 0, SQ2, nthreads=3)[0]
    for i, r in enumerate(picks):
        assert close_closed(reg[r], ref[i], T), (r, reg[r], ref[i])
    eng.release_buffers()
    torch.cuda.empty_cache()
