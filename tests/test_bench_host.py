"""CPU: bench.py's host-side bookkeeping -- the `iterating.turbo_waves` histograms (where the
turbo iterations go, per code block and per packed-decoder wavefront pair) on a synthetic per-code-block
iteration array, without a GPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeBatch:
    def __init__(self, n_groups, n_cb, sched="p2", compact=True):
        self.n_groups, self.n_codeblocks, self.turbo_sched, self.turbo_compact = n_groups, n_cb, sched, compact


def test_wave_iterations_histograms():
    rng = np.random.default_rng(7)
    n_groups = 6                                     # 3 group pairs of 128 lanes
    cb = rng.choice([1, 2, 3, 4], size=64 * n_groups, p=[0.7, 0.2, 0.07, 0.03]).astype(np.uint32)
    cb[-10:] = 0                                     # padding lanes of the last group (no code block)
    w = bench.wave_iterations(FakeBatch(n_groups, 64 * n_groups - 10), cb)
    assert sum(w["cb_its_hist"].values()) == 64 * n_groups - 10
    assert w["cb_its_hist"] == {v: int((cb == v).sum()) for v in (1, 2, 3, 4)}
    assert abs(w["cb_mean_its"] - cb[cb > 0].mean()) < 1e-4
    assert w["codeblocks_past_iteration_0"] == int((cb > 1).sum())
    pm = cb.reshape(3, 128).max(axis=1)
    assert w["pair_max_its_hist"] == {int(v): int((pm == v).sum()) for v in np.unique(pm)}
    assert w["pair_iterations_without_compaction"] == int(pm.sum())
    assert w["compaction"] is True
    assert w["continuation_pairs"] == -(-int((cb > 1).sum()) // 128)


def test_wave_iterations_other_schedules_have_no_pair_fields():
    cb = np.ones(128, np.uint32)
    w = bench.wave_iterations(FakeBatch(2, 128, sched="lanexr", compact=False), cb)
    assert "pair_max_its_hist" not in w and "continuation_pairs" not in w
    assert w["cb_its_hist"] == {1: 128}


class FakeRunner:
    """Counts runs; stage_ms() reports a fixed isolated duration (abi.Batch / TdecBatch profiling interface)."""
    def __init__(self):
        self.runs, self.resets = 0, 0

    def profile_reset(self):
        self.resets += 1
        self.runs = 0

    def stage_ms(self):
        return {"tdec": 6.4, "rm": 2.4}, self.runs


def test_isolated_stages_only_for_overlapped_steps(monkeypatch):
    """--streams S > 1: the roofline divides by isolated re-runs after the timed region (one workspace alone,
    each run synchronised), the overlapped average stays beside it; S == 1 keeps the timed region's events."""
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda dev=None: None)
    r = FakeRunner()
    assert bench.isolated_stages(r, None, "cpu", 1, 200) is None and r.resets == 0

    def run():
        r.runs += 1
    st, n = bench.isolated_stages(r, run, "cpu", 4, 200)
    assert r.resets == 1 and n == 10 and st["tdec"] == 6.4
    assert bench.isolated_stages(r, run, "cpu", 4, 3)[1] == 3
    t = bench.roofline_timing({"tdec": 19.3}, 200, (st, n))
    assert t["avg_launch_ms"] == 6.4 and t["launches_averaged"] == 10
    assert t["avg_launch_ms_overlapped"] == 19.3 and t["launches_averaged_overlapped"] == 200
    assert bench.roofline_timing({"tdec": 6.5}, 200, None) == {"avg_launch_ms": 6.5, "launches_averaged": 200}


def test_split_share():
    """--split F: the front end's CU eighths of a split run (mi_dl_batch_run_split); by default tuned on the box for the
    headline shard and off elsewhere, and off with one stream (a lone workspace's front end waits for its own back
    end: nothing to overlap)."""
    import argparse
    import bench
    ns = lambda f, c=4: argparse.Namespace(split=f, config=c)   # noqa: E731
    assert bench.split_share(ns(-1), 4) == -1                        # headline: tuned on the box (tune_split)
    assert bench.split_share(ns(-1, 5), 16) == 0 and bench.split_share(ns(-1, 3), 16) == 0
    assert bench.split_share(ns(0), 4) == 0
    assert bench.split_share(ns(2), 4) == 2 and bench.split_share(ns(3, 5), 16) == 3
    assert bench.split_share(ns(2), 1) == 0 and bench.split_share(ns(-1), 1) == 0


def test_tune_split_rule(monkeypatch):
    """tune_split keeps split runs only when their best ms per step beats whole runs' by more than SPLIT_MARGIN, timing
    3 S steps of each layout per round (a fake clock advanced by the fake runs)."""
    clock = [0.0]
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda dev=None: None)
    monkeypatch.setattr(bench.time, "perf_counter", lambda: clock[0])

    def runner(ms):
        def run(i):
            clock[0] += ms[0] * 1e-3
        return run

    for whole_ms, split_ms, want in ((8.30, 7.95, bench.AUTO_SPLIT), (7.90, 8.02, 0), (8.00, 7.90, 0)):
        calls = []
        w, s = [whole_ms], [split_ms]
        F, rec = bench.tune_split(lambda i: (calls.append("w"), runner(w)(i)), lambda i: (calls.append("s"), runner(s)(i)),
                                  4, "cpu")
        assert F == want, (whole_ms, split_ms)
        assert calls.count("w") == calls.count("s") == 2 * 12 and rec["steps_each"] == 12
        assert abs(min(rec["whole_ms_per_step"]) - whole_ms) < 1e-6 and rec["chosen"] == ("split" if F else "whole")


def test_hw_queues_argument():
    """--hw-queues N and --hw-queues=N are both honoured, checked to 0..32 (gpurun refuses more than 32), and
    importing bench (as the GPU tests do) leaves GPU_MAX_HW_QUEUES alone."""
    import bench
    assert bench.hw_queues_arg([], {}) == "8"
    assert bench.hw_queues_arg(["--hw-queues", "16"], {}) == "16"
    # 16 by default when the process brings up RCCL (its streams take queues too): N > 1 ranks or --pg, not the
    # gloo --share-gpu rehearsal or the parent that only spawns the ranks (it never touches the GPU)
    assert bench.hw_queues_arg(["--gpus", "8"], {"WORLD_SIZE": "8"}) == "16"
    assert bench.hw_queues_arg(["--pg"], {}) == "16"
    assert bench.hw_queues_arg(["--gpus", "2", "--share-gpu"], {"WORLD_SIZE": "2"}) == "8"
    assert bench.hw_queues_arg(["--gpus", "8", "--hw-queues", "8"], {"WORLD_SIZE": "8"}) == "8"
    assert bench.hw_queues_arg(["--steps", "3", "--hw-queues=0"]) == "0"
    for bad in (["--hw-queues", "33"], ["--hw-queues=-1"], ["--hw-queues=x"]):
        with pytest.raises(SystemExit):
            bench.hw_queues_arg(bad)
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([sys.executable, "-c", "import os, bench; print(os.environ.get('GPU_MAX_HW_QUEUES'))"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.stdout.strip() == "None", out.stdout + out.stderr


@pytest.mark.parametrize("S,want", [(1, 2), (2, 2), (3, 4), (4, 4), (5, 6), (6, 6)])
def test_static_workspaces_count(S, want):
    """The static planning replay keeps one list per workspace on J = 2 lists: S rounded up to a multiple of J, never
    lcm(S, J) = 2 S for odd S (10 workspaces of ~45 GB at S = 5)."""
    W = bench.static_workspaces(S, 2)
    assert W == want
    # every list is kept by some workspace, and every stream is used
    assert {k % 2 for k in range(W)} == {0, 1}
    assert {k % S for k in range(W)} == set(range(S))
