"""CPU: bench.py's host-side bookkeeping -- the `iterating.turbo_waves` histograms (where the
turbo iterations go, per code block and per packed-decoder wavefront pair) on a synthetic per-code-block
iteration array, without a GPU."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
