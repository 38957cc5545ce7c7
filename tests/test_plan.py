"""CPU: the host planner behind mi_dl_plan_build / mi_dl_batch_replan (include/mi_dl.h).

* mi_dl_plan_build is host-only -- it runs here, with no GPU -- for the default shard, varied per-subframe grants
  (bench.varied_cfgs) and configs[4]'s mixed cells, and rejects bad configurations with an error string;
* the planner's output is pinned: tools/plan_dump.cpp builds four seeded scenarios (uniform shard, varied grants,
  mixed cells with partial allocations and TM2, HARQ mix with new_tb = 0 and rv 0-3) and digests everything the
  kernels read, with table offsets resolved to table contents.  The digests below were produced by the round-3
  planner (before the round-4 rewrite that shares RE lists across RNTI / Qm, counting-sorts the code blocks and
  finds the busy rate-matching chunks by binary search), so the rewrite feeds the kernels exactly the same values."""
import ctypes as C
import os
import shutil
import subprocess

import pytest

from srsue_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PINNED_1000 = ["bc5321547fa8b244", "a20cb6b375dcebdd", "270b69ece8902398", "a4272f923aee78f4"]
# round 4: the rate de-matching work list in XCD queues (plan.cpp xcd_order; MI_RM_XCDQ=0 restores launch order,
# whose digests stay the round-3 ones above) -- only the order of the work items and their padding differ
PINNED_1000_XCDQ = ["a8a162fd8056e17c", "98387cdd846c58be", "c0350a36f49274d9", "20f8be341ddcf81c"]


def test_plan_build_host_only(built):
    import bench
    p = abi.Plan()
    for cfgs in (bench.config_cfgs(4, 600, 0), bench.varied_cfgs(600, 0), bench.config_cfgs(5, 600, 0),
                 bench.config_cfgs(3, 100, 0)):
        p.build(cfgs)
        p.build(abi.cfg_array(cfgs))      # prebuilt array, warm caches
    bad = abi.sf_cfg(Qm=5)
    with pytest.raises(RuntimeError, match="Qm"):
        p.build([bad])
    p.close()


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_planner_output_pinned(tmp_path):
    exe = str(tmp_path / "plan_dump")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DMI_EMU", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "srsue_amd", "csrc"), "-w", os.path.join(ROOT, "tools", "plan_dump.cpp"),
                    os.path.join(ROOT, "srsue_amd", "csrc", "plan.cpp"), os.path.join(ROOT, "srsue_amd", "csrc", "tables.cpp"),
                    "-o", exe], check=True, timeout=300)
    for xcdq, pinned in (("0", PINNED_1000), ("1", PINNED_1000_XCDQ)):
        env = dict(os.environ, MI_RM_XCDQ=xcdq)
        out = subprocess.run([exe, "1000"], capture_output=True, text=True, check=True, timeout=120, env=env).stdout
        digests = [ln.split("digest ")[1].split()[0] for ln in out.splitlines() if "digest" in ln]
        assert digests == pinned, (xcdq, out)
