"""Summarise the SQ counter passes of tools/pmc_tdec.sh (per kernel, averaged over launches):
python3 tools/summarize_sq.py gpurun_out/<tag> > profiles/<round>/sq_counters.md

Derived (MI355X_MICROARCH.md 'rocprofv3 PMC slots'): WAIT_ANY = WAVE_CYCLES - ACTIVE_INST_ANY -
WAIT_INST_ANY (wave parked on s_waitcnt); VALU busy = SQ_INSTS_VALU x 2 cycles (wave64 on SIMD32) /
(1,024 SIMDs x kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs."""
import collections
import csv
import glob
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mi::", "").split("<")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | waves | VALU instr / wave | SALU / wave | VMEM rd / wave | VMEM wr / wave | "
          "active % | issue-stall % | parked (s_waitcnt) % | VALU busy % | VMEM LEVEL / instr | SMEM LEVEL / instr |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k, v in acc.items():
        if not k.startswith(("tdec", "rm_", "demap", "ofdm", "chest", "tb_")):
            continue
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVES", 0) or 1
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        act, stall = m.get("SQ_ACTIVE_INST_ANY", 0), m.get("SQ_WAIT_INST_ANY", 0)
        park = wc - act - stall
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
        busy = 100 * m.get("SQ_INSTS_VALU", 0) * 2 / (1024 * cyc)
        # SQ_INST_LEVEL_* accumulate in-flight instructions per sample: / instructions ~ mean latency (counter units)
        vlat = m["SQ_INST_LEVEL_VMEM"] / m["SQ_INSTS_VMEM"] if m.get("SQ_INSTS_VMEM") else float("nan")
        slat = m["SQ_INST_LEVEL_SMEM"] / m["SQ_INSTS_SMEM"] if m.get("SQ_INSTS_SMEM") else float("nan")
        print(f"| {k} | {w:.0f} | {m.get('SQ_INSTS_VALU', 0) / w:.0f} | {m.get('SQ_INSTS_SALU', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | {m.get('SQ_INSTS_VMEM_WR', 0) / w:.0f} | "
              f"{100 * act / wc:.1f} | {100 * stall / wc:.1f} | {100 * park / wc:.1f} | {busy:.1f} | {vlat:.0f} | {slat:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1])
