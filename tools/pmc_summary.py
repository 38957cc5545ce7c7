"""Summary of tools/pmc_ab.sh: per build and kernel, the rocprofv3 average duration, fabric traffic per launch
((2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB: the gfx950 FETCH_SIZE correction, profiles/r4/calib) and the SQ counters
per wave (VALU / SALU / VMEM rd / VMEM wr / LDS / SMEM instructions; wave cycles active / issue-stalled / parked on
s_waitcnt; VALU busy = SQ_INSTS_VALU x 2 cycles / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8)).
    python3 tools/pmc_summary.py gpurun_out/<tag> [kernel-prefix ...]"""
import collections
import csv
import glob
import os
import sys


def short(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").replace("mi::", "")


def build(d, prefixes):
    dur = {}
    p = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            dur[short(r["Name"])] = float(r["AverageNs"]) / 1e6
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k in sorted(set(dur) | set(acc)):
        if not k.startswith(prefixes):
            continue
        m = {c: sum(x) / len(x) for c, x in acc[k].items()}
        w = m.get("SQ_WAVES") or 1
        wc = m.get("SQ_WAVE_CYCLES") or 1
        act, stall = m.get("SQ_ACTIVE_INST_ANY", 0), m.get("SQ_WAIT_INST_ANY", 0)
        cyc = (m.get("GRBM_GUI_ACTIVE") or 0) / 8
        traffic = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in m and "WRITE_SIZE" in m else None
        rows.append((k, dur.get(k), traffic, {n: m.get("SQ_INSTS_" + n, 0) / w for n in ("VALU", "SALU", "VMEM_RD",
                                                                                     "VMEM_WR", "LDS", "SMEM")},
                     100 * act / wc, 100 * stall / wc, 100 * (wc - act - stall) / wc,
                     100 * m.get("SQ_INSTS_VALU", 0) * 2 / (1024 * cyc) if cyc else None, w))
    return rows


def main(root, prefixes):
    print("| build | kernel | ms | traffic GB / launch | waves | VALU / wave | SALU | VMEM rd | VMEM wr | LDS | SMEM | "
          "active % | stalled % | parked % | VALU busy % |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(d):
            continue
        for k, ms, tr, ins, a, s, p, vb, w in build(d, prefixes):
            f = lambda x, n=1: "-" if x is None else f"{x:.{n}f}"   # noqa: E731
            if w <= 1:   # no SQ pass (PMC_SET=traffic)
                print(f"| {os.path.basename(d)} | {k} | {f(ms, 3)} | {f(tr and tr / 1e9, 2)} |" + " - |" * 11)
                continue
            print(f"| {os.path.basename(d)} | {k} | {f(ms, 3)} | {f(tr and tr / 1e9, 2)} | {w:.0f} | {ins['VALU']:.0f} | "
                  f"{ins['SALU']:.0f} | {ins['VMEM_RD']:.0f} | {ins['VMEM_WR']:.0f} | {ins['LDS']:.0f} | {ins['SMEM']:.0f} | "
                  f"{a:.1f} | {s:.1f} | {p:.1f} | {f(vb)} |")


if __name__ == "__main__":
    main(sys.argv[1], tuple(sys.argv[2:]) or ("tdec", "rm_", "ofdm", "chest", "tb_"))
