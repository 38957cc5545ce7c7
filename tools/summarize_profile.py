"""Summarise a tools/profile.sh output directory into summary.json + summary.md.

Per kernel: rocprofv3 kernel-trace average duration, HBM traffic per launch from the PMC passes
(FETCH_SIZE x 2 + WRITE_SIZE, in KiB units -> bytes; the x2 is the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md section HBM, which we checked against the OFDM kernel's known byte count), and
for the dominant kernel the algorithmic bytes / agreement with the bench line's live HIP-event time.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_src_hash  # noqa: E402


def short(name):
    n = name.split("(")[0].split("<")[0]      # template arguments dropped: tdec_kernel<true> -> tdec_kernel
    return n.replace("void ", "").replace("mi::", "")


def main(d):
    bench = json.load(open(os.path.join(d, "bench.json")))
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                   "pct": float(r["Percentage"])}
    pmc = collections.defaultdict(dict)
    for sub, cname in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] == cname:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            pmc[k][cname] = sum(v) / len(v)
    valu = collections.defaultdict(lambda: collections.defaultdict(list))
    vpath = os.path.join(d, "pmc_valu", "run_counter_collection.csv")
    if os.path.exists(vpath):
        for r in csv.DictReader(open(vpath)):
            valu[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, s in stats.items():
        if not k.startswith(("tdec", "rm_", "demap", "ofdm", "chest", "tb_")):
            continue
        f = pmc.get(k, {}).get("FETCH_SIZE")
        w = pmc.get(k, {}).get("WRITE_SIZE")
        traffic = None if f is None or w is None else (2 * f + w) * 1024
        # VALU busy = SQ_INSTS_VALU x 2 cycles (wave64 over two 32-lane passes) / (1,024 SIMDs x kernel cycles),
        # kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs (tools/summarize_sq.py)
        v = {c: sum(x) / len(x) for c, x in valu.get(k, {}).items()}
        busy = (100 * v["SQ_INSTS_VALU"] * 2 / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
                if v.get("SQ_INSTS_VALU") and v.get("GRBM_GUI_ACTIVE") else None)
        kernels[k] = dict(s, traffic_bytes_per_launch=traffic,
                          traffic_GBs=None if traffic is None else traffic / (s["avg_ms"] * 1e-3) / 1e9,
                          valu_busy_pct=None if busy is None else round(busy, 1),
                          valu_instr_per_wave=round(v["SQ_INSTS_VALU"] / v["SQ_WAVES"]) if v.get("SQ_WAVES") else None)
    rl = bench["roofline"]
    same_run_ms = None
    for line in open(os.path.join(d, "prof_trace.log"), errors="replace"):
        if line.startswith("{") and '"roofline"' in line:
            same_run_ms = json.loads(line)["roofline"]["avg_launch_ms"]
    td = next((v for k, v in kernels.items() if k.startswith("tdec_kernel")), {})
    summary = {
        "bench": {k: bench[k] for k in ("value", "unit", "ms_per_step", "stage_ms_per_step", "config")},
        "roofline_bench": rl,
        "kernels": kernels,
        # same command: the JSON line the bench printed inside the rocprofv3 --kernel-trace run
        "tdec_agreement": {"bench_hip_event_avg_ms_same_run": same_run_ms, "rocprof_avg_ms": td.get("avg_ms"),
                           "ratio": None if not (td and same_run_ms) else round(td["avg_ms"] / same_run_ms, 4),
                           "standalone_bench_hip_event_avg_ms": rl["avg_launch_ms"]},
        "tdec_traffic_over_algorithmic": None if not td.get("traffic_bytes_per_launch") else
        round(td["traffic_bytes_per_launch"] / rl["algorithmic_bytes_per_launch"], 3),
    }
    json.dump(summary, open(os.path.join(d, "summary.json"), "w"), indent=1)
    if td.get("traffic_bytes_per_launch"):
        json.dump({"src_hash": kernel_src_hash(), "sf_per_gpu": bench["config"]["subframes_per_gpu"],
                   "tdec": bench["config"].get("turbo_arithmetic", "gen"),
                   "tdec_kernel": rl["kernel"],
                   "tdec_traffic_bytes_per_launch": td["traffic_bytes_per_launch"],
                   "tdec_valu_busy_pct": td.get("valu_busy_pct"),
                   "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same bench command "
                             f"({os.path.basename(d)}); bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024"},
                  open(os.path.join(d, "traffic.json"), "w"), indent=1)
    with open(os.path.join(d, "summary.md"), "w") as f:
        f.write(f"# Profile summary ({os.path.basename(d)})\n\n")
        f.write(f"bench: {bench['value']} {bench['unit']}, {bench['ms_per_step']} ms/step, {bench['config']['workload']}\n\n")
        f.write("| kernel | calls | avg ms (rocprof) | % time | HBM traffic / launch (MB) | GB/s | VALU busy % |\n"
                "|---|---|---|---|---|---|---|\n")
        for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["pct"]):
            t = v["traffic_bytes_per_launch"]
            tmb = "-" if t is None else "%.1f" % (t / 1e6)
            gbs = "-" if t is None else "%.0f" % v["traffic_GBs"]
            f.write("| %s | %d | %.4f | %.2f | %s | %s | %s |\n" % (k, v["calls"], v["avg_ms"], v["pct"], tmb, gbs,
                                                               "-" if v["valu_busy_pct"] is None else v["valu_busy_pct"]))
        f.write(f"\ntdec agreement (rocprof / bench HIP events): {summary['tdec_agreement']}\n")
        f.write(f"\ntdec traffic / algorithmic bytes: {summary['tdec_traffic_over_algorithmic']}\n")
    print(json.dumps(summary["tdec_agreement"]), summary["tdec_traffic_over_algorithmic"])


if __name__ == "__main__":
    main(sys.argv[1])
