"""one line per bench JSON of a gpurun_out directory: value, ms/step, schedule, tdec ms, iterations"""
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(os.path.basename(f), "unreadable", e); continue
    it = d.get("iterating") or {}
    print("%-14s %10s %8s %-34s tdec %8s its %s ok %s | iter tdec %s Mbps %s" % (
        os.path.basename(f), d.get("value"), d.get("ms_per_step"), d["config"].get("turbo_schedule", "")[:34],
        d.get("stage_ms_per_step", {}).get("tdec"), d.get("mean_turbo_iterations"), d.get("crc_ok_rate"),
        it.get("stage_ms_per_step", {}).get("tdec"), it.get("Mbps")))
