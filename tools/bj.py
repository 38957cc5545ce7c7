"""one line per bench JSON file: value, ms/step, tdec / rm ms, roofline, waterfall block, planning"""
import json, os, sys
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(os.path.basename(f), "unreadable", e); continue
    st = d.get("stage_ms_per_step", {})
    rf = d.get("roofline") or {}
    it = d.get("iterating") or {}
    itr = it.get("tdec_roofline") or {}
    print("%-12s %9.1f Mbps %6.3f ms  tdec %s rm %s  launch %s frac %s  | iter %s Mbps tdec %s  | cpu %s" % (
        os.path.basename(f), d.get("value", 0), d.get("ms_per_step", 0), st.get("tdec"), st.get("rm"),
        rf.get("avg_launch_ms"), rf.get("frac"), it.get("Mbps"), itr.get("avg_launch_ms"),
        (d.get("cpu_baseline") or {}).get("value")))
