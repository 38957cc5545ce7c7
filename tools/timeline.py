"""Overlap analysis of a rocprofv3 --kernel-trace CSV of a multi-stream bench run:
python3 tools/timeline.py <kernel_trace.csv> [kernel-substring ...]
Prints, over the window spanned by the turbo-decoder launches: per kernel the count, mean duration, and the
fraction of wall time during which >= 1 of them runs; how much of the window has a turbo decoder running, and the
mean number of turbo launches running concurrently while any runs."""
import csv, sys, collections

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    name = r.get("Kernel_Name", "")
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", ""))))
td = [k for k in ks if "tdec_kernel_p2x" in k[2]]
if not td:
    print("no tdec_kernel_p2x launches"); sys.exit(0)
t0 = min(k[0] for k in td[len(td) // 4:])   # skip warm-up: the last 3/4 of the launches
t1 = max(k[1] for k in td)
win = [k for k in ks if k[1] > t0 and k[0] < t1]
print("window %.3f ms, %d launches" % ((t1 - t0) / 1e6, len(win)))

def cover(iv):
    """union length of intervals clipped to the window, and time-weighted mean concurrency while >= 1 runs"""
    ev = []
    for a, b in iv:
        a, b = max(a, t0), min(b, t1)
        if b > a:
            ev += [(a, 1), (b, -1)]
    ev.sort()
    cur, last, busy, area = 0, None, 0, 0
    for t, d in ev:
        if last is not None and cur > 0:
            busy += t - last
            area += (t - last) * cur
        cur += d
        last = t
    return busy, (area / busy if busy else 0)

groups = collections.defaultdict(list)
for a, b, n, q in win:
    key = n.split("(")[0].replace("void ", "").replace("mi::", "").split("<")[0]
    groups[key].append((a, b))
for key, iv in sorted(groups.items(), key=lambda x: -sum(b - a for a, b in x[1])):
    busy, conc = cover(iv)
    print("%-28s n %4d  mean %.3f ms  covers %5.1f %%  concurrency %.2f" % (
        key[:28], len(iv), sum(b - a for a, b in iv) / len(iv) / 1e6, 100 * busy / (t1 - t0), conc))
