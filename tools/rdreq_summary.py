"""Summarise tools/pmc_rdreq.sh: per kernel, the average per dispatch of each TCC counter, and read bytes counted as
32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (checked against the calibration kernels' known byte counts)."""
import collections, csv, glob, sys

out = sys.argv[1]
for part in ("calib", "bench", "bench_hit"):
    f = glob.glob(out + "/" + part + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print(part, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        agg[r["Kernel_Name"].split("(")[0][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", part)
    for k, cs in agg.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        line = "  ".join("%s %.4g" % (c.replace("TCC_EA0_", "").replace("_sum", ""), v) for c, v in sorted(avg.items()))
        if "TCC_EA0_RDREQ_128B_sum" in avg:
            b = 32 * avg.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * avg.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                128 * avg.get("TCC_EA0_RDREQ_128B_sum", 0)
            line += "  | bytes(by size) %.4g GB" % (b / 1e9)
        print("%-48s %s" % (k, line))
