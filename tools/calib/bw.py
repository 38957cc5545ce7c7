"""Bandwidth of each calibration kernel (tools/calib/pmc_calib.hip) from a rocprofv3 kernel-stats CSV."""
import csv, sys
B = 2 ** 31
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    b = B // 2 if "wr16_rows" in n else (B // 8 if "wr_partial" in n else B)
    ns = float(r["AverageNs"])
    print("%-60s %8.3f ms  %6.2f TB/s" % (n[:60], ns / 1e6, b / ns / 1e3))
