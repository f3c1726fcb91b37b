"""Summarise rocprofv3 counter-collection CSVs (per-dispatch mean of each counter) under a directory."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print("%-42s %-22s %.4g  (n=%d)" % (k, c, sum(v) / len(v), len(v)))
