"""Per-launch means of every counter in one or more rocprofv3 --pmc output trees, grouped by (kernel, grid size).

Usage: pmc_group.py <out.json> <pmc dir> [<pmc dir> ...]
Each directory is one --pmc pass (rocprofv3 does not split counters over passes); the groups of all passes are
merged, so a counter collected in two passes (GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES as a cross-check) keeps both means.
"""
import collections
import csv
import glob
import json
import re
import sys


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    groups = collections.defaultdict(dict)
    for i, root in enumerate(dirs):
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        files = (glob.glob(root + "/run_counter_collection.csv") + glob.glob(root + "/*/run_counter_collection.csv")
                 + glob.glob(root + "/*/*/run_counter_collection.csv"))
        for f in files:
            for r in csv.DictReader(open(f)):
                m = re.search(r"\bk_\w+", r["Kernel_Name"])
                name = m.group(0) if m else r["Kernel_Name"][:40]
                per[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for (name, grid), cs in per.items():
            g = groups["%s@grid%d" % (name, grid)]
            for c, v in cs.items():
                key = c if c not in g else "%s#pass%d" % (c, i + 1)
                g[key] = sum(v) / len(v)
                g.setdefault("dispatches_pass%d" % (i + 1), len(v))
    json.dump({"passes": dirs, "kernels": groups}, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
