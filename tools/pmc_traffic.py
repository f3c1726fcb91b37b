"""Per-launch HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh).

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): both counters are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read (128-B requests tallied at 64 B), so it is doubled;
WRITE_SIZE is taken as is.  Dispatches are grouped by (kernel, grid size) so the config-2 BA launches and
the scaled-sweep launches of k_linearize stay apart; a kernel that early-exits on some launches
(k_linearize after a rejected LM step) is summarised over its active launches (write traffic above half
of the group's maximum).  Usage: pmc_traffic.py <pmc dir> <out.json> [command that was profiled]
"""
import collections
import csv
import glob
import json
import re
import sys


def load(path):
    per = collections.defaultdict(list)
    for f in glob.glob(path + "/run_counter_collection.csv") + glob.glob(path + "/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"\bk_\w+", r["Kernel_Name"])
            name = m.group(0) if m else r["Kernel_Name"][:40]
            per[(name, int(r["Grid_Size"]), r["Counter_Name"])].append(
                (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return per


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch = load(root + "/p1")
    write = load(root + "/p2")
    groups = {}
    for (name, grid, c), v in fetch.items():
        w = write.get((name, grid, "WRITE_SIZE"))
        if c != "FETCH_SIZE" or not w:
            continue
        fv = [x for _, x in sorted(v)]
        wv = [x for _, x in sorted(w)]
        n = min(len(fv), len(wv))
        fv, wv = fv[:n], wv[:n]
        wmax = max(wv) if wv else 0.0
        act = [i for i in range(n) if wv[i] >= 0.5 * wmax] if wmax > 0 else list(range(n))
        fb = 2.0 * 1024.0 * sum(fv[i] for i in act) / len(act)
        wb = 1024.0 * sum(wv[i] for i in act) / len(act)
        groups["%s@grid%d" % (name, grid)] = {
            "kernel": name, "grid_size": grid, "dispatches": n, "active_dispatches": len(act),
            "fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb}
    cmd = sys.argv[3] if len(sys.argv) > 3 else "bench.py --steps 20 --warmup 4 --cpu-seconds 0"
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over %s; FETCH_SIZE "
                     "doubled (gfx950), KiB -> bytes" % cmd,
           "kernels": groups}
    json.dump(res, open(out, "w"), indent=1)
    for k, g in sorted(groups.items()):
        print("%-40s n=%4d act=%4d fetch %10.3f MB write %10.3f MB" % (
            k, g["dispatches"], g["active_dispatches"], g["fetch_bytes"] / 1e6, g["write_bytes"] / 1e6))


if __name__ == "__main__":
    main()
