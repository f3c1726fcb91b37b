"""Matrix-core utilisation per launch from one rocprofv3 pass of SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
SQ_WAVE_CYCLES and GRBM_GUI_ACTIVE (tools/profile_round.sh).

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over the SIMDs (one v_mfma_f64_16x16x4f64 keeps
a SIMD's matrix core busy 64 cycles: profiles/r4_schur_bench_pmc.log); GRBM_GUI_ACTIVE is the launch's GPU
cycles summed over the 8 XCDs (MI355X_MICROARCH.md).  mfma_busy_frac = MFMA busy / (1024 SIMDs x GRBM_GUI_ACTIVE
/ 8): the share of the chip's matrix-core cycles the launch kept busy; mfma_busy_cycles_per_launch = the
busy cycles (64 per 16x16x4 f64 MFMA; k_schur's rhs slots run v_mfma_f64_4x4x4_4b_f64 since round 5).
Dispatches are grouped by (kernel, grid size).  Usage: pmc_mfma.py <pmc dir> <out.json> [profiled command]
"""
import collections
import csv
import glob
import json
import re
import sys


def main():
    root, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/run_counter_collection.csv") + glob.glob(root + "/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"\bk_\w+", r["Kernel_Name"])
            name = m.group(0) if m else r["Kernel_Name"][:40]
            per[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    groups = {}
    for (name, grid), cs in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in cs or "GRBM_GUI_ACTIVE" not in cs:
            continue
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        busy, gui = mean["SQ_VALU_MFMA_BUSY_CYCLES"], mean["GRBM_GUI_ACTIVE"]
        groups["%s@grid%d" % (name, grid)] = {
            "kernel": name, "grid_size": grid, "dispatches": len(cs["GRBM_GUI_ACTIVE"]), **mean,
            "mfma_busy_frac": busy / (1024.0 * gui / 8.0) if gui else None, "mfma_busy_cycles_per_launch": busy}
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    json.dump({"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE over "
                         + cmd, "formula": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": groups},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
