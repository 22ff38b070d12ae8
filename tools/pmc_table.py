#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (one CSV or directory).
  tools/pmc_table.py DIR [--kernel SUBSTR]
Prints per dispatch-average counter values and derived ratios (clock from
GRBM_GUI_ACTIVE / 8 XCDs / kernel time, SQ wait/issue fractions)."""
import argparse
import collections
import csv
import glob
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="k_sym")
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        p = sorted(glob.glob(os.path.join(p, "**", "*counter_collection*.csv"), recursive=True))[-1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    with open(p) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            if a.kernel not in k:
                continue
            d = row["Dispatch_Id"]
            per[d][row["Counter_Name"]] += float(row["Counter_Value"])
            dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
            names[d] = k.split("(")[0][:60]
    by = collections.defaultdict(list)
    for d in per:
        by[names[d]].append(d)
    for k, ds in by.items():
        n = len(ds)
        avg = collections.defaultdict(float)
        for d in ds:
            for c, v in per[d].items():
                avg[c] += v / n
        t = sum(dur[d] for d in ds) / n
        print("%s  dispatches=%d  avg %.3f ms" % (k, n, t * 1e3))
        for c in sorted(avg):
            print("   %-28s %.4g" % (c, avg[c]))
        if "GRBM_GUI_ACTIVE" in avg and t > 0:
            print("   clock(GUI_ACTIVE/8/t)       %.3f GHz" % (avg["GRBM_GUI_ACTIVE"] / 8 / t / 1e9))
        w = avg.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if c in avg:
                    print("   %-28s %.3f of wave cycles" % (c, avg[c] / w))
        b = avg.get("SQ_BUSY_CYCLES")
        if b and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            print("   MFMA busy / SQ busy          %.3f" % (avg["SQ_VALU_MFMA_BUSY_CYCLES"] / b))


if __name__ == "__main__":
    main()
