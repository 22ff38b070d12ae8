#!/usr/bin/env python3
"""Per-dispatch effective shader clock and stall mix from rocprofv3 --pmc runs.

Effective clock = GRBM_GUI_ACTIVE / 8 / dispatch wall time (rocprofv3 sums the
8 XCDs; MI355X_MICROARCH.md, "DVFS give-back").  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES
/ 1024 SIMDs / (wall time x clock).  WAIT_INST / WAIT_ANY are fractions of
SQ_WAVE_CYCLES (issue stalls / s_waitcnt-barrier waits).

  python tools/clock_summary.py [--filter k_sym] DIR [DIR ...]
Each DIR holds pmc_counter_collection.csv; dispatches shorter than 0.3 ms are skipped."""
import argparse
import collections
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for d in a.dirs:
        rows = list(csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))))
        per = collections.defaultdict(dict)
        meta = {}
        for r in rows:
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[did] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print("== %s" % d)
        for did in sorted(per):
            name, ns = meta[did]
            if ns < 300000 or a.filter not in name:
                continue
            c = per[did]
            out = "  %-58s %8.3f ms" % (name[:58], ns / 1e6)
            clk = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 / ns
            if clk:
                out += "  clk %.2f GHz" % clk
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    out += "  mfma-busy %.2f" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (ns * clk))
            w = c.get("SQ_WAVE_CYCLES", 0.0)
            if w:
                for k, lab in (("SQ_WAIT_INST_ANY", "wait-inst"), ("SQ_WAIT_ANY", "wait-any"),
                               ("SQ_ACTIVE_INST_ANY", "active")):
                    if k in c:
                        out += "  %s %.2f" % (lab, c[k] / w)
            print(out)


if __name__ == "__main__":
    main()
