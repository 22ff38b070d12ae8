#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc runs: one row per kernel name.

  python tools/kernel_pmc_table.py [--filter k_band] DIR [DIR ...]

Each DIR holds a pmc_counter_collection.csv (one --pmc pass); rows of the same
kernel name are merged across DIRs (the passes of one workload).  Printed per
kernel: dispatches, mean duration, and what the counters present give --
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall time), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / cycles), the wave-time split
(SQ_WAIT_INST_ANY issue stalls, SQ_WAIT_ANY s_waitcnt/barrier waits,
SQ_WAIT_INST_LDS of the issue stalls), LDS bank-conflict cycles per LDS-array
cycle, and HBM bytes per dispatch (FETCH_SIZE x1024 x2 for 16-B streaming
reads, WRITE_SIZE x1024; MI355X_MICROARCH.md's HBM section).  Dispatches shorter
than --min-us are skipped."""
import argparse
import collections
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--min-us", type=float, default=50.0)
    ap.add_argument("--json", action="store_true", help="one JSON object per kernel")
    a = ap.parse_args()
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    dur = collections.defaultdict(list)
    for d in a.dirs:
        path = d if d.endswith(".csv") else os.path.join(d, "pmc_counter_collection.csv")
        per, meta = collections.defaultdict(dict), {}
        for r in csv.DictReader(open(path)):
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[did] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for did, c in per.items():
            name, ns = meta[did]
            if ns < a.min_us * 1e3 or a.filter not in name:
                continue
            dur[name].append(ns)
            for k, v in c.items():
                sums[name][k] += v
                cnt[name][k] += 1
                sums[name]["_ns_" + k] += ns
    for name in sorted(dur):
        s, n = sums[name], cnt[name]
        mean = {k: s[k] / n[k] for k in n}
        ns_of = {k: s["_ns_" + k] / n[k] for k in n}
        o = {"kernel": name[:90], "dispatches": len(dur[name]),
             "mean_ms": round(sum(dur[name]) / len(dur[name]) / 1e6, 4)}
        if "GRBM_GUI_ACTIVE" in mean:
            clk = mean["GRBM_GUI_ACTIVE"] / 8 / ns_of["GRBM_GUI_ACTIVE"]
            o["clock_GHz"] = round(clk, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                o["mfma_busy"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024
                                       / (ns_of["SQ_VALU_MFMA_BUSY_CYCLES"] * clk), 3)
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for k, lab in (("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_WAIT_ANY", "waitcnt_barrier"),
                           ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "lds_issue_stall")):
                if k in mean:
                    o[lab] = round(mean[k] / wc, 3)
        if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
            o["lds_conflict_per_active"] = round(mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"], 4)
        for k in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_MFMA"):
            if k in mean:
                o[k] = mean[k]
        if "FETCH_SIZE" in mean:
            o["fetch_GB"] = round(mean["FETCH_SIZE"] * 1024 * 2 / 1e9, 4)
        if "WRITE_SIZE" in mean:
            o["write_GB"] = round(mean["WRITE_SIZE"] * 1024 / 1e9, 4)
        print(json.dumps(o) if a.json else "  ".join("%s=%s" % kv for kv in o.items()))


if __name__ == "__main__":
    main()
