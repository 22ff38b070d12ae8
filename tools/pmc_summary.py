#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs into per-launch HBM traffic for one kernel.

Usage:
  tools/pmc_summary.py --fetch DIR_OR_CSV --write DIR_OR_CSV --kernel k_ld_pass \
      --label r01 [--algorithmic-bytes B] [--K K --M M] > profiles/pmc_ld_pass_r01.json
(bench.py attaches a summary's traffic only to a run of the same kernel, K, M and
algorithmic bytes per launch.)

Corrections (MI355X_MICROARCH.md, HBM section; cdna_hip_programming.md section 7):
* FETCH_SIZE and WRITE_SIZE are in KiB (x1024);
* on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide coalesced
  streaming read (16 B/lane global_load / buffer_load ... lds): x2.  The LD
  pass reads R with 16-B nontemporal loads per lane, so the x2 applies;
* WRITE_SIZE reads exact for 16-B-per-lane streaming stores (the LD pass's
  stores are 8 B per lane and few: they are reported uncorrected).
FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slot limits).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys


def find_csv(path):
    if os.path.isfile(path):
        return path
    c = glob.glob(os.path.join(path, "**", "*counter_collection*.csv"), recursive=True)
    if not c:
        sys.exit("no counter_collection csv under %s" % path)
    return sorted(c)[-1]


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(find_csv(path)) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[int(d)] = vals.get(int(d), 0.0) + float(row["Counter_Value"])
    return [vals[d] for d in sorted(vals)]


def grouped(vals, n):
    """sums of n consecutive dispatches: one pass launched as n block groups"""
    return [sum(vals[i:i + n]) for i in range(0, len(vals) - n + 1, n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_ld_pass")
    ap.add_argument("--label", default="")
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("--K", type=int, default=None, help="cohorts of the profiled bench run")
    ap.add_argument("--M", type=int, default=None, help="markers of the profiled bench run")
    ap.add_argument("--group", type=int, default=1,
                    help="launches per pass (block groups, round 5): traffic is summed per pass")
    a = ap.parse_args()
    fetch = grouped(per_dispatch(a.fetch, "FETCH_SIZE", a.kernel), a.group)
    write = grouped(per_dispatch(a.write, "WRITE_SIZE", a.kernel), a.group)
    if not fetch:
        sys.exit("no FETCH_SIZE rows for kernel %s" % a.kernel)
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write) if write else 0.0
    read_b = f_kib * 1024 * 2
    write_b = w_kib * 1024
    out = {
        "kernel": a.kernel,
        "label": a.label,
        "K": a.K,
        "M": a.M,
        "launches_per_pass": a.group,
        "dispatches_fetch": len(fetch),
        "dispatches_write": len(write),
        "FETCH_SIZE_kib_median": f_kib,
        "WRITE_SIZE_kib_median": w_kib,
        "read_bytes_per_launch": read_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "correction": "FETCH_SIZE x1024 x2 (gfx950 wide-stream half count), WRITE_SIZE x1024",
    }
    if a.algorithmic_bytes:
        out["algorithmic_bytes_per_launch"] = a.algorithmic_bytes
        out["traffic_over_algorithmic"] = (read_b + write_b) / a.algorithmic_bytes
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
