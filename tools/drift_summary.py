#!/usr/bin/env python3
"""Per-dispatch durations of the LD pass's main kernel over a kernel trace, in
time bins: does the pass slow down as the run goes on (the clock the chip holds
under sustained load)?
    python tools/drift_summary.py TRACE_DIR [bin_ms]"""
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    bin_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 250.0
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(f)))
    main_k = [(s, e) for s, e, n in rows if ("k_sym_mfma" in n or "k_sym_pass" in n)
              and e - s > 100000]
    if not main_k:
        print("no pass dispatches")
        return
    t0 = main_k[0][0]
    bins = {}
    for s, e in main_k:
        bins.setdefault(int((s - t0) / 1e6 // bin_ms), []).append((e - s) / 1e6)
    print("%s: %d passes over %.2f s" % (d, len(main_k), (main_k[-1][1] - t0) / 1e9))
    for b in sorted(bins):
        v = bins[b]
        print("  t = %6.0f ms  passes %3d  median %.4f ms  min %.4f  max %.4f" % (
            b * bin_ms, len(v), statistics.median(v), min(v), max(v)))


if __name__ == "__main__":
    main()
