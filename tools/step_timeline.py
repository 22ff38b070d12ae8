#!/usr/bin/env python3
"""Per-step GPU timeline from a rocprofv3 --kernel-trace (+ --memory-copy-trace)
CSV of bench.py: span, busy time, launches and idle gaps between consecutive
VAMP steps (delimited by sgv::k_denoise).
  python tools/step_timeline.py gpurun_out/trace [--last 3] [--gap-us 15]"""
import argparse
import collections
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--gap-us", type=float, default=15.0)
    a = ap.parse_args()
    K = list(csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv"))))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:44]) for r in K]
    cp = os.path.join(a.dir, "run_memory_copy_trace.csv")
    if os.path.exists(cp):
        ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"])
               for r in csv.DictReader(open(cp))]
    ev.sort()
    den = [e for e in ev if "k_denoise" in e[2]]
    for i in range(max(0, len(den) - a.last - 1), len(den) - 1):
        t0, t1 = den[i][0], den[i + 1][0]
        seg = [e for e in ev if t0 <= e[0] < t1]
        busy = sum(e[1] - e[0] for e in seg)
        dur = collections.defaultdict(int)
        cnt = collections.Counter(e[2] for e in seg)
        for e in seg:
            dur[e[2]] += e[1] - e[0]
        gaps = [((b[0] - x[1]) / 1e3, x[2], b[2]) for x, b in zip(seg, seg[1:])
                if b[0] - x[1] > a.gap_us * 1e3]
        print("step span %.3f ms  busy %.3f ms  launches %d  gaps>%gus: %d (%.1f us)"
              % ((t1 - t0) / 1e6, busy / 1e6, len(seg), a.gap_us, len(gaps),
                 sum(g[0] for g in gaps)))
        for k, v in sorted(dur.items(), key=lambda x: -x[1]):
            print("   %-44s %3d %9.1f us" % (k, cnt[k], v / 1e3))
        for g in gaps:
            print("   gap %6.1f us  %s -> %s" % g)


if __name__ == "__main__":
    main()
