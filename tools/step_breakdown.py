"""Where a bench step's GPU time goes: per kernel name, the summed duration over
the timed steps of a rocprofv3 kernel trace of bench.py, per step and as a share
of the step's wall span (steps start at k_em_prep; the last --steps of them).
    python tools/step_breakdown.py TRACE.csv [--steps 10]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(a.trace)))
    starts = [i for i, r in enumerate(rows) if "k_em_prep" in r[2]]
    lo, hi = starts[-a.steps - 1], starts[-1]      # the last `steps` complete steps
    seg = rows[lo:hi]
    span = (rows[hi][0] - rows[lo][0]) / 1e6 / a.steps
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in seg:
        name = n.split("(")[0].replace("void ", "").replace("sgv::", "")
        tot[name] += (e - s) / 1e6 / a.steps
        cnt[name] += 1
    busy = sum(tot.values())
    print("%d steps: %.3f ms per step (wall), %.3f ms busy, %.3f ms idle" % (a.steps, span, busy,
                                                                             span - busy))
    print("%-40s %9s %7s %9s" % ("kernel", "ms/step", "share", "launches"))
    for name, t in sorted(tot.items(), key=lambda x: -x[1]):
        print("%-40s %9.3f %6.1f%% %9.1f" % (name[:40], t, 100 * t / span, cnt[name] / a.steps))


if __name__ == "__main__":
    main()
