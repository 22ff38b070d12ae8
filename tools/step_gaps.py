"""Per-step GPU busy/idle time from a rocprofv3 kernel trace of bench.py.

Steps start at each k_em_prep launch (the first kernel of a VAMP step); the
last `--steps` of them are the timed ones.  Idle = wall span of the step minus
the union of its kernels' [start, end) intervals.
    python tools/step_gaps.py TRACE.csv [TRACE.csv ...] [--steps 10]
"""
import argparse
import csv


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def steps(rows, n):
    starts = [i for i, r in enumerate(rows) if "k_em_prep" in r[2]]
    out = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        seg = rows[a:b]
        busy, cur_s, cur_e = 0, seg[0][0], seg[0][1]
        for s, e, _ in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        nxt = rows[b][0] if b < len(rows) else cur_e
        out.append((nxt - seg[0][0], busy, len(seg)))
    return out[-n - 1:-1] if len(out) > n else out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    for p in a.traces:
        st = steps(load(p), a.steps)
        span = sum(s for s, _, _ in st) / len(st) / 1e6
        busy = sum(b for _, b, _ in st) / len(st) / 1e6
        print(f"{p}: {len(st)} steps, span {span:.3f} ms, busy {busy:.3f} ms, "
              f"idle {span - busy:.3f} ms, kernels/step {st[0][2]}")


if __name__ == "__main__":
    main()
