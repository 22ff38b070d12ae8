"""LD-pass times from a rocprofv3 kernel trace of bench.py, for comparison with
the bench line's HIP-event average (roofline.avg_launch_ms).

The pipelined CG enqueues one pass past its stop test; that pass exits at once
(~5 us), and rocprofv3's --stats average mixes it in.  This summary keeps the
passes that ran: k_sym_mfma / k_sym_pass / k_ld_pass dispatches of >= 100 us,
each with the k_pack (k_pack16 before round 3) before it and the finalize after it.
    python tools/trace_pass_summary.py TRACE.csv [BENCH.json]
"""
import csv
import json
import statistics
import sys

MAIN = ("k_sym_mfma", "k_sym_pass", "k_ld_pass")


def main():
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(sys.argv[1])))
    passes = []
    for i, (s, e, n) in enumerate(rows):
        if any(m in n for m in MAIN) and "finalize" not in n and e - s >= 100_000:
            t0 = rows[i - 1][0] if i and "k_pack" in rows[i - 1][2] else s
            t1 = rows[i + 1][1] if i + 1 < len(rows) and "finalize" in rows[i + 1][2] else e
            passes.append(((e - s) / 1e6, (t1 - t0) / 1e6, n.split("(")[0]))
    if not passes:
        sys.exit("no LD pass dispatches in the trace")
    d = None
    if len(sys.argv) > 2:   # the timed passes: the last `launches` of the run
        d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
        passes = passes[-int(d["roofline"]["launches"]):]
    main_ms = [p[0] for p in passes]
    full_ms = [p[1] for p in passes]
    print("passes that ran%s: %d (%s)" % (" (timed steps)" if d else "", len(passes),
                                          sorted({p[2] for p in passes})))
    print("main kernel: mean %.4f ms, median %.4f, min %.4f, max %.4f"
          % (statistics.mean(main_ms), statistics.median(main_ms), min(main_ms), max(main_ms)))
    print("pass (pack + main + finalize, first start to last end): mean %.4f ms"
          % statistics.mean(full_ms))
    if d:
        print("bench line (HIP events, same command): avg_launch_ms %.4f over %d launches"
              % (d["roofline"]["avg_launch_ms"], d["roofline"]["launches"]))


if __name__ == "__main__":
    main()
