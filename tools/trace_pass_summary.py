"""LD-pass times from a rocprofv3 kernel trace of bench.py, for comparison with
the bench line's HIP-event average (roofline.avg_launch_ms).

The pipelined CG enqueues one pass past its stop test; that pass exits at once
(~5 us), and rocprofv3's --stats average mixes it in.  This summary keeps the
passes that ran: k_sym_mfma / k_sym_pass / k_ld_pass dispatches of >= 100 us,
each with the k_pack (k_pack16 before round 3) before it and the finalize after it;
since round 5 a pass may be several main-kernel launches (block groups) with their
finalizes on a second stream: the pass is first start to last end of them all.
    python tools/trace_pass_summary.py TRACE.csv [BENCH.json]
"""
import csv
import glob
import os
import json
import statistics
import sys

MAIN = ("k_sym_mfma", "k_sym_pass", "k_ld_pass", "k_band_walk")
PART = MAIN + ("k_pack", "finalize", "k_walk_fin", "k_coupling")


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "*kernel_trace.csv"))[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    # a pass = a maximal run of consecutive pass dispatches (pack, the main
    # kernel's launches -- one per block group since round 5 -- and the
    # finalizes on the side stream); it counts if its main launches ran >= 100 us
    passes, cur = [], []

    def close():
        if cur:
            mains = [(e - s) for s, e, n in cur if any(m in n for m in MAIN) and "finalize" not in n]
            if sum(mains) >= 100_000:
                t0 = min(s for s, _, _ in cur)
                t1 = max(e for _, e, _ in cur)
                name = next(n for _, _, n in cur if any(m in n for m in MAIN)).split("(")[0]
                passes.append((sum(mains) / 1e6, (t1 - t0) / 1e6, name, len(mains)))
        cur.clear()

    for s, e, n in rows:
        if any(m in n for m in PART):
            cur.append((s, e, n))
        else:
            close()
    close()
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
    print("main kernel launches per pass: %s" % sorted({p[3] for p in passes}))
    print("main kernel (sum over its launches): mean %.4f ms, median %.4f, min %.4f, max %.4f"
          % (statistics.mean(main_ms), statistics.median(main_ms), min(main_ms), max(main_ms)))
    print("pass (pack + main + finalize, first start to last end): mean %.4f ms"
          % statistics.mean(full_ms))
    if d:
        print("bench line (HIP events, same command): avg_launch_ms %.4f over %d launches"
              % (d["roofline"]["avg_launch_ms"], d["roofline"]["launches"]))


if __name__ == "__main__":
    main()
