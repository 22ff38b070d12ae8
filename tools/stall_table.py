#!/usr/bin/env python3
"""Per-kernel table of the `gpu_recipes.sh stall` passes (two --pmc runs of one
workload): clock, VMEM and LDS instruction levels per instruction (outstanding
instructions summed per cycle / instructions issued), the active-instruction
mix and LDS issue waits as fractions of wave cycles, TA busy (GRBM) and the TA
stall counters summed over the TA instances.  Raw ratios: read them next to
each other (north star vs band walk), not as absolute latencies.
  python tools/stall_table.py gpurun_out/stall1_TAG gpurun_out/stall2_TAG"""
import collections
import csv
import json
import sys


def load(d, min_ns=200000):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(d + "/pmc_counter_collection.csv")):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for did, c in per.items():
        name, ns = meta[did]
        if ns < min_ns:
            continue
        key = name.split("(")[0].replace("void ", "").replace("sgv::", "")
        n[key] += 1
        for k, v in c.items():
            agg[key][k] += v
        agg[key]["_ns"] += ns
    return agg, n


def main():
    a1, n1 = load(sys.argv[1])
    a2, _ = load(sys.argv[2])
    for k, c in sorted(a1.items()):
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        out = dict(kernel=k[:48], dispatches=n1[k], mean_ms=round(c["_ns"] / n1[k] / 1e6, 3),
                   clock_GHz=round(c["GRBM_GUI_ACTIVE"] / 8 / c["_ns"], 3),
                   vmem_level_per_inst=round(c["SQ_INST_LEVEL_VMEM"] / max(c["SQ_INSTS_VMEM_RD"], 1), 1),
                   active_valu=round(c["SQ_ACTIVE_INST_VALU"] / wc, 3),
                   active_lds=round(c["SQ_ACTIVE_INST_LDS"] / wc, 3),
                   wait_inst_lds=round(c["SQ_WAIT_INST_LDS"] / wc, 3))
        d = a2.get(k)
        if d:
            gui = d["GRBM_GUI_ACTIVE"] or 1.0
            out.update(ta_busy=round(d["GRBM_TA_BUSY"] / gui, 3),
                       ta_addr_stalled_by_tc_sum_per_busy=round(
                           d["TA_ADDR_STALLED_BY_TC_CYCLES"] / max(d["GRBM_TA_BUSY"], 1), 3),
                       ta_data_stalled_by_tc_sum_per_busy=round(
                           d["TA_DATA_STALLED_BY_TC_CYCLES"] / max(d["GRBM_TA_BUSY"], 1), 3),
                       lds_fifo_full=round(d["SQ_LDS_DATA_FIFO_FULL"] / (d["SQ_WAVE_CYCLES"] or 1), 4),
                       lds_level_per_inst=round(d["SQ_INST_LEVEL_LDS"] / max(d["SQ_INSTS_LDS"], 1), 2))
        print(json.dumps(out))


if __name__ == "__main__":
    main()
