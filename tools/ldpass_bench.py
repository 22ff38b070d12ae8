#!/usr/bin/env python3
"""LD-pass microbenchmark: kernel time per pass (HIP events inside the shim)
for dense vs packed-symmetric storage and 1..16 right-hand sides.

  python tools/ldpass_bench.py [--blocks 8] [--block-size 25000] [--nsamp 2000] [--reps 5]
Prints one JSON object per (format, ncol)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

from engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--block-size", type=int, default=25000)
    ap.add_argument("--nsamp", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ncols", default="1,2,3,4,8,12,16")
    ap.add_argument("--lib", default=None, help="A/B: load this build of libsgvamp_hip.so")
    ap.add_argument("--formats", default="packed,packed_valu,dense",
                    help="packed (f64 MFMA pass from 3 columns), packed_valu, dense")
    a = ap.parse_args()
    if a.lib:
        import hip_backend
        hip_backend.load(a.lib)
    sizes = [a.block_size] * a.blocks
    M = sum(sizes)
    for fmt in a.formats.split(","):
        eng = Engine(sizes, K=1)
        eng.set_ld_packing(fmt.startswith("packed"))
        if fmt == "packed_valu":
            eng.set_mfma_min(0)
        eng.synth_ld_g(0, 11, a.nsamp, np.zeros(M))
        rs = np.random.RandomState(0)
        for nc in [int(x) for x in a.ncols.split(",")]:
            V = rs.normal(size=(nc, M))
            eng.ld_matvec(0, V)                       # warm
            eng.timers(reset=True)
            for _ in range(a.reps):
                eng.ld_matvec(0, V)
            t = eng.timers()
            ms = t["ld_ms"] / t["ld_launches"]
            print(json.dumps(dict(
                format=fmt, ncol=nc, ms_per_pass=ms,
                stored_GBs=t["ld_bytes"] / t["ld_launches"] / ms / 1e6,
                dense_equiv_GBs=t["dense_bytes"] / t["ld_launches"] / ms / 1e6,
                stored_GB=t["ld_bytes"] / t["ld_launches"] / 1e9,
                aux_MB=t["aux_bytes"] / t["ld_launches"] / 1e6)), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
