#!/usr/bin/env python3
"""A/B of LD-pass kernel variants (selected by SGV_AB=1 environment switches,
one variant per process): ms per pass (HIP events in the shim, pack + pass +
finalize) on several block structures, and a SHA-256 of the products so that
runs of different variants can be checked bitwise against each other.

  SGV_AB=1 SGV_MF_GLDS=2 python tools/ldpass_ab.py --tag glds2 --shapes 64x15625,8x25000
Prints one JSON object per (shape, ncol)."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

from engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--shapes", default="64x15625")
    ap.add_argument("--ncols", default="4,8")
    ap.add_argument("--nsamp", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="A/B of builds: load this libsgvamp_hip.so")
    ap.add_argument("--rhs", default="normal", choices=["normal", "zero", "ones"],
                    help="right-hand sides (zero/ones: the pass's data-dependent power, not its products)")
    a = ap.parse_args()
    if a.lib:
        import hip_backend
        hip_backend.load(a.lib, strict=False)
    for shape in a.shapes.split(","):
        nb, n = (int(x) for x in shape.split("x"))
        sizes = [n] * nb
        M = sum(sizes)
        eng = Engine(sizes, K=1)
        eng.synth_ld_g(0, 11, a.nsamp, np.zeros(M))
        rs = np.random.RandomState(0)
        for nc in [int(x) for x in a.ncols.split(",")]:
            V = rs.normal(size=(nc, M))
            if a.rhs == "zero":
                V[:] = 0.0
            elif a.rhs == "ones":
                V[:] = 1.0
            Y = eng.ld_matvec(0, V)                       # warm
            eng.timers(reset=True)
            for _ in range(a.reps):
                eng.ld_matvec(0, V)
            t = eng.timers()
            ms = t["ld_ms"] / t["ld_launches"]
            print(json.dumps(dict(tag=a.tag, shape=shape, ncol=nc, ms_per_pass=round(ms, 4),
                                  stored_GBs=round(t["ld_bytes"] / t["ld_launches"] / ms / 1e6, 1),
                                  sha=hashlib.sha256(Y.tobytes()).hexdigest()[:16])), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
