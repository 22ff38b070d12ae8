#!/usr/bin/env python3
"""Per-workgroup timeline of the NC <= 8 MFMA LD pass (diagnostic library built
with -DSGV_MF_TRACE, see tools/README.md): when each strip's workgroup started
and ended (wall clock, 100 MHz), so the launch's tail -- the time after the first
workgroup slot runs out of strips -- can be read off.

  python tools/strip_trace.py --lib tools/diaglib/libsgvamp_trace.so --shape 8x15625 --ncol 8
Prints one JSON object per shape."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

import hip_backend  # noqa: E402
from engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--shapes", default="8x15625,64x15625")
    ap.add_argument("--ncol", type=int, default=8)
    ap.add_argument("--env", default="", help="VAR=VALUE pairs set before the library loads")
    a = ap.parse_args()
    lib = hip_backend.load(a.lib)
    lib.sgv_diag_mf_trace.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.sgv_diag_mf_trace.restype = ctypes.c_int
    for shape in a.shapes.split(","):
        nb, n = (int(x) for x in shape.split("x"))
        sizes = [n] * nb
        M = sum(sizes)
        eng = Engine(sizes, K=1)
        eng.synth_ld_g(0, 11, 2000, np.zeros(M))
        V = np.random.RandomState(0).normal(size=(a.ncol, M))
        for _ in range(3):
            eng.ld_matvec(0, V)
        buf = (ctypes.c_ulonglong * (3 * 65536))()
        got = lib.sgv_diag_mf_trace(buf, 65536)
        tr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3)[:got]
        live = tr[tr[:, 1] > 0]
        t0 = live[:, 0].min()
        st = (live[:, 0] - t0) / 100.0   # us
        en = (live[:, 1] - t0) / 100.0
        span = en.max()
        dur = en - st
        # the slot view: sort end times; the tail starts when strips stop starting
        last_start = st.max()
        busy = dur.sum()
        cus = np.unique(live[:, 2]).size
        # concurrency over time (active workgroups, sampled every 5 us) and the
        # per-CU hand-over gap: from a workgroup's end to the next start on that CU
        ts = np.arange(0.0, span, 5.0)
        act = np.array([np.count_nonzero((st <= t) & (en > t)) for t in ts])
        gaps = []
        for cu in np.unique(live[:, 2]):
            m = live[:, 2] == cu
            s_cu, e_cu = np.sort(st[m]), np.sort(en[m])
            # with two slots per CU: the k-th start after the first two follows the (k-2)-th end
            if s_cu.size > 2:
                gaps.extend((s_cu[2:] - e_cu[:-2]).tolist())
        gaps = np.array(gaps) if gaps else np.zeros(1)
        # per XCD: workgroup i is assumed dispatched to XCD i % 8 (round robin);
        # the CU id tells where it ran -- the table checks the assumption, and
        # each XCD's first start / last end / busy show whether the tail is an
        # XCD running out of work while others still have strips
        idx = np.nonzero(tr[:, 1] > 0)[0]
        xcd_of = idx % 8
        cu = live[:, 2].astype(np.int64)
        per_xcd = []
        for x in range(8):
            m = xcd_of == x
            if not m.any():
                continue
            per_xcd.append(dict(xcd=x, strips=int(m.sum()), busy_us=round(float(dur[m].sum()), 1),
                                last_start=round(float(st[m].max()), 1),
                                last_end=round(float(en[m].max()), 1),
                                mean_us=round(float(dur[m].mean()), 1),
                                cus=int(np.unique(cu[m]).size),
                                cu_ids=[int(cu[m].min()), int(cu[m].max())]))
        if os.environ.get("SGV_TRACE_RAW"):
            np.save(os.environ["SGV_TRACE_RAW"] + "_%s.npy" % shape, live)
        print(json.dumps(dict(
            per_xcd=per_xcd,
            active_mean=round(float(act.mean()), 1),
            active_pctl={p: int(np.percentile(act, p)) for p in (1, 10, 50, 90)},
            handover_gap_us={p: round(float(np.percentile(gaps, p)), 1) for p in (10, 50, 90, 99)},
            shape=shape, ncol=a.ncol, strips=int(live.shape[0]), cus_seen=int(cus),
            span_us=round(float(span), 1), last_start_us=round(float(last_start), 1),
            tail_us=round(float(span - last_start), 1),
            strip_us_median=round(float(np.median(dur)), 1), strip_us_max=round(float(dur.max()), 1),
            slot_util=round(float(busy / (span * 512)), 3),
            end_pctl_us={p: round(float(np.percentile(en, p)), 1) for p in (50, 90, 99, 100)})),
              flush=True)
        eng.close()


if __name__ == "__main__":
    main()
