"""The profile summarisers the bench line's evidence comes from (CPU, synthetic
rocprofv3 CSVs): tools/pmc_summary.py sums the block-group launches of a pass
(--group) before taking the median per pass and applies the gfx950 corrections;
tools/trace_pass_summary.py measures a pass from its first launch to its last
finalize across both streams."""
import csv
import json
import os
import subprocess
import sys

from tests.conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def _counters(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name",
                                          "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for did, name, counter, value in rows:
            w.writerow(dict(Dispatch_Id=did, Kernel_Name=name, Counter_Name=counter,
                            Counter_Value=value, Start_Timestamp=1000 * did,
                            End_Timestamp=1000 * did + 500000))


def test_pmc_summary_groups_launches(tmp_path):
    k = "void sgv::k_sym_mfma<2, 2, false, true>(...)"
    # 3 passes of 4 group launches; FETCH_SIZE in KiB, counted per XCD (summed)
    fetch, write = [], []
    for p in range(3):
        for g in range(4):
            did = 10 * p + g
            for xcd in range(2):
                fetch.append((did, k, "FETCH_SIZE", 1000.0 * (g + 1) + p))
                write.append((did, k, "WRITE_SIZE", 10.0 * (g + 1)))
            fetch.append((did + 5, "sgv::k_pack", "FETCH_SIZE", 7.0))   # another kernel
    _counters(tmp_path / "f.csv", fetch)
    _counters(tmp_path / "w.csv", write)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "pmc_summary.py"), "--fetch",
                          str(tmp_path / "f.csv"), "--write", str(tmp_path / "w.csv"),
                          "--kernel", "k_sym_mfma<2", "--group", "4",
                          "--algorithmic-bytes", "1e7"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["launches_per_pass"] == 4 and d["dispatches_fetch"] == 3
    # per pass: 2 XCDs x sum_g 1000 (g + 1) + 4 p -> median over p = 1 (p = 1)
    fetch_kib = 2 * (1000.0 * 10 + 4 * 1)
    assert d["FETCH_SIZE_kib_median"] == fetch_kib
    assert d["read_bytes_per_launch"] == fetch_kib * 1024 * 2      # x1024, gfx950 x2
    assert d["write_bytes_per_launch"] == 2 * 10.0 * 10 * 1024
    assert abs(d["traffic_over_algorithmic"]
               - (d["read_bytes_per_launch"] + d["write_bytes_per_launch"]) / 1e7) < 1e-12


def test_trace_pass_spans_both_streams(tmp_path):
    # one pass: pack, 4 group launches, 4 finalizes overlapping on the side
    # stream; then a CG kernel; then a no-op pass (short launches) to skip
    rows = [(0, 10, "sgv::k_pack(...)")]
    t = 10
    for g in range(4):
        rows.append((t, t + 2_000_000, "void sgv::k_sym_mfma<2, 2, false, true>(...)"))
        rows.append((t + 2_000_000, t + 2_300_000, "void sgv::k_sym_finalize_strip<8>(...)"))
        t += 2_000_000
    rows.append((t + 400_000, t + 500_000, "sgv::k_cg_xr(...)"))
    rows.append((t + 600_000, t + 600_010, "sgv::k_pack(...)"))
    for g in range(4):
        rows.append((t + 600_100 + g, t + 600_105 + g, "void sgv::k_sym_mfma<2, 2, false, true>(...)"))
    path = tmp_path / "kernel_trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for s, e, n in rows:
            w.writerow(dict(Kernel_Name=n, Start_Timestamp=s, End_Timestamp=e))
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "trace_pass_summary.py"), str(path)],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "passes that ran: 1" in out.stdout
    assert "main kernel launches per pass: [4]" in out.stdout
    assert "mean 8.0000 ms" in out.stdout                       # 4 x 2 ms of MFMA kernel
    assert "first start to last end): mean 8.3000 ms" in out.stdout
