"""bench.py's roofline bookkeeping (CPU): the PMC traffic attached to a bench
line must come from a summary of the same workload."""
import json
import os
import sys

from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _summaries():
    out = {}
    for f in sorted(os.listdir(os.path.join(ROOT, "profiles"))):
        if "pmc" in f and f.endswith(".json"):
            out[f] = json.load(open(os.path.join(ROOT, "profiles", f)))
    return out


def test_traffic_matches_workload_bytes():
    sums = _summaries()
    assert sums, "no PMC summaries committed under profiles/"
    for name, d in sums.items():
        alg = d.get("algorithmic_bytes_per_launch")
        if not alg:
            continue
        kern = "k_sym_mfma" if "k_sym_mfma" in d["kernel"] else d["kernel"].split("<")[0]
        traffic, src = bench.read_traffic(kern, alg, d["K"], d["M"])
        assert src is not None
        got = sums[src]
        assert abs(got["algorithmic_bytes_per_launch"] - alg) <= 0.01 * alg
        assert (got["K"], got["M"]) == (d["K"], d["M"])
        assert traffic == got["hbm_bytes_per_launch"]


def test_traffic_none_for_unprofiled_workload():
    # the C2 pass bytes at ten times the size: no summary, so no traffic claimed
    assert bench.read_traffic("k_sym_pass", 2.0e11, 1, 200000) == (None, None)
    assert bench.read_traffic("k_no_such_kernel", 20210140245.0, 1, 200000) == (None, None)
    # C5 and the north star store the same LD (bytes within 0.2 %): K tells them apart
    src = bench.read_traffic("k_sym_mfma", 63779430912.0, 8, 1000000)[1]
    assert src.startswith("pmc_sym_mfma_") and src.endswith("_c5.json"), src
    src = bench.read_traffic("k_sym_mfma", 63651430912.0, 4, 1000000)[1]
    assert src.startswith("pmc_sym_mfma_") and src.endswith("_northstar.json"), src


def test_northstar_and_c2_summaries_present():
    sums = _summaries()
    kinds = {(d["kernel"].split("<")[0], round(d.get("algorithmic_bytes_per_launch") or 0, -9))
             for d in sums.values()}
    assert ("k_sym_pass", 2.0e10) in kinds          # C2, K = 1
    assert ("k_sym_mfma", 6.4e10) in kinds          # north star, M = 1e6, K = 4


def test_workload_label_names_non_default_flags():
    """the bench line's workload names every reference CLI
    flag (src/main.py:27-50) it sets away from the CLI default, instead of
    claiming the defaults."""
    import argparse

    def args(**kw):
        d = dict(band=None, prior="matched", ridge=0.0, lmmse_damp=0)
        d.update(kw)
        return argparse.Namespace(**d)

    matched = dict(prior_vars=[0.0, 3.2e-6], prior_probs=[0.5, 0.5])
    lab = bench.flags_label(args(), matched)
    assert "--prior-vars 0,3.2e-06 --prior-probs 0.5,0.5" in lab and "except" in lab
    assert "default flags" not in lab
    lab = bench.flags_label(args(ridge=0.1, lmmse_damp=1), matched)
    assert "--s 0.1" in lab and "--lmmse-damp 1" in lab
    cli = dict(prior_vars=[0.0, 1.0], prior_probs=[0.99, 0.01])
    assert bench.flags_label(args(prior="cli"), cli) == \
        "reference CLI default flags (src/main.py:27-50)"
