"""The BASELINE.json configurations themselves on the GPU (C2-C5, full size).

* ``test_baseline_config_vs_oracle``: the HIP VAMP path (src/sgvamp.py:222-389
  replaced through the C ABI) on each configuration's full problem -- the bench's
  device-generated LD and r, the CLI's default flags with the simulated prior --
  for 2-3 outer iterations, against the CPU oracle run on the SAME inputs read
  back from the device: the LD blocks as packed upper-triangle panels
  (oracle.PanelLD: 20 GB at C2/C3, 63.5 GB at C4/C5) and the 2K CG solves of an
  iteration in lockstep (oracle.cg_track_batch: each column exactly scipy's cg,
  the products of the columns on the LD taken together; pinned to the
  reference's fixtures in tests/test_oracle_golden.py).  Bar: xhat <= 1e-8
  relative per iteration (the north star's is 1e-5), CG iteration counts and EM
  steps exact.
* ``test_sharded_bench_equals_one_rank``: ``bench.py --gpus 8 --share-device``
  (the N = 8 partition of C4 / C5: 8 of the 64 blocks per rank, 8 ranks
  self-launched on the one device, host exchange) writes output files bitwise
  identical to the one-rank run -- the ordered per-block reductions make the
  trajectory independent of the GPU count, which also carries the oracle
  parity above to the 8-GPU configurations.
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import hip_backend as hb
from engine import Engine
from oracle import vamp_oracle as vo
from sgvamp import VAMP, BlockLD
from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

# BASELINE.json configs[1..4]
CONFIGS = {
    "C2": dict(blocks=8, size=25000, K=1, s=0.0, damp=False, its=3),
    "C3": dict(blocks=8, size=25000, K=4, s=0.0, damp=False, its=3),
    "C4": dict(blocks=64, size=15625, K=1, s=0.0, damp=False, its=2),
    "C5": dict(blocks=64, size=15625, K=8, s=0.1, damp=True, its=2),
}
SEED, NSAMP = 2025, 10000
_LD = {}      # the host copy of the last configuration's LD (C2 -> C3, C4 -> C5 share it)


def _log(*a):
    print("[configs]", *a, file=sys.stderr, flush=True)
    path = os.environ.get("SGV_GATE_LOG")   # the gates' numbers for profiles/ (GPU suite runs)
    if path:
        with open(path, "a") as f:
            print("[configs]", *a, file=f)


def maxrel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


def _host_ld(eng, key, nblk):
    """The engine's LD as oracle.PanelLD (block by block: one dense block at a
    time on the host).  Reused by the next configuration with the same LD after
    checking its first block reads back identically."""
    if key in _LD:
        L = _LD[key]
        B = eng.get_ld_block(0, 0)
        np.testing.assert_array_equal(L.blocks[0][2][0], B[:256, :])   # first panel
        return L
    _LD.clear()
    L = vo.PanelLD()
    for b in range(nblk):
        L.add_block(eng.get_ld_block(0, b))
    _LD[key] = L
    return L


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_baseline_config_vs_oracle(name, tmp_path):
    cfg = CONFIGS[name]
    K, its = cfg["K"], cfg["its"]
    sizes = [cfg["size"]] * cfg["blocks"]
    eng = Engine(sizes, K=K, ld_of=[0] * K)
    args = argparse.Namespace(seed=SEED, nsamp=NSAMP)
    beta, _ = bench.make_problem(eng, eng.comm, args)        # the bench's own problem
    M, N = eng.M, NSAMP
    cm = int(M * 0.5)
    prior = dict(prior_vars=[0.0, 0.8 / cm * N / (N * K)], prior_probs=[0.5, 0.5])
    eng.set_ridge(cfg["s"])
    x0 = beta * np.sqrt(N)
    r_list = [eng.get_vector(hb.VEC_R, k) for k in range(K)]
    _log(name, "problem generated on the device")
    L = _host_ld(eng, (cfg["blocks"], cfg["size"]), cfg["blocks"])
    L.s = cfg["s"]
    _log(name, "LD read back (%d blocks)" % cfg["blocks"])

    v = VAMP(N=[N] * K, Nt=N * K, M=M, K=K, rho=0.5, gamw=5.0, gam1=1e-6, a=[1.0 / K] * K,
             out_dir=str(tmp_path), out_name=name, seed=SEED, write_files=False, **prior)
    v.attach_engine(eng, x0=x0)
    run = dict(cg_maxit=500, em_prior_maxit=100, learn_gamw=True, lmmse_damp=cfg["damp"],
               prior_update="em", update_prior_from=1)
    xh = v.infer(None, None, its, x0=x0, **run)
    hist = [(h["cg_iters"], h.get("em_steps")) for h in v.history]
    eng.close()
    _log(name, "GPU run done", hist)

    t = vo.infer([L], [0] * K, r_list, [N] * K, its, rho=0.5, gamw=5.0, gam1=1e-6, x0=x0,
                 seed=SEED, reducer=vo.Reducer("blocked", bounds=L.bounds), rs_recurrence=True,
                 batched=True, **prior, **run)
    _log(name, "oracle done", t["cg_iters"], t["em_steps"])
    for it in range(its):
        got = xh[it].ravel() / np.sqrt(N * K)
        ref = np.asarray(t["xhat"][it])
        assert np.isfinite(ref).all()
        assert maxrel(got, ref) < 1e-8, (name, it, maxrel(got, ref))
    assert [list(map(list, h[0])) for h in hist] == [list(map(list, x)) for x in t["cg_iters"]]
    assert [h[1] for h in hist][1:] == list(t["em_steps"])
    if name in ("C3", "C5"):        # K >= 2 shares one LD: the f64 MFMA pass was exercised
        assert max(max(c) for c in hist[0][0]) >= 1


@pytest.mark.timeout(900)
@pytest.mark.parametrize("K", [4, pytest.param(1, marks=pytest.mark.skipif(
    os.environ.get("SGV_FULL_GATE") != "1",
    reason="C4's 50-iteration gate (~3 min of host oracle): run with SGV_FULL_GATE=1 "
           "(profiles/r05/c4_k1_50it_gate_r05.log)"))])
def test_north_star_50_iterations_vs_oracle(K, tmp_path):
    """The north star's own gate at its own size, in the driver's suite (VERDICT
    round 5 item 3): M = 1e6 in 64 blocks of 15,625, K = 4 cohorts sharing one
    LD (the f64 MFMA pass; K = 1: C4, the VALU pass, opt-in), the bench's
    problem and flags, 50 outer iterations of the HIP path against the CPU
    oracle on the same inputs read back from the device (the host LD of the C4 /
    C5 cases above, reused: the oracle's panel products run in C on the job's
    CPU share, oracle/panel_ld.c).  Bar (BASELINE.json north_star): xhat within
    1e-5 relative of the oracle at every one of the 50 iterations (reference
    loop: src/sgvamp.py:196-389), with CG iteration counts and EM steps equal at
    every iteration."""
    errs, cg, em = _gate_50(64, 15625, K, tmp_path)
    assert max(errs) < 1e-5, max(errs)
    assert cg[0] == cg[1]
    assert em[0] == em[1]


def _bench(out_dir, *extra, gpus=None, timeout=600):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--cpu-baseline", "off", "--read-bw", "0", "--out-dir", str(out_dir)] + list(extra)
    if gpus:
        cmd += ["--gpus", str(gpus), "--share-device"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,flags", [
    ("C4", ["--K", "1"]),
    ("C5", ["--K", "8", "--ridge", "0.1", "--lmmse-damp", "1"]),
])
def test_sharded_bench_equals_one_rank(name, flags, tmp_path):
    one = _bench(tmp_path / "one", *flags)
    _log(name, "one rank", one["cg_iters_per_step"])
    eight = _bench(tmp_path / "eight", *flags, gpus=8)
    _log(name, "eight ranks", eight["cg_iters_per_step"])
    assert one["n_gpus"] == 1 and eight["n_gpus"] == 8
    assert eight["config"]["share_device"] and eight["config"]["K"] == one["config"]["K"]
    assert eight["cg_iters_per_step"] == one["cg_iters_per_step"]
    assert one["config"]["cg_column_sets"] == eight["config"]["cg_column_sets"]
    # the 8-rank line says where its exchange went: collectives per
    # step, their time, the EM loop's exchange mode; one rank has no communicator
    x1, x8 = one["exchange"], eight["exchange"]
    assert x1["transport"] is None and x1["allgathers_per_step"] == 0 and x1["em_mode"] is None
    assert x8["transport"] == "host" and x8["allgathers_per_step"] > 0 and x8["ms_per_step"] > 0
    # the EM exchange mode is the cost model's, from the latency the probe measured
    m = x8["em_model"]
    assert m["latency_source"].startswith("measured") and m["latency_us"] > 0
    assert x8["em_mode"] == ("replicated" if m["predicted_replicated_us"] < m["predicted_per_step_us"]
                             else "per-step")
    assert x8["em_loops"]["replicated"] + x8["em_loops"]["per_step"] >= 2
    assert x8["host_wait_ms_per_step"] >= 0
    # the line says who ran: the host transport labelled
    # as such, no RCCL rank count, every rank on the one device with its own wait
    assert x8["rccl_ranks"] is None and "not RCCL" in x8["transport_note"]
    assert [r["rank"] for r in x8["ranks"]] == list(range(8))
    assert all(r["transport"] == "host" and r["comm_ranks"] == 8 and r["comm_rank"] == r["rank"]
               and r["device"] == 0 and r["host_wait_ms_per_step"] >= 0 for r in x8["ranks"])
    assert x8["distinct_devices"] == 1 and x1["ranks"][0]["comm_ranks"] == 1
    _log(name, "eight-rank exchange", x8)
    files = sorted(f for f in os.listdir(tmp_path / "one") if f.endswith(".bin"))
    K = one["config"]["K"]
    assert len(files) == 3 * (K + 1)          # warmup + 2 steps: xhat and r1 per cohort
    for f in files:
        a = (tmp_path / "one" / f).read_bytes()
        b = (tmp_path / "eight" / f).read_bytes()
        assert len(a) == 8 * 1000000 and a == b, f
    for f in sorted(f for f in os.listdir(tmp_path / "one") if f.endswith(".csv")):
        assert (tmp_path / "one" / f).read_bytes() == (tmp_path / "eight" / f).read_bytes(), f


@pytest.mark.timeout(600)
def test_band_bench_over_ranks_equals_one_rank(tmp_path):
    """bench.py --band: one chromosome of windowed LD as a CSR through the class
    seam, cut into coupled pieces (65,536 + 84,464); 2 ranks on one device (a
    piece each, a halo all-gather per pass) write output files bitwise equal to
    one rank's, and the line names the band workload."""
    flags = ["--band", "150000,500", "--K", "2"]
    one = _bench(tmp_path / "one", *flags)
    two = _bench(tmp_path / "two", *flags, gpus=2)
    _log("band", "one rank", one["cg_iters_per_step"], one["roofline"]["frac"])
    assert one["config"]["band"] == "150000,500" and one["config"]["ld_blocks"] >= 2
    assert "windowed LD" in one["config"]["workload"] and one["cpu_baseline"] is None
    assert two["n_gpus"] == 2 and two["cg_iters_per_step"] == one["cg_iters_per_step"]
    assert two["exchange"]["allgathers_per_step"] > 0
    files = sorted(f for f in os.listdir(tmp_path / "one") if f.endswith((".bin", ".csv")))
    assert len([f for f in files if f.endswith(".bin")]) == 3 * (2 + 1)
    for f in files:
        assert (tmp_path / "one" / f).read_bytes() == (tmp_path / "two" / f).read_bytes(), f


def _gate_50(nblk, size, K, tmp_path, its=50, ref_algebra=False):
    """50 outer iterations of the HIP path against the CPU oracle on the same
    inputs read back from the device (the bench's problem, prior and flags);
    returns the per-iteration max relative xhat errors, the CG counts (GPU,
    oracle) and EM steps (GPU, oracle).  ref_algebra: the oracle runs the
    reference's own algebra -- dense LD blocks, np.dot reductions, R_s xhat2
    and R_s Sigma2u as direct products (src/sgvamp.py:352,359) and the two
    con_grad solves of each cohort one column at a time (:316,332) -- instead
    of the build's (carried R_s x, batched columns, blocked sums)."""
    sizes = [size] * nblk
    eng = Engine(sizes, K=K, ld_of=[0] * K)
    args = argparse.Namespace(seed=SEED, nsamp=NSAMP)
    beta, _ = bench.make_problem(eng, eng.comm, args)
    M, N = eng.M, NSAMP
    cm = int(M * 0.5)
    prior = dict(prior_vars=[0.0, 0.8 / cm * N / (N * K)], prior_probs=[0.5, 0.5])
    x0 = beta * np.sqrt(N)
    r_list = [eng.get_vector(hb.VEC_R, k) for k in range(K)]
    if ref_algebra is True:
        L = vo.BlockLD([eng.get_ld_block(0, b) for b in range(nblk)], s=0.0)
    else:
        L = _host_ld(eng, (nblk, size), nblk)
        L.s = 0.0
    v = VAMP(N=[N] * K, Nt=N * K, M=M, K=K, rho=0.5, gamw=5.0, gam1=1e-6, a=[1.0 / K] * K,
             out_dir=str(tmp_path), out_name="gate50", seed=SEED, write_files=False, **prior)
    v.attach_engine(eng, x0=x0)
    run = dict(cg_maxit=500, em_prior_maxit=100, learn_gamw=True, lmmse_damp=False,
               prior_update="em", update_prior_from=1)
    xh = v.infer(None, None, its, x0=x0, **run)
    hist = [(h["cg_iters"], h.get("em_steps")) for h in v.history]
    eng.close()
    _log("%dx%d K=%d: GPU %d iterations done" % (nblk, size, K, its))
    if ref_algebra:
        # True: dense blocks and np.dot products, con_grad one column at a time;
        # "batched": the same algebra on the packed host LD, the columns' CG in
        # lockstep with each column's products the bits it gets alone
        # (oracle.cg_scipy_batch) -- fast enough for C3's full size
        t = vo.infer([L], [0] * K, r_list, [N] * K, its, rho=0.5, gamw=5.0, gam1=1e-6, x0=x0,
                     seed=SEED, reducer=vo.Reducer("numpy"), rs_recurrence=False,
                     batched=ref_algebra == "batched",
                     progress=lambda it: _log("oracle (reference algebra) iteration %d" % it),
                     **prior, **run)
    else:
        t = vo.infer([L], [0] * K, r_list, [N] * K, its, rho=0.5, gamw=5.0, gam1=1e-6, x0=x0,
                     seed=SEED, reducer=vo.Reducer("blocked", bounds=L.bounds), rs_recurrence=True,
                     batched=True, progress=lambda it: _log("oracle iteration %d" % it),
                     **prior, **run)
    errs = []
    for it in range(its):
        got = xh[it].ravel() / np.sqrt(N * K)
        ref = np.asarray(t["xhat"][it])
        assert np.isfinite(ref).all()
        errs.append(maxrel(got, ref))
    cg = ([list(map(list, h[0])) for h in hist], [list(map(list, x)) for x in t["cg_iters"]])
    em = ([h[1] for h in hist][1:], list(t["em_steps"]))
    same_cg = sum(a == b for a, b in zip(*cg))
    same_em = sum(a == b for a, b in zip(*em))
    _log("%dx%d K=%d %d it: max rel xhat err per iteration" % (nblk, size, K, its),
         ["%.2e" % e for e in errs])
    _log("%dx%d K=%d %d it: CG counts equal in %d/%d iterations, EM steps in %d/%d"
         % (nblk, size, K, its, same_cg, its, same_em, its - 1))
    _log("CG counts", cg[0])
    return errs, cg, em


@pytest.mark.timeout(900)
@pytest.mark.parametrize("nblk,size", [(4, 12500)])
def test_50_iterations_mid_size_vs_oracle(nblk, size, tmp_path):
    """The north star's 50-iteration gate in the driver's suite, above toy size
    (VERDICT round 3): 4 LD blocks of 12,500 markers (M = 50,000, each block
    wider than the MFMA pass's strips of 8 panels), K = 4 cohorts sharing the
    LD (8 CG columns: the f64 MFMA pass), rho 0.5, the bench's generator and
    prior (C3's full problem: in the reference's algebra, below).
    Bar (BASELINE.json north_star): xhat within 1e-5 relative of the oracle,
    asserted at every one of the 50 iterations; CG iteration counts and EM steps
    equal at every iteration."""
    errs, cg, em = _gate_50(nblk, size, 4, tmp_path)
    assert max(errs) < 1e-5, max(errs)
    assert cg[0] == cg[1]
    assert em[0] == em[1]


@pytest.mark.timeout(900)
def test_50_iterations_vs_reference_algebra(tmp_path):
    """The build's algebra against the reference's above toy size (VERDICT round
    4): the GPU default path -- R_s x carried through the CG (DESIGN.md section 2,
    item 4), both solves of every cohort batched into one pass per CG
    iteration, per-block ordered sums -- for 50 iterations at 4 x 12,500 (M =
    50,000), K = 4 sharing the LD (the f64 MFMA pass), against the oracle in the
    reference's own algebra: dense blocks, np.dot, R_s xhat2 and R_s Sigma2u by
    direct products (src/sgvamp.py:352,359), con_grad one column at a time
    (:316,332).  Bar: xhat within 1e-5 relative at every iteration, CG iteration
    counts and EM steps equal at every iteration."""
    errs, cg, em = _gate_50(4, 12500, 4, tmp_path, ref_algebra=True)
    assert max(errs) < 1e-5, max(errs)
    assert cg[0] == cg[1]
    assert em[0] == em[1]


@pytest.mark.timeout(900)
def test_c3_50_iterations_vs_reference_algebra(tmp_path):
    """the reference's own algebra at C3's full size (8 x
    25,000, K = 4 sharing the LD: the f64 MFMA pass), 50 iterations -- the oracle
    with direct R_s xhat2 / R_s Sigma2u products (src/sgvamp.py:352,359),
    scipy's cg per column with its warm-start residual from a direct product
    (:316,332) and np.dot reductions, against the GPU default path (carried
    R_s x, batched passes, blocked sums).  Bar: xhat within 1e-5 relative at
    every iteration, CG iteration counts and EM steps equal at every iteration
    (~105 s on the box: profiles/r06/c3_ref_algebra_gate.log, <= 3.1e-15).  It
    replaces round 5's gate at this size in the build's own algebra."""
    errs, cg, em = _gate_50(8, 25000, 4, tmp_path, ref_algebra="batched")
    assert max(errs) < 1e-5, max(errs)
    assert cg[0] == cg[1]
    assert em[0] == em[1]


@pytest.mark.timeout(900)
def test_band_full_size_vs_oracle(tmp_path):
    """The band path at full size: bench.py --band's problem (one chromosome of
    windowed LD, M = 1e6, bw = 1,000, K = 4, cut into 15 coupled pieces) through
    the class seam, 10 outer iterations against the oracle running scipy's CSR
    mat-vec on the same matrix (the reference's operator for .npz LD,
    src/main.py:199-200, src/sgvamp.py:316,332), same probes and flags: xhat within
    1e-8 relative per iteration, CG and EM counts equal (~45 s on the box:
    profiles/r04/band_gate_full_size.log)."""
    its, K, N = 10, 4, NSAMP
    A, r, x0, cm = bench.band_problem(argparse.Namespace(band="1000000,1000", seed=SEED,
                                                         nsamp=N), K)
    M = A.shape[0]
    prior = dict(prior_vars=[0.0, 0.5 / cm * N / (N * K)], prior_probs=[0.95, 0.05])
    run = dict(cg_maxit=500, em_prior_maxit=100, learn_gamw=True, lmmse_damp=False,
               prior_update="em", update_prior_from=1)
    v = VAMP(N=[N] * K, Nt=N * K, M=M, K=K, rho=0.5, gamw=5.0, gam1=1e-6, a=[1.0 / K] * K,
             out_dir=str(tmp_path), out_name="band", seed=SEED, write_files=False, **prior)
    xh = v.infer(BlockLD.from_csr(A), r, its, x0=x0, **run)
    hist = [(h["cg_iters"], h.get("em_steps")) for h in v.history]
    pieces = list(v.engine.block_sizes)
    v.engine.close()
    assert len(pieces) == 15
    _log("band 1e6 K=4: GPU %d iterations done" % its)
    t = vo.infer([vo.CsrLD(A)], [0] * K, [r[k] for k in range(K)], [N] * K, its, rho=0.5, gamw=5.0,
                 gam1=1e-6, x0=x0, seed=SEED,
                 reducer=vo.Reducer("blocked", bounds=np.concatenate([[0], np.cumsum(pieces)])),
                 rs_recurrence=True, **prior, **run)
    errs = [maxrel(xh[it].ravel() / np.sqrt(N * K), np.asarray(t["xhat"][it]).ravel())
            for it in range(its)]
    _log("band 1e6 K=4: max rel xhat err per iteration", ["%.2e" % e for e in errs])
    cg = ([list(map(list, h[0])) for h in hist], [list(map(list, x)) for x in t["cg_iters"]])
    _log("band 1e6 K=4: CG counts equal in %d/%d iterations" % (
        sum(a == b for a, b in zip(*cg)), its))
    assert max(errs) < 1e-8, errs
    assert cg[0] == cg[1]
    assert [h[1] for h in hist][1:] == list(t["em_steps"])
