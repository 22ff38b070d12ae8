#!/usr/bin/env python3
"""Benchmark: VAMP iterations/s on the north-star configuration.

Default workload = the configuration BASELINE.json's north_star states its
target on ("70 % of the HBM roofline on the LD mat-vec at M=1e6, K=4"):
M = 1,000,000 markers in 64 LD blocks of 15,625 (C4's block structure), K = 4
cohorts sharing one LD (8 CG right-hand sides per LD pass: the f64-MFMA pass),
N = 10,000 samples per cohort, one GPU (63.5 GB of packed LD fits one MI355X).
Other configurations are flags: C2 (configs[1]) ``--blocks 8 --block-size 25000
--K 1``; C3 adds ``--K 4``; C4 ``--K 1``; C5 ``--K 8 --ridge 0.1 --lmmse-damp 1``.
The reference CLI's default flags (gamw 5, gam1 1e-6,
rho 0.5, cg-maxit 500, EM prior from it 1 with <= 100 steps, learn-gamw 1,
lmmse-damp 0, s 0) except the prior: --prior matched (default) sets
--prior-vars 0,0.8/cm --prior-probs 0.5,0.5, the simulated mixture.  With the
CLI default prior (0,1 / 0.99,0.01: slab variance 1*Nt = 1e4 against a
simulated effect variance of 0.08) the reference algorithm's EM drives lam to 0
and the run turns NaN within a few iterations (tests/test_gpu_parity.py::
test_vamp_medium_scale_vs_oracle[cli_default] shows the oracle does the same),
after which every CG runs to cg-maxit: not a meaningful benchmark.  Synthetic data generated on the
device following simulation/sim_gen_phen_mult.py (X ~ Bin(2, 0.4), 50 %
causal markers, h2 = 0.8).  A "step" is one VAMP outer iteration
(src/sgvamp.py:222-387): EM prior update, denoiser, both CG solves, gamw
learning, output files.  Inputs are resident in HBM before timing starts.

Multi-GPU: ``python bench.py --gpus N`` starts N ranks itself, one process per
GPU (sgvamp-py_amd/launch.py: child processes, started before anything touches
the GPU); an external one-process-per-GPU launcher (RANK/WORLD_SIZE/LOCAL_RANK,
mpirun, srun) is accepted too, and then --gpus must equal its world size.  The
LD blocks are sharded over the N ranks (strong scaling, one problem); CG dot
products are ordered per-block sums exchanged with RCCL all-gathers.  The host
communicator is the build's own TCP rendezvous (sgvamp-py_amd/comm.py), torch
is never imported.

Prints ONE JSON line on rank 0 (other output goes to stderr).
"""
import argparse
import glob
import json
import os
import re
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, MI355X_MICROARCH.md chip table
F64_MFMA_PEAK_TFS = 78.6   # MI355X dense f64 matrix peak (AMD spec; not in the guide)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPU ranks (default: the launcher's world size, else 1); N > 1 without "
                        "a launcher starts N local ranks")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=64)
    p.add_argument("--block-size", type=int, default=15625)
    p.add_argument("--nsamp", type=int, default=10000)
    p.add_argument("--K", type=int, default=4)
    p.add_argument("--distinct-ld", action="store_true",
                   help="one LD matrix per cohort (the reference's per-rank ld_fpaths_list[rank], "
                        "src/main.py:173,199-202) instead of K cohorts sharing one")
    p.add_argument("--seed", type=int, default=2025)
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-blocks", type=int, default=4,
                   help="LD blocks of the CPU-baseline sample (see cpu_baseline)")
    p.add_argument("--cpu-iters", type=int, default=3)
    p.add_argument("--no-files", action="store_true", help="skip the per-iteration output files")
    p.add_argument("--out-dir", default=None, help="keep the output files here (default: a temp dir)")
    p.add_argument("--share-device", action="store_true",
                   help="rehearsal: every rank on device 0 with the host exchange (RCCL refuses "
                        "two ranks on one device); timings are then not a multi-GPU result")
    p.add_argument("--exchange", choices=["auto", "rccl", "host"], default="auto",
                   help="cross-rank exchange; auto = RCCL when N > 1, none at N = 1.  An explicit "
                        "choice at N = 1 runs a one-rank communicator (measures the exchange cost)")
    p.add_argument("--prior", choices=["matched", "cli"], default="matched")
    p.add_argument("--ridge", type=float, default=0.0, help="--s of the CLI (C5: 0.1)")
    p.add_argument("--lmmse-damp", type=int, default=0, help="--lmmse-damp of the CLI (C5: 1)")
    p.add_argument("--pause", type=float, default=0.0,
                   help="seconds the device idles after set-up, before the warm-up steps "
                        "(clock/thermal studies: the set-up's generator kernels heat the chip)")
    p.add_argument("--read-bw", type=int, default=1,
                   help="1: after the timed steps, measure the GPU's streaming-read rate "
                        "(roofline.box_stream_GBs)")
    p.add_argument("--dry-run", action="store_true",
                   help="start the ranks and report each one's rank/device as one JSON line, "
                        "without touching the GPU (checks the launch)")
    p.add_argument("--ld-format", choices=["packed", "dense"], default="packed",
                   help="LD block storage: packed symmetric panels (default) or full squares")
    p.add_argument("--band", default=None, metavar="M,BW",
                   help="one chromosome of windowed LD instead of the device-generated blocks: "
                        "M markers, bandwidth BW (simulate.windowed_ld, CSR on the host: the "
                        "reference's .npz / PLINK .ld path, src/main.py:199-200,251-257); long "
                        "bands are cut into coupled pieces the ranks share")
    return p.parse_args()


def band_problem(args, K):
    """--band: the windowed LD (every rank builds the same CSR), r_k = R x0 +
    N(0, 1) noise per cohort, x0 = beta * sqrt(N) with 5 % causal markers."""
    from simulate import windowed_ld

    M, bw = (int(x) for x in args.band.split(","))
    A = windowed_ld(M, bw, seed=args.seed)
    rs = np.random.RandomState(args.seed)
    cm = max(1, M // 20)
    beta = np.zeros(M)
    beta[rs.choice(M, cm, replace=False)] = rs.normal(0, np.sqrt(0.5 / cm), cm)
    x0 = beta * np.sqrt(args.nsamp)
    Ax0 = A @ x0
    r = np.stack([Ax0 + np.random.RandomState(args.seed + 1000 + k).normal(0.0, 1.0, M)
                  for k in range(K)])
    return A, r, x0, cm


def make_problem(eng, comm, args):
    """beta and noise on the host (RandomState, as the reference recipe);
    genotypes, LD blocks, g and r on the device.  Cohorts sharing an LD matrix
    share its genotypes (their own noise); with one LD matrix per cohort
    (--distinct-ld, the reference's native layout: ld_fpaths_list[rank],
    src/main.py:173,199-202) cohort k has its own genotypes, the same beta."""
    M, N = eng.M, args.nsamp
    rs = np.random.RandomState(args.seed)
    cm = int(M * 0.5)                                   # sim_gen_phen_mult.py:28-32
    beta = np.zeros(M)
    beta[rs.choice(M, cm, replace=False)] = rs.normal(0, np.sqrt(0.8 / cm), cm)
    gs = {}
    for ld in range(eng.nld):
        geno_seed = args.seed + 1 + 7919 * ld
        g_loc = eng.synth_ld_g(ld, geno_seed, N, beta)      # (nblk_local, N)
        g_all = np.concatenate(comm.allgather(g_loc)) if comm.Get_size() > 1 else g_loc
        g = g_all[0].copy()
        for b in range(1, g_all.shape[0]):                  # global block order
            g = g + g_all[b]
        gs[ld] = (geno_seed, g)
    ys = []
    for k in range(eng.K):
        geno_seed, g = gs[eng.ld_of[k]]
        w = np.random.RandomState(args.seed + 1000 + k).normal(0.0, np.sqrt(0.2), N)
        y = g + w
        eng.synth_r(k, geno_seed, N, y)
        ys.append(y)
    return beta, ys


def read_traffic(kernel_prefix, bytes_launch, K, M):
    """HBM bytes per LD-pass launch from the committed PMC summary of the same
    workload (profiles/*pmc*.json written by tools/pmc_summary.py): the newest
    summary for this kernel, K and M whose algorithmic bytes per launch agree
    with this run's within 1 %.  None when no summary was collected on this
    workload."""
    # by round label, numbers compared as numbers (r02s10 after r02s7)
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")),
                   key=lambda p: [int(x) if x.isdigit() else x
                                  for x in re.split(r"(\d+)", os.path.basename(p))])
    for path in reversed(cands):
        try:
            d = json.load(open(path))
            alg = float(d.get("algorithmic_bytes_per_launch") or 0)
            if (kernel_prefix in d.get("kernel", "") and d.get("K") == K and d.get("M") == M
                    and abs(alg - bytes_launch) <= 0.01 * bytes_launch):
                return float(d["hbm_bytes_per_launch"]), os.path.basename(path)
        except Exception:
            continue
    return None, None


def matvecs_per_step(recs, learn_gamw=True):
    """Single-column LD mat-vecs the reference performs for one outer iteration
    with the CG counts the GPU run recorded: per cohort CG #1 + CG #2 iterations
    (src/sgvamp.py:316,332), the two warm-start residuals (iterative.py:392:
    x0.any() holds from iteration 1 on) and the two gamw products (:352,359)."""
    tot = 0
    for rec in recs:
        for n1, n2 in rec["cg_iters"]:
            tot += n1 + n2 + 2 + (2 if learn_gamw else 0)
    return tot / max(len(recs), 1)


# The reference's per-marker Python loops (measured by
# importing src/sgvamp.py): denoiser_meta + der_denoiser_meta per marker and
# iteration (src/sgvamp.py:273,285), and one EM step (:116-136) per 200k
# markers per cohort count (1 core each).
REF_DENOISE_S_PER_MARKER = 17.7e-6 + 27.7e-6
REF_EM_S_PER_200K = {1: 0.013, 4: 0.034, 8: 0.064}


def _ref_em_step_s(M, K):
    ks = sorted(REF_EM_S_PER_200K)
    k0 = max([k for k in ks if k <= K] or [ks[0]])
    k1 = min([k for k in ks if k >= K] or [ks[-1]])
    t0, t1 = REF_EM_S_PER_200K[k0], REF_EM_S_PER_200K[k1]
    t = t0 if k1 == k0 else t0 + (t1 - t0) * (K - k0) / (k1 - k0)
    return t * M / 200000.0


def usable_cores():
    """The host threads this process is given: OMP_NUM_THREADS when the box
    sets it (its CPU share: 16 per GPU on the MI355X pool, whose os.cpu_count()
    reports the whole machine), else the CPUs it may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _oracle_sample(eng, args, ref_flags, x0, S):
    """The oracle on LD blocks 0 .. S-1 of every LD matrix (dense f64, as the
    reference stores them) with all cohorts' r and x0 on those markers, for
    cpu_iters outer iterations; LD mat-vecs timed separately.  Returns the
    wall time, the mat-vec time per single-column product per block, the
    non-LD time per step scaled to M, and the oracle's own mat-vecs per step."""
    from oracle import vamp_oracle as vo
    import hip_backend as hb

    n = int(sum(eng.block_sizes[:S]))
    r_list = [eng.get_vector(hb.VEC_R, k)[:n].copy() for k in range(eng.K)]
    t_mv = [0.0, 0]
    lds = []
    for ld in range(eng.nld):
        L = vo.BlockLD([eng.get_ld_block(ld, b) for b in range(S)], s=args.ridge)
        raw = L.matvec_R

        def timed(v, raw=raw):
            t = time.perf_counter()
            out = raw(v)
            t_mv[0] += time.perf_counter() - t
            t_mv[1] += 1
            return out

        L.matvec_R = timed
        lds.append(L)
    its = args.cpu_iters
    t0 = time.perf_counter()
    traj = vo.infer(lds, eng.ld_of, r_list, [args.nsamp] * eng.K, its, x0=x0[:n],
                    reducer=vo.Reducer(), seed=args.seed, **ref_flags)
    dt = time.perf_counter() - t0
    return dict(n=n, dt=dt, traj=traj, mv_block=t_mv[0] / max(t_mv[1], 1) / S,
                other=(dt - t_mv[0]) / its * (eng.M / float(n)), nmv=t_mv[1] / its)


def cpu_baseline(eng, args, ref_flags, recs, x0):
    """Two CPU figures for the same workload, neither run on the GPU box by
    the reference itself (it never travels there):

    * ``value`` -- the oracle (the build's NumPy restatement of the reference,
      OpenBLAS on every usable core) TIMED on a bounded sample of the workload
      and extrapolated.  Sample: LD blocks 0 .. cpu_blocks-1 (dense f64, as the
      reference stores them) with all K cohorts' r and x0 on those markers, run
      for cpu_iters outer iterations; its LD mat-vecs timed separately.  Full
      step = (non-LD time per step) x (M / sample markers) + (mat-vec time per
      block) x (LD blocks) x (single-column mat-vecs per step of the reference
      with the CG counts recorded in the timed GPU steps).  When the sample is
      the whole problem the measured step is reported beside the model
      (``measured_step_s``, ``model_error``).
    * ``reference_formula`` -- the reference's own cost structure (SURVEY.md
      section 8d(i)): its mat-vecs streamed at the dgemv rate this box just
      measured (dense blocks; its .npz CSR path runs single-threaded at ~4 GB/s,
      ~10x slower), plus its per-marker denoiser loops (45.4 us per marker and
      iteration on each MPI rank, the K ranks in parallel), plus its EM steps
      (the GPU run's step counts, one core per rank)."""
    import threadpoolctl

    cores = usable_cores()
    its = args.cpu_iters
    # host memory: at most cpu_blocks dense blocks over all LD matrices
    S = max(1, min(args.cpu_blocks // eng.nld, len(eng.block_sizes)))
    with threadpoolctl.threadpool_limits(limits=cores):
        info = threadpoolctl.threadpool_info()
        threads = max([i.get("num_threads", 1) for i in info if i.get("internal_api") in
                       ("openblas", "mkl", "blis")] or [1])
        smp = _oracle_sample(eng, args, ref_flags, x0, S)
        # the sample is the whole problem: validate the extrapolation from a
        # two-block sub-sample against it (same basis: the full oracle run's
        # mat-vecs per step)
        sub = _oracle_sample(eng, args, ref_flags, x0, 2) \
            if S == len(eng.block_sizes) and S > 2 else None
    n, dt, mv_block, other = smp["n"], smp["dt"], smp["mv_block"], smp["other"]
    dense_block_bytes = sum(b * b for b in eng.block_sizes[:S]) * 8.0 / S
    dgemv_GBs = dense_block_bytes / mv_block / 1e9
    nmv = matvecs_per_step(recs, ref_flags.get("learn_gamw", True))
    step = other + mv_block * len(eng.block_sizes) * nmv
    out = dict(value=1.0 / step, unit="VAMP it/s", cores=int(threads), kind="port",
               host_cpus=os.cpu_count(), cores_given=cores,
               cores_note="threads = the box's CPU share (OMP_NUM_THREADS), not the machine's "
                          "%d CPUs" % (os.cpu_count() or 0),
               extrapolated=S < len(eng.block_sizes),
               sample="oracle/vamp_oracle.py (NumPy + OpenBLAS, %d threads) on LD blocks 0-%d (%d "
                      "markers, %.1f GB dense), all %d cohorts, %d iterations in %.2f s: %.1f ms per "
                      "single-column mat-vec per LD block (%.0f GB/s), %.1f ms of non-LD work per "
                      "step scaled to M=%d; full step = %.1f ms non-LD + %d blocks x %.1f mat-vecs "
                      "per step (the reference's count with the GPU run's CG iterations) = %.2f s" % (
                          threads, S - 1, n, dense_block_bytes * S / 1e9, eng.K, its, dt,
                          mv_block * 1e3, dgemv_GBs, other * 1e3, eng.M, other * 1e3,
                          len(eng.block_sizes), nmv, step))
    if sub is not None:
        meas = dt / its
        model = sub["other"] + sub["mv_block"] * len(eng.block_sizes) * smp["nmv"]
        out.update(measured_step_s=meas, model_from_2_blocks_step_s=model,
                   model_error=model / meas - 1.0, oracle_cg_iters=smp["traj"]["cg_iters"],
                   model_note="the extrapolation the sample line uses, from LD blocks 0-1 "
                              "(%d markers), against the oracle measured on the whole problem; "
                              "both with the whole run's %.1f mat-vecs per step"
                              % (sub["n"], smp["nmv"]))
    # the reference's cost structure, with this box's dgemv rate
    M, K = eng.M, eng.K
    dense_pass = sum(float(b) * b for b in eng.block_sizes) * 8.0   # one LD matrix
    em_steps = np.mean([r.get("em_steps") or 0 for r in recs])
    t_mv_ref = nmv * dense_pass / (dgemv_GBs * 1e9)
    t_den = M * REF_DENOISE_S_PER_MARKER
    t_em = em_steps * _ref_em_step_s(M, K)
    t_ref = t_mv_ref + t_den + t_em
    out["reference_formula"] = dict(
        value=1.0 / t_ref, unit="VAMP it/s", kind="reference cost model (extrapolated)",
        step_s=t_ref, matvec_s=t_mv_ref, denoiser_loops_s=t_den, em_s=t_em,
        formula="%.1f single-column mat-vecs x %.1f GB dense / %.0f GB/s (this box's dgemv) "
                "+ %d markers x 45.4 us (src/sgvamp.py:273,285 per-marker loops, K ranks in "
                "parallel) + %.1f EM steps x %.0f ms (src/sgvamp.py:116-136 at M=%d, K=%d)" % (
                    nmv, dense_pass / 1e9, dgemv_GBs, M, em_steps, _ref_em_step_s(M, K) * 1e3,
                    M, K))
    return out


def flags_label(args, prior):
    """The reference CLI flags (src/main.py:27-50) this run uses, naming every
    one that differs from the CLI's default."""
    diff = []
    if args.band or args.prior != "cli":
        diff.append("--prior-vars %s --prior-probs %s (%s; the CLI default 0,1 / 0.99,0.01 "
                    "collapses the reference algorithm on this data, DESIGN.md section 6)" % (
                        ",".join("%.6g" % x for x in prior["prior_vars"]),
                        ",".join("%.6g" % x for x in prior["prior_probs"]),
                        "the simulated mixture" if not args.band else "the band problem's mixture"))
    if args.ridge:
        diff.append("--s %g" % args.ridge)
    if args.lmmse_damp:
        diff.append("--lmmse-damp 1")
    if not diff:
        return "reference CLI default flags (src/main.py:27-50)"
    return ("reference CLI flags (src/main.py:27-50) at their defaults except " + ", ".join(diff))


def main():
    args = parse()
    from launch import relaunch

    rc = relaunch(args.gpus)               # before anything touches the GPU
    if rc is not None:
        sys.exit(rc)
    import hip_backend as hb  # noqa: F401  (fails loudly if the library is missing)
    from comm import world_from_env
    from engine import Engine
    from sgvamp import VAMP

    comm = world_from_env()
    rank, world = comm.Get_rank(), comm.Get_size()
    device = 0 if args.share_device else comm.local_rank
    if args.dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                "SGV_LAUNCHED_BY", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID")
        ranks = comm.allgather(dict(rank=rank, world=world, local_rank=comm.local_rank,
                                    device=device, pid=os.getpid(),
                                    env={k: os.environ[k] for k in keys if k in os.environ}))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": ranks}), flush=True)
        comm.close()
        return
    sizes = [args.block_size] * args.blocks
    K = args.K
    t_setup = time.perf_counter()
    ld_of = list(range(K)) if args.distinct_ld else [0] * K
    exchange = "host" if args.share_device else (None if args.exchange == "auto" else args.exchange)
    N_list = [args.nsamp] * K
    Nt = sum(N_list)
    a = np.array(N_list) / Nt
    if args.band:
        band_A, band_r, x0, cm = band_problem(args, K)
        M_run = band_A.shape[0]
        eng = None
    else:
        eng = Engine(sizes, K, ld_of=ld_of, comm=comm, device=device, exchange=exchange)
        eng.set_ld_packing(args.ld_format == "packed")
        beta, _ = make_problem(eng, comm, args)
        M_run = eng.M
        cm = int(eng.M * 0.5)
    if args.band:
        prior = dict(prior_vars=[0.0, 0.5 / cm * N_list[0] / Nt], prior_probs=[0.95, 0.05])
    elif args.prior == "matched":
        # simulated effect variance 0.8/cm in x = beta*sqrt(N_k) scale is 0.8/cm * N_k; the
        # reference scales slab variances by Nt (src/sgvamp.py:27): 0.8/cm * N_k / Nt
        prior = dict(prior_vars=[0.0, 0.8 / cm * N_list[0] / Nt], prior_probs=[0.5, 0.5])
    else:
        prior = dict(prior_vars=[0.0, 1.0], prior_probs=[0.99, 0.01])
    flags = dict(rho=0.5, gamw=5.0, gam1=1e-6, **prior)
    run = dict(cg_maxit=500, em_prior_maxit=100, learn_gamw=True, lmmse_damp=bool(args.lmmse_damp),
               prior_update="em", update_prior_from=1)
    tmp = args.out_dir or tempfile.mkdtemp(prefix="sgvamp_bench_")
    os.makedirs(tmp, exist_ok=True)
    v = VAMP(N=N_list if K > 1 else N_list[0], Nt=Nt, M=M_run, K=K, a=a, out_dir=tmp,
             out_name="bench", comm=comm, seed=args.seed, write_files=not args.no_files,
             device=device, exchange=exchange, ld_packing=args.ld_format == "packed", **flags)
    # the warm-up steps queue no step past their last: the timers are reset
    # between the two loops while no step runs
    if args.band:   # the class seam's own set-up: the CSR, cut into coupled pieces when long
        from sgvamp import BlockLD

        v.begin(BlockLD.from_csr(band_A, s=args.ridge), band_r, x0=x0, return_xhat=False,
                iterations=args.warmup, **run)
        eng = v.engine
        del band_A
    else:
        eng.set_ridge(args.ridge)
        x0 = beta * np.sqrt(N_list[0])                      # main.py:276-279
        v.attach_engine(eng, x0=x0)
        v.begin(x0=x0, return_xhat=False, iterations=args.warmup, **run)
    eng.sync()
    comm.barrier()
    log("[bench] setup (device data generation) %.1f s, M=%d, blocks=%d x %d, N=%d, K=%d, ranks=%d"
        % (time.perf_counter() - t_setup, eng.M, len(eng.block_sizes), max(eng.block_sizes),
           args.nsamp, K, world))

    if args.pause > 0:
        time.sleep(args.pause)
        comm.barrier()
    for it in range(args.warmup):
        rec = v.step(it)
        log("[bench] warmup it=%d cg=%s passes=%d %.1f ms" % (it, rec["cg_iters"], rec["ld_passes"],
                                                              rec["wall_s"] * 1e3))
    eng.timers(reset=True)
    eng.exchange_stats(reset=True)
    eng.sync()
    v.set_iterations(args.warmup + args.steps)
    comm.barrier()
    t0 = time.perf_counter()
    recs = []
    for it in range(args.warmup, args.warmup + args.steps):
        recs.append(v.step(it))
    v.drain()                                           # output files and CSV rows of the timed steps
    eng.sync()
    t1 = time.perf_counter()
    comm.barrier()
    dt = max(comm.allgather(t1 - t0))
    tm = eng.timers()
    xs = eng.exchange_stats()
    xs_all = comm.allgather(xs) if world > 1 else [xs]
    # each rank's view of the exchange (sgv_comm_info: RCCL's own rank count and
    # this rank in it, the HIP device and its PCI bus id) and its exact-CG host
    # wait, so an N-GPU line proves which devices and which communicator ran
    ci = eng.comm_info()
    ci.update(rank=rank, host_wait_ms_per_step=xs["host_wait_ms"] / args.steps)
    ci_all = comm.allgather(ci) if world > 1 else [ci]
    # this box's own streaming-read rate (after the timed region; context only:
    # the roofline peak stays the guide's 8 TB/s); the slowest rank's
    box_bw = None
    if args.read_bw:
        try:
            bw = eng.read_bw(8 << 30, 5)
        except Exception as e:  # noqa: BLE001 -- context only: the bench line stays valid
            log("[bench] streaming-read probe failed: %s" % e)
            bw = 0.0
        bws = comm.allgather(bw)
        box_bw = min(bws) if min(bws) > 0 else None
    for rec in recs:
        log("[bench] it=%d cg=%s em=%s passes=%d %.1f ms l2=%s waits(ms): probes %.2f outputs %.2f "
            "writes %.2f" % (
                rec["it"], rec["cg_iters"], rec.get("em_steps"), rec["ld_passes"],
                rec["wall_s"] * 1e3, "%.4f" % rec["metrics"][1] if "metrics" in rec else "-",
                rec.get("wait_probes_ms", 0.0), rec.get("outputs_ms", 0.0),
                rec.get("wait_write_ms", 0.0)))

    steps = args.steps
    value = steps / dt
    launches = max(tm["ld_launches"], 1)
    avg_s = tm["ld_ms"] / 1e3 / launches
    ld_bytes_launch = tm["ld_bytes"] / launches            # stored LD bytes actually read
    bytes_launch = ld_bytes_launch + tm["rhs_bytes"] / launches
    achieved = bytes_launch / avg_s / 1e9 if avg_s > 0 else None
    dense_equiv = (tm["dense_bytes"] / launches + tm["rhs_bytes"] / launches) / avg_s / 1e9
    nc_pass = 2 * K // eng.nld                         # columns per LD pass
    mfma = args.ld_format == "packed" and nc_pass >= 3  # NC >= 3: the f64 MFMA pass
    traffic, traffic_src = read_traffic(("k_sym_mfma" if mfma else "k_sym_pass")
                                        if args.ld_format == "packed" else "k_ld_pass",
                                        bytes_launch, K, eng.M)
    if args.band:
        cname = ("one chromosome of windowed LD (bandwidth %s, CSR -> packed band, %d coupled "
                 "piece(s))" % (args.band.split(",")[1], len(eng.block_sizes)))
    elif args.distinct_ld and K > 1:
        cname = "distinct per-cohort LD (the reference's ld_fpaths_list[rank] layout)"
    elif eng.M == 200000 and args.ridge == 0 and not args.lmmse_damp:
        cname = {1: "C2 (BASELINE.json configs[1])", 4: "C3 (BASELINE.json configs[2])"}.get(K, "custom")
    elif eng.M == 1000000 and K == 4 and args.ridge == 0 and not args.lmmse_damp:
        cname = ("north-star configuration (BASELINE.json north_star: LD mat-vec at M=1e6, K=4) "
                 "on %d GPU(s)" % world)
    elif eng.M == 1000000 and K == 1 and args.ridge == 0 and not args.lmmse_damp:
        cname = "C4 (BASELINE.json configs[3]) on %d GPU(s)" % world
    elif eng.M == 1000000 and K == 8 and args.ridge == 0.1 and args.lmmse_damp:
        cname = "C5 (BASELINE.json configs[4]) on %d GPU(s)" % world
        if args.nsamp >= max(eng.block_sizes):   # full-rank LD blocks: the run converges
            cname += (", N >= LD block size (full-rank blocks: a converging run, unlike the "
                      "N = 10,000 C5 line)")
    else:
        cname = "custom"
    passes = sum(r["ld_passes"] for r in recs)
    ld_bytes_total = ld_bytes_launch * comm.Get_size()
    result = {
        "metric": "VAMP iterations/sec (and effective LD-matvec GB/s) at M markers, K cohorts",
        "value": value,
        "unit": "VAMP it/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": dt / steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: windowed LD (simulate.windowed_ld), r = R x0 + N(0,1), 5%% causal, "
                 "seed %d" % args.seed) if args.band else
                ("synthetic: device generator following simulation/sim_gen_phen_mult.py "
                 "(Bin(2,0.4) genotypes, 50%% causal, h2=0.8), seed %d" % args.seed),
        "config": {
            "workload": "%s: K=%d cohort(s) %s, M=%d markers in %d LD blocks "
                        "of %d, N=%d per cohort, output files written each iteration, %s"
                        % (cname, K, "with one LD matrix each" if args.distinct_ld
                           else "sharing one LD", eng.M, len(eng.block_sizes),
                           max(eng.block_sizes), args.nsamp, flags_label(args, prior)),
            "K": K, "M": eng.M, "ld_blocks": len(eng.block_sizes),
            "block_size": args.block_size if not args.band else max(eng.block_sizes),
            "band": args.band,
            "ld_matrices": eng.nld,
            "s": args.ridge, "lmmse_damp": bool(args.lmmse_damp),
            "N": args.nsamp, "parallelism": "LD blocks sharded over %d GPU rank(s)" % world,
            "share_device": bool(args.share_device),
            "cg_column_sets": "exact" if eng.cg_exact else "look-ahead",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "kernel": (("sgv::k_sym_mfma (f64 MFMA, >= 3 RHS)" if mfma else "sgv::k_sym_pass")
                       + " + k_sym_finalize (packed symmetric LD pass, per GPU)"
                       if args.ld_format == "packed" else "sgv::k_ld_pass (dense LD pass, per GPU)"),
            "bytes_per_launch": bytes_launch,
            "ld_format": args.ld_format,
            "dense_equivalent_GBs": dense_equiv,
            "aux_partial_bytes_per_launch": tm["aux_bytes"] / launches,
            "avg_launch_ms": avg_s * 1e3,
            "launches": int(launches),
            "traffic_source": traffic_src,
            "box_stream_GBs": box_bw,
            "frac_of_box_stream": (achieved / box_bw) if (achieved and box_bw) else None,
        },
        # the 9..16-column passes (C5: 16 CG columns on one LD) are bound by the
        # f64 matrix core (v_mfma_f64_16x16x4f64), not by HBM: their algorithmic
        # flops (sgv_timers: 2 per multiply-add, row part of every stored element
        # + transpose part of the off-diagonal-block ones) over their HIP-event
        # time, against the dense f64 matrix peak (AMD's MI355X figure; the
        # guide lists no f64 row)
        "compute_roofline": ({
            "bound": "mfma",
            "achieved": tm["wide_flops"] / (tm["wide_ms"] / 1e3) / 1e12,
            "peak": F64_MFMA_PEAK_TFS,
            "unit": "TFLOP/s",
            "frac": tm["wide_flops"] / (tm["wide_ms"] / 1e3) / 1e12 / F64_MFMA_PEAK_TFS,
            "passes": tm["wide_launches"],
            "avg_launch_ms": tm["wide_ms"] / tm["wide_launches"],
            "hbm_frac_of_these_passes": None,
        } if tm["wide_launches"] > 0 and tm["wide_ms"] > 0 else None),
        "exchange": {
            # cross-rank all-gathers of the timed steps (sgv_exchange_stats): the
            # ordered CG/EM reductions and r1 gathers that replace the reference's
            # bcast all-gather (src/sgvamp.py:228-233); ms = HIP events around each
            # ncclAllGather (the wait for the slowest peer included) or the host
            # callback's wall time; the slowest rank's
            "transport": xs["transport"],
            "allgathers_per_step": xs["allgathers"] / steps,
            "ms_per_step": max(x["ms"] for x in xs_all) / steps,
            "frac_of_step": (max(x["ms"] for x in xs_all) / steps) / (dt / steps * 1e3),
            "bytes_per_step_per_rank": xs["bytes"] / steps,
            # the EM prior loop's exchange mode per loop, chosen by the cost model
            # (capi.hip em_costs) from the per-all-gather latency measured at
            # set-up (sgv_exchange_probe, the slowest rank's): the last decision
            # with both predicted costs, and the loops run in each mode
            "em_mode": xs["em_mode"],
            "em_loops": {"replicated": xs["em_loops_replicated"],
                         "per_step": xs["em_loops_per_step"]},
            "em_model": {"latency_us": xs["latency_us"], "latency_source": xs["latency_source"],
                         "predicted_steps": xs["em_pred_steps"],
                         "predicted_replicated_us": xs["em_pred_replicated_us"],
                         "predicted_per_step_us": xs["em_pred_per_step_us"],
                         "replicated_possible": xs["em_replicated_possible"],
                         # the device-driven EM loops as they ran (HIP events), the
                         # slowest rank's mean per loop, to check the prediction
                         "measured_us_per_loop": (max(x["em_ms"] / max(x["em_loops_timed"], 1)
                                                      for x in xs_all) * 1e3
                                                  if xs["em_loops_timed"] else None),
                         "loops_timed": xs["em_loops_timed"]},
            # exact CG column sets: the device's idle time between an iteration's
            # p update and its passes, which the host enqueues after reading the
            # stop test (HIP events; the slowest rank's)
            "host_wait_ms_per_step": max(x["host_wait_ms"] for x in xs_all) / steps,
            "K_times_M": K * eng.M,
            # who ran: RCCL's own count of ranks in the communicator (None unless
            # the transport is RCCL), and per rank its place in the communicator,
            # HIP device, PCI bus id and exact-CG host wait
            "transport_note": {"rccl": "RCCL all-gathers (ncclAllGather) on each rank's device",
                               "host": "host exchange: per-block partials all-gathered by the "
                                       "host communicator (a rehearsal when --share-device puts "
                                       "every rank on one device; not RCCL)",
                               None: "one rank, no communicator"}[xs["transport"]],
            "rccl_ranks": ci_all[0]["comm_ranks"] if xs["transport"] == "rccl" else None,
            "ranks": ci_all,
            "distinct_devices": len({c["pci_bus_id"] for c in ci_all}),
        },
        "ld_passes_per_step": passes / steps,
        "effective_ld_gbps_end_to_end": passes * ld_bytes_total / dt / 1e9,
        "cg_iters_per_step": [r["cg_iters"] for r in recs],
    }
    if rank == 0 and world == 1 and args.cpu_baseline == "auto" and not args.band:
        log("[bench] cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline(eng, args, dict(flags, **run), recs, x0)
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    v.finish()
    eng.close()


if __name__ == "__main__":
    main()
