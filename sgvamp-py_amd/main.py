"""sgVAMP command line -- drop-in for the reference's src/main.py.

Same flags, defaults, validation messages, log lines and output files
({out}/{name}.bim, {name}_xhat_it_{it}.bin, {name}_r1_cohort_{k}_it_{it}.bin,
{name}_cohort_{k}.csv, {name}_metrics.csv).  Differences:

* one process per GPU instead of one MPI rank per cohort: a single process
  handles all K cohorts (python main.py ...); ``--gpus G`` starts G local
  ranks (launch.py) and the LD blocks are sharded over them.  The reference's
  own launch (mpirun -np K python main.py ..., src/main.py:16-18) also works:
  its K processes become K GPU ranks of ONE job (comm.launch_from_env maps
  Open MPI / Hydra / srun ranks; rank 0 alone writes the shared files), not K
  copies of it;
* --seed (extension): seeds the Hutchinson probes per cohort, RandomState(seed+k)
  (the reference draws from the unseeded global RNG, src/sgvamp.py:326);
* --bim-files may be omitted when every cohort has the same marker order;
* LD may also be given as a block manifest (*.blocks.json, see ldio.py).
"""
import argparse
import logging
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from comm import world_from_env  # noqa: E402
from ldio import load_ld, load_plink_ld_all, load_r, load_true_signal, merge_bims  # noqa: E402
from sgvamp import BlockLD  # noqa: E402
from sgvamp import VAMP  # noqa: E402


def build_parser():
    # src/main.py:27-50
    parser = argparse.ArgumentParser()
    parser.add_argument("-ld_files", "--ld-files", help="Path to LD matrices in .npz files, separated by comma ")
    parser.add_argument("-r_files", "--r-files", help="Path to XTy .npy files separated by comma")
    parser.add_argument("-true_signal_file", "--true-signal-file", help="Path to true signal .npy file", default=None)
    parser.add_argument("-out_dir", "--out-dir", help="Output directory")
    parser.add_argument("-out_name", "--out-name", help="Output file name")
    parser.add_argument("-N", "--N", help="Number of samples in each cohort, saparated by comma")
    parser.add_argument("-M", "--M", help="Number of markers in each cohort, separated by comma")
    parser.add_argument("-K", "--K", help="Number of cohorts", default=1)
    parser.add_argument("-L", "--L", help="Number of prior mixture components", default=2)
    parser.add_argument("-iterations", "--iterations", help="Number of iterations", default=10)
    parser.add_argument("-prior_vars", "--prior-vars", help="Prior mixture variances of different cohorts", default="0,1")
    parser.add_argument("-prior_probs", "--prior-probs", help="Prior mixture probabilites of different cohorts", default="0.99,0.01")
    parser.add_argument("-gamw", "--gamw", help="Initial noise precision", default=5)
    parser.add_argument("-gam1", "--gam1", help="Initial signal precision", default=0.000001)
    parser.add_argument("-lmmse_damp", "--lmmse-damp", help="Use LMMSE damping", default=False)
    parser.add_argument("-learn_gamw", "--learn-gamw", help="Learn or fix gamw", default=True)
    parser.add_argument("-rho", "--rho", help="Damping factor rho", default=0.5)
    parser.add_argument("-cg_maxit", "--cg-maxit", help="CG max iterations", default=500)
    parser.add_argument("-s", "--s", help="Rused = (1-s) * R + s * Id", default=0.0)
    parser.add_argument("-prior_update", "--prior-update", help="Learning prior probabilities", default="em")
    parser.add_argument("-update_prior_from", "--update-prior-from", help="Learn prior probabilities from specific iteration onwards", default=1)
    parser.add_argument("-em_prior_maxit", "--em-prior-maxit", help="Maximal number of iterations that prior-learning EM is allowed to perform", default=100)
    parser.add_argument("-bim_files", "--bim-files", help="Path to files containing list of snps", default=None)
    # extensions
    parser.add_argument("--seed", help="Seed of the Hutchinson probes (RandomState(seed + k))", default=None)
    parser.add_argument("--device", help="HIP device (default: the node-local rank)", default=None)
    parser.add_argument("--gpus", help="GPU ranks to start on this node (default: the launcher's "
                        "world size, else 1)", default=None)
    return parser


def main(argv=None):
    args = build_parser().parse_args(argv)
    if argv is None:            # command line: --gpus N starts the ranks (before any GPU call)
        from launch import relaunch

        rc = relaunch(None if args.gpus is None else int(args.gpus))
        if rc is not None:
            sys.exit(rc)
    comm = world_from_env()
    rank = comm.Get_rank()
    logging.basicConfig(format="%(message)s", level=logging.DEBUG)   # main.py:21
    if rank == 0:
        logging.info(" ### VAMP for summary statistics ###\n")

    # main.py:54-97
    ld_fpaths, r_fpaths = args.ld_files, args.r_files
    true_signal_fpath = args.true_signal_file
    out_dir, out_name = args.out_dir, args.out_name
    Ms, Ns = args.M, args.N
    iterations = int(args.iterations)
    K = int(args.K)
    L = int(args.L)
    prior_vars, prior_probs = args.prior_vars, args.prior_probs
    gamw = float(args.gamw)
    gam1 = float(args.gam1)
    rho = float(args.rho)
    lmmse_damp = bool(int(args.lmmse_damp))
    learn_gamw = bool(int(args.learn_gamw))
    cg_maxit = int(args.cg_maxit)
    s = float(args.s)
    prior_update = args.prior_update
    update_prior_from = int(args.update_prior_from)
    em_prior_maxit = int(args.em_prior_maxit)
    bim_fpaths = args.bim_files
    seed = None if args.seed is None else int(args.seed)

    ld_fpaths_list = ld_fpaths.split(",")
    r_fpaths_list = r_fpaths.split(",")
    N_list = [int(n) for n in Ns.split(",")]
    M_list = [int(m) for m in Ms.split(",")]
    Nt = sum(N_list)
    prior_vars_list = [float(x) for x in prior_vars.split(",")]
    prior_probs_list = [float(x) for x in prior_probs.split(",")]
    if len(ld_fpaths_list) != K:
        raise Exception("Specified number of cohorts is not equal to number of LD matrices provided!")
    if len(r_fpaths_list) != K:
        raise Exception("Specified number of cohorts is not equal to number of marginal estimates provided!")
    if len(prior_vars_list) != L:
        raise Exception("Number of prior variances must be L!")
    if len(prior_probs_list) != L:
        raise Exception("Number of prior mixture probabilites must be L!")

    if rank == 0:
        logging.info("Input arguments:")
        for flag, val in [("--ld-files", ld_fpaths), ("--r-files", r_fpaths),
                          ("--out-name", out_name), ("--out-dir", out_dir),
                          ("--true-signal-file", true_signal_fpath), ("--N", Ns), ("--M", Ms),
                          ("--K", K), ("--L", L), ("--iterations", iterations),
                          ("--prior-vars", prior_vars), ("--prior-probs", prior_probs),
                          ("--gam1", gam1), ("--gamw", gamw), ("--lmmse-damp", lmmse_damp),
                          ("--learn-gamw", learn_gamw), ("--rho", rho), ("--cg-maxit", cg_maxit),
                          ("--s", s), ("--prior-update", prior_update),
                          ("--update-prior-from", update_prior_from)]:
            logging.info(f"{flag} {val}")
        if prior_update == "em":
            logging.info(f"--em_prior_maxit {em_prior_maxit}")
        logging.info(f"--bim-files {bim_fpaths}\n")

    # .bim merge (main.py:126-165)
    ts = time.time()
    if bim_fpaths is not None:
        if rank == 0:
            logging.info("...loading .bim files\n")
        bim_ref_df, bim_list = merge_bims(bim_fpaths.split(","))
        bim_ref = list(bim_ref_df["Variant"])
        M = len(bim_ref)
        idx = {rs: i for i, rs in enumerate(bim_ref)}
        i_maps = [[idx[rs] for rs in bim_list[k]] for k in range(K)]
        if rank == 0:
            logging.info(f"Total number of markers in reference is {M} \n")
            logging.info("...Saving refenrence .bim file \n")
            bim_ref_df.iloc[:, :6].to_csv(os.path.join(out_dir, out_name + ".bim"), header=None,
                                          sep="\t", index=False)
    else:
        if len(set(M_list)) != 1:
            raise Exception("--bim-files is required when cohorts have different markers")
        M = M_list[0]
        i_maps = [list(range(M))] * K
    logging.debug(f"Rank {rank}: Handling .bim file took {time.time() - ts} seconds \n")   # main.py:165

    # r and R (main.py:167-266)
    if rank == 0:
        logging.info("...loading R matrix and r vector\n")
    ts = time.time()
    r = np.stack([load_r(r_fpaths_list[k], M_list[k], N_list[k], i_maps[k], M) for k in range(K)])
    # per-rank lines of main.py:193-194 (every rank holds all K cohorts' r here)
    logging.info(f"Rank {rank} loaded r vector with shape {r.shape}\n")
    logging.debug(f"Rank {rank}: Loading r vector took {time.time() - ts} seconds \n")
    ts = time.time()
    by_path = {}
    lds = []
    if any(p.endswith(".ld") for p in ld_fpaths_list):
        # PLINK text LD: every cohort's table plus the missing-marker exchange (main.py:203-257)
        if bim_fpaths is None or not all(p.endswith(".ld") for p in ld_fpaths_list):
            raise Exception("PLINK .ld LD needs --bim-files and a .ld file for every cohort")
        mats, r = load_plink_ld_all(ld_fpaths_list, r, bim_ref, bim_list, N_list)
        for k in range(K):
            by_path[k] = BlockLD.from_csr(mats[k], s=s)
            lds.append(by_path[k])
    else:
        for k in range(K):
            p = ld_fpaths_list[k]
            if p not in by_path:
                by_path[p] = load_ld(p, s)
            lds.append(by_path[p])
    for L in lds:
        if L.M != M:
            raise Exception(f"LD matrix has {L.M} markers, expected {M}")
    if rank == 0:
        logging.info(f"Loaded {len(by_path)} LD matrix/matrices, blocks {lds[0].block_sizes[:8]}"
                     f"{'...' if len(lds[0].block_sizes) > 8 else ''}\n")
    # main.py:262-263 (the LD is uploaded per rank: its blocks of the partition)
    logging.info(f"Rank {rank} loaded R matrix with shape {(lds[0].M, lds[0].M)}\n")
    logging.debug(f"Rank {rank}: Loading R matrix took {time.time() - ts} seconds \n")

    x0 = None
    if true_signal_fpath is not None:
        x0 = load_true_signal(true_signal_fpath, M, N_list[0])
        if rank == 0:
            logging.info(f"True signals loaded. Shape: {x0.shape}\n")

    a = np.array(N_list) / sum(N_list)   # main.py:287
    sgv = VAMP(N=N_list, Nt=Nt, M=M, K=K, rho=rho, gam1=gam1, gamw=gamw, a=a,
               prior_vars=prior_vars_list, prior_probs=prior_probs_list, out_dir=out_dir,
               out_name=out_name, comm=comm, seed=seed,
               device=None if args.device is None else int(args.device))
    if rank == 0:
        logging.info("...Running sgVAMP\n")
    ts = time.time()
    R = lds[0] if len(by_path) == 1 else lds
    xhat1 = sgv.infer(R, r, iterations, x0=x0, cg_maxit=cg_maxit, em_prior_maxit=em_prior_maxit,
                      learn_gamw=learn_gamw, lmmse_damp=lmmse_damp, prior_update=prior_update,
                      update_prior_from=update_prior_from)
    te = time.time()
    if rank == 0:
        logging.info(f"sgVAMP inference running time: {(te - ts):0.4f}s\n")   # main.py:324
    if x0 is not None:
        alignments, l2s = [], []
        for it in range(iterations):
            x = xhat1[it].squeeze()
            alignments.append(np.inner(x, x0.squeeze()) / np.linalg.norm(x) / np.linalg.norm(x0.squeeze()))
            l2s.append(np.linalg.norm(x - x0.squeeze()) / np.linalg.norm(x0.squeeze()))
        if rank == 0:
            logging.info(f"Alignment(x1hat, x0) over iterations: \n {alignments}\n")
            logging.info(f"L2 error(x1hat, x0) over iterations: \n {l2s}\n")
    sgv.engine.close()
    return xhat1


if __name__ == "__main__":
    main()
