"""Synthetic cohorts generated on the device, written as the CLI's input files
(simulation/sim_gen_phen_mult.py:1-61 of the reference, restated for LD of any
size).

The reference draws X ~ Binomial(2, 0.4) (N x M) per cohort, standardises the
columns, sets y = X beta + N(0, 1 - h2), and saves beta, y, r = X^T y / sqrt(N)
and the dense R = X^T X / N.  Here the genotypes are drawn per LD block on the
device (the build's counter-based generator, `oracle/synth_oracle.py` restates
it), R is block-diagonal (one block per --block-size markers; the whole matrix
when it is not given, as the reference) and is formed by the device GEMM, so
M = 1e6 (125 GB of blocks) takes minutes instead of hours.  beta uses
RandomState(seed) instead of the unseeded global RNG.

Outputs (prefix --out):
  {out}_bet.npy               beta (M, 1)
  {out}_{k}_phen.npy          y of cohort k (N, 1)
  {out}_{k}_r.npy             r of cohort k (M, 1)
  {out}_{k}_R.npy             LD of cohort k, one block  (or {out}_R.npy with --shared-ld 1)
  {out}_{k}_R.blocks.json     several blocks: the manifest main.py reads, one .npy per block
  {out}_{k}.bim               variants rs0.. at coordinates 1..M (main.py's --bim-files)

    python simulate.py --out sim/c --N 10000 --M 1000000 --K 4 --block-size 15625 --shared-ld 1
"""
import argparse
import json
import os

import numpy as np

import hip_backend as hb
from engine import Engine


def windowed_ld(n, bw, seed=0, taps=12):
    """Synthetic windowed LD (PLINK --ld-window's shape, one chromosome): an
    exactly symmetric positive semi-definite CSR matrix with unit diagonal and
    entries only within bw of the diagonal, R = D B B^T D with B lower-banded
    (each marker mixes `taps` earlier 'haplotype factors' at fixed offsets,
    0 and bw among them, decaying with distance).  Built on the host with
    scipy in O(n * taps^2); M = 1e6, bw = 1,000 takes ~15 s."""
    import scipy.sparse

    rs = np.random.RandomState(seed)
    decay = max(bw / 3.0, 1.0)
    offs = {0, bw}
    if bw > 1:
        offs |= set(rs.choice(np.arange(1, bw), min(bw - 1, taps), replace=False).tolist())
    rows, cols, vals = [], [], []
    for k in sorted(offs):
        i = np.arange(k, n)
        rows.append(i)
        cols.append(i - k)
        vals.append(rs.normal(size=n - k) * np.exp(-k / decay) + (1.0 if k == 0 else 0.0))
    B = scipy.sparse.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                                shape=(n, n))
    R = (B @ B.T).tocsr()
    d = 1.0 / np.sqrt(R.diagonal())
    R = scipy.sparse.diags(d) @ R @ scipy.sparse.diags(d)
    R = ((R + R.T) * 0.5).tocsr()
    R.sum_duplicates()
    R.sort_indices()
    return R


def _write_ld(eng, ld, sizes, prefix):
    """One cohort's LD from the device: a .npy, or a manifest and one .npy per block."""
    if len(sizes) == 1:
        path = prefix + ".npy"
        np.save(path, eng.get_ld_block(ld, 0))
        return path
    files = []
    for b in range(len(sizes)):
        fn = "%s_b%d.npy" % (os.path.basename(prefix), b)
        np.save(os.path.join(os.path.dirname(os.path.abspath(prefix)), fn), eng.get_ld_block(ld, b))
        files.append(fn)
    path = prefix + ".blocks.json"
    with open(path, "w") as f:
        json.dump({"block_sizes": [int(n) for n in sizes], "files": files}, f)
    return path


def simulate(out, N, M, K=2, h2=0.8, lam=0.5, block_size=None, shared_ld=False, seed=2025,
             device=None):
    """Writes the files listed in the module docstring; returns their paths."""
    bs = int(block_size or M)
    sizes = [bs] * (M // bs) + ([M % bs] if M % bs else [])
    rs = np.random.RandomState(seed)
    cm = int(M * lam)                                   # :28-32
    beta = np.zeros(M)
    beta[rs.choice(M, cm, replace=False)] = rs.normal(0, np.sqrt(h2 / cm), cm)
    paths = {"beta": out + "_bet.npy", "phen": [], "r": [], "ld": [], "bim": []}
    np.save(paths["beta"], beta.reshape(M, 1))
    nld = 1 if shared_ld else K
    ld_of = [0 if shared_ld else k for k in range(K)]
    geno_seed = [seed + 1 + 7919 * ld for ld in range(nld)]   # one genotype stream per LD
    eng = Engine(sizes, K=K, ld_of=ld_of, device=device)
    try:
        g = [eng.synth_ld_g(ld, geno_seed[ld], N, beta).sum(axis=0) for ld in range(nld)]
        ld_path = [_write_ld(eng, ld, sizes, out + ("_R" if shared_ld else "_%d_R" % ld))
                   for ld in range(nld)]
        for k in range(K):
            w = np.random.RandomState(seed + 1000 + k).normal(0.0, np.sqrt(1 - h2), N)   # :46
            y = g[ld_of[k]] + w
            eng.synth_r(k, geno_seed[ld_of[k]], N, y)
            r = eng.get_vector(hb.VEC_R, k)
            paths["phen"].append("%s_%d_phen.npy" % (out, k))
            paths["r"].append("%s_%d_r.npy" % (out, k))
            np.save(paths["phen"][-1], y.reshape(N, 1))
            np.save(paths["r"][-1], r.reshape(M, 1))
            paths["ld"].append(ld_path[ld_of[k]])
            bim = "%s_%d.bim" % (out, k)
            with open(bim, "w") as f:
                for j in range(M):
                    f.write("1\trs%d\t0\t%d\tA\tG\n" % (j, j + 1))
            paths["bim"].append(bim)
    finally:
        eng.close()
    return paths


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-out", "--out", help="Output path")
    p.add_argument("-N", "--N", help="Number of samples")
    p.add_argument("-M", "--M", help="Number of markers")
    p.add_argument("-h2", "--h2", help="Heritability used in simulations", default=0.8)
    p.add_argument("-lam", "--lam", help="Sparsity (lambda) used in simulations", default=0.5)
    p.add_argument("-K", "--K", help="Number of cohorts", default=2)
    p.add_argument("--block-size", help="LD block size (default: M, one dense block)", default=None)
    p.add_argument("--shared-ld", help="1: all cohorts share one genotype draw (one LD)", default=0)
    p.add_argument("--seed", help="beta, genotype and noise seed", default=2025)
    p.add_argument("--device", help="HIP device", default=None)
    a = p.parse_args(argv)
    print("...Simulating data for sgVAMP\n")
    paths = simulate(a.out, int(a.N), int(a.M), K=int(a.K), h2=float(a.h2), lam=float(a.lam),
                     block_size=int(a.block_size) if a.block_size else None,
                     shared_ld=bool(int(a.shared_ld)), seed=int(a.seed),
                     device=int(a.device) if a.device is not None else None)
    print("main.py inputs: --ld-files %s --r-files %s --bim-files %s --true-signal-file %s"
          % (",".join(paths["ld"]), ",".join(paths["r"]), ",".join(paths["bim"]), paths["beta"]))


if __name__ == "__main__":
    main()
