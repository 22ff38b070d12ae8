"""Offline PLINK converter (scripts/plink2np.py:1-50 of the reference):
``.assoc.linear`` BETA column -> ``.npy``; ``.ld`` pair table -> CSR ``.npz``
with a unit diagonal and every listed pair in both triangles (duplicates summed,
as scipy's COO -> CSR conversion does), markers indexed in the ``.linear``
file's SNP order.  The outputs are what main.py's ``--r-files`` / ``--ld-files``
read.  Same flags and output paths as the reference script:

    python plink2np.py --ld-file X.ld --r-file Y.assoc.linear
"""
import argparse

import numpy as np
import scipy.sparse

from ldio import read_plink_ld


def convert(ld_file, r_file):
    """Writes the two outputs; returns their paths (r .npy, R .npz)."""
    import pandas as pd

    out_r = r_file.split(".assoc.linear")[0] + ".npy"      # :22-23
    out_R = ld_file.split(".ld")[0] + ".npz"
    print(out_r)
    print(out_R)
    df_r = pd.read_table(r_file, sep=r"\s+")
    print(f".linear file loaded. Shape: {df_r.shape}", flush=True)
    print(f"storing r vector to {out_r}")
    np.save(out_r, df_r["BETA"].values)                     # :30 (NaN kept, no sqrt(N))
    M = len(df_r)
    idx = {rs: i for i, rs in enumerate(df_r["SNP"])}      # :35-36
    indA, indB, vals = read_plink_ld(ld_file, idx)
    print(f".ld file loaded. Pairs: {len(vals)}", flush=True)
    rows = np.concatenate([np.arange(M), np.asarray(indA, dtype=np.int64),
                           np.asarray(indB, dtype=np.int64)])
    cols = np.concatenate([np.arange(M), np.asarray(indB, dtype=np.int64),
                           np.asarray(indA, dtype=np.int64)])
    v = np.concatenate([np.ones(M), np.asarray(vals, dtype=np.float64),
                        np.asarray(vals, dtype=np.float64)])
    R = scipy.sparse.csr_matrix((v, (rows, cols)), shape=(M, M))   # :41-47
    print(f"storing R matrix to {out_R}")
    scipy.sparse.save_npz(out_R, R, compressed=True)
    return out_r, out_R


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-ld_file", "--ld-file", help="Path to .ld file", default=None)
    p.add_argument("-r_file", "--r-file", help="Path to .linear file", default=None)
    a = p.parse_args(argv)
    print("Input arguments:")
    print("--ld-file", a.ld_file)
    print("--r-file", a.r_file)
    print("\n", flush=True)
    convert(a.ld_file, a.r_file)


if __name__ == "__main__":
    main()
