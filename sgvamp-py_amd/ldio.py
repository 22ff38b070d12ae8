"""Input loaders of the CLI (src/main.py:126-285), host side.

* .bim files: union of variants over cohorts, sorted by Coordinate (main.py:132-143)
* r vectors:  .txt / .npy / PLINK .linear (BETA, NaN -> 0, x sqrt(N)) (main.py:176-191)
* LD:         .npy dense (block structure detected), .npz CSR (block-diagonal
              detected from indptr/indices), or the build's block manifest
              ``*.blocks.json`` = {"block_sizes": [...], "files": [one .npy per
              block]} for LD that cannot exist as one dense array (M = 1e6).
* true signal: .bin (f64) / .npy, multiplied by sqrt(N) (main.py:268-285)
"""
import json
import os
import struct

import numpy as np

from sgvamp import BlockLD


def merge_bims(bim_paths):
    """Returns (bim_ref DataFrame, per-cohort variant lists).  src/main.py:132-143."""
    import pandas as pd

    bim_list, bim_ref_df = [], None
    for k, path in enumerate(bim_paths):
        df = pd.read_table(path, sep=r"\s+", header=None,
                           names=["Chromosome", "Variant", "Position", "Coordinate", "Allele1",
                                  "Allele2"])
        bim_list.append(list(df["Variant"]))
        if k == 0:
            bim_ref_df = df
        else:
            bim_ref_df = pd.merge(bim_ref_df, df, on=["Variant"], how="outer", suffixes=("", "_y"))
    bim_ref_df = bim_ref_df.sort_values(by=["Coordinate"])
    return bim_ref_df, bim_list


def load_r(path, M_k, N_k, i_map, M):
    """One cohort's r in the merged marker order (src/main.py:176-191)."""
    if path.endswith(".txt"):
        r_k = np.loadtxt(path).reshape((M_k,))
    elif path.endswith(".npy"):
        r_k = np.load(path).reshape((M_k,))
    elif path.endswith(".linear"):
        import pandas as pd

        df = pd.read_table(path, sep=r"\s+")
        r_k = np.array(df["BETA"], dtype=np.float64).reshape((M_k,))
        r_k[np.isnan(r_k)] = 0
        r_k *= np.sqrt(N_k)
    else:
        raise Exception("Unsupported r vector format!")
    r = np.zeros(M)
    r[np.asarray(i_map, dtype=np.int64)] = r_k
    return r


def load_ld(path, s):
    """One cohort's LD matrix as a BlockLD with ridge s (src/main.py:199-265)."""
    if path.endswith(".npz"):
        import scipy.sparse

        return BlockLD.from_csr(scipy.sparse.load_npz(path), s=s)
    if path.endswith(".npy"):
        R = np.load(path, mmap_mode="r")
        return BlockLD.from_dense(R, s=s)
    if path.endswith(".blocks.json"):
        man = json.load(open(path))
        base = os.path.dirname(os.path.abspath(path))
        files = [f if os.path.isabs(f) else os.path.join(base, f) for f in man["files"]]
        sizes = [int(b) for b in man["block_sizes"]]
        return BlockLD(block_sizes=sizes, loader=lambda b: np.load(files[b], mmap_mode="r"), s=s)
    if path.endswith(".ld"):
        raise Exception("PLINK .ld text LD is not supported yet; convert it to .npz")
    raise Exception("Unsupported R matrix format!")


def load_true_signal(path, M, N):
    if path.endswith(".bin"):
        with open(path, "rb") as f:
            buf = f.read(M * 8)
        x0 = np.array(struct.unpack(str(M) + "d", buf)).reshape((M, 1))
        return x0 * np.sqrt(N)
    if path.endswith(".npy"):
        return np.load(path) * np.sqrt(N)
    raise Exception("Unsupported true signal format!")
