"""Input loaders of the CLI (src/main.py:126-285), host side.

* .bim files: union of variants over cohorts, sorted by Coordinate (main.py:132-143)
* r vectors:  .txt / .npy / PLINK .linear (BETA, NaN -> 0, x sqrt(N)) (main.py:176-191)
* LD:         .npy dense (block structure detected), .npz CSR (block-diagonal
              detected from indptr/indices), or the build's block manifest
              ``*.blocks.json`` = {"block_sizes": [...], "files": [one .npy per
              block]} for LD that cannot exist as one dense array (M = 1e6).
* PLINK .ld text LD (main.py:203-257): per cohort a CSR matrix with a unit
              diagonal and every listed pair in both triangles (duplicates summed, as
              scipy's COO -> CSR does); markers a cohort lacks are filled from another
              cohort (the reference's MPI point-to-point exchange, emulated here in one
              process: load_plink_ld_all)
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
        raise Exception("PLINK .ld LD needs every cohort's .ld and .bim: use load_plink_ld_all")
    raise Exception("Unsupported R matrix format!")


def plink_ld_sources(bim_ref, bim_list, N_list):
    """src/main.py:151-162: for cohort k and reference marker i, the cohort k asks
    for marker i (== k: k holds it).  Reproduced as the reference computes it:
    kx = argmax of N over the OTHER cohorts holding the marker is a position in
    that list, used as a cohort id (main.py:161-162), so a marker may be asked of
    a cohort that lacks it (then nothing arrives and r stays 0), or of k itself
    (never requested)."""
    M = len(bim_ref)
    K = len(bim_list)
    idx = {rs: i for i, rs in enumerate(bim_ref)}
    sets = [set(b) for b in bim_list]
    out = []
    for k in range(K):
        source = np.ones(M) * k
        for rs in list(set(bim_ref) - sets[k]):
            idx_rs = [j for j in range(K) if j != k and rs in sets[j]]
            kx = np.argmax(np.array(N_list)[idx_rs])
            source[idx[rs]] = kx
        out.append(source)
    return out


def read_plink_ld(path, idx):
    """One PLINK --r table (columns SNP_A, SNP_B, R): reference-indexed pairs."""
    import pandas as pd

    df = pd.read_table(path, sep=r"\s+")
    indA = [idx[rs] for rs in list(df["SNP_A"])]
    indB = [idx[rs] for rs in list(df["SNP_B"])]
    return indA, indB, list(df["R"])


def load_plink_ld_all(ld_paths, r, bim_ref, bim_list, N_list):
    """All cohorts' .ld files -> (per-cohort scipy CSR R, updated r (K, M)).

    src/main.py:203-257 with the exchange between cohort ranks done in one
    process, in the reference's order: cohort k asks cohort j (j != k) for the
    markers with source[k] == j; j answers with every entry of ITS OWN .ld that
    touches a requested marker -- once per requested endpoint, so a pair whose
    two markers were both requested arrives twice and, summed, doubles -- and
    with its r at those markers; k appends the answers of j = 0..K-1 to its own
    entries and overwrites r[source == j].  R = I + pairs + transposed pairs.

    The reference scans j's whole table once per requested marker
    (O(requests x pairs), main.py:221-225); here one vectorised pass per (k, j)
    selects the same entries in the same order (requested marker ascending,
    then table order; oracle/ldio_oracle.py keeps the loop, tests compare)."""
    import scipy.sparse

    K = len(ld_paths)
    M = len(bim_ref)
    idx = {rs: i for i, rs in enumerate(bim_ref)}
    own = [tuple(np.asarray(a) for a in read_plink_ld(p, idx)) for p in ld_paths]
    own = [(A.astype(np.int64), B.astype(np.int64), C.astype(np.float64)) for A, B, C in own]
    sources = plink_ld_sources(bim_ref, bim_list, N_list)
    r_in = np.asarray(r, dtype=np.float64)
    r_out = r_in.copy()
    mats = []
    for k in range(K):
        parts_a, parts_b, parts_c = [own[k][0]], [own[k][1]], [own[k][2]]
        source = sources[k]
        for j in range(K):
            if j == k or j not in source:
                continue
            req = np.flatnonzero(source == j)
            jA, jB, jC = own[j]
            want = np.zeros(M, dtype=bool)
            want[req] = True
            inA, inB = want[jA], want[jB] & (jB != jA)    # a self pair answers once
            e = np.concatenate([np.flatnonzero(inA), np.flatnonzero(inB)])
            key = np.concatenate([jA[inA], jB[inB]])          # the requested endpoint
            order = np.lexsort((e, key))                      # by marker, then table order
            e = e[order]
            parts_a.append(jA[e])
            parts_b.append(jB[e])
            parts_c.append(jC[e])
            r_out[k][source == j] = r_in[j][req]
        indA, indB, R_col = (np.concatenate(x) for x in (parts_a, parts_b, parts_c))
        ar = np.arange(M)
        ind_r = np.concatenate([ar, indA, indB])
        ind_c = np.concatenate([ar, indB, indA])
        v = np.concatenate([np.ones(M), R_col, R_col])
        mats.append(scipy.sparse.csr_matrix((v, (ind_r, ind_c)), shape=(M, M)))
    return mats, r_out


def load_true_signal(path, M, N):
    if path.endswith(".bin"):
        with open(path, "rb") as f:
            buf = f.read(M * 8)
        x0 = np.array(struct.unpack(str(M) + "d", buf)).reshape((M, 1))
        return x0 * np.sqrt(N)
    if path.endswith(".npy"):
        return np.load(path) * np.sqrt(N)
    raise Exception("Unsupported true signal format!")
