"""Marker / LD-block partitioning across GPU ranks (pure host logic).

The reference gives every MPI rank one cohort and the full marker range
(src/main.py:85,173-174).  Here every rank owns a contiguous range of LD blocks
for ALL cohorts, so the reference's per-iteration K x M all-gather
(src/sgvamp.py:228-233) disappears; only ordered per-block partial sums travel.
"""
import numpy as np


def partition_blocks(block_sizes, nranks):
    """Contiguous block ranges [(b0, b1)] per rank, balanced by LD bytes
    (sum n_b^2).  Every rank gets at least one block."""
    sizes = np.asarray(block_sizes, dtype=np.int64)
    nb = len(sizes)
    if nranks < 1:
        raise ValueError("nranks must be >= 1")
    if nb < nranks:
        raise ValueError("%d LD blocks cannot be spread over %d ranks" % (nb, nranks))
    w = sizes.astype(np.float64) ** 2
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, nranks):
        target = total * r / nranks
        b = int(np.searchsorted(cum, target, side="left"))
        # choose the nearer boundary, keep >= 1 block per rank on both sides
        if b > 0 and abs(cum[b - 1] - target) <= abs(cum[min(b, nb)] - target):
            b -= 1
        b = max(b, cuts[-1] + 1)
        b = min(b, nb - (nranks - r))
        cuts.append(b)
    cuts.append(nb)
    return [(cuts[r], cuts[r + 1]) for r in range(nranks)]


def marker_offsets(block_sizes):
    return np.concatenate([[0], np.cumsum(np.asarray(block_sizes, dtype=np.int64))])


def detect_blocks_dense(R, tol=0.0):
    """Finest contiguous block-diagonal partition of a dense symmetric-pattern
    matrix: block ends at j when no nonzero links rows/cols <= j with > j."""
    M = R.shape[0]
    nz = np.abs(np.asarray(R)) > tol
    nz |= nz.T
    rows_any = nz.any(axis=1)
    last = np.where(rows_any, M - 1 - np.argmax(nz[:, ::-1], axis=1), np.arange(M))
    return _blocks_from_reach(np.maximum(last, np.arange(M)))


def detect_blocks_csr(indptr, indices, M):
    """Same for a CSR matrix (scipy.sparse .npz LD, src/main.py:200)."""
    indptr = np.asarray(indptr)
    indices = np.asarray(indices)
    reach = np.arange(M)
    counts = np.diff(indptr)
    rows = np.repeat(np.arange(M), counts)
    if len(indices):
        np.maximum.at(reach, rows, indices)
        # symmetric pattern: column c reaches row r as well
        np.maximum.at(reach, indices, rows)
    return _blocks_from_reach(reach)


def coarsen_blocks(sizes, min_size=128):
    """Merge runs of consecutive blocks smaller than min_size (PADV markers, one
    padded vector segment) into blocks of at least min_size: a diagonal or
    near-diagonal LD (e.g. a PLINK .ld without pairs: R = I) would otherwise
    become M blocks of one marker, each padded to 128 in every device vector.
    Blocks already >= min_size are kept as they are -- a small run is never
    merged into one (that would grow its n x n storage and change its row
    stride) -- and the merged blocks hold zeros between their parts (same
    matrix, coarser partition).  A trailing small run joins the previous block
    only when that one is itself merged from small blocks."""
    out, merged, acc, nacc = [], [], 0, 0
    for n in sizes:
        n = int(n)
        if acc and n >= min_size:     # a pending run of small blocks stays apart from a big one
            out.append(acc)
            merged.append(True)
            acc, nacc = 0, 0
        acc += n
        nacc += 1
        if acc >= min_size:
            out.append(acc)
            merged.append(nacc > 1)
            acc, nacc = 0, 0
    if acc:
        if out and merged[-1]:
            out[-1] += acc
        else:
            out.append(acc)
    return out


def _blocks_from_reach(reach):
    sizes = []
    start = 0
    far = -1
    for i, r in enumerate(reach):
        far = max(far, int(r))
        if far == i:
            sizes.append(i + 1 - start)
            start = i + 1
            far = -1
    return sizes
