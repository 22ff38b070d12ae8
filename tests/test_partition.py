"""Host logic: block partitioning, block-structure detection, LD regrouping."""
import numpy as np
import pytest
import scipy.sparse

from partition import (detect_blocks_csr, detect_blocks_dense, marker_offsets,
                       partition_blocks)


@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
def test_equal_blocks_split_evenly(nranks):
    r = partition_blocks([25000] * 8, nranks)
    assert r[0][0] == 0 and r[-1][1] == 8
    assert all(b1 - b0 == 8 // nranks for b0, b1 in r)
    assert all(r[i][1] == r[i + 1][0] for i in range(nranks - 1))


def test_uneven_blocks_balanced_by_bytes():
    sizes = [100, 100, 100, 400, 50, 50, 300, 200]
    r = partition_blocks(sizes, 3)
    w = [sum(s * s for s in sizes[b0:b1]) for b0, b1 in r]
    assert all(b1 > b0 for b0, b1 in r)
    assert max(w) <= 0.6 * sum(w)


def test_every_rank_gets_a_block():
    r = partition_blocks([1000, 1, 1, 1], 4)
    assert [b1 - b0 for b0, b1 in r] == [1, 1, 1, 1]
    with pytest.raises(ValueError):
        partition_blocks([5, 5], 3)


def test_marker_offsets():
    np.testing.assert_array_equal(marker_offsets([3, 4, 5]), [0, 3, 7, 12])


def _blockdiag(sizes, seed=0):
    rs = np.random.RandomState(seed)
    M = sum(sizes)
    R = np.zeros((M, M))
    o = 0
    for n in sizes:
        B = rs.normal(size=(n, n))
        R[o:o + n, o:o + n] = B + B.T
        o += n
    return R


def test_detect_blocks_dense_and_csr():
    sizes = [5, 1, 7, 3]
    R = _blockdiag(sizes)
    assert detect_blocks_dense(R) == sizes
    A = scipy.sparse.csr_matrix(R)
    assert detect_blocks_csr(A.indptr, A.indices, R.shape[0]) == sizes


def test_detect_blocks_sparse_pattern_inside_block():
    # a block whose first and last marker are linked only through the corner
    R = np.eye(6)
    R[0, 3] = R[3, 0] = 0.5
    R[4, 5] = R[5, 4] = 0.1
    assert detect_blocks_dense(R) == [4, 2]
    A = scipy.sparse.csr_matrix(R)
    assert detect_blocks_csr(A.indptr, A.indices, 6) == [4, 2]


def test_blockld_regroup_and_common_partition():
    from sgvamp import BlockLD, common_partition

    R = _blockdiag([130, 140, 150])
    L = BlockLD.from_dense(R)
    assert L.block_sizes == [130, 140, 150]
    assert common_partition([[130, 140, 150], [270, 150]]) == [270, 150]
    G = L.regroup([270, 150])
    np.testing.assert_array_equal(G.block(0), R[:270, :270])
    np.testing.assert_array_equal(G.block(1), R[270:, 270:])
    with pytest.raises(ValueError):
        L.regroup([150, 270])
    # blocks below 128 markers are merged (no 1-marker blocks padded to 128)
    assert BlockLD.from_dense(_blockdiag([3, 2, 4])).block_sizes == [9]


def test_coarsen_blocks_merges_tiny_blocks():
    from partition import coarsen_blocks

    assert coarsen_blocks([200, 250, 150]) == [200, 250, 150]      # golden CSR layout unchanged
    c = coarsen_blocks([1] * 3000 + [2050])                        # R = I beside a band
    assert sum(c) == 5050 and c[-2:] == [56, 2050] and min(c[:-2]) >= 128 and len(c) == 25
    # a small run is never merged into a big block (its n x n storage would grow)
    assert coarsen_blocks([1] * 100 + [5000] + [3] * 10) == [100, 5000, 30]
    assert coarsen_blocks([5, 20000]) == [5, 20000]
    assert coarsen_blocks([20000, 5]) == [20000, 5]
    assert coarsen_blocks([20000, 100, 100, 5]) == [20000, 205]      # joins a merged block
    assert coarsen_blocks([60, 70, 5]) == [135]
    assert coarsen_blocks([5] * 10) == [50]
    assert coarsen_blocks([]) == []


def test_cg_exact_mode_from_stored_bytes():
    """The run's CG column-set mode (engine.cg_exact_from_stored):
    decided by the bytes the shared LD actually stores, so a banded LD whose
    block sizes alone would suggest >= 24 GB keeps the look-ahead; a matrix used
    by one cohort (2 columns: the VALU pass) never narrows."""
    from engine import cg_exact_from_stored, cg_exact_mode

    assert cg_exact_mode([15625] * 64) == 1                      # north star: 63.5 GB triangle
    assert cg_exact_mode([1_000_000]) == 1                       # one 1e6 block by size ...
    assert cg_exact_from_stored([10.2e9], [0, 0, 0, 0]) == 0     # ... but a bw=1000 band stores 10 GB
    assert cg_exact_from_stored([63.5e9], [0, 0, 0, 0]) == 1
    assert cg_exact_from_stored([63.5e9, 1e9], [0, 1]) == 0      # distinct LD: 2 columns per matrix
    assert cg_exact_from_stored([1e9, 30e9], [0, 0, 1, 1]) == 1
