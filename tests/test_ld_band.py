"""Host side of sparse / banded LD (CPU): a symmetric CSR LD matrix of any
sparsity goes to the library as the CSR of each block's upper triangle and is
never densified; non-symmetric blocks are densified only within a size limit,
with a clear error instead of an n x n allocation (src/main.py:199-200,251-257
hand the reference's cg such matrices)."""
import numpy as np
import pytest
import scipy.sparse

from oracle import vamp_oracle as vo
from sgvamp import BlockLD


class FakeEngine:
    def __init__(self):
        self.csr, self.dense = {}, {}

    def set_ld_block_csr(self, ld, b, U):
        self.csr[(ld, b)] = U

    def set_ld_block(self, ld, b, B):
        self.dense[(ld, b)] = B


def test_banded_ld_goes_up_as_upper_csr_without_densifying():
    M, bw = 200_000, 40            # dense: 320 GB; band: ~70 MB of CSR
    A = vo.banded_ld(M, bw, seed=2)
    L = BlockLD.from_csr(A)
    assert L.block_sizes == [M]    # one block: the band links every marker
    eng = FakeEngine()
    L.upload(eng, 0, 0)
    assert not eng.dense
    U = eng.csr[(0, 0)]
    rows = np.repeat(np.arange(M), np.diff(U.indptr))
    assert np.all(U.indices >= rows) and np.max(U.indices - rows) == bw
    assert abs(U.nnz - (A.nnz + M) // 2) == 0          # the upper triangle, diagonal included
    np.testing.assert_array_equal((U + scipy.sparse.triu(U, 1).T).tocsr()[:50, :50].toarray(),
                                  A[:50, :50].toarray())


def test_block_diagonal_csr_splits_into_blocks():
    A = scipy.sparse.block_diag([vo.banded_ld(300, 10, seed=1), vo.banded_ld(500, 60, seed=2)],
                                format="csr")
    L = BlockLD.from_csr(A)
    assert L.block_sizes == [300, 500]
    eng = FakeEngine()
    for b in range(2):
        L.upload(eng, 0, b)
    assert set(eng.csr) == {(0, 0), (0, 1)} and not eng.dense
    np.testing.assert_array_equal(L.block(1), A[300:, 300:].toarray())


def test_nonsymmetric_large_block_fails_fast(monkeypatch):
    import sgvamp

    M = 50_000
    A = vo.banded_ld(M, 8, seed=3).tolil()
    A[0, 7] = A[0, 7] + 1e-3                 # no longer symmetric
    L = BlockLD.from_csr(A.tocsr())
    monkeypatch.setattr(sgvamp, "DENSE_BLOCK_LIMIT", 1 << 30)
    with pytest.raises(ValueError, match="not symmetric"):
        L.upload(FakeEngine(), 0, 0)
    # dense storage forced (packing off) on a huge sparse block: same clear error
    B = BlockLD.from_csr(vo.banded_ld(M, 8, seed=4))
    with pytest.raises(ValueError, match="dense LD storage requested"):
        B.upload(FakeEngine(), 0, 0, packed=False)


def test_regroup_keeps_csr():
    A1 = scipy.sparse.block_diag([vo.banded_ld(200, 4, seed=5), vo.banded_ld(100, 4, seed=6)],
                                 format="csr")
    L = BlockLD.from_csr(A1)
    G = L.regroup([300])
    eng = FakeEngine()
    G.upload(eng, 0, 0)
    np.testing.assert_array_equal(eng.csr[(0, 0)].toarray(), scipy.sparse.triu(A1).toarray())


def test_banded_ld_generator_properties():
    R = vo.banded_ld(1200, 100, seed=7)
    assert (R != R.T).nnz == 0
    np.testing.assert_allclose(R.diagonal(), 1.0, rtol=0, atol=1e-15)
    rows = np.repeat(np.arange(1200), np.diff(R.indptr))
    assert np.max(np.abs(R.indices - rows)) == 100
    assert np.linalg.eigvalsh(R.toarray()).min() > -1e-12


def test_band_cut_into_coupled_pieces():
    """One band block (one chromosome of windowed LD) is cut into pieces that
    ranks can own (sgvamp.band_cuts / BlockLD.pieces): pieces of P markers (the
    last up to 2P), consecutive ones coupled by the band's corner; the pieces'
    diagonal blocks plus the couplings (and their transposes) are the matrix
    itself.  The cut is a function of the matrix only: no rank count enters."""
    from sgvamp import BAND_CUT_MAX_BW, band_cuts

    A = vo.banded_ld(70_000, 600, seed=9, taps=12)
    L = BlockLD.from_csr(A)
    assert L.band_width(0) == 600
    cuts = band_cuts([L], L.block_sizes, piece=16384)
    assert cuts == [[16384, 16384, 16384, 70_000 - 3 * 16384]]
    P, cpl = L.pieces(cuts)
    assert P.block_sizes == cuts[0] and sorted(cpl) == [0, 1, 2]
    offs = np.cumsum([0] + P.block_sizes)
    B = scipy.sparse.block_diag([P.block_csr(k) for k in range(4)], format="lil")
    for gb, (nr, nc, C) in cpl.items():
        assert (nr, nc) == (600, 600)
        cut = offs[gb + 1]
        B[cut - nr:cut, cut:cut + nc] = C
        B[cut:cut + nc, cut - nr:cut] = C.T
    assert abs(B.tocsr() - A).max() == 0.0
    # not cut: too short, too wide a band, or no piece length
    assert band_cuts([L], L.block_sizes, piece=65536) == [[70_000]]
    assert band_cuts([L], L.block_sizes, piece=2048) == [[70_000]]          # bw > piece / 4
    W = BlockLD.from_csr(vo.banded_ld(40_000, BAND_CUT_MAX_BW + 8, seed=1, taps=4))
    assert band_cuts([W], W.block_sizes, piece=16384) == [[40_000]]         # bw > 4,096
    assert band_cuts([L], L.block_sizes, piece=0) == [[70_000]]
    # dense sources are never cut
    D = BlockLD(blocks=[np.eye(2)])
    assert band_cuts([D], D.block_sizes, piece=1) == [[2]]


def test_product_windowed_ld_matches_the_oracle_generator():
    """bench --band builds its LD with simulate.windowed_ld (product side); the
    oracle's banded_ld is the same recipe, so band parity tests and the band
    bench run the same matrices."""
    from simulate import windowed_ld

    for M, bw, taps in ((3000, 40, 12), (5000, 300, 4)):
        A = windowed_ld(M, bw, seed=3, taps=taps)
        B = vo.banded_ld(M, bw, seed=3, taps=taps)
        assert A.nnz == B.nnz
        assert abs(A - B).max() == 0.0


def test_bench_band_problem_shapes():
    import bench

    class Args:
        band, seed, nsamp = "4000,50", 2, 10_000

    A, r, x0, cm = bench.band_problem(Args, 3)
    assert A.shape == (4000, 4000) and r.shape == (3, 4000) and x0.shape == (4000,)
    assert cm == 200 and np.count_nonzero(x0) == cm


def test_fewer_pieces_than_ranks_is_refused_with_a_hint(tmp_path):
    """Ranks own whole LD blocks / band pieces: a chromosome cut into 2 pieces
    cannot run on 3 ranks -- refused before any device work, naming the
    piece-length switch (the cut itself never depends on the rank count)."""
    import scipy.sparse  # noqa: F401
    from comm import SingleComm
    from sgvamp import VAMP

    class ThreeRanks(SingleComm):
        def Get_size(self):
            return 3

    M = 150_000
    A = vo.banded_ld(M, 300, seed=4, taps=4)
    L = BlockLD.from_csr(A)
    v = VAMP(N=1000, Nt=1000, M=M, K=1, rho=0.5, gamw=1.0, gam1=1e-6, a=[1.0],
             prior_vars=[0.0, 1e-3], prior_probs=[0.9, 0.1], out_dir=str(tmp_path),
             out_name="x", comm=ThreeRanks(), write_files=False)
    with pytest.raises(ValueError, match=r"2 LD block\(s\) cannot be spread over 3 ranks.*SGV_BAND_PIECE"):
        v._setup(L, np.zeros(M), None)
