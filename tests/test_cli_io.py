"""CLI input plumbing of src/main.py, restated in sgvamp-py_amd/ldio.py + main.py
(host only, no GPU)."""
import json

import numpy as np
import pytest
import scipy.sparse

from ldio import load_ld, load_r, load_true_signal, merge_bims
from main import build_parser


def write_bim(path, variants, coords):
    with open(path, "w") as f:
        for v, c in zip(variants, coords):
            f.write("1 %s 0 %d A G\n" % (v, c))


def test_merge_bims_union_sorted_by_coordinate(tmp_path):
    """src/main.py:139-141 merges on Variant only with suffixes ('', '_y') and sorts
    by cohort 0's Coordinate: variants absent from cohort 0 have NaN there and
    sort last (a reference quirk, reproduced)."""
    write_bim(tmp_path / "a.bim", ["rs1", "rs3", "rs5"], [100, 300, 500])
    write_bim(tmp_path / "b.bim", ["rs2", "rs3", "rs4"], [200, 300, 400])
    df, lists = merge_bims([str(tmp_path / "a.bim"), str(tmp_path / "b.bim")])
    assert list(df["Variant"]) == ["rs1", "rs3", "rs5", "rs2", "rs4"]
    write_bim(tmp_path / "c.bim", ["rs0", "rs3"], [50, 300])
    df, _ = merge_bims([str(tmp_path / "c.bim")])
    assert list(df["Variant"]) == ["rs0", "rs3"]
    assert lists == [["rs1", "rs3", "rs5"], ["rs2", "rs3", "rs4"]]


def test_load_r_formats(tmp_path):
    r_k = np.array([1.5, -2.0, 0.25])
    np.save(tmp_path / "r.npy", r_k)
    np.savetxt(tmp_path / "r.txt", r_k)
    with open(tmp_path / "r.linear", "w") as f:
        f.write("CHR SNP BP A1 TEST NMISS BETA STAT P\n")
        for i, b in enumerate([0.1, float("nan"), -0.3]):
            f.write("1 rs%d %d A ADD 100 %s 1 0.5\n" % (i, i, "NA" if b != b else b))
    i_map = [4, 0, 2]
    for name in ("r.npy", "r.txt"):
        r = load_r(str(tmp_path / name), 3, 100, i_map, 5)
        np.testing.assert_array_equal(r, [-2.0, 0, 0.25, 0, 1.5])
    r = load_r(str(tmp_path / "r.linear"), 3, 100, i_map, 5)
    np.testing.assert_allclose(r, [0.0, 0, -3.0, 0, 1.0])   # BETA * sqrt(N), NaN -> 0
    with pytest.raises(Exception, match="Unsupported r vector format"):
        load_r(str(tmp_path / "r.csv"), 3, 100, i_map, 5)


def _bd(sizes, seed=1):
    rs = np.random.RandomState(seed)
    M = sum(sizes)
    R = np.zeros((M, M))
    o = 0
    for n in sizes:
        X = rs.normal(size=(2 * n, n))
        R[o:o + n, o:o + n] = X.T @ X / (2 * n)
        o += n
    return R


def test_load_ld_formats(tmp_path):
    sizes = [140, 160, 130]
    R = _bd(sizes)
    np.save(tmp_path / "R.npy", R)
    scipy.sparse.save_npz(tmp_path / "R.npz", scipy.sparse.csr_matrix(R))
    offs = np.cumsum([0] + sizes)
    files = []
    for b in range(3):
        np.save(tmp_path / ("b%d.npy" % b), R[offs[b]:offs[b + 1], offs[b]:offs[b + 1]])
        files.append("b%d.npy" % b)
    with open(tmp_path / "R.blocks.json", "w") as f:
        json.dump({"block_sizes": sizes, "files": files}, f)
    for name in ("R.npy", "R.npz", "R.blocks.json"):
        L = load_ld(str(tmp_path / name), s=0.1)
        assert L.block_sizes == sizes and L.s == 0.1
        for b in range(3):
            np.testing.assert_array_equal(L.block(b), R[offs[b]:offs[b + 1], offs[b]:offs[b + 1]])
    with pytest.raises(Exception, match="Unsupported R matrix format"):
        load_ld(str(tmp_path / "R.mat"), 0.0)


def test_true_signal(tmp_path):
    x = np.array([0.5, -1.0, 2.0])
    x.tofile(tmp_path / "x.bin")
    np.save(tmp_path / "x.npy", x)
    np.testing.assert_allclose(load_true_signal(str(tmp_path / "x.bin"), 3, 4).ravel(), 2 * x)
    np.testing.assert_allclose(load_true_signal(str(tmp_path / "x.npy"), 3, 4).ravel(), 2 * x)


def test_cli_flags_and_defaults_match_reference():
    """Every flag of src/main.py:27-50 with its default."""
    p = build_parser()
    a = p.parse_args([])
    assert (a.K, a.L, a.iterations, a.prior_vars, a.prior_probs) == (1, 2, 10, "0,1", "0.99,0.01")
    assert (a.gamw, a.gam1, a.lmmse_damp, a.learn_gamw, a.rho) == (5, 0.000001, False, True, 0.5)
    assert (a.cg_maxit, a.s, a.prior_update, a.update_prior_from, a.em_prior_maxit) == (
        500, 0.0, "em", 1, 100)
    assert a.bim_files is None and a.true_signal_file is None
    a = p.parse_args(["-ld_files", "x", "--r-files", "y", "-N", "10,20", "--M", "5,5", "-K", "2",
                      "--lmmse-damp", "1", "--learn-gamw", "0", "--prior-update", "none"])
    assert (a.ld_files, a.r_files, a.N, a.M, a.K, a.lmmse_damp, a.learn_gamw,
            a.prior_update) == ("x", "y", "10,20", "5,5", "2", "1", "0", "none")


# ---------------------------------------------------------------------------
# PLINK .ld text LD (src/main.py:151-162, 203-257).  The reference's exchange
# runs over mpi4py point-to-point messages; mpi4py is absent here, so these
# expectations are derived by hand from that code (parity unpinned by a run of
# the reference), including its two quirks.
# ---------------------------------------------------------------------------
def write_ld(path, rows):
    with open(path, "w") as f:
        f.write(" CHR_A BP_A SNP_A CHR_B BP_B SNP_B R\n")
        for a, b, r in rows:
            f.write(" 1 0 %s 1 0 %s %r\n" % (a, b, r))


def test_plink_ld_exchange_two_cohorts(tmp_path):
    from ldio import load_plink_ld_all, plink_ld_sources

    names = ["A", "B", "C", "D", "E"]
    write_bim(tmp_path / "c0.bim", names, [1, 2, 3, 4, 5])
    write_bim(tmp_path / "c1.bim", ["A", "B", "C"], [1, 2, 3])
    df, lists = merge_bims([str(tmp_path / "c0.bim"), str(tmp_path / "c1.bim")])
    ref = list(df["Variant"])
    assert ref == names
    write_ld(tmp_path / "c0.ld", [("A", "B", 0.5), ("B", "E", 0.1), ("C", "D", 0.3),
                                  ("D", "E", 0.2)])
    write_ld(tmp_path / "c1.ld", [("A", "C", 0.4)])
    N = [100, 200]
    src = plink_ld_sources(ref, lists, N)
    np.testing.assert_array_equal(src[0], [0, 0, 0, 0, 0])
    np.testing.assert_array_equal(src[1], [1, 1, 1, 0, 0])      # D, E asked of cohort 0
    r = np.array([[1.0, 2, 3, 4, 5], [10.0, 20, 30, 0, 0]])
    mats, r_out = load_plink_ld_all([str(tmp_path / "c0.ld"), str(tmp_path / "c1.ld")], r, ref,
                                    lists, N)
    E0 = np.eye(5)
    for (i, j, v) in [(0, 1, 0.5), (1, 4, 0.1), (2, 3, 0.3), (3, 4, 0.2)]:
        E0[i, j] = E0[j, i] = v
    np.testing.assert_array_equal(mats[0].toarray(), E0)
    # cohort 1: own (A,C); from cohort 0 every entry touching D, then every entry
    # touching E -- (D,E) touches both, arrives twice and sums to 0.4
    E1 = np.eye(5)
    for (i, j, v) in [(0, 2, 0.4), (2, 3, 0.3), (3, 4, 0.4), (1, 4, 0.1)]:
        E1[i, j] = E1[j, i] = v
    np.testing.assert_allclose(mats[1].toarray(), E1, rtol=0, atol=1e-15)
    np.testing.assert_array_equal(r_out[0], r[0])
    np.testing.assert_array_equal(r_out[1], [10, 20, 30, 4, 5])


def test_plink_ld_exchange_source_quirk(tmp_path):
    """main.py:161-162: kx indexes the list of other cohorts holding the marker,
    and is used as a cohort id."""
    from ldio import load_plink_ld_all, plink_ld_sources

    write_bim(tmp_path / "c0.bim", ["A", "B", "C", "D"], [1, 2, 3, 4])
    write_bim(tmp_path / "c1.bim", ["A", "B", "D", "E"], [1, 2, 4, 5])
    write_bim(tmp_path / "c2.bim", ["B", "C", "D", "E"], [2, 3, 4, 5])
    df, lists = merge_bims([str(tmp_path / ("c%d.bim" % k)) for k in range(3)])
    ref = list(df["Variant"])
    assert ref == ["A", "B", "C", "D", "E"]
    N = [100, 300, 200]
    src = plink_ld_sources(ref, lists, N)
    # cohort 0 lacks E: holders [1, 2], N [300, 200] -> kx = 0 = cohort 0 itself: never asked
    np.testing.assert_array_equal(src[0], [0, 0, 0, 0, 0])
    # cohort 1 lacks C: holders [0, 2], N [100, 200] -> kx = 1 = itself
    np.testing.assert_array_equal(src[1], [1, 1, 1, 1, 1])
    # cohort 2 lacks A: holders [0, 1], N [100, 300] -> kx = 1: asks cohort 1 (holds A)
    np.testing.assert_array_equal(src[2], [1, 2, 2, 2, 2])
    write_ld(tmp_path / "c0.ld", [("A", "C", 0.6)])
    write_ld(tmp_path / "c1.ld", [("A", "B", 0.5), ("D", "E", 0.2), ("A", "D", 0.1)])
    write_ld(tmp_path / "c2.ld", [("B", "C", 0.7)])
    r = np.array([[1.0, 2, 3, 4, 0], [11.0, 12, 0, 14, 15], [0, 22.0, 23, 24, 25]])
    mats, r_out = load_plink_ld_all([str(tmp_path / ("c%d.ld" % k)) for k in range(3)], r, ref,
                                    lists, N)
    E2 = np.eye(5)
    for (i, j, v) in [(1, 2, 0.7), (0, 1, 0.5), (0, 3, 0.1)]:
        E2[i, j] = E2[j, i] = v
    np.testing.assert_array_equal(mats[2].toarray(), E2)
    np.testing.assert_array_equal(r_out[2], [11, 22, 23, 24, 25])
    np.testing.assert_array_equal(r_out[0], r[0])                # E never filled: r = 0
    assert mats[0].toarray()[4].tolist() == [0, 0, 0, 0, 1]


def test_plink_exchange_vectorised_equals_reference_loop(tmp_path):
    """The vectorised .ld exchange selects the same entries in the same order
    as the reference's per-marker table scan (oracle/ldio_oracle.py restates
    src/main.py:203-257): identical COO triplets, identical CSR (bitwise), on
    three cohorts with missing markers, pairs whose both ends are requested
    (sent twice) and self pairs."""
    import scipy.sparse

    from ldio import load_plink_ld_all, plink_ld_sources
    from oracle import ldio_oracle

    rs = np.random.RandomState(12)
    M, K = 300, 3
    ref = ["rs%d" % i for i in range(M)]
    missing = [set(), set(rs.choice(M, 40, replace=False)), set(rs.choice(M, 25, replace=False))]
    lists = [[x for i, x in enumerate(ref) if i not in missing[k]] for k in range(K)]
    N = [1000, 1500, 1200]
    tables = []
    for k in range(K):
        have = [i for i in range(M) if i not in missing[k]]
        pairs = set()
        while len(pairs) < 900:
            a, b = sorted(rs.choice(have, 2))
            if abs(a - b) < 30:
                pairs.add((a, b))
        pairs = sorted(pairs) + [(have[3], have[3])]          # a self pair
        tables.append(pairs)
        with open(tmp_path / ("c%d.ld" % k), "w") as fh:
            fh.write(" CHR_A BP_A SNP_A CHR_B BP_B SNP_B R\n")
            for a, b in pairs:
                fh.write(" 1 %d %s 1 %d %s %r\n" % (a, ref[a], b, ref[b], float(rs.uniform(-.9, .9))))
    r = rs.normal(size=(K, M))
    paths = [str(tmp_path / ("c%d.ld" % k)) for k in range(K)]
    mats, r_out = load_plink_ld_all(paths, r, ref, lists, N)
    import pandas as pd

    idx = {x: i for i, x in enumerate(ref)}
    own = []
    for p in paths:
        df = pd.read_table(p, sep=r"\s+")
        own.append(([idx[x] for x in df["SNP_A"]], [idx[x] for x in df["SNP_B"]], list(df["R"])))
    trip, r_ref = ldio_oracle.exchange(own, plink_ld_sources(ref, lists, N), r, M)
    np.testing.assert_array_equal(r_out, r_ref)
    for k in range(K):
        ind_r, ind_c, v = trip[k]
        want = scipy.sparse.csr_matrix((np.array(v), (ind_r, ind_c)), shape=(M, M))
        got = mats[k]
        assert (got != want).nnz == 0
        np.testing.assert_array_equal(got.toarray(), want.toarray())


def test_plink2np_converter(tmp_path):
    """scripts/plink2np.py:22-49: BETA -> .npy as read (NaN kept); .ld pairs ->
    CSR .npz in the .linear file's SNP order, unit diagonal, both triangles,
    a pair listed twice summed; the .npz is what --ld-files reads."""
    from plink2np import main as plink2np_main

    lin = tmp_path / "c.assoc.linear"
    with open(lin, "w") as f:
        f.write(" CHR SNP BP A1 TEST NMISS BETA STAT P\n")
        for snp, beta in [("rs3", 0.5), ("rs1", float("nan")), ("rs7", -1.25), ("rs2", 2.0)]:
            f.write(" 1 %s 0 A ADD 100 %r 0 0\n" % (snp, beta))
    write_ld(tmp_path / "c.ld", [("rs3", "rs1", 0.25), ("rs1", "rs2", -0.5), ("rs3", "rs1", 0.125)])
    plink2np_main(["--ld-file", str(tmp_path / "c.ld"), "--r-file", str(lin)])
    r = np.load(tmp_path / "c.npy")
    np.testing.assert_array_equal(r[[0, 2, 3]], [0.5, -1.25, 2.0])
    assert np.isnan(r[1])
    R = scipy.sparse.load_npz(tmp_path / "c.npz").toarray()
    E = np.eye(4)
    E[0, 1] = E[1, 0] = 0.25 + 0.125
    E[1, 3] = E[3, 1] = -0.5
    np.testing.assert_array_equal(R, E)
    L = load_ld(str(tmp_path / "c.npz"), 0.0)
    assert L.block_sizes == [4]
    np.testing.assert_array_equal(L.block(0), E)
