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
    sizes = [4, 6, 3]
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
