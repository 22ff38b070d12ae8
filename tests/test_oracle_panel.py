"""The oracle's host LD product (test infrastructure): oracle/panel_ld.c, which
the full-size gates use, against NumPy's dense product of the same symmetric
blocks (the reference's np.dot on its .npy LD, src/main.py:199-202,
src/sgvamp.py:312), and independent of the worker count."""
import numpy as np
import pytest

from oracle import vamp_oracle as vo


@pytest.fixture(autouse=True)
def _fresh_lib():
    vo._PANEL_LIB.clear()
    yield
    vo._PANEL_LIB.clear()


def _blocks(sizes, seed=0):
    rs = np.random.RandomState(seed)
    out = []
    for n in sizes:
        X = rs.standard_normal((n, n))
        out.append((X + X.T) / 2)
    return out


@pytest.mark.parametrize("ncol", [1, 3, 8, 16])
def test_c_panel_product_vs_dense(ncol, monkeypatch):
    assert vo._panel_lib() is not None, "build first: make -C oracle"
    blocks = _blocks([700, 256, 1, 513, 4500])   # 4500: 18 panels, two ranges
    L = vo.PanelLD()
    for B in blocks:
        L.add_block(B)
    M = sum(b.shape[0] for b in blocks)
    V = np.random.RandomState(1).standard_normal((M, ncol))
    ref = np.zeros_like(V)
    off = 0
    for B in blocks:
        n = B.shape[0]
        ref[off:off + n] = B @ V[off:off + n]
        off += n
    outs = {}
    for th in ("1", "4", "8"):   # 8 > 5 blocks: the panel ranges on the inner pool
        monkeypatch.setenv("SGV_ORACLE_THREADS", th)
        outs[th] = L.matmat_R(V)
    np.testing.assert_array_equal(outs["1"], outs["4"])
    np.testing.assert_array_equal(outs["1"], outs["8"])
    # a column gives the same bits alone as with others (the batched reference
    # algebra relies on it)
    monkeypatch.setenv("SGV_ORACLE_THREADS", "4")
    np.testing.assert_array_equal(L.matmat_R(V[:, :1])[:, 0], outs["1"][:, 0])
    assert np.max(np.abs(outs["1"] - ref)) <= 1e-12 * np.max(np.abs(ref))
    monkeypatch.setenv("SGV_ORACLE_NUMPY", "1")
    vo._PANEL_LIB.clear()
    np.testing.assert_allclose(L.matmat_R(V), ref, rtol=0, atol=1e-12 * np.max(np.abs(ref)))


def test_c_panel_rejects_bad_args():
    lib = vo._panel_lib()
    assert lib is not None
    buf = np.zeros(4)
    assert lib.oracle_panel_block_matmat(4, 256, None, 17, buf.ctypes.data, buf.ctypes.data) == -1
    assert lib.oracle_panel_block_matmat(4, 512, None, 1, buf.ctypes.data, buf.ctypes.data) == -1
