"""INTEGRATION.md section 3 executed: the reference-side ctypes binding (the stub a
maintainer would add next to src/sgvamp.py) and the reference's infer loop
driven through it, against the reference's own golden run (k1_dense: xhat1 of
every iteration, CG counts and info, the cohort CSV scalars).  The code blocks
are taken from the document itself, so the documented binding -- its argtypes
and argument order against include/sgvamp_hip.h -- is what runs."""
import os
import re

import numpy as np
import pytest

from tests.conftest import PKG, ROOT
from tests.golden import Case


def stub_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 3. Operator seam"):text.index("## Building")]
    return re.findall(r"```python\n(.*?)```", sec, flags=re.S)


def test_integration_stub_blocks_present():
    """CPU: section 3 holds the binding and the host loop, and they compile."""
    blocks = stub_blocks()
    assert len(blocks) == 2
    assert "sgv_lmmse" in blocks[0] and "argtypes" in blocks[0]
    assert "def infer(" in blocks[1]
    for b in blocks:
        compile(b, "INTEGRATION.md", "exec")


def maxrel(a, b):
    a, b = np.asarray(a).ravel(), np.asarray(b).ravel()
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["k1_dense", "k1_blocks_csr_s_damp"])
def test_integration_stub_matches_reference_golden(name, monkeypatch):
    monkeypatch.setenv("SGVAMP_HIP_LIB", os.path.join(PKG, "libsgvamp_hip.so"))
    ns = {"__name__": "sgvamp_hip_stub"}
    for b in stub_blocks():
        exec(compile(b, "INTEGRATION.md", "exec"), ns)
    c = Case(name)
    f = c.flags
    assert c.K == 1
    if f["sparse"]:
        import scipy.sparse

        blocks = [scipy.sparse.csr_matrix(B) for B in c.ld_blocks[0]]
    else:
        blocks = c.ld_blocks[0]
    xhat1s, rows, cgs = ns["infer"](
        blocks, c.r[0] if np.ndim(c.r) == 2 else c.r, float(c.N[0]), f["s"], f["iterations"],
        f["rho"], f["gamw"], f["gam1"], f["prior_vars"], f["prior_probs"], f["seed"],
        cg_maxit=f["cg_maxit"], em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
        lmmse_damp=f["lmmse_damp"], update_prior_from=f["update_prior_from"])
    Nt = sum(c.N)
    for it in range(f["iterations"]):
        assert maxrel(xhat1s[it] / np.sqrt(Nt), c.xhat[it]) < 1e-8, it
    cg = np.array(cgs)
    np.testing.assert_array_equal(cg[:, [0, 2]], c.cg_iters[0])
    np.testing.assert_array_equal(cg[:, [1, 3]], c.cg_info[0])
    np.testing.assert_allclose(np.array(rows, dtype=np.float64), c.cohort_csv[0], rtol=1e-5, atol=0)
