"""The C-ABI library loads and exports every entry point include/*.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import glob
import os
import re

import pytest

from tests.conftest import PKG, ROOT

LIB = os.path.join(PKG, "libsgvamp_hip.so")


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(sgv_\w+)\s*\(", text))
    return names


def test_header_declares_entry_points():
    names = declared_symbols()
    for must in ("sgv_create", "sgv_destroy", "sgv_lmmse", "sgv_denoise", "sgv_em",
                 "sgv_ld_matvec", "sgv_cg_solve", "sgv_comm_init", "sgv_comm_unique_id"):
        assert must in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make -C sgvamp-py_amd/csrc"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in sorted(declared_symbols()) if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    import hip_backend as hb

    assert set(hb.EXPORTS) == declared_symbols()
    hb.load()  # types every symbol


def test_binding_constants_match_header():
    """The ctypes binding's constants are the header's #defines."""
    import hip_backend as hb

    text = open(os.path.join(ROOT, "include", "sgvamp_hip.h")).read()
    defs = {m.group(1): int(m.group(2))
            for m in re.finditer(r"^#define (SGV_\w+)\s+\(?(-?\d+)\)?", text, flags=re.M)}
    pairs = {"SGV_OK": hb.SGV_OK, "SGV_MAX_COHORTS": hb.MAX_COHORTS,
             "SGV_MAX_SLABS": hb.MAX_SLABS, "SGV_LMMSE_NOUT": hb.LMMSE_NOUT,
             "SGV_ABI_VERSION": hb.ABI_VERSION, "SGV_TIMERS_N": hb.TIMERS_N,
             "SGV_EXCHANGE_STATS_N": hb.EXCHANGE_STATS_N, "SGV_COMM_INFO_N": hb.COMM_INFO_N}
    for n in ("R", "R1", "XHAT1", "XHAT2", "SIG2U", "X0"):
        pairs["SGV_VEC_" + n] = getattr(hb, "VEC_" + n)
    for n in ("TRSIGMA2", "ALPHA2", "GAM1", "Z", "TRRSIGMA2", "GAMW", "XR", "XRX"):
        pairs["SGV_O_" + n] = getattr(hb, "O_" + n)
    for n in ("EM", "DENOISE_DAMP", "ALPHA1_DAMP", "LMMSE_DAMP", "LEARN_GAMW", "METRICS", "CHAIN",
              "MLE"):
        pairs["SGV_STEP_" + n] = getattr(hb, "STEP_" + n)
    for n in ("NOT_CONVERGED", "NEGATIVE"):
        pairs["SGV_MLE_" + n] = getattr(hb, "MLE_" + n)
    for name, value in pairs.items():
        assert defs[name] == value, (name, defs[name], value)


def test_abi_version():
    """The library reports the header's ABI revision (no device needed)."""
    import hip_backend as hb

    assert hb.load().sgv_abi_version() == hb.ABI_VERSION


def test_library_is_gfx950_only():
    """The code object embedded in the library targets gfx950 and nothing else."""
    data = open(LIB, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx\w+)", data))
    assert targets == {b"gfx950"}, targets


def _hip_device_count():
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return 0
    n = ctypes.c_int(0)
    return n.value if hip.hipGetDeviceCount(ctypes.byref(n)) == 0 else 0


def test_no_cpu_fallback_without_device():
    """The product path fails loudly when no HIP device is present."""
    if _hip_device_count() > 0:
        pytest.skip("a HIP device is visible")
    import hip_backend as hb

    with pytest.raises(hb.HipError):
        hb.Context(0, 1, [0], [100], 0, 1, 100)


def test_missing_library_raises(tmp_path):
    import hip_backend as hb

    with pytest.raises(hb.HipError):
        saved = hb._lib
        hb._lib = None
        try:
            hb.load(str(tmp_path / "nope.so"))
        finally:
            hb._lib = saved


def test_product_does_not_import_oracle():
    for p in glob.glob(os.path.join(PKG, "*.py")):
        src = open(p).read()
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), p


def test_product_and_bench_do_not_import_torch():
    """PyTorch is neither the product nor its launcher: the package and bench.py
    import no torch module (the multi-rank bootstrap is comm.SocketComm)."""
    for p in glob.glob(os.path.join(PKG, "*.py")) + [os.path.join(ROOT, "bench.py")]:
        mods = re.findall(r"^\s*(?:from|import)\s+([\w.]+)", open(p).read(), flags=re.M)
        assert not [m for m in mods if m.split(".")[0] == "torch"], p


@pytest.mark.parametrize("seed", [0, 1, 2025, 987654321])
def test_probe_stream_matches_numpy_binomial(seed):
    """sgv_probe_draw (host only) reproduces src/sgvamp.py:326's
    RandomState.binomial(p=1/2, n=1, size=M)*2-1 bit for bit, stream position
    included: whole draws, rank slices, empty slices, successive iterations."""
    import numpy as np
    import hip_backend as hb

    rs = np.random.RandomState(seed)
    ps = hb.ProbeStream(np.random.RandomState(seed))
    for n, lo, hi in [(200000, 0, 200000), (12345, 100, 9000), (1, 0, 1), (0, 0, 0),
                      (77777, 77777, 77777), (5000, 0, 0), (3001, 1, 3000), (100000, 60000, 100000)]:
        ref = (rs.binomial(p=1 / 2, n=1, size=n) * 2 - 1).astype(np.int8)[lo:hi]
        np.testing.assert_array_equal(ps.draw(n, lo, hi), ref)


def test_probe_stream_odd_position():
    """A stream left at an odd 32-bit position (a 32-bit draw made before)."""
    import numpy as np
    import hip_backend as hb

    rs = np.random.RandomState(5)
    rs.randint(0, 10, dtype=np.int32)   # one 32-bit output
    ps = hb.ProbeStream(rs)
    assert ps.pos[0] % 2 == 1
    for n in (5000, 1248, 3):
        ref = (rs.binomial(p=1 / 2, n=1, size=n) * 2 - 1).astype(np.int8)
        np.testing.assert_array_equal(ps.draw(n, 0, n), ref)


def _em_costs(km, n, lat, steps):
    import numpy as np
    import hip_backend as hb

    out = np.zeros(2)
    assert hb.load().sgv_em_cost_model(km, n, lat, steps, hb.dptr(out)) == hb.SGV_OK
    return out


def test_em_cost_model_host_only():
    """The EM exchange cost model (sgv_em_cost_model, host arithmetic): the
    replicated loop's cost is one latency
    plus the r1 bytes plus the steps over all markers, the per-step loop's one
    latency per step; raising the latency moves the choice to replicated at a
    crossover the formula predicts; bad arguments are refused."""
    import hip_backend as hb

    km = 4e6   # the north star: K = 4, M = 1e6
    rep1, ps1 = _em_costs(km, 1, 25.0, 10)
    assert rep1 == pytest.approx(ps1 + 25.0 + 10 * (35.0 - 15.0 - 25.0))
    # per-step cost grows with L once per step, replicated once per loop
    rep_a, ps_a = _em_costs(km, 8, 10.0, 10)
    rep_b, ps_b = _em_costs(km, 8, 110.0, 10)
    assert rep_b - rep_a == pytest.approx(100.0)
    assert ps_b - ps_a == pytest.approx(10 * 100.0)
    # the crossover latency: rep(L*) == ps(L*), with L per step vs once
    lo, hi = 0.0, 1e4
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        r, p = _em_costs(km, 8, mid, 10)
        lo, hi = (mid, hi) if p < r else (lo, mid)
    r, p = _em_costs(km, 8, hi * 1.01, 10)
    assert r < p
    r, p = _em_costs(km, 8, lo * 0.99, 10)
    assert p < r
    # replicated bytes: 8 K M (N-1)/N at 100 GB/s
    r2, _ = _em_costs(km, 2, 0.0, 0)
    assert r2 == pytest.approx(8 * km * 0.5 / 1e5)
    out = (ctypes.c_double * 2)()
    lib = hb.load()
    assert lib.sgv_em_cost_model(km, 0, 25.0, 10, out) != hb.SGV_OK
    assert lib.sgv_em_cost_model(-1.0, 8, 25.0, 10, out) != hb.SGV_OK
    assert lib.sgv_em_cost_model(km, 8, 25.0, 10, None) != hb.SGV_OK
