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
