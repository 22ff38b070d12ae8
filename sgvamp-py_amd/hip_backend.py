"""ctypes binding of libsgvamp_hip.so (C ABI declared in include/sgvamp_hip.h).

There is no CPU fallback: if the library or a HIP device is missing, every entry
point raises.  Build the library with ``make -C sgvamp-py_amd/csrc`` (or
``python -c "import __graft_entry__ as g; g.build()"``).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsgvamp_hip.so")   # the in-tree build, nothing else

SGV_OK = 0
VEC_R, VEC_R1, VEC_XHAT1, VEC_XHAT2, VEC_SIG2U, VEC_X0 = range(6)
LMMSE_NOUT = 8
O_TRSIGMA2, O_ALPHA2, O_GAM1, O_Z, O_TRRSIGMA2, O_GAMW, O_XR, O_XRX = range(8)
STEP_EM, STEP_DENOISE_DAMP, STEP_ALPHA1_DAMP, STEP_LMMSE_DAMP, STEP_LEARN_GAMW, STEP_METRICS, \
    STEP_CHAIN, STEP_MLE = 1, 2, 4, 8, 16, 32, 64, 128
MLE_NOT_CONVERGED, MLE_NEGATIVE = 1, 2
OUT_SLOTS = 3
MAX_COHORTS = 1024
MAX_SLABS = 8
ABI_VERSION = 2          # the header's SGV_ABI_VERSION this binding is typed against
TIMERS_N, EXCHANGE_STATS_N, COMM_INFO_N = 10, 16, 5

_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_i64_p = ctypes.POINTER(ctypes.c_int64)
_c_dbl_p = ctypes.POINTER(ctypes.c_double)
_c_i8_p = ctypes.POINTER(ctypes.c_int8)
_vp = ctypes.c_void_p

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "sgv_create": [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_int_p, ctypes.c_int, _c_i64_p,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(_vp)],
    "sgv_destroy": [_vp],
    "sgv_last_error": [_vp],
    "sgv_comm_unique_id": [ctypes.c_char_p],
    "sgv_comm_init": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _c_int_p],
    "sgv_comm_init_host": [_vp, ctypes.c_int, ctypes.c_int, _c_int_p, ctypes.c_void_p, _vp],
    "sgv_set_mfma_min": [_vp, ctypes.c_int],
    "sgv_set_cg_pipeline": [_vp, ctypes.c_int],
    "sgv_set_cg_exact": [_vp, ctypes.c_int],
    "sgv_set_rs_recurrence": [_vp, ctypes.c_int],
    "sgv_reset_solver": [_vp],
    "sgv_outputs_begin": [_vp, ctypes.c_int],
    "sgv_outputs_wait": [_vp, ctypes.c_int, ctypes.POINTER(_c_dbl_p)],
    "sgv_mle_exp_max": [_vp, _c_dbl_p, ctypes.c_int, _c_dbl_p, _c_dbl_p],
    "sgv_mle_terms": [_vp, _c_dbl_p, _c_dbl_p, ctypes.c_int, _c_dbl_p, _c_dbl_p, ctypes.c_double,
                      _c_dbl_p],
    "sgv_mle_update": [_vp, _c_dbl_p, _c_dbl_p, ctypes.c_int, _c_dbl_p, _c_dbl_p, _c_dbl_p,
                       _c_dbl_p, _c_int_p],
    "sgv_fsolve": [ctypes.c_int, ctypes.c_void_p, _vp, _c_dbl_p, _c_dbl_p, _c_int_p],
    "sgv_set_mle_gam": [_vp, ctypes.c_double],
    "sgv_set_ld_block": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p, ctypes.c_int64],
    "sgv_get_ld_block": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p, ctypes.c_int64],
    "sgv_set_ld_block_csr": [_vp, ctypes.c_int, ctypes.c_int, _c_i64_p, _c_i64_p, _c_dbl_p],
    "sgv_set_ld_packing": [_vp, ctypes.c_int],
    "sgv_ld_block_format": [_vp, ctypes.c_int, ctypes.c_int, _c_int_p],
    "sgv_ld_stored_bytes": [_vp, ctypes.c_int, _c_dbl_p],
    "sgv_set_ld_coupling": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dbl_p],
    "sgv_set_ridge": [_vp, ctypes.c_double],
    "sgv_set_cohort_n": [_vp, ctypes.c_int, ctypes.c_double],
    "sgv_set_vector": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p],
    "sgv_get_vector": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p],
    "sgv_synth_ld_g": [_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, _c_dbl_p,
                       _c_dbl_p],
    "sgv_synth_r": [_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, _c_dbl_p],
    "sgv_denoise": [_vp, _c_dbl_p, _c_dbl_p, ctypes.c_double, ctypes.c_int, _c_dbl_p, _c_dbl_p,
                    ctypes.c_double, ctypes.c_int, _c_dbl_p],
    "sgv_em": [_vp, _c_dbl_p, _c_dbl_p, ctypes.c_int, _c_dbl_p, ctypes.c_int, _c_dbl_p, _c_dbl_p,
               _c_int_p, _c_dbl_p],
    "sgv_lmmse": [_vp, ctypes.c_int, _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_i8_p, ctypes.c_int,
                  ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int, _c_dbl_p, _c_int_p,
                  _c_int_p],
    "sgv_metrics": [_vp, _c_dbl_p],
    "sgv_metrics_begin": [_vp],
    "sgv_metrics_end": [_vp, _c_dbl_p],
    "sgv_ld_matvec": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p, _c_dbl_p],
    "sgv_cg_solve": [_vp, ctypes.c_int, ctypes.c_int, _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_dbl_p,
                     ctypes.c_int, ctypes.c_double, _c_int_p, _c_int_p],
    "sgv_abi_version": [],
    "sgv_timers": [_vp, _c_dbl_p, ctypes.c_int, ctypes.c_int],
    "sgv_exchange_stats": [_vp, _c_dbl_p, ctypes.c_int, ctypes.c_int],
    "sgv_comm_info": [_vp, _c_int_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int],
    "sgv_exchange_probe": [_vp, ctypes.c_int, _c_dbl_p],
    "sgv_em_cost_model": [ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                          _c_dbl_p],
    "sgv_step": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dbl_p, _c_dbl_p,
                 _c_dbl_p, _c_dbl_p, _c_dbl_p, ctypes.c_double, _c_dbl_p, _c_dbl_p, _c_dbl_p,
                 _c_i8_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, _c_dbl_p, _c_int_p,
                 _c_dbl_p, _c_int_p],
    "sgv_step_begin": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dbl_p,
                       _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_dbl_p, ctypes.c_double, _c_dbl_p,
                       _c_dbl_p, _c_dbl_p, _c_i8_p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                       _c_dbl_p, _c_int_p, _c_dbl_p, _c_int_p],
    "sgv_step_end": [_vp],
    "sgv_probe_draw": [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32),
                       ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _c_i8_p],
    "sgv_sync": [_vp],
    "sgv_read_bw": [_vp, ctypes.c_int64, ctypes.c_int, _c_dbl_p],
}
_RESTYPES = {"sgv_destroy": None, "sgv_last_error": ctypes.c_char_p}
EXPORTS = tuple(_SIGS)

_lib = None


class HipError(RuntimeError):
    pass


def ab_env(name):
    """A/B tuning switch from the environment, honoured only with SGV_AB=1 (as
    the library's own overrides); a set switch without it is ignored loudly."""
    v = os.environ.get(name)
    if v is None:
        return None
    if os.environ.get("SGV_AB") != "1":
        import warnings

        warnings.warn("%s=%s ignored: A/B overrides need SGV_AB=1" % (name, v))
        return None
    return v


def load(path=LIB_PATH, strict=True):
    """Load and type the library (cached).  Raises if it is absent.  strict=False
    (A/B tools loading an older build): symbols the build lacks are left untyped."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HipError("libsgvamp_hip.so not found at %s -- build it with "
                       "`make -C sgvamp-py_amd/csrc` (there is no CPU fallback)" % path)
    lib = ctypes.CDLL(path)
    for name, args in _SIGS.items():
        if not hasattr(lib, name):
            if not strict:
                continue
            raise HipError("%s does not export %s: stale build -- rebuild with "
                           "`make -C sgvamp-py_amd/csrc`" % (path, name))
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if strict and lib.sgv_abi_version() != ABI_VERSION:
        raise HipError("%s has ABI version %d, this binding expects %d: rebuild with "
                       "`make -C sgvamp-py_amd/csrc`" % (path, lib.sgv_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


FSOLVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int, _c_dbl_p, _c_dbl_p)


def fsolve(func, x0):
    """sgv_fsolve (the library's scipy.optimize.fsolve, MINPACK hybrd with
    fsolve's defaults) on a Python function: returns (x, info, nfev).  For the
    tests; the product path calls it from C (sgv_mle_update)."""
    lib = load()
    x = np.array(x0, dtype=np.float64)
    n = x.size
    err = []

    def cb(_user, nn, xp, fp):
        try:
            xv = np.ctypeslib.as_array(xp, shape=(nn,)).copy()
            fp_arr = np.ctypeslib.as_array(fp, shape=(nn,))
            fp_arr[:] = np.asarray(func(xv), dtype=np.float64)
            return 0
        except Exception as e:  # noqa: BLE001 -- reported after the solver returns
            err.append(e)
            return -1

    cfn = FSOLVE_FN(cb)
    nfev = np.zeros(1, dtype=np.int32)
    info = lib.sgv_fsolve(int(n), ctypes.cast(cfn, ctypes.c_void_p), None, dptr(x), None, iptr(nfev))
    if err:
        raise err[0]
    return x, int(info), int(nfev[0])


def dptr(a):
    return a.ctypes.data_as(_c_dbl_p)


def iptr(a):
    return a.ctypes.data_as(_c_int_p)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Context:
    """Owns one sgv_ctx (one GPU, one rank)."""

    def __init__(self, device, K, ld_of, block_sizes_local, blk0, nblk_global, M_total):
        self.lib = load()
        ld_of = np.ascontiguousarray(ld_of, dtype=np.int32)
        sizes = np.ascontiguousarray(block_sizes_local, dtype=np.int64)
        nld = int(ld_of.max()) + 1
        h = _vp()
        rc = self.lib.sgv_create(int(device), int(K), nld, iptr(ld_of), len(sizes),
                                 sizes.ctypes.data_as(_c_i64_p), int(blk0), int(nblk_global),
                                 int(M_total), ctypes.byref(h))
        if rc != SGV_OK:
            raise HipError("sgv_create failed (%d): %s" % (
                rc, self.lib.sgv_last_error(None).decode(errors="replace")))
        self.h = h
        self.K, self.nld = K, nld
        self.Mloc = int(sizes.sum())

    def check(self, rc, what):
        if rc != SGV_OK:
            msg = self.lib.sgv_last_error(self.h).decode(errors="replace")
            raise HipError("%s failed (%d): %s" % (what, rc, msg))

    def close(self):
        if self.h:
            self.lib.sgv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __getattr__(self, name):
        """ctx.sgv_xxx(args...) -> checked call with the handle prepended."""
        if not name.startswith("sgv_"):
            raise AttributeError(name)
        fn = getattr(self.lib, name)

        def call(*args):
            self.check(fn(self.h, *args), name)

        return call


class ProbeStream:
    """One cohort's Hutchinson probe stream (src/sgvamp.py:326): the legacy
    RandomState `rs`'s binomial(p=1/2, n=1) draws, advanced and sliced in C
    (sgv_probe_draw, bit for bit numpy's stream).  `rs` is not advanced."""

    def __init__(self, rs):
        name, key, pos = rs.get_state()[:3]
        if name != "MT19937":
            raise HipError("probe stream: %s is not a legacy MT19937 RandomState" % name)
        self.key = np.ascontiguousarray(key, dtype=np.uint32).copy()
        self.pos = np.array([pos], dtype=np.int32)
        self.lib = load()

    def draw(self, n, lo, hi):
        """Advance by n samples; return u[lo:hi] as int8 +-1."""
        out = np.empty(max(hi - lo, 1), dtype=np.int8)
        rc = self.lib.sgv_probe_draw(self.key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                     self.pos.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                     int(n), int(lo), int(hi), out.ctypes.data_as(_c_i8_p))
        if rc != SGV_OK:
            raise HipError("sgv_probe_draw failed (%d)" % rc)
        return out[:hi - lo]


# int fn(void* user, const double* send, double* recv, int64_t count)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double), ctypes.c_int64)


def make_allgather(comm, nranks):
    """Wrap comm.allgather_f64 as the library's host all-gather callback.  Keep
    the returned object alive for as long as the context uses it."""
    import numpy as np

    def cb(_user, send, recv, count):
        try:
            a = np.ctypeslib.as_array(send, shape=(count,)).copy()
            out = np.ctypeslib.as_array(recv, shape=(count * nranks,))
            out[:] = comm.allgather_f64(a)
            return 0
        except Exception:  # noqa: BLE001 -- reported as a nonzero status by the library
            import traceback

            traceback.print_exc()
            return 1

    return ALLGATHER_FN(cb)


def unique_id():
    lib = load()
    buf = ctypes.create_string_buffer(128)
    rc = lib.sgv_comm_unique_id(buf)
    if rc != SGV_OK:
        raise HipError("sgv_comm_unique_id failed: %s" % lib.sgv_last_error(None).decode())
    return buf.raw
