"""ctypes binding of libmcg.so (the C-ABI in include/mcg.h).

The HIP library is the only compute path: if it is missing or no GPU is visible, every
entry point raises (McgError / RuntimeError) -- there is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("MCG_LIBRARY", os.path.join(PKG_ROOT, "lib", "libmcg.so"))

MCG_OK, MCG_EINVAL, MCG_EFAIL, MCG_EDEVICE, MCG_ENOMEM, MCG_ESTATE = 0, -1, -2, -3, -4, -5
LIK_FLAT, LIK_DIAG_GAUSS, LIK_FULLCOV_GAUSS, LIK_GAUSS_SHELL, LIK_GAUSS_DATA, LIK_CAUCHY_DATA, LIK_GAUSS_MIX = range(7)
LIK_MIX_MAX = 64
PRIOR_FLAT, PRIOR_BOX, PRIOR_OPEN_BOX, PRIOR_DIAG_GAUSS = 0, 1, 2, 3
PROP_GAUSS, PROP_WRAP_UNIFORM, PROP_KD_INTERP, PROP_DE, PROP_MIXTURE = 1, 2, 3, 4, 5
MIX_GAUSS, MIX_SHIFT_UNIFORM, MIX_WRAP_UNIFORM, MIX_KD_INTERP = 1, 2, 3, 4
RJ_JUMP_GAUSS, RJ_JUMP_WRAP, RJ_JUMP_INDEP_GAUSS, RJ_JUMP_KD = 1, 2, 3, 4
FLAG_NESTED_FIXED_STOP = 1

_dp = C.POINTER(C.c_double)
_u64p = C.POINTER(C.c_uint64)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)


class McgOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32), ("seed", C.c_uint64),
                ("chain_offset", C.c_uint64), ("lanes_per_chain", C.c_int32),
                ("steps_per_launch", C.c_int32)]


class McgRunOpts(C.Structure):
    _fields_ = [("nbin", C.c_int64), ("nskip", C.c_int64), ("n_rec", C.c_int64),
                ("record_x", C.c_int32), ("record_llp", C.c_int32),
                ("record_accept", C.c_int32), ("accumulate", C.c_int32), ("append", C.c_int32)]


class McgNestedOpts(C.Structure):
    _fields_ = [("nlive", C.c_int64), ("nmcmc", C.c_int64), ("k", C.c_int64),
                ("epsrel", C.c_double), ("mode_hop", C.c_double), ("max_dead", C.c_int64)]


class McgNestedResult(C.Structure):
    _fields_ = [("log_ev", C.c_double), ("log_dev", C.c_double), ("n_dead", C.c_int64),
                ("n_total", C.c_int64), ("n_gen", C.c_int64), ("converged", C.c_int32)]


class McgRjModel(C.Structure):
    _fields_ = [("ndim", C.c_int32),
                ("lik_kind", C.c_int32), ("lik_params", _dp), ("n_lik", C.c_size_t),
                ("prior_kind", C.c_int32), ("prior_params", _dp), ("n_prior", C.c_size_t),
                ("jump_kind", C.c_int32), ("jump_params", _dp), ("n_jump", C.c_size_t),
                ("into_kind", C.c_int32), ("into_params", _dp), ("n_into", C.c_size_t),
                ("kd_pts", _dp), ("kd_M", C.c_int64), ("kd_low", _dp), ("kd_high", _dp),
                ("model_prior", C.c_double)]


class McgKernelTiming(C.Structure):
    _fields_ = [("launches", C.c_int64), ("total_ms", C.c_double), ("last_ms", C.c_double)]


OBSERVER = C.CFUNCTYPE(None, C.c_void_p, _dp, _dp, _dp, C.c_int64)

# every symbol include/mcg.h declares, with its ctypes signature
SIGNATURES = {
    "mcg_abi_version": ([], C.c_int),
    "mcg_device_arch": ([], C.c_char_p),
    "mcg_ctx_create": ([C.POINTER(C.c_void_p), C.POINTER(McgOpts)], C.c_int),
    "mcg_ctx_destroy": ([C.c_void_p], None),
    "mcg_last_error": ([C.c_void_p], C.c_char_p),
    "mcg_set_likelihood": ([C.c_void_p, C.c_int32, C.c_int32, _dp, C.c_size_t], C.c_int),
    "mcg_set_prior": ([C.c_void_p, C.c_int32, _dp, C.c_size_t], C.c_int),
    "mcg_set_proposal": ([C.c_void_p, C.c_int32, _dp, C.c_size_t], C.c_int),
    "mcg_set_kd_proposal": ([C.c_void_p, _dp, C.c_int64, _dp, _dp], C.c_int),
    "mcg_kd_info": ([C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], C.c_int),
    "mcg_kd_export": ([C.c_void_p, _i32p, _dp, _i32p, _i32p, _i32p, _dp, _dp], C.c_int),
    "mcg_init": ([C.c_void_p, C.c_int64, _dp, _dp, _dp], C.c_int),
    "mcg_get_state": ([C.c_void_p, _dp, _dp, _dp], C.c_int),
    "mcg_run": ([C.c_void_p, C.POINTER(McgRunOpts)], C.c_int),
    "mcg_get_records": ([C.c_void_p, _dp, _dp, _dp, _u64p], C.c_int),
    "mcg_last_run_steps": ([C.c_void_p], C.c_int64),
    "mcg_last_run_lanes": ([C.c_void_p], C.c_int),
    "mcg_get_counters": ([C.c_void_p, _u64p, _u64p], C.c_int),
    "mcg_reset_counters": ([C.c_void_p], C.c_int),
    "mcg_num_tiles": ([C.c_void_p], C.c_int64),
    "mcg_tile_stats": ([C.c_void_p, _dp], C.c_int),
    "mcg_tile_stats_device": ([C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)], C.c_int),
    "mcg_tile_stats_into": ([C.c_void_p, C.c_void_p], C.c_int),
    "mcg_combine_tiles": ([C.c_int32, C.c_int64, _dp, _dp, _dp, _dp], C.c_int),
    "mcg_stats": ([C.c_void_p, _dp, _dp, _dp], C.c_int),
    "mcg_nested": ([C.c_void_p, C.POINTER(McgNestedOpts), C.POINTER(McgNestedResult), OBSERVER,
                    C.c_void_p], C.c_int),
    "mcg_nested_get": ([C.c_void_p, _dp, _dp, _dp, _dp], C.c_int),
    "mcg_nested_take": ([C.c_void_p, C.POINTER(_dp), C.POINTER(_dp), C.POINTER(_dp)], C.c_int),
    "mcg_free": ([C.c_void_p], None),
    "mcg_state_token": ([C.c_void_p], C.c_uint64),
    "mcg_nested_rows_into": ([C.c_void_p, C.c_void_p, C.c_int64, C.c_int32], C.c_int),
    "mcg_log_total_error_estimate": ([C.c_double, C.c_double, C.c_int64], C.c_double),
    "mcg_set_de_proposal": ([C.c_void_p, _dp, C.c_int64, C.c_double], C.c_int),
    "mcg_posterior_samples": ([C.c_void_p, _dp, C.c_int64, C.c_int64, _i64p], C.c_int),
    "mcg_evidence_direct": ([C.c_int32, C.c_int64, _dp, _dp, _dp, C.c_int64, _dp], C.c_int),
    "mcg_evidence_lebesgue": ([C.c_int32, C.c_int64, _dp, _dp, _dp, C.c_int64, C.c_double, _dp], C.c_int),
    "mcg_write_rows": ([C.c_char_p, C.c_int32, C.c_char_p, C.c_int64, C.c_int32, _dp], C.c_int),
    "mcg_read_rows_shape": ([C.c_char_p, C.c_int64, _i64p, _i32p], C.c_int),
    "mcg_read_rows": ([C.c_char_p, C.c_int64, C.c_int64, C.c_int32, _dp, _dp, C.c_int32], C.c_int),
    "mcg_set_rjmcmc": ([C.c_void_p, C.POINTER(McgRjModel), C.POINTER(McgRjModel)], C.c_int),
    "mcg_rj_init": ([C.c_void_p, C.c_int64, C.POINTER(C.c_uint8), _dp, _dp], C.c_int),
    "mcg_rj_get_models": ([C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)], C.c_int),
    "mcg_rj_model_counts": ([C.c_void_p, _u64p, _u64p], C.c_int),
    "mcg_nested_merge": ([C.c_int32, _i64p, _i64p, _i64p, _dp, _i64p, _dp, _dp, _dp], C.c_int),
    "mcg_evidence_weights": ([C.c_int64, C.c_int64, C.c_int64, _dp, C.c_int64, _dp, _dp, _dp], C.c_int),
    "mcg_get_kernel_timing": ([C.c_void_p, C.c_char_p, C.POINTER(McgKernelTiming)], C.c_int),
    "mcg_set_timing": ([C.c_void_p, C.c_int32], C.c_int),
    "mcg_sync": ([C.c_void_p], C.c_int),
    "mcg_reseed": ([C.c_void_p, C.c_uint64], C.c_int),
    "mcg_rng_step": ([C.c_void_p], C.c_uint64),
}


class McgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("mcg error %d: %s" % (code, msg))
        self.code = code


class InvalidArgument(McgError):
    """Raised where the reference raises Invalid_argument."""


class Failure(McgError):
    """Raised where the reference raises Failure (e.g. nested.ml:70-72)."""


_lib = None


def _one_hip_runtime():
    """Keep ONE HIP runtime in the process.  The ROCm torch wheel bundles its own libamdhip64.so
    (SONAME libamdhip64.so.7) and HSA runtime; libmcg.so needs libamdhip64.so.7.  With torch
    loaded first the dynamic loader serves libmcg's dependency from torch's copy (same SONAME), so
    torch's collectives (RCCL) and libmcg share one runtime and one device address space.  With
    libmcg loaded first it maps /opt/rocm's runtime, and a later `import torch` (its libraries name
    the unversioned libamdhip64.so) maps a second HIP + HSA runtime, which then finds no GPU.  So
    torch, when installed, is imported before libmcg.so is loaded (MCG_NO_TORCH_PRELOAD=1 skips)."""
    if os.environ.get("MCG_NO_TORCH_PRELOAD"):
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libmcg.so not built (%s): run `python -c 'import __graft_entry__ as g; "
                               "g.build()'` -- there is no CPU fallback" % LIB_PATH)
        _one_hip_runtime()
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc, ctx_ptr=None):
    if rc == MCG_OK:
        return
    msg = lib().mcg_last_error(ctx_ptr).decode() if ctx_ptr else ""
    if rc == MCG_EINVAL:
        raise InvalidArgument(rc, msg)
    if rc == MCG_EFAIL:
        raise Failure(rc, msg)
    raise McgError(rc, msg)


def dptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def u64ptr(a):
    return None if a is None else a.ctypes.data_as(_u64p)


def u8ptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_uint8))


def i64ptr(a):
    return None if a is None else a.ctypes.data_as(_i64p)


def i32ptr(a):
    return None if a is None else a.ctypes.data_as(_i32p)
