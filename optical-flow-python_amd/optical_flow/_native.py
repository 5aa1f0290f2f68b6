"""ctypes binding of liboptflow.so (the HIP/gfx950 library behind include/optflow.h).

This is the only way the package computes flow: there is no CPU fallback.  If
the library is missing or no HIP device is visible, the first compute call
raises RuntimeError.
"""
import ctypes as C
import os
import threading

import numpy as np

from optical_flow._abi import (OfParams, OfStats, OfCgGeometry, OfSolveRecord, OfProgressFn, OF_ABI_VERSION,
                               OF_EINVAL, OF_ENOTSUP)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OPTFLOW_LIB", os.path.join(_HERE, "_lib", "liboptflow.so"))

_lib = None
_lock = threading.Lock()
_tls = threading.local()

_fp = C.POINTER(C.c_float)
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_vp = C.c_void_p

_SIGS = {
    "of_abi_version": ([], C.c_int),
    "of_device_count": ([_ip], C.c_int),
    "of_ctx_create": ([C.c_int, C.POINTER(_vp)], C.c_int),
    "of_ctx_destroy": ([_vp], C.c_int),
    "of_last_error": ([_vp], C.c_char_p),
    "of_synchronize": ([_vp], C.c_int),
    "of_set_profiling": ([_vp, C.c_int], C.c_int),
    "of_set_option": ([_vp, C.c_int, C.c_int], C.c_int),
    "of_get_option": ([_vp, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "of_set_progress": ([_vp, OfProgressFn, _vp, C.c_int], C.c_int),
    "of_kernel_times": ([_vp, C.c_int, C.POINTER(C.c_char_p), _dp, C.POINTER(C.c_int64), _dp, _ip], C.c_int),
    "of_kernel_timeline": ([_vp, C.c_int, C.POINTER(C.c_char_p), _dp, _dp, _dp, _ip], C.c_int),
    "of_estimate_flow": ([_vp, C.POINTER(OfParams), _fp, _fp, C.c_int, C.c_int, C.c_int, _fp, _fp,
                          C.POINTER(OfStats)], C.c_int),
    "of_compute_flow": ([_vp, C.POINTER(OfParams), _fp, C.c_int, C.c_int, C.c_int, _fp, C.c_int, _fp, _fp,
                         C.POINTER(OfStats)], C.c_int),
    "of_compute_flow_base": ([_vp, C.POINTER(OfParams), _fp, C.c_int, C.c_int, C.c_int, _fp, C.c_int,
                              C.c_double, _fp, _fp], C.c_int),
    "of_alt_ba_flow_base": ([_vp, C.POINTER(OfParams), _fp, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, _fp,
                             _fp, _fp, _fp], C.c_int),
    "of_pair_upload": ([_vp, C.c_int, _fp, _fp, C.c_int, C.c_int, C.c_int], C.c_int),
    "of_pair_run": ([_vp, C.c_int, C.POINTER(OfParams), C.POINTER(OfStats)], C.c_int),
    "of_pairs_run": ([_vp, C.c_int, C.POINTER(OfParams), C.c_int, C.POINTER(OfStats)], C.c_int),
    "of_pairs_run_host": ([_vp, C.c_int, C.POINTER(_vp), C.POINTER(_vp), C.c_int, C.c_int, C.c_int,
                           C.POINTER(OfParams), C.c_int, C.POINTER(_vp), C.POINTER(OfStats)], C.c_int),
    "of_pair_download": ([_vp, C.c_int, _fp], C.c_int),
    "of_pairs_open": ([_vp, C.c_int, C.c_int, C.c_int, C.POINTER(OfParams), C.c_int], C.c_int),
    "of_pairs_submit": ([_vp, C.c_int, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(C.c_int64)],
                        C.c_int),
    "of_pairs_wait": ([_vp, C.c_int64], C.c_int),
    "of_pairs_submit_slots": ([_vp, C.c_int, _ip, C.POINTER(C.c_int64)], C.c_int),
    "of_pairs_close": ([_vp], C.c_int),
    "of_rccl_unique_id": ([C.c_char_p], C.c_int),
    "of_rccl_init": ([_vp, C.c_char_p, C.c_int, C.c_int], C.c_int),
    "of_rccl_gather_flows": ([_vp, C.c_int, _fp], C.c_int),
    "of_rccl_gather_slots": ([_vp, C.c_int, C.c_int, _fp], C.c_int),
    "of_rccl_finalize": ([_vp], C.c_int),
    "of_preprocess": ([_vp, _fp, _fp, C.c_int, C.c_int, _fp, _fp], C.c_int),
    "of_rof_texture": ([_vp, _fp, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_double, _fp], C.c_int),
    "of_pyramid_level": ([_vp, _fp, C.c_int, C.c_int, C.c_int, _dp, C.c_int, C.c_double, _fp, _ip, _ip], C.c_int),
    "of_resample_flow": ([_vp, _fp, C.c_int, C.c_int, C.c_int, C.c_int, _fp], C.c_int),
    "of_partial_deriv": ([_vp, _fp, C.c_int, C.c_int, C.c_int, _fp, C.c_int, _dp, C.c_double, _fp, _fp, _fp],
                         C.c_int),
    "of_flow_operator": ([_vp, C.POINTER(OfParams), C.c_double, _fp, _fp, _fp, _fp, _fp, C.c_int, C.c_int,
                          C.c_int, _fp, _fp], C.c_int),
    "of_solve": ([_vp, C.POINTER(OfParams), _fp, _fp, C.c_int, C.c_int, _fp, _ip, _dp], C.c_int),
    "of_flow_operator_dia": ([_vp, C.POINTER(OfParams), C.c_double, _fp, _fp, _fp, _fp, _fp, C.c_int, C.c_int,
                              C.c_int, _ip, _fp, _fp], C.c_int),
    "of_solve_dia": ([_vp, C.POINTER(OfParams), C.c_int, _fp, _fp, C.c_int, C.c_int, _fp, _ip, _dp], C.c_int),
    "of_detect_occlusion": ([_vp, _fp, _fp, C.c_int, C.c_int, C.c_int, _fp], C.c_int),
    "of_weighted_median": ([_vp, _fp, _fp, C.c_int, _fp, C.c_int, C.c_int, C.c_int, C.c_double, _fp], C.c_int),
    "of_median_filter": ([_vp, _fp, C.c_int, C.c_int, C.c_int, C.c_int, _fp], C.c_int),
    "of_flow_to_color": ([_vp, _vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, _vp], C.c_int),
    "of_solver_geometry": ([C.c_int, C.c_int, C.c_int, C.POINTER(OfCgGeometry)], C.c_int),
    "of_set_solve_log": ([_vp, C.c_int], C.c_int),
    "of_solve_log": ([_vp, C.c_int, C.POINTER(OfSolveRecord), _ip], C.c_int),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def load_library(path=None):
    """dlopen liboptflow.so and declare every C-ABI signature.  Raises
    RuntimeError (never falls back) when the library is absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"liboptflow.so not found at {p}: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.of_abi_version() != OF_ABI_VERSION:
            raise RuntimeError("liboptflow.so ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


class NativeError(RuntimeError):
    pass


class Context:
    """One HIP device + stream (of_ctx)."""

    def __init__(self, device=0):
        self.lib = load_library()
        h = _vp()
        rc = self.lib.of_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"of_ctx_create(device={device}) failed ({rc}): no usable HIP device? "
                               "The optical_flow package runs only on the GPU.")
        self.handle = h
        self.device = device

    def check(self, rc):
        if rc == 0:
            return
        msg = self.lib.of_last_error(self.handle)
        msg = msg.decode() if msg else f"error {rc}"
        if rc == OF_EINVAL:
            raise ValueError(msg)
        if rc == OF_ENOTSUP:
            raise NotImplementedError(msg)
        raise NativeError(msg)

    def set_option(self, option, value):
        """of_set_option (include/optflow.h), e.g. OF_OPT_SOR_PIPELINE."""
        self.check(self.lib.of_set_option(self.handle, int(option), int(value)))

    def get_option(self, option):
        """of_get_option: an option's value or a read-only counter (OF_OPT_SOR_FALLBACKS)."""
        v = C.c_int64(0)
        self.check(self.lib.of_get_option(self.handle, int(option), C.byref(v)))
        return v.value

    def progress(self, fn, flags):
        """Context manager: of_set_progress(fn, flags) for the calls inside it
        (fn(OfProgress) -> None; see include/optflow.h), NULL afterwards."""
        ctx = self

        class _P:
            def __enter__(self):
                self.cb = OfProgressFn(lambda user, ev: fn(ev.contents))
                ctx.check(ctx.lib.of_set_progress(ctx.handle, self.cb, None, int(flags)))
                return self

            def __exit__(self, *exc):
                ctx.lib.of_set_progress(ctx.handle, OfProgressFn(), None, 0)
                return False
        return _P()

    def set_solve_log(self, enable=True):
        """Log the fp64 true residual of every linear solve (of_set_solve_log)."""
        self.check(self.lib.of_set_solve_log(self.handle, int(bool(enable))))

    def solve_log(self):
        """Records of the solves since set_solve_log(True) (of_solve_log)."""
        n = C.c_int(0)
        self.check(self.lib.of_solve_log(self.handle, 0, None, C.byref(n)))
        recs = (OfSolveRecord * max(1, n.value))()
        self.check(self.lib.of_solve_log(self.handle, n.value, recs, C.byref(n)))
        return [recs[i].as_dict() for i in range(n.value)]

    def close(self):
        if self.handle:
            self.lib.of_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solver_geometry(H, W, solver):
    """Launch geometry of the solver kernels for an H x W level (of_solver_geometry;
    no device needed).  Raises NotImplementedError when the level is too large."""
    from optical_flow._abi import SOLVER
    lib = load_library()
    g = OfCgGeometry()
    rc = lib.of_solver_geometry(int(H), int(W), SOLVER[solver], C.byref(g))
    if rc == OF_EINVAL:
        raise ValueError(f"bad geometry request {H}x{W} {solver}")
    if rc == OF_ENOTSUP:
        raise NotImplementedError(f"{H}x{W} is too large for the {solver} kernels")
    return {f: getattr(g, f) for f, _ in OfCgGeometry._fields_}


def context():
    """Per-thread default context on device $OPTFLOW_DEVICE (default 0)."""
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        ctx = Context(int(os.environ.get("OPTFLOW_DEVICE", "0")))
        _tls.ctx = ctx
    return ctx


# ---- numpy <-> C helpers -------------------------------------------------

def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def ptr(a):
    return None if a is None else a.ctypes.data_as(_fp)


def dptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def planar(a):
    """(H, W, C) -> contiguous float32 (C, H, W); (H, W) -> (1, H, W)."""
    a = np.asarray(a)
    if a.ndim == 2:
        return f32(a[None])
    return f32(np.moveaxis(a, 2, 0))


def interleaved(a):
    """(C, H, W) planar -> (H, W, C) float64."""
    return np.moveaxis(np.asarray(a, dtype=np.float64), 0, 2).copy()
