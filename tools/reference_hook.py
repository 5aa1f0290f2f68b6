"""The reference-side binding: what a maintainer of
jordanshivers/optical-flow-python would add to route `estimate_flow`
(interface.py:11-71) to liboptflow.so through ctypes.  This repository's
package is the drop-in (same name `optical_flow`, same registry and attribute
bag), so the hook takes the method object from `optical_flow.load_of_method`,
applies `params` with the reference's own `parse_input_parameter` semantics
('lambda' -> lambda_, unknown keys ignored, dict or flat [key, val, ...];
base.py:65-85), flattens it with `to_params()` into the C ABI's of_params
(include/optflow.h) and calls `of_estimate_flow`.  tests/test_api_cpu.py runs
the parameter handling below.

    OPTFLOW_BACKEND=mi355x  ->  interface.estimate_flow():
        from optical_flow._mi355x import estimate_flow as _gpu   # this file
        return _gpu(im1, im2, method, params)
"""
import ctypes as C
import os

import numpy as np

from optical_flow import _abi
from optical_flow.methods.config import load_of_method

_fp = C.POINTER(C.c_float)


def params_for(method, params=None):
    """(method object, of_params) for estimate_flow(..., method, params)."""
    ope = load_of_method(method)  # ValueError on an unknown name, as the reference
    if params is not None:
        ope.parse_input_parameter(params)
    P = ope.to_params()
    return ope, P


def load_lib(path=None):
    path = path or os.environ.get("OPTFLOW_LIB") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "optical-flow-python_amd", "optical_flow", "_lib",
        "liboptflow.so")
    lib = C.CDLL(path)
    lib.of_last_error.restype = C.c_char_p
    lib.of_last_error.argtypes = [C.c_void_p]
    if lib.of_abi_version() != _abi.OF_ABI_VERSION:
        raise RuntimeError("liboptflow.so ABI version mismatch")
    return lib


def estimate_flow(im1, im2, method="classic+nl-fast", params=None, lib=None):
    """interface.py:11-71 on the GPU: (H, W, 2) float64 flow."""
    lib = lib or load_lib()
    im1 = np.asarray(im1, dtype=float)
    im2 = np.asarray(im2, dtype=float)
    ope, P = params_for(method, params)
    if im1.ndim == 3 and im1.shape[2] < 3:
        raise NotImplementedError("1-2 channel stacks go through optical_flow.estimate_flow")
    H, W = im1.shape[:2]
    Cn = 3 if im1.ndim == 3 else 1
    a = np.ascontiguousarray(im1[..., :3] if Cn == 3 else im1, np.float32)
    b = np.ascontiguousarray(im2[..., :3] if Cn == 3 else im2, np.float32)
    # colour-guided weighted median for Classic+NL (interface.py:49-64)
    P.guide_mode = int(ope._METHOD == "classic_nl" and Cn == 3)
    ctx = C.c_void_p()
    rc = lib.of_ctx_create(0, C.byref(ctx))
    if rc != 0:
        raise RuntimeError(lib.of_last_error(None).decode())
    try:
        out = np.empty((2, H, W), np.float32)
        rc = lib.of_estimate_flow(ctx, C.byref(P), a.ctypes.data_as(_fp), b.ctypes.data_as(_fp), H, W, Cn, None,
                                  out.ctypes.data_as(_fp), None)
        if rc != 0:
            msg = lib.of_last_error(ctx).decode()
            raise (ValueError if rc == _abi.OF_EINVAL else NotImplementedError if rc == _abi.OF_ENOTSUP
                   else RuntimeError)(msg)
    finally:
        lib.of_ctx_destroy(ctx)
    return np.moveaxis(out, 0, 2).astype(np.float64)
