"""Micro-benchmark of the weighted median kernel at 1080p (one launch per
call, HIP-event timing from the library).  Prints mean ms per launch and a
checksum of the output so variants can be compared bitwise.

usage: python tools/wmf_bench.py [--h 1080 --w 1920 --reps 5 --save out.npy]
"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
import numpy as np  # noqa: E402

from optical_flow import _native  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gc", type=int, default=3)
    ap.add_argument("--save", default=None)
    ap.add_argument("--lib", default=None, help="alternative liboptflow.so (variant builds)")
    a = ap.parse_args()
    H, W = a.h, a.w
    if a.lib:
        _native._lib = _native.load_library(a.lib)
    im1, _, gt = synth_pair(H, W, 0)
    rng = np.random.default_rng(0)
    uv = (gt + 0.05 * rng.standard_normal(gt.shape)).astype(np.float32)
    uv = _native.f32(np.moveaxis(uv, 2, 0))
    guide = _native.f32(np.moveaxis(im1, 2, 0)[: a.gc])
    occ = _native.f32(rng.uniform(0.0, 1.0, (H, W)))
    out = np.empty_like(uv)
    ctx = _native.Context(0)
    lib = ctx.lib
    args = (ctx.handle, _native.ptr(uv), _native.ptr(guide), a.gc, _native.ptr(occ), H, W, 7, 7.0, _native.ptr(out))
    ctx.check(lib.of_weighted_median(*args))  # warm-up
    ctx.check(lib.of_set_profiling(ctx.handle, 1))
    for _ in range(a.reps):
        ctx.check(lib.of_weighted_median(*args))
    n = C.c_int(0)
    names = (C.c_char_p * 64)()
    ms = (C.c_double * 64)()
    cnt = (C.c_int64 * 64)()
    ctx.check(lib.of_kernel_times(ctx.handle, 64, names, ms, cnt, None, C.byref(n)))
    rec = {names[i].decode(): ms[i] / cnt[i] for i in range(n.value)}
    print(json.dumps({"variant": a.lib or "default", "H": H, "W": W, "gc": a.gc,
                      "ms_per_launch": rec, "sha1": hashlib.sha1(out.tobytes()).hexdigest()}), flush=True)
    if a.save:
        np.save(a.save, out)


if __name__ == "__main__":
    main()
