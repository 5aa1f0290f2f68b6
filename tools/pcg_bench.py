"""Per-iteration cost of the fused CG kernel on a 1080p operator with the
structure of a Classic+NL stage-2 system (random robust edge weights over
three decades, rank-1 data term).  Runs a fixed number of iterations
(rtol 0) so variants can be compared launch for launch.

usage: python tools/pcg_bench.py [--h 1080 --w 1920 --iters 200 --solver backslash]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
import numpy as np  # noqa: E402

from optical_flow import _native  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402


def operator(H, W, seed=0):
    rng = np.random.default_rng(seed)
    w = 10.0 ** rng.uniform(-1, 2, (4, H, W))
    w[0][:, -1] = 0
    w[2][:, -1] = 0
    w[1][-1, :] = 0
    w[3][-1, :] = 0
    gx, gy = rng.standard_normal((2, H, W))
    psi = rng.uniform(0.1, 10, (H, W))

    def esum(wx, wy):
        s = wx.copy()
        s[:, 1:] += wx[:, :-1]
        s += wy
        s[1:, :] += wy[:-1, :]
        return s
    coef = np.stack([w[0], w[1], w[2], w[3], psi * gx * gx + esum(w[0], w[1]), psi * gx * gy,
                     psi * gy * gy + esum(w[2], w[3])])
    rhs = rng.standard_normal((2, H, W))
    return _native.f32(coef), _native.f32(rhs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--solver", default="backslash")
    a = ap.parse_args()
    coef, rhs = operator(a.h, a.w)
    ope = load_of_method("classic+nl-fast")
    ope.solver = a.solver
    P = ope.to_params()
    P.exact_rtol = 0.0
    P.exact_maxiter = a.iters
    P.pcg_rtol = 0.0
    P.pcg_maxiter = a.iters
    ctx = _native.Context(0)
    lib = ctx.lib
    x = np.empty((2, a.h, a.w), np.float32)
    it = C.c_int()
    rr = C.c_double()
    call = lambda: ctx.check(lib.of_solve(ctx.handle, C.byref(P), _native.ptr(coef), _native.ptr(rhs), a.h, a.w,  # noqa
                                          _native.ptr(x), C.byref(it), C.byref(rr)))
    call()
    try:  # instrumented builds (CGS_PHASE_TIMING): per-role k_cgs timers
        dbg = lib.of_debug_cgs_times
    except AttributeError:
        dbg = None
    buf = (C.c_ulonglong * 12)()
    if dbg:
        dbg(buf)
    import time
    t0 = time.perf_counter()
    for _ in range(5):
        call()  # of_solve returns the host-side solution: synchronised
    wall_ms = (time.perf_counter() - t0) / 5 * 1e3
    ctx.check(lib.of_set_profiling(ctx.handle, 1))
    call()
    call()
    if dbg:
        dbg(buf)
        for r in range(4):
            w, t, n = buf[3 * r], buf[3 * r + 1], max(1, buf[3 * r + 2])
            print(json.dumps({"role": r, "work_cycles_per_wave": w / n, "barrier_wait_cycles_per_wave": t / n,
                              "waves": n}), flush=True)
    n = C.c_int(0)
    names = (C.c_char_p * 64)()
    ms = (C.c_double * 64)()
    cnt = (C.c_int64 * 64)()
    ctx.check(lib.of_kernel_times(ctx.handle, 64, names, ms, cnt, None, C.byref(n)))
    rec = {names[i].decode(): {"ms_per_launch": ms[i] / cnt[i], "launches": cnt[i]} for i in range(n.value)}
    k = rec.get("pcg_iter") or rec.get("pcg_small") or rec.get("sor_sweep")
    # whole solve (2 timed calls): every kernel of the solve
    ms_solve = sum(v["ms_per_launch"] * v["launches"] for v in rec.values()) / 2
    bpp = 76 if os.environ.get("OF_PCG_VARIANT", "2") != "1" else 92
    print(json.dumps({"variant": os.environ.get("OF_PCG_VARIANT", "default"), "waves": os.environ.get("OF_PCG_WAVES"),
                      "iters": it.value, "rel_res": rr.value, "ms_per_solve": ms_solve, "wall_ms_per_solve": wall_ms, "kernels": rec,
                      "alg_GBps_at_%dB" % bpp: bpp * a.h * a.w / (k["ms_per_launch"] * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
