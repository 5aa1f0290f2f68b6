"""Why are of_pairs_run steps slower after a pair pool ran on the same
context?  Times K steps of of_pairs_run (8 1080p pairs, 4 lanes) on a fresh
context, then after of_pairs_open/submit_slots/close on that context, then
on a second fresh context; and the device-slot pool itself on a fresh
context.  usage: python tools/order_probe.py [K]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
import numpy as np  # noqa: E402

from optical_flow import _native  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
H, W, NP, LANES = 1080, 1920, 8, 4
ope = load_of_method("classic+nl-fast")
P0 = ope.to_params()
P0.guide_mode = 1
P0.display = 0
frames = [synth_pair(H, W, s)[:2] for s in range(NP)]


def new_ctx(nsets=1):
    ctx = _native.Context(0)
    for k in range(nsets):
        for s, (a, b) in enumerate(frames):
            ctx.check(ctx.lib.of_pair_upload(ctx.handle, k * NP + s, _native.ptr(_native.f32(a)),
                                             _native.ptr(_native.f32(b)), H, W, 3))
    return ctx


def run_steps(ctx, k):
    ctx.check(ctx.lib.of_pairs_run(ctx.handle, NP, C.byref(P0), LANES, None))  # warm-up
    ctx.check(ctx.lib.of_synchronize(ctx.handle))
    t = time.perf_counter()
    for _ in range(k):
        ctx.check(ctx.lib.of_pairs_run(ctx.handle, NP, C.byref(P0), LANES, None))
    ctx.check(ctx.lib.of_synchronize(ctx.handle))
    return NP * k / (time.perf_counter() - t)


def pool_steps(ctx, k):
    lib = ctx.lib
    ctx.check(lib.of_pairs_open(ctx.handle, H, W, 3, C.byref(P0), LANES))
    sets = [(C.c_int * NP)(*range(j * NP, (j + 1) * NP)) for j in range(2)]

    def sub(s):
        t = C.c_int64(0)
        ctx.check(lib.of_pairs_submit_slots(ctx.handle, NP, sets[s % 2], C.byref(t)))
        return t.value

    def wait(t0):
        for t in range(t0, t0 + NP):
            ctx.check(lib.of_pairs_wait(ctx.handle, t))
    wait(sub(0))
    t = time.perf_counter()
    prev = sub(0)
    for s in range(1, k):
        cur = sub(s)
        wait(prev)
        prev = cur
    wait(prev)
    r = NP * k / (time.perf_counter() - t)
    ctx.check(lib.of_pairs_close(ctx.handle))
    return r


out = {}
a = new_ctx(1)
out["run_fresh_ctx"] = run_steps(a, K)
out["run_fresh_ctx_again"] = run_steps(a, K)
b = new_ctx(2)
out["pool_fresh_ctx"] = pool_steps(b, K)
out["run_after_pool_same_ctx"] = run_steps(b, K)
out["run_first_ctx_after_pool"] = run_steps(a, K)
c = new_ctx(2)
out["run_third_ctx_16slots"] = run_steps(c, K)
out["pool_third_ctx_after_run"] = pool_steps(c, K)
out["run_third_ctx_after_its_pool"] = run_steps(c, K)
d = new_ctx(1)
out["run_new_ctx_after_pools"] = run_steps(d, K)
out["run_after_pool_same_ctx_again"] = run_steps(b, K)
print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)
