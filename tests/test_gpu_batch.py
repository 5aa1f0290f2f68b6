"""Device-resident batch path (bench.py / config 5): of_pair_upload/run/
download and the RCCL gather, on one GPU.

A world-size-1 RCCL communicator exercises of_rccl_init and the gather's
send/recv group; the multi-rank sharding logic around it is covered on CPU by
tests/test_dist_cpu.py (gloo, world size 2)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _params(method):
    from optical_flow.methods.config import load_of_method
    ope = load_of_method(method)
    P = ope.to_params()
    P.guide_mode = int(ope._METHOD == "classic_nl" and ope.color_images is not None)
    P.display = 0
    return P


def _run_slots(ctx, P0, n):
    from optical_flow import _abi
    for s in range(n):
        P = _abi.OfParams()
        C.memmove(C.byref(P), C.byref(P0), C.sizeof(P0))
        ctx.check(ctx.lib.of_pair_run(ctx.handle, s, C.byref(P), None))


def test_pair_slots_match_estimate_flow():
    """A slot run equals estimate_flow on the same pair (same kernels)."""
    import optical_flow
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    H, W = 60, 88
    pairs = [synth_pair(H, W, k) for k in range(3)]
    for s, (a, b, _) in enumerate(pairs):
        ctx.check(ctx.lib.of_pair_upload(ctx.handle, s, _native.ptr(_native.f32(a)), _native.ptr(_native.f32(b)),
                                         H, W, 3))
    _run_slots(ctx, _params("classic+nl-fast"), 3)
    for s, (a, b, _) in enumerate(pairs):
        uv = np.empty((2, H, W), np.float32)
        ctx.check(ctx.lib.of_pair_download(ctx.handle, s, _native.ptr(uv)))
        ref = optical_flow.estimate_flow(a, b, "classic+nl-fast")
        np.testing.assert_allclose(np.moveaxis(uv, 0, 2), ref, atol=1e-5)
    ctx.close()


def test_pairs_run_lanes_bitwise():
    """of_pairs_run: the flow of every slot is bitwise the same whether the
    slots run one after another (lanes=1), on 3 concurrent pipelines, or one
    slot per of_pair_run call; argument errors raise ValueError."""
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    lib = ctx.lib
    H, W = 72, 100
    n = 5
    for s in range(n):
        a, b, _ = synth_pair(H, W, 20 + s)
        ctx.check(lib.of_pair_upload(ctx.handle, s, _native.ptr(_native.f32(a)), _native.ptr(_native.f32(b)),
                                     H, W, 3))
    P0 = _params("classic+nl-fast")

    def flows():
        out = np.empty((n, 2, H, W), np.float32)
        for s in range(n):
            ctx.check(lib.of_pair_download(ctx.handle, s, _native.ptr(out[s])))
        return out

    _run_slots(ctx, P0, n)
    ref = flows()
    assert np.all(np.isfinite(ref)) and np.abs(ref).max() > 0.1
    for lanes in (1, 3, 8):
        ctx.check(lib.of_pairs_run(ctx.handle, n, C.byref(P0), lanes, None))
        np.testing.assert_array_equal(flows(), ref)
    with pytest.raises(ValueError):
        ctx.check(lib.of_pairs_run(ctx.handle, n + 1, C.byref(P0), 2, None))
    with pytest.raises(ValueError):
        ctx.check(lib.of_pairs_run(ctx.handle, n, C.byref(P0), 0, None))
    ctx.close()


def test_pairs_submit_slots_matches_pairs_run():
    """The pair pool over device-resident slots (of_pairs_submit_slots, the
    bench's timed form): two sets of slots queued back to back, host pairs
    interleaved in the same pool, waited out of order -- every slot's flow is
    bitwise of_pairs_run's with the same lanes, the host pairs' flows equal
    of_pairs_run_host's; bad slots raise."""
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    lib = ctx.lib
    H, W, n, lanes = 60, 88, 3, 2
    frames = [synth_pair(H, W, 40 + s)[:2] for s in range(n)]
    for k in range(2):
        for s, (a, b) in enumerate(frames):
            ctx.check(lib.of_pair_upload(ctx.handle, k * n + s, _native.ptr(_native.f32(a)),
                                         _native.ptr(_native.f32(b)), H, W, 3))
    P0 = _params("classic+nl-fast")
    ctx.check(lib.of_pairs_run(ctx.handle, n, C.byref(P0), lanes, None))
    ref = np.empty((n, 2, H, W), np.float32)
    for s in range(n):
        ctx.check(lib.of_pair_download(ctx.handle, s, _native.ptr(ref[s])))
    u8 = [(np.ascontiguousarray(a.astype(np.uint8)), np.ascontiguousarray(b.astype(np.uint8))) for a, b in frames]
    hout = [np.empty((2, H, W), np.float32) for _ in range(n)]
    vp = C.c_void_p
    p1 = (vp * n)(*[x[0].ctypes.data for x in u8])
    p2 = (vp * n)(*[x[1].ctypes.data for x in u8])
    po = (vp * n)(*[o.ctypes.data for o in hout])
    hwant = [np.empty((2, H, W), np.float32) for _ in range(n)]
    pw = (vp * n)(*[o.ctypes.data for o in hwant])
    ctx.check(lib.of_pairs_run_host(ctx.handle, n, p1, p2, H, W, 3, C.byref(P0), lanes, pw, None))
    # of_pairs_run_host released the slots' frames: upload both sets again
    for k in range(2):
        for s, (a, b) in enumerate(frames):
            ctx.check(lib.of_pair_upload(ctx.handle, k * n + s, _native.ptr(_native.f32(a)),
                                         _native.ptr(_native.f32(b)), H, W, 3))
    ctx.check(lib.of_pairs_open(ctx.handle, H, W, 3, C.byref(P0), lanes))
    try:
        t = []
        for k in range(2):
            first = C.c_int64(0)
            ctx.check(lib.of_pairs_submit_slots(ctx.handle, n, (C.c_int * n)(*range(k * n, (k + 1) * n)),
                                                C.byref(first)))
            t.append(first.value)
        th = C.c_int64(0)
        ctx.check(lib.of_pairs_submit(ctx.handle, n, p1, p2, po, C.byref(th)))
        for tk in [t[1] + 2, t[0], th.value + 1, t[1], t[0] + 1, th.value, t[1] + 1, t[0] + 2, th.value + 2]:
            ctx.check(lib.of_pairs_wait(ctx.handle, tk))
        with pytest.raises(ValueError):
            ctx.check(lib.of_pairs_submit_slots(ctx.handle, 1, (C.c_int * 1)(2 * n + 3), None))
    finally:
        ctx.check(lib.of_pairs_close(ctx.handle))
    for k in range(2):
        for s in range(n):
            uv = np.empty((2, H, W), np.float32)
            ctx.check(lib.of_pair_download(ctx.handle, k * n + s, _native.ptr(uv)))
            np.testing.assert_array_equal(uv, ref[s], err_msg=f"set {k} slot {s}")
    for s in range(n):
        np.testing.assert_array_equal(hout[s], hwant[s])
        np.testing.assert_array_equal(hwant[s], ref[s])
    ctx.close()


def test_rccl_gather_single_rank():
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    lib = ctx.lib
    H, W = 40, 56
    for s in range(2):
        a, b, _ = synth_pair(H, W, 10 + s)
        ctx.check(lib.of_pair_upload(ctx.handle, s, _native.ptr(_native.f32(a)), _native.ptr(_native.f32(b)),
                                     H, W, 3))
    _run_slots(ctx, _params("hs"), 2)
    uid = C.create_string_buffer(128)
    ctx.check(lib.of_rccl_unique_id(uid))
    ctx.check(lib.of_rccl_init(ctx.handle, uid.raw, 1, 0))
    try:
        out = np.full((2, 2, H, W), np.nan, np.float32)
        ctx.check(lib.of_rccl_gather_flows(ctx.handle, 2, _native.ptr(out)))
        for s in range(2):
            uv = np.empty((2, H, W), np.float32)
            ctx.check(lib.of_pair_download(ctx.handle, s, _native.ptr(uv)))
            np.testing.assert_array_equal(out[s], uv)
        out1 = np.full((1, 2, H, W), np.nan, np.float32)
        ctx.check(lib.of_rccl_gather_slots(ctx.handle, 1, 1, _native.ptr(out1)))
        np.testing.assert_array_equal(out1[0], out[1])
        with pytest.raises(ValueError):
            ctx.check(lib.of_rccl_gather_flows(ctx.handle, 5, None))  # more slots than uploaded
        with pytest.raises(ValueError):
            ctx.check(lib.of_rccl_gather_slots(ctx.handle, 1, 2, None))
    finally:
        lib.of_rccl_finalize(ctx.handle)
        ctx.close()


def test_rccl_gather_while_pool_computes():
    """bench.py's N > 1 pattern: step s's slots are gathered with RCCL while
    step s + 1 computes on the pool, whose lane 0 is the context itself.  The
    gather must not touch the context's arena, stream or pending solves (it
    runs on a stream of its own): every slot's flow, gathered or computed
    meanwhile, equals of_pairs_run's bitwise (single-rank communicator).
    Slot downloads work meanwhile; entries that compute on the context are
    refused (ValueError) instead of resetting lane 0's arena."""
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    lib = ctx.lib
    H, W, n, lanes = 120, 160, 3, 3
    frames = [synth_pair(H, W, 60 + s)[:2] for s in range(n)]

    def upload():
        for k in range(2):
            for s, (a, b) in enumerate(frames):
                ctx.check(lib.of_pair_upload(ctx.handle, k * n + s, _native.ptr(_native.f32(a)),
                                             _native.ptr(_native.f32(b)), H, W, 3))
    upload()
    P0 = _params("classic+nl-fast")
    ctx.check(lib.of_pairs_run(ctx.handle, n, C.byref(P0), lanes, None))
    ref = np.empty((n, 2, H, W), np.float32)
    for s in range(n):
        ctx.check(lib.of_pair_download(ctx.handle, s, _native.ptr(ref[s])))
    upload()
    uid = C.create_string_buffer(128)
    ctx.check(lib.of_rccl_unique_id(uid))
    ctx.check(lib.of_rccl_init(ctx.handle, uid.raw, 1, 0))
    from optical_flow import _abi
    nr = C.c_int64(0)
    ctx.check(lib.of_get_option(ctx.handle, _abi.OF_OPT_RCCL_NRANKS, C.byref(nr)))
    assert nr.value == 1  # RCCL's own count (ncclCommCount)
    sets = [(C.c_int * n)(*range(k * n, (k + 1) * n)) for k in range(2)]
    gathered = []
    try:
        ctx.check(lib.of_pairs_open(ctx.handle, H, W, 3, C.byref(P0), lanes))
        try:
            first = []
            for step in range(4):
                t = C.c_int64(0)
                ctx.check(lib.of_pairs_submit_slots(ctx.handle, n, sets[step % 2], C.byref(t)))
                first.append(t.value)
                if step:
                    prev = step - 1
                    for tk in range(first[prev], first[prev] + n):
                        ctx.check(lib.of_pairs_wait(ctx.handle, tk))
                    out = np.full((n, 2, H, W), np.nan, np.float32)
                    ctx.check(lib.of_rccl_gather_slots(ctx.handle, (prev % 2) * n, n, _native.ptr(out)))
                    gathered.append(out)
                    # slot copies are pool-safe too; compute entries refuse
                    uv = np.empty((2, H, W), np.float32)
                    ctx.check(lib.of_pair_download(ctx.handle, (prev % 2) * n + 1, _native.ptr(uv)))
                    np.testing.assert_array_equal(uv, ref[1])
                    with pytest.raises(ValueError):
                        ctx.check(lib.of_pair_run(ctx.handle, 0, C.byref(P0), None))
            for tk in range(first[3], first[3] + n):
                ctx.check(lib.of_pairs_wait(ctx.handle, tk))
        finally:
            ctx.check(lib.of_pairs_close(ctx.handle))
        for out in gathered:
            np.testing.assert_array_equal(out, ref)
        for k in range(2):
            for s in range(n):
                uv = np.empty((2, H, W), np.float32)
                ctx.check(lib.of_pair_download(ctx.handle, k * n + s, _native.ptr(uv)))
                np.testing.assert_array_equal(uv, ref[s])
    finally:
        lib.of_rccl_finalize(ctx.handle)
        ctx.close()


@pytest.mark.parametrize("lanes,n,H,W", [(1, 3, 60, 88), (2, 5, 60, 88), (3, 4, 270, 480), (3, 3, 540, 960)])
def test_pairs_run_host_matches_estimate_flow(lanes, n, H, W):
    """of_pairs_run_host (uint8 frames in host memory -> flows in host
    memory, uploads/downloads overlapped on copy streams) equals
    estimate_flow on every pair bitwise (same kernels; the bytes path
    computes gray/Lab from the same integer values), for any lane count;
    the flows also stay in device slots 0..n-1.  At 540x960 three lanes run
    3 x 504 k_cgs blocks at once, more than the 512 that are resident: the
    ping-ponged CG partials must keep every lane's result exact."""
    import optical_flow
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    pairs = [synth_pair(H, W, 10 + k) for k in range(n)]
    a = [p[0].astype(np.uint8) for p in pairs]
    b = [p[1].astype(np.uint8) for p in pairs]
    got = optical_flow.estimate_flow_batch(a, b, "classic+nl-fast", lanes=lanes)
    for k in range(n):
        ref = optical_flow.estimate_flow(pairs[k][0], pairs[k][1], "classic+nl-fast")
        assert np.array_equal(got[k], ref), (k, np.abs(got[k] - ref).max())
    ctx = _native.context()
    uv = np.empty((2, H, W), np.float32)
    ctx.check(ctx.lib.of_pair_download(ctx.handle, n - 1, _native.ptr(uv)))
    assert np.array_equal(np.moveaxis(uv, 0, 2), got[n - 1])
    with pytest.raises(ValueError):
        optical_flow.estimate_flow_batch([a[0] + 0.5], [b[0]])


def test_pairs_run_host_fine_solves_side_by_side():
    """Lanes mode at 1080p: two fine solves hold the token's two slots at
    once, each with 252 k_cgs blocks (CGS_LANES_BLOCKS) instead of a single
    estimate_flow's 504, so the band geometry and the CG partial-sum order
    differ; both meet the 1e-6 true residual, so the flows agree to CG
    rounding (measured below), and lane counts >= 2 agree bitwise."""
    import optical_flow
    from optical_flow.utils.synthetic import synth_pair
    pairs = [synth_pair(1080, 1920, 40 + k) for k in range(3)]
    a = [p[0].astype(np.uint8) for p in pairs]
    b = [p[1].astype(np.uint8) for p in pairs]
    got2 = optical_flow.estimate_flow_batch(a, b, "classic+nl-fast", lanes=2)
    got3 = optical_flow.estimate_flow_batch(a, b, "classic+nl-fast", lanes=3)
    for k in range(3):
        assert np.array_equal(got2[k], got3[k]), k
    ref = optical_flow.estimate_flow(pairs[0][0], pairs[0][1], "classic+nl-fast")
    # the documented contract (include/optflow.h, of_pairs_run_host): one
    # lane keeps estimate_flow's single-solve geometry, bitwise
    got1 = optical_flow.estimate_flow_batch(a[:1], b[:1], "classic+nl-fast", lanes=1)
    assert np.array_equal(got1[0], ref)
    e = np.sqrt(((got2[0] - ref) ** 2).sum(-1))
    aepe = lambda uv: float(np.sqrt(((uv - pairs[0][2]) ** 2).sum(-1)).mean())  # noqa: E731
    print(f"lanes vs single 1080p: mean {e.mean():.2e} p99 {np.percentile(e, 99):.2e} "
          f"dAEPE {abs(aepe(got2[0]) - aepe(ref)):.2e}")
    assert e.mean() < 1e-3 and abs(aepe(got2[0]) - aepe(ref)) < 1e-4


def test_pool_refuses_settings_and_busy_slots():
    """While a pair stream is open (lane 0 = the context), the settings and
    profiling calls the lanes read are refused, and a slot queued in the
    stream cannot be submitted again, re-uploaded or downloaded until its
    ticket is done (a re-upload could free the frames under a
    running lane).  One lane, two 540x960 pairs: the second pair waits
    behind the first for tens of ms, inside which every check runs."""
    from optical_flow import _abi, _native
    from optical_flow.utils.synthetic import synth_pair
    ctx = _native.Context(0)
    lib = ctx.lib
    H, W = 540, 960
    a, b = synth_pair(H, W, 5)[:2]
    fa, fb = _native.f32(a), _native.f32(b)
    for s in range(2):
        ctx.check(lib.of_pair_upload(ctx.handle, s, _native.ptr(fa), _native.ptr(fb), H, W, 3))
    P0 = _params("classic+nl-fast")
    slots = (C.c_int * 2)(0, 1)
    dup = (C.c_int * 2)(0, 0)
    ctx.check(lib.of_pairs_open(ctx.handle, H, W, 3, C.byref(P0), 1))
    try:
        with pytest.raises(ValueError):
            ctx.check(lib.of_pairs_submit_slots(ctx.handle, 2, dup, None))
        t = C.c_int64(0)
        ctx.check(lib.of_pairs_submit_slots(ctx.handle, 2, slots, C.byref(t)))
        uv = np.empty((2, H, W), np.float32)
        with pytest.raises(ValueError, match="queued"):
            ctx.check(lib.of_pairs_submit_slots(ctx.handle, 1, (C.c_int * 1)(1), None))
        with pytest.raises(ValueError, match="queued"):
            ctx.check(lib.of_pair_upload(ctx.handle, 1, _native.ptr(fa), _native.ptr(fb), H, W, 3))
        with pytest.raises(ValueError, match="queued"):
            ctx.check(lib.of_pair_download(ctx.handle, 1, _native.ptr(uv)))
        n = C.c_int(0)
        for call in (lambda: lib.of_set_option(ctx.handle, _abi.OF_OPT_FUSED_WARP, 0),
                     lambda: lib.of_set_profiling(ctx.handle, 1),
                     lambda: lib.of_set_solve_log(ctx.handle, 1),
                     lambda: lib.of_kernel_times(ctx.handle, 0, None, None, None, None, C.byref(n)),
                     lambda: lib.of_kernel_timeline(ctx.handle, 0, None, None, None, None, C.byref(n))):
            with pytest.raises(ValueError, match="pair stream is open"):
                ctx.check(call())
        for tk in (t.value, t.value + 1):
            ctx.check(lib.of_pairs_wait(ctx.handle, tk))
        # done: the slot is free again
        ctx.check(lib.of_pair_download(ctx.handle, 1, _native.ptr(uv)))
        ctx.check(lib.of_pairs_submit_slots(ctx.handle, 1, (C.c_int * 1)(1), C.byref(t)))
        ctx.check(lib.of_pairs_wait(ctx.handle, t.value))
    finally:
        ctx.check(lib.of_pairs_close(ctx.handle))
    ctx.check(lib.of_set_option(ctx.handle, _abi.OF_OPT_FUSED_WARP, 1))
    v = C.c_int64(-1)
    ctx.check(lib.of_get_option(ctx.handle, _abi.OF_OPT_RCCL_NRANKS, C.byref(v)))
    assert v.value == 0  # no communicator on this context
