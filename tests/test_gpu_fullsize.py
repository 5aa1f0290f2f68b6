"""Full-size GPU parity for BASELINE.json configs 2-4.

Each case runs `estimate_flow` on `synth_pair(H, W, 0)` at the config's size
and compares with the reference's own output on the same input, generated in
the build container by `tests/golden/gen_golden.py full480sor|full720|
full1080pcg|full1080` (uv stored subsampled, AEPE against the analytic
ground truth on the full field):

  config 2  'hs'              640x480,   solver 'sor'  (hs.py:49-99, base.py:138-172)
  config 3  'classic-c'       1280x720,  solver 'pcg'  (ba.py:57-138, base.py:116-136)
  config 4  'classic+nl-fast' 1920x1080, solver 'pcg' and the default 'backslash'
                                                        (classic_nl.py:89-198, base.py:87-114)

Gates are the north-star ones (|dAEPE| <= 1e-3 against the reference's AEPE)
plus EPE-to-reference statistics on the stored samples, with per-case
tolerances written next to each case (fp32 vs the reference's float64: CG at
rtol 1e-3 / SOR at tol 1e-2 stop at a different iterate when the arithmetic
differs, so those solvers' outputs differ by more than the tight 'backslash'
surrogate's).  The 1080p default-solver case also logs the fp64 TRUE relative
residual ||b - A x|| / ||b|| of every solve (of_solve_log) next to the CG
recurrence's own estimate.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, epe_stats

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _aepe(uv, gt):
    return float(np.sqrt(((uv - gt) ** 2).sum(-1)).mean())


# name -> (fixture, H, W, method, params, sub, (mean, median, p99) EPE-to-reference gates)
CASES = {
    "cfg2_hs_sor_480": ("ref480_hs_sor_sub2.npz", 480, 640, "hs", {"solver": "sor"}, 2,
                        (1e-3, 5e-5, 1e-2)),  # measured 2.0e-4 / 4.7e-6 / 2.2e-3
    # charbonnier GNC is chaotic: the reference itself moves by 8.1e-3 / 5.8e-3 /
    # 4.1e-2 under a 1e-12 perturbation of frame 1 (chaos720.npz); measured
    # GPU 9.1e-3 / 6.6e-3 / 4.2e-2, gated at ~2x the reference's own spread
    "cfg3_classic_c_pcg_720": ("ref720_classic_c_pcg_sub4.npz", 720, 1280, "classic-c", {"solver": "pcg"}, 4,
                               (1.6e-2, 1.2e-2, 8e-2)),
    "cfg4_classic_nl_fast_pcg_1080": ("ref1080_pcg_sub4.npz", 1080, 1920, "classic+nl-fast", {"solver": "pcg"}, 4,
                                      (1e-3, 2e-4, 1e-2)),  # measured 2.3e-4 / 4.6e-5 / 2.9e-3
    # the reference's own default solver (spsolve) at 1080p, 2 h on the build host
    "cfg4_classic_nl_fast_1080": ("ref1080_backslash_sub4.npz", 1080, 1920, "classic+nl-fast", None, 4,
                                  (6e-4, 1.2e-4, 8e-3)),  # measured 2.0e-4 / 3.7e-5 / 2.8e-3, |dAEPE| 9.9e-6
}


def _run(method, params, H, W, log=False):
    import optical_flow
    from optical_flow import _native
    from optical_flow.utils.synthetic import synth_pair
    im1, im2, gt = synth_pair(H, W, 0)
    ctx = _native.context()
    ctx.set_solve_log(log)
    try:
        uv = optical_flow.estimate_flow(im1, im2, method, params)
        recs = ctx.solve_log() if log else []
    finally:
        ctx.set_solve_log(False)
    return uv, gt, recs


@pytest.mark.parametrize("case", list(CASES))
def test_fullsize_vs_reference(case):
    fix, H, W, method, params, sub, (g_mean, g_med, g_p99) = CASES[case]
    path = os.path.join(GOLDEN, fix)
    if not os.path.exists(path):
        pytest.skip(f"{fix} not generated (gen_golden.py)")
    d = dict(np.load(path))
    uv, gt, recs = _run(method, params, H, W, log=params is None)
    assert uv.shape == (H, W, 2) and np.all(np.isfinite(uv))
    ref = d[f"uv_sub{sub}"].astype(np.float64)
    s = epe_stats(uv[::sub, ::sub], ref)
    a_gpu, a_ref = _aepe(uv, gt), float(d["aepe_gt"])
    print(f"{case}: AEPE gpu {a_gpu:.6f} ref {a_ref:.6f} d {a_gpu - a_ref:+.2e}  EPE-to-ref {s}")
    if recs:
        fine = [r for r in recs if r["h"] * r["w"] >= H * W // 2]
        worst = max(r["true_rel"] for r in fine)
        print(f"  {len(recs)} solves; finest-level true rel residual max {worst:.3e}; per solve "
              + ", ".join(f"{r['h']}x{r['w']}:{r['iters']}it true {r['true_rel']:.2e} est {r['est_rel']:.2e} "
                          f"out {r['true_rel_out']:.2e}" for r in fine))
        # the 'backslash' surrogate stops at rtol 1e-6: with its residual
        # replacement the solver's iterate must meet that in the fp64 true
        # residual; the returned fp32 x adds its rounding (~2e-6 floor)
        assert worst <= 1.5e-6, worst  # measured max 9.9e-7
        assert max(r["true_rel_out"] for r in fine) <= 3e-6  # measured max 1.44e-6
    assert abs(a_gpu - a_ref) <= 1e-3, (a_gpu, a_ref)
    assert s["mean"] <= g_mean and s["median"] <= g_med and s["p99"] <= g_p99, s
    if case.startswith("cfg3"):
        ch = dict(np.load(os.path.join(GOLDEN, "chaos720.npz")))
        print(f"  reference's own spread under a 1e-12 perturbation: mean {float(ch['mean']):.2e} "
              f"median {float(ch['median']):.2e} p99 {float(ch['p99']):.2e}")
        assert s["mean"] <= 2 * float(ch["mean"]) and s["median"] <= 2 * float(ch["median"])


def test_fullsize_1080_default_solve_log():
    """Config 4 with the default solver: every solve's true fp64 residual
    (of_solve_log) within 1.5x the surrogate's rtol (1e-6) for the solver's
    iterate, within 3x for the returned fp32 x (rounding a solution of these
    systems to fp32 alone leaves ~2e-6 on robust stages: |A||x|/|b| ~ 145,
    tools/fp32_floor.py), and the AEPE against the analytic GT within 1e-3 of
    the reference's pcg run (the reference's own 'backslash' run at 1080p is
    the ref1080_backslash fixture above)."""
    d = dict(np.load(os.path.join(GOLDEN, "ref1080_pcg_sub4.npz")))
    uv, gt, recs = _run("classic+nl-fast", None, 1080, 1920, log=True)
    assert np.all(np.isfinite(uv))
    assert len(recs) == 27, len(recs)  # 7 levels x 3 + 2 GNC levels x 3
    for r in recs:
        print(f"  {r['h']}x{r['w']} iters {r['iters']} done {r['done']} true {r['true_rel']:.3e} est {r['est_rel']:.3e} "
              f"out {r['true_rel_out']:.3e}")
    assert all(r["done"] in (1, 3) for r in recs), [r for r in recs if r["done"] not in (1, 3)]
    worst = max(r["true_rel"] for r in recs)
    assert worst <= 1.5e-6, worst  # measured max 9.9e-7 (the est agrees to 4 digits)
    # solves long enough to get the residual replacement (>= 16 iterations):
    # the CG estimate tracks the true residual (measured to 4 digits); the
    # short quadratic-stage solves drift by < 10 % without it
    assert all(abs(r["true_rel"] - r["est_rel"]) <= 0.05 * r["true_rel"] for r in recs if r["iters"] >= 16)
    assert all(abs(r["true_rel"] - r["est_rel"]) <= 0.15 * r["true_rel"] for r in recs)
    assert max(r["true_rel_out"] for r in recs) <= 3e-6  # measured max 1.44e-6
    a_gpu = _aepe(uv, gt)
    print(f"AEPE gpu backslash {a_gpu:.6f}  ref pcg {float(d['aepe_gt']):.6f}")
    assert abs(a_gpu - float(d["aepe_gt"])) <= 1e-3  # measured 1.2e-5


def test_fullsize_1080_timed_geometry():
    """The path bench.py times: of_pairs_run_host on
    uint8 1080p pairs with several lanes, where the fine CG solves of two
    pairs run side by side at 252 blocks each.  Pair 0 is
    synth_pair(1080, 1920, 0), compared with the reference's own default-solver
    run (ref1080_backslash_sub4.npz) under the cfg4 gates; the other lanes'
    pairs (seeds 1..3) keep the side-by-side token busy."""
    import optical_flow
    from optical_flow.utils.synthetic import synth_pair
    d = dict(np.load(os.path.join(GOLDEN, "ref1080_backslash_sub4.npz")))
    pairs = [synth_pair(1080, 1920, s) for s in range(4)]
    a = [p[0].astype(np.uint8) for p in pairs]
    b = [p[1].astype(np.uint8) for p in pairs]
    flows = optical_flow.estimate_flow_batch(a, b, "classic+nl-fast", lanes=4)
    uv, gt = flows[0], pairs[0][2]
    assert np.all(np.isfinite(uv))
    s = epe_stats(uv[::4, ::4], d["uv_sub4"].astype(np.float64))
    a_gpu, a_ref = _aepe(uv, gt), float(d["aepe_gt"])
    print(f"timed geometry: AEPE gpu {a_gpu:.6f} ref {a_ref:.6f} d {a_gpu - a_ref:+.2e}  EPE-to-ref {s}")
    assert abs(a_gpu - a_ref) <= 1e-3
    g_mean, g_med, g_p99 = CASES["cfg4_classic_nl_fast_1080"][-1]
    assert s["mean"] <= g_mean and s["median"] <= g_med and s["p99"] <= g_p99, s


def test_fullsize_4k_largest_frame():
    """The largest frame size exercised (2160x3840, 4x config 4's pixels): the
    pyramid depth, the k_cgs band geometry (single solve and the lanes
    mode's side-by-side fine solves) and the arena sizing at 8.3 Mpx.  No
    reference run exists at this size (the reference needs hours per 1080p
    pair), so the checks are size-independent properties: every solve's fp64
    true residual within 1.5x the surrogate's rtol, the AEPE against the
    analytic ground truth of the same order as at 1080p (0.0526 there), and
    a 2-lane batch of the pair equal to estimate_flow to CG rounding."""
    import optical_flow
    from optical_flow.utils.synthetic import synth_pair
    uv, gt, recs = _run("classic+nl-fast", None, 2160, 3840, log=True)
    assert uv.shape == (2160, 3840, 2) and np.all(np.isfinite(uv))
    assert len(recs) >= 27, len(recs)
    assert all(r["done"] in (1, 3) for r in recs), [r for r in recs if r["done"] not in (1, 3)]
    worst = max(r["true_rel"] for r in recs)
    a = _aepe(uv, gt)
    print(f"4k: {len(recs)} solves, worst true residual {worst:.3e}, AEPE {a:.5f}")
    assert worst <= 1.5e-6, worst
    assert a <= 0.15, a
    im1, im2, _ = synth_pair(2160, 3840, 0)
    f = optical_flow.estimate_flow_batch([im1.astype(np.uint8)] * 2, [im2.astype(np.uint8)] * 2,
                                         "classic+nl-fast", lanes=2)
    for x in f:
        s = epe_stats(x, uv)
        print(f"4k batch vs estimate_flow: {s}")
        assert s["mean"] <= 1e-4, s
    np.testing.assert_array_equal(f[0], f[1])
