"""GPU end-to-end parity: estimate_flow on the GPU vs the reference outputs
(golden) and the float64 oracle.

The pipeline is non-smooth (clipping + medians), so u/v parity is stated
statistically: mean / median / p99 end-point difference to the
reference flow, and |delta AEPE| against ground truth."""
import numpy as np
import pytest

from conftest import epe_stats

pytestmark = pytest.mark.gpu

METHODS = ["classic+nl-fast", "classic+nl", "classic+nl-full", "hs-brightness", "hs", "ba-brightness", "ba",
           "classic-l", "classic-c-a", "classic-c-brightness", "classic-c", "classic++"]


def _aepe(uv, gt):
    return float(np.sqrt(((uv - gt) ** 2).sum(-1)).mean())


# Tolerances per method family: about 3-8x the mean / median EPE to the
# reference measured on the GPU (round 2, profiles/r2j_*; the kernels are
# deterministic, so a rerun reproduces those numbers exactly):
#  - stable (HS, BA-Lorentzian): float32 vs float64 only (<= 2.6e-6 / 1.3e-6);
#  - nlfast (Classic+NL-fast): 2.9e-5 / 4.4e-6 on the crop, 1.8e-4 / 1.2e-5 on
#    the synthetic pair (the weighted median amplifies single-pixel flips);
#  - nl (Classic+NL, gnc 3 with the 0.5 blend): 2.9e-3 / 4.0e-4;
#  - chaotic (classic-c*, classic++): charbonnier GNC amplifies last-bit
#    differences.  On the crop the reference itself moves by 4.7e-3 / 5.4e-3
#    px mean when its direct solve is perturbed by 1e-12 (relative).  On the
#    synthetic pair (tests/golden/chaos_synth.npz: frame 1's gray image
#    perturbed after the uint8 quantization, 3 seeds) the reference moves by
#    1.3-1.4e-2 mean / 8.7-8.8e-3 median (classic-c) and 8.6-8.9e-3 / 4.1-4.6e-3
#    (classic++) at 1e-12, and by 1.9-2.1e-2 / 1.2-1.4e-2 (classic-c) at 6e-8
#    (float32 rounding); the GPU's classic-c sits at 2.0e-2 / 1.33e-2 (round
#    3), i.e. at the reference's own float32-level spread, and
#    test_e2e_synthetic gates it at 1.5x that spread;
#  - classic-c-a: the reference diverges (|uv| ~ 3.6e36); so must we.
TOL = {"stable": (2e-5, 1e-5), "nlfast": (5e-4, 4e-5), "nl": (1e-2, 2e-3), "chaotic": (3e-2, 2e-2)}
FAMILY = {"classic+nl-fast": "nlfast", "classic+nl": "nl", "classic+nl-full": "nl", "hs-brightness": "stable",
          "hs": "stable", "ba-brightness": "stable", "ba": "stable", "classic-l": "stable",
          "classic-c-brightness": "chaotic", "classic-c": "chaotic", "classic++": "chaotic"}


@pytest.mark.parametrize("method", METHODS)
def test_e2e_small_crop(golden, method):
    import optical_flow
    d = golden("e2e_small.npz")
    uv = optical_flow.estimate_flow(d["im1"], d["im2"], method)
    if method == "classic-c-a":
        assert np.abs(d[method]).max() > 1e20
        assert (~np.isfinite(uv)).any() or np.abs(uv).max() > 1e20
        return
    s = epe_stats(uv, d[method])
    print(method, s)
    assert np.all(np.isfinite(uv))
    mean_tol, med_tol = TOL[FAMILY[method]]
    assert s["mean"] < mean_tol and s["median"] < med_tol, s


def test_e2e_gray_and_pcg(golden):
    import optical_flow
    d = golden("e2e_small.npz")
    for key, args in (("gray:classic+nl-fast", (d["gray1"], d["gray2"], "classic+nl-fast")),
                      ("gray:hs-brightness", (d["gray1"], d["gray2"], "hs-brightness"))):
        s = epe_stats(optical_flow.estimate_flow(*args), d[key])
        assert s["mean"] < 2e-2, (key, s)
    uv = optical_flow.estimate_flow(d["im1"], d["im2"], "classic+nl-fast", {"solver": "pcg"})
    assert epe_stats(uv, d["pcg:classic+nl-fast"])["mean"] < 3e-2
    uv = optical_flow.estimate_flow(d["im1"], d["im2"], "hs", {"solver": "pcg"})
    assert epe_stats(uv, d["pcg:hs"])["mean"] < 3e-2


@pytest.mark.parametrize("method", ["classic+nl-fast", "hs", "classic-c", "hs-brightness", "classic++"])
def test_e2e_synthetic(golden, method):
    """synth_pair(120, 160, 0) end to end vs the reference.  Chaotic methods
    are gated at 1.5x the reference's own spread under a float32-level (6e-8
    relative) perturbation of its gray input (max over 3 seeds,
    chaos_synth.npz).  The 1e-12 spread is printed beside; measured (round 4)
    classic-c 2.0e-2 / 1.33e-2 vs the reference's 6e-8 spread 2.1e-2 /
    1.43e-2 (1e-12: 1.4e-2 / 8.8e-3), classic++ 1.97e-2 / 1.04e-2 vs 2.0e-2 /
    9.8e-3 (1e-12: 8.9e-3 / 4.6e-3).

    What the gap is made of (round 5; tools/rtol_chaos.py,
    profiles/r5_rtol_chaos.jsonl, mean EPE to the reference, classic-c /
    classic++): the fp64 oracle with its 'backslash' stopped at the GPU's
    1e-6 lands where the GPU does, 1.98e-2 / 2.11e-2; stopped at 1e-12 it is
    at 1.22e-2 / 0.50e-2, at 1e-8 1.77e-2 / 1.61e-2.  With every solution
    rounded to float32 (the form the GPU returns x in) and solved to 1e-12:
    1.76e-2 / 1.34e-2.  On the GPU, solving every level <= 65536 px 100x
    tighter (1e-8) moved the flow only to 1.85e-2 / 1.96e-2
    (profiles/r5ab_small_rtol_probe.log): the fp32 CG's returned x has a true
    residual of ~1e-7 however far its iterate goes (k_cg_reg iterate 6e-9,
    returned x 3e-8 .. 2e-7; k_cgs quadratic-stage solves 9e-8 with an
    estimate of 4e-9), and at 1e-7 the fp64 oracle is already at 2.0e-2 /
    1.78e-2.  So below the 1e-6 stop the limit is fp32 -- x and the flow
    state it updates -- and 2x the reference's 1e-12 spread (2.8e-2 /
    1.78e-2) is out of reach for classic++ without fp64 solves and flow
    state; the gate stays at the reference's float32-level spread.  Other
    methods by TOL."""
    import optical_flow
    d = golden("e2e_synth.npz")
    ch = golden("chaos_synth.npz")
    ref = d[method] if method in d else ch[method]
    uv = optical_flow.estimate_flow(d["im1"], d["im2"], method)
    s = epe_stats(uv, ref)
    da = abs(_aepe(uv, d["gt"]) - _aepe(ref, d["gt"]))
    fam = FAMILY[method]
    print(method, s, "dAEPE", da)
    if method in ch:
        spread = {eps: (max(float(ch[f"{method}:eps{eps}:seed{k}:mean"]) for k in range(3)),
                        max(float(ch[f"{method}:eps{eps}:seed{k}:median"]) for k in range(3)))
                  for eps in ("1e-12", "6e-08")}
        print("  reference spread (mean, median): 1e-12", spread["1e-12"], " 6e-8", spread["6e-08"])
    if fam == "chaotic":
        mean_tol, med_tol = 1.5 * spread["6e-08"][0], 1.5 * spread["6e-08"][1]
    else:
        mean_tol, med_tol = TOL[fam]
    assert s["mean"] < mean_tol and s["median"] < med_tol, (s, mean_tol, med_tol)
    assert da < (3e-3 if fam == "chaotic" else 1e-3)


@pytest.mark.slow
@pytest.mark.parametrize("method", ["classic+nl-fast", "hs-brightness"])
def test_rubberwhale(golden, rubberwhale, method):
    """The north-star parity target: |dAEPE| <= 1e-3 vs the NumPy reference on
    RubberWhale; |dAAE| <= 0.02 deg; mean EPE to the reference uv <= 5e-3 px,
    median <= 1e-3, p99 <= 0.05."""
    import optical_flow
    from optical_flow.evaluation.metrics import flow_angular_error as fae
    im1, im2, gt = rubberwhale
    ref = golden("rubberwhale_ref.npz")[method].astype(np.float64)
    uv = optical_flow.estimate_flow(im1, im2, method)
    a_gpu = fae(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1])
    a_ref = fae(gt[..., 0], gt[..., 1], ref[..., 0], ref[..., 1])
    s = epe_stats(uv, ref)
    print(method, "gpu AAE/AEPE", a_gpu[0], a_gpu[2], "ref", a_ref[0], a_ref[2], s)
    assert abs(a_gpu[2] - a_ref[2]) <= 1e-3
    assert abs(a_gpu[0] - a_ref[0]) <= 0.02
    assert s["mean"] <= 5e-3 and s["median"] <= 1e-3 and s["p99"] <= 0.05, s
