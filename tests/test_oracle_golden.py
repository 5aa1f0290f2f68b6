"""The float64 CPU oracle (test infrastructure) pinned against the golden
vectors generated from the reference (tests/golden/gen_golden.py).  Runs on
CPU; every stage of SURVEY.md §8a must agree to float64 rounding."""
import numpy as np
import pytest

import oracle as O
from conftest import epe_stats

FILT = np.array([1, -8, 0, 8, -1]) / 12.0
PEN_CASES = [
    ("quadratic", [1.0]), ("quadratic", [2.5]), ("quadratic", [1e-3]),
    ("lorentzian", [0.03]), ("lorentzian", [1.5]),
    ("charbonnier", [1e-3]), ("charbonnier", [0.5]),
    ("generalized_charbonnier", [1e-3, 0.45]), ("generalized_charbonnier", [0.1, 1.0]),
    ("geman_mcclure", [0.7]), ("huber", [0.8]), ("tukey", [1.2]), ("gaussian", [0.9]),
    ("tdist", [5.0, 1.0]), ("tdist_unnorm", [5.0, 1.0]),
]


def test_penalties(golden):
    d = golden("penalties.npz")
    for k, (name, p) in enumerate(PEN_CASES):
        for dt in range(3):
            ref = d[f"c{k}_d{dt}"]
            np.testing.assert_allclose(O.penalty(name, p, d["x"], dt), ref, rtol=1e-13, atol=1e-300)


def test_preprocess(golden):
    d = golden("preprocess.npz")
    np.testing.assert_array_equal(O.rgb2gray(d["rgb1"]), d["gray1"])
    np.testing.assert_array_equal(O.rgb2gray(d["frac"] * 255.3), d["gray_frac"])
    np.testing.assert_allclose(O.rgb2lab(d["rgb1"]), d["lab"], atol=1e-11)
    np.testing.assert_allclose(O.rgb2lab(d["frac"]), d["lab_frac"], atol=1e-11)
    lab = O.rgb2lab(d["rgb1"])
    for c in range(3):
        lab[..., c] = O.scale_image(lab[..., c], 0, 255)
    np.testing.assert_allclose(lab, d["lab_scaled"], atol=1e-10)


def test_rof(golden):
    d = golden("rof.npz")
    np.testing.assert_allclose(O.rof_texture(d["images"]), d["texture"], atol=1e-10)
    np.testing.assert_allclose(O.rof_texture(d["images"][..., 0]), d["texture_2d"], atol=1e-10)
    np.testing.assert_allclose(O.rof_texture(d["images4"], 1 / 8, 37, 0.8), d["texture4"], atol=1e-10)


def test_gaussian_and_pyramid(golden):
    g = golden("gauss.npz")
    np.testing.assert_allclose(O.gaussian(5, 1.0), g["g_2.0"], atol=1e-15)
    np.testing.assert_allclose(O.gaussian(3, np.sqrt(1.25) / np.sqrt(2)), g["g_1.25"], atol=1e-15)
    np.testing.assert_allclose(O.gaussian(5, 1.5), g["g_5_1.5"], atol=1e-15)
    d = golden("pyramid.npz")
    for sp, ratio in ((2.0, 0.5), (1.25, 0.8)):
        p = O.pyramid(d["img"], g[f"g_{sp}"], 4, ratio)
        for lv in range(4):
            np.testing.assert_allclose(p[lv], d[f"p_{sp}_{lv}"], atol=1e-10)
        p = O.pyramid(d["lab"], g[f"g_{sp}"], 3, ratio)
        for lv in range(3):
            np.testing.assert_allclose(p[lv], d[f"lab_{sp}_{lv}"], atol=1e-10)


def test_resample(golden):
    d = golden("resample.npz")
    for (h, w) in ((46, 62), (18, 25), (37, 53), (23, 31)):
        np.testing.assert_allclose(O.resample_flow(d["uv"], (h, w)), d[f"r_{h}_{w}"], atol=1e-13)


def test_interp2_bicubic(golden):
    d = golden("deriv.npz")
    H, W = d["uv"].shape[:2]
    xg, yg = np.meshgrid(np.arange(1, W + 1.0), np.arange(1, H + 1.0))
    zi, zx, zy = O.interp2_bicubic(d["images"][..., 1], xg + d["uv"][..., 0], yg + d["uv"][..., 1], FILT)
    assert np.array_equal(np.isnan(zi), np.isnan(d["ZI"]))
    np.testing.assert_allclose(zi[~np.isnan(zi)], d["ZI"][~np.isnan(zi)], atol=1e-10)
    np.testing.assert_allclose(zx, d["ZXI"], atol=1e-10)
    np.testing.assert_allclose(zy, d["ZYI"], atol=1e-10)


def test_bspline_prefilter_matches_scipy():
    from scipy.ndimage import spline_filter
    rng = np.random.default_rng(5)
    for shape in ((7, 9), (1, 5), (2, 3), (40, 33)):
        a = rng.normal(size=shape)
        np.testing.assert_allclose(O.bspline_prefilter(a), spline_filter(a, 3, mode="mirror"), atol=1e-12)


@pytest.mark.parametrize("method", ["bi-cubic", "cubic", "bi-linear"])
def test_partial_deriv(golden, method):
    d = golden("deriv.npz")
    for b, suf in ((0.5, ""), (0.3, "_b03")):
        out = O.partial_deriv(d["images"], d["uv"], method, FILT, b)
        for got, name in zip(out, ("It", "Ix", "Iy")):
            np.testing.assert_allclose(got, d[f"{method}{suf}_{name}"], atol=1e-10)
    if method != "bi-linear":
        out = O.partial_deriv(d["images4"], d["uv"], method, FILT, 0.5)
        for got, name in zip(out, ("It", "Ix", "Iy")):
            np.testing.assert_allclose(got, d[f"mc_{method}_{name}"], atol=1e-10)


OPS = [("nl_robust", "classic+nl", 0.0), ("nl_qua", "classic+nl", 1.0), ("nl_blend05", "classic+nl", 0.5),
       ("ba_lor", "ba", 0.0), ("ba_charb", "classic-c", 0.0), ("ba_pp", "classic++", 0.0), ("hs", "hs", 0.0)]


@pytest.mark.parametrize("tag,meth,alpha", OPS)
def test_operator_and_direct_solve(golden, tag, meth, alpha):
    from scipy import sparse
    from optical_flow.methods.config import load_of_method
    from optical_flow.methods.base import planes_to_sparse
    d = golden("operator.npz")
    H, W = d["uv"].shape[:2]
    N = H * W
    P = load_of_method(meth).to_params()
    if tag == "hs":
        It, Ix, Iy = O.partial_deriv(d["images"], d["uv"], "cubic")
    else:
        It, Ix, Iy = d["It"], d["Ix"], d["Iy"]
    coef, rhs = O.flow_operator(P, alpha, d["uv"], None, It, Ix, Iy)
    Ar = sparse.coo_matrix((d[tag + "_val"], (d[tag + "_row"], d[tag + "_col"])), shape=(2 * N, 2 * N)).tocsc()
    assert abs(planes_to_sparse(coef) - Ar).max() <= 1e-13 * abs(Ar).max()
    b = np.concatenate([rhs[0].ravel(order="F"), rhs[1].ravel(order="F")])
    np.testing.assert_allclose(b, d[tag + "_b"], atol=1e-12 * np.abs(d[tag + "_b"]).max())
    x, it, _ = O.solve(P, coef, rhs)  # 'backslash' -> fp64 PCG to rtol 1e-12
    xf = np.concatenate([x[0].ravel(order="F"), x[1].ravel(order="F")])
    assert np.abs(xf - d[tag + "_x"]).max() <= 1e-8 * max(1.0, np.abs(d[tag + "_x"]).max())


def test_pcg_matches_scipy_cg(golden):
    from scipy import sparse
    from scipy.sparse.linalg import cg, LinearOperator
    from optical_flow.methods.config import load_of_method
    d = golden("operator.npz")
    H, W = d["uv"].shape[:2]
    N = H * W
    for tag, meth, alpha in OPS:
        P = load_of_method(meth).to_params()
        P.solver, P.pcg_rtol, P.pcg_maxiter = 1, 1e-3, 200
        It, Ix, Iy = (O.partial_deriv(d["images"], d["uv"], "cubic") if tag == "hs" else (d["It"], d["Ix"], d["Iy"]))
        coef, rhs = O.flow_operator(P, alpha, d["uv"], None, It, Ix, Iy)
        x, it, _ = O.solve(P, coef, rhs)
        A = sparse.coo_matrix((d[tag + "_val"], (d[tag + "_row"], d[tag + "_col"])), shape=(2 * N, 2 * N)).tocsc()
        dg = A.diagonal()
        xs, _ = cg(A, d[tag + "_b"], M=LinearOperator(A.shape, matvec=lambda v: v / dg), maxiter=200, rtol=1e-3)
        xf = np.concatenate([x[0].ravel(order="F"), x[1].ravel(order="F")])
        np.testing.assert_allclose(xf, xs, atol=1e-10 * np.abs(xs).max())


def test_occlusion(golden):
    d = golden("occlusion.npz")
    np.testing.assert_allclose(O.detect_occlusion(d["uv"], d["images"]), d["occ"], atol=1e-14)
    np.testing.assert_allclose(O.detect_occlusion(d["uv"], d["images4"]), d["occ4"], atol=1e-14)


def test_weighted_median(golden):
    d = golden("wmf.npz")
    np.testing.assert_array_equal(O.weighted_median(d["uv"], d["lab"], d["occ"], 7, 7.0), d["out_lab"])
    np.testing.assert_array_equal(O.weighted_median(d["uv"], d["gray"], d["occ"], 7, 7.0), d["out_gray"])
    np.testing.assert_array_equal(O.weighted_median(d["uv"], None, d["occ"], 7, 7.0), d["out_none"])
    np.testing.assert_array_equal(O.weighted_median(d["uv"], d["lab"], d["occ"], 3, 4.0), d["out_lab_h3"])


def test_median(golden):
    d = golden("median.npz")
    np.testing.assert_array_equal(O.median_filter(d["a"]), d["a_med"])
    np.testing.assert_array_equal(O.median_filter(d["t"]), d["t_med"])
    np.testing.assert_array_equal(O.median_filter(d["a"], 3), d["a3"])


# end-to-end: stable methods agree to float64 rounding; the charbonnier
# methods are chaotic (the reference itself moves by ~5e-3 px mean when its
# solve is perturbed by 1e-12 relative) and classic-c-a diverges
# in the reference (|uv| ~ 1e36), which the oracle reproduces.
E2E_TIGHT = ["classic+nl-fast", "hs-brightness", "hs", "ba-brightness", "ba", "classic-l"]


@pytest.mark.parametrize("method", E2E_TIGHT)
def test_e2e_small(golden, method):
    d = golden("e2e_small.npz")
    s = epe_stats(O.estimate_flow(d["im1"], d["im2"], method), d[method])
    assert s["max"] < 1e-6, s


def test_e2e_chaotic_and_divergent(golden):
    d = golden("e2e_small.npz")
    s = epe_stats(O.estimate_flow(d["im1"], d["im2"], "classic++"), d["classic++"])
    assert s["mean"] < 2e-2 and s["median"] < 1e-2, s
    ref = d["classic-c-a"]
    assert np.abs(ref).max() > 1e20  # the reference diverges
    out = O.estimate_flow(d["im1"], d["im2"], "classic-c-a")
    assert (~np.isfinite(out)).any() or np.abs(out).max() > 1e20


def test_e2e_gray_and_pcg(golden):
    d = golden("e2e_small.npz")
    assert epe_stats(O.estimate_flow(d["gray1"], d["gray2"], "hs-brightness"), d["gray:hs-brightness"])["max"] < 1e-6
    s = epe_stats(O.estimate_flow(d["im1"], d["im2"], "hs", {"solver": "pcg"}), d["pcg:hs"])
    assert s["max"] < 1e-8


def test_e2e_synth_hs(golden):
    d = golden("e2e_synth.npz")
    s = epe_stats(O.estimate_flow(d["im1"], d["im2"], "hs-brightness"), d["hs-brightness"])
    assert s["max"] < 1e-6, s


@pytest.mark.parametrize("tag", ["hs", "ba_lor", "nl_robust"])
def test_oracle_sor_matches_reference(golden, tag):
    """The oracle's lexicographic SOR (base.py:138-172) reproduces the
    reference's Python row loop: same sweep count, x to 1e-10."""
    from scipy import sparse
    from optical_flow.methods.base import sparse_to_planes
    from optical_flow.methods.config import load_of_method
    d, s = golden("operator.npz"), golden("sor.npz")
    H, W = d["uv"].shape[:2]
    n = 2 * H * W
    A = sparse.coo_matrix((d[tag + "_val"], (d[tag + "_row"], d[tag + "_col"])), shape=(n, n)).tocsr()
    coef = sparse_to_planes(A, H, W)
    b = d[tag + "_b"]
    rhs = np.stack([b[:H * W].reshape(H, W, order="F"), b[H * W:].reshape(H, W, order="F")])
    o = load_of_method("hs")
    o.solver = "sor"
    x, it, _ = O.solve(o.to_params(), coef, rhs)
    xf = np.concatenate([x[0].ravel(order="F"), x[1].ravel(order="F")])
    assert it == int(s[tag + "_sweeps"])
    assert np.linalg.norm(xf - s[tag + "_x"]) <= 1e-10 * np.linalg.norm(s[tag + "_x"])


def test_oracle_altba_nondivergent(golden):
    """classic-c-a with lambda2 = 0.01 (tests/golden/altba.npz): the oracle
    within the reference's own chaos (a 1e-12 input perturbation moves the
    reference by 3.3e-3 px mean, 1.5e-3 median)."""
    from conftest import epe_stats
    d = golden("altba.npz")
    s = epe_stats(O.estimate_flow(d["im1"], d["im2"], "classic-c-a", {"lambda2": 0.01}), d["e2e_lam2_0.01"])
    assert s["mean"] < 1e-2 and s["median"] < 5e-3, s


@pytest.mark.parametrize("alpha,rep", [(1.0, True), (1.0, False), (0.0, True), (0.0, False)])
def test_oracle_altba_compute_flow_base(golden, alpha, rep):
    """The oracle's AltBA compute_flow_base(uv, uvhat) vs the reference
    (tests/golden/altba.npz, gen_golden.py altba): float64 to 1e-8."""
    from optical_flow.methods.config import load_of_method
    d = golden("altba.npz")
    o = load_of_method("classic-c-a")
    o.images = d["base_images"]
    o.lambda2 = 0.01
    o.max_iters = 4
    o.alpha = alpha
    o.replacement = rep
    u, uh = O.alt_ba_flow_base(o, d["base_uv"], d["base_uvhat"])
    key = f"base_a{int(alpha)}_r{int(rep)}"
    np.testing.assert_allclose(u, d[key + "_uv"], atol=1e-6)
    np.testing.assert_allclose(uh, d[key + "_uvhat"], atol=1e-6)
