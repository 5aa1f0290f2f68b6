"""GPU stage parity: every hot-path row of SURVEY.md §8a, HIP kernel (through
the C ABI) vs the reference's golden vectors and the float64 oracle.

Tolerances are float32 tolerances against float64 references, stated per
test (pointwise stages rtol 1e-5 / atol 1e-4 x scale)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

FILT = np.array([1, -8, 0, 8, -1]) / 12.0


def test_library_loads_on_gpu():
    from optical_flow import _native
    ctx = _native.context()
    assert ctx.handle


def test_preprocess_gray_lab(golden):
    from optical_flow.interface import _preprocess
    d = golden("preprocess.npz")
    gray, lab = _preprocess(d["rgb1"], d["rgb2"])
    np.testing.assert_array_equal(gray[0], d["gray1"])       # integer-valued: exact
    np.testing.assert_array_equal(gray[1], d["gray2"])
    np.testing.assert_allclose(np.moveaxis(lab, 0, 2), d["lab_scaled"], atol=255 * 2e-5)


def test_rof_texture(golden):
    from optical_flow.utils.image_processing import structure_texture_decomposition_rof as rof
    d = golden("rof.npz")
    np.testing.assert_allclose(rof(d["images"]), d["texture"], atol=2e-3)
    np.testing.assert_allclose(rof(d["images"][..., 0]), d["texture_2d"], atol=2e-3)
    np.testing.assert_allclose(rof(d["images4"], 1 / 8, 37, 0.8), d["texture4"], atol=2e-3)


def test_pyramid(golden):
    from optical_flow.utils.pyramid import compute_image_pyramid
    d, g = golden("pyramid.npz"), golden("gauss.npz")
    for sp, ratio in ((2.0, 0.5), (1.25, 0.8)):
        p = compute_image_pyramid(d["img"], g[f"g_{sp}"], 4, ratio)
        for lv in range(4):
            np.testing.assert_allclose(p[lv], d[f"p_{sp}_{lv}"], atol=2e-4 * 255)
        p = compute_image_pyramid(d["lab"], g[f"g_{sp}"], 3, ratio)
        for lv in range(3):
            np.testing.assert_allclose(p[lv], d[f"lab_{sp}_{lv}"], atol=1e-3)


def test_resample_flow(golden):
    from optical_flow.utils.warping import resample_flow
    d = golden("resample.npz")
    for (h, w) in ((46, 62), (18, 25), (37, 53), (23, 31)):
        np.testing.assert_allclose(resample_flow(d["uv"], (h, w)), d[f"r_{h}_{w}"], atol=2e-5)


@pytest.mark.parametrize("method", ["bi-cubic", "cubic", "bi-linear"])
@pytest.mark.parametrize("blend", [0.5, 0.3])
def test_partial_deriv(golden, method, blend):
    from optical_flow.utils.derivatives import partial_deriv
    d = golden("deriv.npz")
    suf = "" if blend == 0.5 else "_b03"
    out = partial_deriv(d["images"], d["uv"], method, FILT, blend)
    for got, name in zip(out, ("It", "Ix", "Iy")):
        ref = d[f"{method}{suf}_{name}"]
        bad = np.abs(got - ref) > 5e-3 + 1e-5 * np.abs(ref)
        # fp32 vs fp64 warped coordinates may flip an in/out-of-bounds test on
        # a pixel that lies within 1 ulp of the image border
        assert bad.sum() <= 2, (name, np.argwhere(bad)[:5], np.abs(got - ref).max())


@pytest.mark.parametrize("method", ["bi-cubic", "cubic"])
def test_partial_deriv_multichannel(golden, method):
    from optical_flow.utils.derivatives import partial_deriv
    d = golden("deriv.npz")
    out = partial_deriv(d["images4"], d["uv"], method, FILT, 0.5)
    for got, name in zip(out, ("It", "Ix", "Iy")):
        ref = d[f"mc_{method}_{name}"]
        assert (np.abs(got - ref) > 5e-3 + 1e-5 * np.abs(ref)).sum() <= 4


OPS = [("nl_robust", "classic+nl", 0.0), ("nl_qua", "classic+nl", 1.0), ("nl_blend05", "classic+nl", 0.5),
       ("ba_lor", "ba", 0.0), ("ba_charb", "classic-c", 0.0), ("ba_pp", "classic++", 0.0), ("hs", "hs", 0.0)]


def _ref_A(d, tag, n2):
    from scipy import sparse
    return sparse.coo_matrix((d[tag + "_val"], (d[tag + "_row"], d[tag + "_col"])), shape=(n2, n2)).tocsc()


@pytest.mark.parametrize("tag,meth,alpha", OPS)
def test_flow_operator(golden, tag, meth, alpha):
    """GPU planes vs the float64 oracle evaluated on the same float32-rounded
    inputs (elementwise rtol 1e-4), and vs the reference's A, b (relative to
    max|A|).  Robust weights are steep near |du| ~ sigma^2, so rounding uv to
    float32 alone moves single entries by up to ~1e-5 max|A| (charbonnier)."""
    from optical_flow.methods.config import load_of_method
    from optical_flow.methods.base import planes_to_sparse
    d = golden("operator.npz")
    o = load_of_method(meth)
    o.images = d["images"]
    if tag == "hs":
        It, Ix, Iy = O.partial_deriv(d["images"], d["uv"], "cubic")
    else:
        It, Ix, Iy = d["It"], d["Ix"], d["Iy"]
    f32 = lambda a: np.asarray(a, dtype=np.float32).astype(np.float64)  # noqa: E731
    coef, rhs = o._operator_planes(d["uv"], None, It, Ix, Iy, alpha)
    oc, orhs = O.flow_operator(o.to_params(), alpha, f32(d["uv"]), None, f32(It), f32(Ix), f32(Iy))
    scale = np.abs(oc).max(axis=(1, 2), keepdims=True)
    assert np.all(np.abs(coef - oc) <= 1e-4 * np.abs(oc) + 1e-6 * scale), np.abs(coef - oc).max()
    bscale = np.abs(orhs).max()
    assert np.all(np.abs(rhs - orhs) <= 1e-4 * np.abs(orhs) + 2e-5 * bscale)
    H, W = d["uv"].shape[:2]
    A = planes_to_sparse(coef)
    Ar = _ref_A(d, tag, 2 * H * W)
    assert abs(A - Ar).max() <= 5e-5 * abs(Ar).max()
    b = np.concatenate([rhs[0].ravel(order="F"), rhs[1].ravel(order="F")])
    assert np.abs(b - d[tag + "_b"]).max() <= 1e-4 * np.abs(d[tag + "_b"]).max()


@pytest.mark.parametrize("tag,meth,alpha", OPS)
def test_solve_backslash_and_pcg(golden, tag, meth, alpha):
    """'backslash' (GPU block-Jacobi PCG surrogate) vs SuperLU's x; 'pcg' vs
    scipy cg (Jacobi, rtol 1e-3, maxiter 200) on the reference's A, b."""
    from optical_flow.methods.config import load_of_method
    from optical_flow import _native as nat
    import ctypes as C
    d = golden("operator.npz")
    H, W = d["uv"].shape[:2]
    N = H * W
    o = load_of_method(meth)
    Ar = _ref_A(d, tag, 2 * N)
    xr = d[tag + "_x"]
    x = o._solve_linear_system(Ar, d[tag + "_b"], (H, W, 2))
    xf = np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])
    assert np.linalg.norm(xf - xr) <= 5e-4 * np.linalg.norm(xr), np.linalg.norm(xf - xr) / np.linalg.norm(xr)
    from scipy.sparse.linalg import cg, LinearOperator
    dg = Ar.diagonal()
    xs, _ = cg(Ar, d[tag + "_b"], M=LinearOperator(Ar.shape, matvec=lambda v: v / dg), maxiter=200, rtol=1e-3)
    o.solver = "pcg"
    x = o._solve_linear_system(Ar, d[tag + "_b"], (H, W, 2))
    xf = np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])
    assert np.linalg.norm(xf - xs) <= 2e-2 * np.linalg.norm(xs)


@pytest.mark.parametrize("tag,meth", [("hs", "hs"), ("ba_lor", "ba"), ("nl_robust", "classic+nl")])
def test_sor_matches_reference_sor(golden, tag, meth):
    """'sor' is the reference's own lexicographic SOR (base.py:138-172), not a
    reordering: same sweep count and the same iterate as the reference's
    Python row loop (tests/golden/sor.npz) to fp32 rounding."""
    from optical_flow.methods.config import load_of_method
    d, s = golden("operator.npz"), golden("sor.npz")
    H, W = d["uv"].shape[:2]
    o = load_of_method(meth)
    o.solver = "sor"
    Ar = _ref_A(d, tag, 2 * H * W)
    x = o._solve_linear_system(Ar, d[tag + "_b"], (H, W, 2))
    xf = np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])
    xr = s[tag + "_x"]
    assert o.last_solve["iters"] == int(s[tag + "_sweeps"]), (o.last_solve, int(s[tag + "_sweeps"]))
    err = np.linalg.norm(xf - xr) / np.linalg.norm(xr)
    assert err <= 2e-5, err


@pytest.mark.parametrize("H,W", [(40, 56), (64, 64), (150, 200), (200, 131), (300, 90)])
def test_sor_synthetic_vs_oracle(H, W):
    """Multi-strip SOR launches (64-row strips handing rows to each other
    inside one launch) vs the float64 oracle's lexicographic SOR on random
    flow systems: same sweep count (+-1 at the stopping threshold), same x to
    fp32 rounding."""
    import oracle as Or
    from optical_flow.methods.config import load_of_method
    from optical_flow.methods.base import sparse_to_planes
    A, b = _spd_flow_system(H, W, seed=7 * H + W)
    o = load_of_method("hs")
    o.solver = "sor"
    x = o._solve_linear_system(A, b, (H, W, 2))
    coef = sparse_to_planes(A, H, W)
    rhs = np.stack([b[:H * W].reshape(H, W, order="F"), b[H * W:].reshape(H, W, order="F")])
    P = o.to_params()
    xo, it, _ = Or.solve(P, coef, rhs)
    assert abs(o.last_solve["iters"] - it) <= 1, (o.last_solve, it)
    xg = np.moveaxis(x, 2, 0)
    err = np.linalg.norm(xg - xo) / np.linalg.norm(xo)
    assert err <= 1e-4, err


def _sor_both(fn):
    """fn() with the pipelined SOR (k_sor_pipe, default) and with one launch
    per sweep (k_sor_lex) on this thread's context."""
    from optical_flow import _native as nat
    from optical_flow._abi import OF_OPT_SOR_PIPELINE
    ctx = nat.context()
    try:
        ctx.set_option(OF_OPT_SOR_PIPELINE, 0)
        ref = fn()
        ctx.set_option(OF_OPT_SOR_PIPELINE, 1)
        return fn(), ref
    finally:
        ctx.set_option(OF_OPT_SOR_PIPELINE, 2)  # the default


@pytest.mark.parametrize("H,W,maxit", [(40, 56, 10000), (64, 64, 10000), (150, 200, 10000), (300, 90, 10000),
                                       (520, 70, 10000), (130, 333, 7), (200, 131, 1)])
def test_sor_pipelined_bitwise(H, W, maxit):
    """k_sor_pipe (sweeps in flight side by side in one persistent launch)
    gives the same iterate and sweep count bitwise as k_sor_lex (one launch
    per sweep): every point is relaxed from the same operands.  Sizes cover
    1..9 strips, the ring wrapping many times, and the sweep limit (done=2)."""
    from optical_flow.methods.config import load_of_method
    A, b = _spd_flow_system(H, W, seed=11 * H + W)
    o = load_of_method("hs")
    o.solver = "sor"
    o.sor_max_iters = maxit

    def run():
        x = o._solve_linear_system(A, b, (H, W, 2))
        return x, dict(o.last_solve)
    (x1, s1), (x0, s0) = _sor_both(run)
    assert s1["iters"] == s0["iters"] and s1.get("done") == s0.get("done"), (s1, s0)
    if maxit < 10000:
        assert s1["iters"] == maxit
    np.testing.assert_array_equal(x1, x0)


def test_sor_pipelined_bitwise_e2e(golden):
    """HS with 'sor' end to end (every level, every warp) on the synthetic
    pair: the pipelined and per-sweep kernels give bitwise the same flow."""
    import optical_flow
    d = golden("e2e_synth.npz")
    uv1, uv0 = _sor_both(lambda: optical_flow.estimate_flow(d["im1"], d["im2"], "hs", {"solver": "sor"}))
    np.testing.assert_array_equal(uv1, uv0)


def _sor_modes(fn, modes=(0, 2)):
    """fn() under each OF_OPT_SOR_PIPELINE mode (0 per sweep, 1 pipelined,
    2 pipelined + the one-workgroup LDS kernel for levels of <= 64 rows);
    returns the results and, per mode, the kernel names that ran."""
    import ctypes as C
    from optical_flow import _native as nat
    from optical_flow._abi import OF_OPT_SOR_PIPELINE
    ctx = nat.context()
    out, ran = [], []
    try:
        for m in modes:
            ctx.set_option(OF_OPT_SOR_PIPELINE, m)
            ctx.check(ctx.lib.of_set_profiling(ctx.handle, 1))
            out.append(fn())
            n = C.c_int(0)
            names = (C.c_char_p * 256)()
            ctx.check(ctx.lib.of_kernel_times(ctx.handle, 256, names, None, None, None, C.byref(n)))
            ran.append({names[i].decode() for i in range(min(n.value, 256))})
            ctx.check(ctx.lib.of_set_profiling(ctx.handle, 0))
    finally:
        ctx.set_option(OF_OPT_SOR_PIPELINE, 2)  # the default
    return out, ran


@pytest.mark.parametrize("H,W,maxit", [(40, 56, 10000), (64, 64, 10000), (30, 40, 10000), (60, 80, 10000),
                                       (17, 30, 10000), (5, 300, 10000), (30, 40, 7), (60, 80, 1), (64, 200, 10000)])
def test_sor_workgroup_bitwise(H, W, maxit):
    """k_sor_wg (a level of <= 64 rows solved in one workgroup, sweep ring and
    progress stamps in LDS) gives the same iterate and sweep count bitwise as
    k_sor_lex, including the sweep limit; levels whose LDS ring would hold
    fewer than 8 sweeps (60x80, 64x64, 64x200) stay on k_sor_pipe."""
    from optical_flow import _abi, _native as nat
    from optical_flow.methods.config import load_of_method
    A, b = _spd_flow_system(H, W, seed=13 * H + W)
    o = load_of_method("hs")
    o.solver = "sor"
    o.sor_max_iters = maxit

    def run():
        x = o._solve_linear_system(A, b, (H, W, 2))
        return x, dict(o.last_solve)
    fb0 = nat.context().get_option(_abi.OF_OPT_SOR_FALLBACKS)
    ((x0, s0), (x2, s2)), (r0, r2) = _sor_modes(run)
    assert nat.context().get_option(_abi.OF_OPT_SOR_FALLBACKS) == fb0
    assert s2["iters"] == s0["iters"] and s2.get("done") == s0.get("done"), (s2, s0)
    if maxit < 10000:
        assert s2["iters"] == maxit
    np.testing.assert_array_equal(x2, x0)
    assert "sor_sweep" in r0
    assert ("sor_wg" in r2) == (H * W * 8 * 8 <= 144 * 1024), r2  # a ring of >= 8 sweeps


def test_sor_workgroup_bitwise_e2e(golden):
    """HS with 'sor' end to end with the one-workgroup kernel on its small
    levels: the flow equals the per-sweep kernel's bitwise."""
    import optical_flow
    d = golden("e2e_synth.npz")
    (uv0, uv2), (r0, r2) = _sor_modes(lambda: optical_flow.estimate_flow(d["im1"], d["im2"], "hs", {"solver": "sor"}))
    assert "sor_wg" in r2
    np.testing.assert_array_equal(uv2, uv0)


def test_sor_device_memory_flat(golden):
    """the pipelined SOR's ring of sweep buffers is one grow-only
    buffer per context (was carved from the per-pair arena on every solve:
    one more ring per warp / level).  HS with 'sor' end to end, three times
    in one context: the context's device bytes (OF_OPT_DEVICE_BYTES: arena
    chunks + SOR ring + gather buffer) do not grow after the first call, and
    no pipelined solve fell back to the per-sweep kernel."""
    import optical_flow
    from optical_flow import _abi, _native
    d = golden("e2e_synth.npz")
    ctx = _native.context()
    held = []
    for _ in range(3):
        optical_flow.estimate_flow(d["im1"], d["im2"], "hs", {"solver": "sor"})
        held.append(ctx.get_option(_abi.OF_OPT_DEVICE_BYTES))
    print("device bytes per call", held)
    assert held[0] > 0 and held[1] == held[0] and held[2] == held[0], held
    assert ctx.get_option(_abi.OF_OPT_SOR_FALLBACKS) == 0


def test_occlusion(golden):
    from optical_flow.utils.occlusion import detect_occlusion
    d = golden("occlusion.npz")
    np.testing.assert_allclose(detect_occlusion(d["uv"], d["images"]), d["occ"], atol=1e-5)
    np.testing.assert_allclose(detect_occlusion(d["uv"], d["images4"]), d["occ4"], atol=1e-5)


@pytest.mark.parametrize("guide,hsz,sig,key", [("lab", 7, 7.0, "out_lab"), ("gray", 7, 7.0, "out_gray"),
                                               ("lab", 3, 4.0, "out_lab_h3")])
def test_weighted_median(golden, guide, hsz, sig, key):
    from optical_flow.utils.weighted_median import denoise_color_weighted_medfilt2
    d = golden("wmf.npz")
    out = denoise_color_weighted_medfilt2(d["uv"], d[guide], d["occ"], hsz, [5, 5], sig)
    ref = d[key]
    same = np.abs(out - ref) <= 1e-6 * (1 + np.abs(ref))
    # float32 weights may pick a neighbouring order statistic when the
    # half-weight crossing is within rounding; everything else exact
    print(f"wmf {key}: exact fraction {same.mean():.5f}")
    assert same.mean() >= 0.999, same.mean()


# sort keys per lane (NPER) by window: hsz 0 -> 1, 1 -> 2, 3 -> 4, 5 / 7 -> 8
# (7: the compile-time instance), 12 -> 16 -- every k_wmf instance's sort
@pytest.mark.parametrize("gc,hsz,sig", [(3, 7, 7.0), (1, 7, 7.0), (3, 3, 4.0), (3, 12, 7.0), (3, 0, 7.0),
                                        (3, 1, 7.0), (1, 1, 7.0), (3, 5, 7.0)])
def test_weighted_median_synthetic_vs_oracle(gc, hsz, sig):
    """Weighted median of a 96x136 synthetic flow (smooth field + noise +
    a motion edge, so sorted chunks and window crossings vary) against the
    float64 oracle on the same fp32-rounded inputs: >= 99.9 % of pixels
    exact, the rest a neighbouring order statistic."""
    import oracle as Or
    from optical_flow.utils.weighted_median import denoise_color_weighted_medfilt2
    from optical_flow.utils.synthetic import synth_pair
    H, W = 96, 136
    im1, _, gt = synth_pair(H, W, 5)
    rng = np.random.default_rng(11)
    uv = gt + 0.3 * rng.standard_normal(gt.shape)
    uv[:, W // 2:] += 1.5
    uv = uv.astype(np.float32).astype(np.float64)
    guide = (Or.rgb2lab(im1) if gc == 3 else im1.mean(-1)).astype(np.float32).astype(np.float64)
    occ = rng.uniform(0.0, 1.0, (H, W)).astype(np.float32).astype(np.float64)
    occ[:20, :30] = 0.0  # weights at the 1e-10 floor
    out = denoise_color_weighted_medfilt2(uv, guide, occ, hsz, [5, 5], sig)
    ref = Or.weighted_median(uv, guide, occ, hsz, sig)
    same = np.abs(out - ref) <= 1e-6 * (1 + np.abs(ref))
    print(f"wmf synthetic gc={gc} hsz={hsz}: exact fraction {same.mean():.5f}")
    assert same.mean() >= 0.999, same.mean()


def test_weighted_median_no_guide_is_median(golden):
    from optical_flow.utils.weighted_median import denoise_color_weighted_medfilt2
    d = golden("wmf.npz")
    out = denoise_color_weighted_medfilt2(d["uv"], None, d["occ"], 7, [5, 5], 7.0)
    np.testing.assert_allclose(out, d["out_none"], atol=1e-6)


def test_median_filter(golden):
    from optical_flow.utils.weighted_median import median_filter2
    d = golden("median.npz")
    np.testing.assert_allclose(median_filter2(d["a"], 5), d["a_med"], atol=1e-6)
    np.testing.assert_allclose(median_filter2(d["t"], 5), d["t_med"], atol=1e-6)
    np.testing.assert_allclose(median_filter2(d["a"], 3), d["a3"], atol=1e-6)


def _spd_flow_system(H, W, seed):
    """A random flow system of the shape flow_operator assembles: positive
    edge weights spanning 4 decades (robust IRLS weights), PSD 2x2 data blocks,
    diagonal = data block + sum of incident edge weights."""
    from optical_flow.methods.base import planes_to_sparse
    rng = np.random.default_rng(seed)
    coef = np.zeros((7, H, W))
    for pl in range(4):
        coef[pl] = 10.0 ** rng.uniform(-2, 2, (H, W))
    coef[0][:, -1] = coef[2][:, -1] = 0.0   # no edge right of the last column
    coef[1][-1, :] = coef[3][-1, :] = 0.0   # nor below the last row
    ix, iy = rng.normal(0, 3, (H, W)), rng.normal(0, 3, (H, W))
    psi = 10.0 ** rng.uniform(-1, 1, (H, W))
    deg = [coef[2 * c].copy() + coef[2 * c + 1] for c in range(2)]
    for c in range(2):
        deg[c][:, 1:] += coef[2 * c][:, :-1]
        deg[c][1:, :] += coef[2 * c + 1][:-1, :]
    coef[4] = psi * ix * ix + deg[0]
    coef[5] = psi * ix * iy
    coef[6] = psi * iy * iy + deg[1]
    return planes_to_sparse(coef), rng.normal(0, 1, 2 * H * W)


@pytest.mark.parametrize("H,W", [(17, 30), (40, 56), (64, 96), (150, 200)])
def test_solve_synthetic_both_cg_paths(H, W):
    """'backslash' and 'pcg' on systems below (one-workgroup k_cg_small) and
    above (fused k_cgs / k_cg launches) the coarse-level size limit
    (CG_SMALL_PX = 4096 px): 'backslash' to <= 1e-4 relative error of the
    direct solve, 'pcg' within 2e-2 of scipy cg (Jacobi, rtol 1e-3)."""
    from optical_flow.methods.config import load_of_method
    from scipy.sparse.linalg import spsolve, cg, LinearOperator
    A, b = _spd_flow_system(H, W, seed=H * W)
    o = load_of_method("classic+nl-fast")

    def flat(x):
        return np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])

    xr = spsolve(A.tocsc(), b)
    x = flat(o._solve_linear_system(A, b, (H, W, 2)))
    assert np.linalg.norm(x - xr) <= 1e-4 * np.linalg.norm(xr), np.linalg.norm(x - xr) / np.linalg.norm(xr)
    dg = A.diagonal()
    xs, _ = cg(A, b, M=LinearOperator(A.shape, matvec=lambda v: v / dg), maxiter=200, rtol=1e-3)
    o.solver = "pcg"
    x = flat(o._solve_linear_system(A, b, (H, W, 2)))
    assert np.linalg.norm(x - xs) <= 2e-2 * np.linalg.norm(xs), np.linalg.norm(x - xs) / np.linalg.norm(xs)


@pytest.mark.parametrize("H,W", [(40, 56), (64, 96), (150, 200)])
def test_solve_rtol0_stops_at_noise_floor(H, W):
    """rtol 0 runs CG past the fp32-representable residual: the solve must stop
    there (prologue test on p.Ap, r.z and the recurrence's next r.z) or
    restart (beta = 0) when the r.z a sweep formed departs from the
    recurrence's prediction, with a finite iterate near direct-solve accuracy
    (1e-3; the rtol 1e-6 solves of test_solve_synthetic_both_cg_paths reach
    1e-4), never return NaN or diverge (both happened before the test
    existed: NaN at 1080p, 1.6e18 for 'pcg' at 64x96; profiles/r2t_cgs_ab.md).
    Covers k_cg_small (40x56), the fused k_cgs launches and 'pcg' (k_cg)."""
    from optical_flow.methods.config import load_of_method
    from scipy.sparse.linalg import spsolve
    A, b = _spd_flow_system(H, W, seed=H + W)
    xr = spsolve(A.tocsc(), b)
    o = load_of_method("classic+nl-fast")
    o.backslash_rtol = 0.0
    o.backslash_maxiter = 3000
    o.pcg_rtol = 0.0
    o.pcg_maxiter = 3000

    def flat(x):
        return np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])

    for solver in ("backslash", "pcg"):
        o.solver = solver
        x = flat(o._solve_linear_system(A, b, (H, W, 2)))
        assert np.all(np.isfinite(x)), solver
        err = np.linalg.norm(x - xr) / np.linalg.norm(xr)
        assert err <= 1e-3, (solver, err)


@pytest.mark.parametrize("method", ["classic+nl-fast", "hs", "classic-c", "ba", "classic+nl"])
def test_fused_warp_operator_matches_two_kernels(golden, method):
    """The fused warp + assembly (k_warp_operator, OF_OPT_FUSED_WARP = 1, the
    default) and partial_deriv + flow_operator as two kernels compute the
    same system bitwise: neither form contracts products into fma
    (OF_WARP_NOCONTRACT, round 6; before, the two forms contracted
    different products and the flows differed by up to 1.4e-4 px), so the
    flows are bitwise equal; both meet the e2e parity gates against the
    reference (test_gpu_e2e's TOL)."""
    import optical_flow
    from optical_flow import _abi, _native
    from test_gpu_e2e import FAMILY, TOL
    from conftest import epe_stats
    d = golden("e2e_small.npz")
    ctx = _native.context()
    assert ctx.get_option(_abi.OF_OPT_FUSED_WARP) == 1
    fused = optical_flow.estimate_flow(d["im1"], d["im2"], method)
    ctx.set_option(_abi.OF_OPT_FUSED_WARP, 0)
    try:
        two = optical_flow.estimate_flow(d["im1"], d["im2"], method)
    finally:
        ctx.set_option(_abi.OF_OPT_FUSED_WARP, 1)
    mean_tol, med_tol = TOL[FAMILY[method]]
    s = epe_stats(fused, two)
    print(method, "fused vs two kernels", s, "bitwise", bool(np.array_equal(fused, two)))
    np.testing.assert_array_equal(fused, two)
    for uv in (fused, two):
        r = epe_stats(uv, d[method])
        assert r["mean"] < mean_tol and r["median"] < med_tol, r
