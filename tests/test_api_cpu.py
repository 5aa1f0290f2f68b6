"""CPU tests of the host-side API mirror and the C ABI surface (no GPU).

Mirrors the reference's own tests (tests/test_classic_nl.py, test_robust_
functions.py, test_flo_io.py, test_metrics.py, ...) against this package,
plus the C-ABI library check: liboptflow.so loads and exports every symbol
include/optflow.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest

from conftest import ROOT


# ---- C ABI --------------------------------------------------------------
def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "optflow.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(of_\w+)\(", txt, flags=re.M)))


def test_library_exports_every_header_symbol():
    from optical_flow import _native
    lib_path = _native.LIB_PATH
    assert os.path.exists(lib_path), "build() first"
    lib = ctypes.CDLL(lib_path)
    syms = _header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_native.EXPORTED_SYMBOLS)
    assert lib.of_abi_version() == 3


def test_struct_layout_matches_header():
    """of_params / of_stats sizes agree between ctypes and the C compiler."""
    from optical_flow import _abi
    import subprocess
    import tempfile
    src = ('#include "optflow.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(){printf("%zu %zu %zu %zu %zu %zu\\n",'
           'sizeof(of_params), sizeof(of_stats), offsetof(of_params, rho_couple), offsetof(of_params, lambda_),'
           'offsetof(of_params, filters), sizeof(of_filter_set));}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", os.path.join(d, "t")], check=True)
        out = subprocess.run([os.path.join(d, "t")], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(_abi.OfParams)
    assert int(out[1]) == ctypes.sizeof(_abi.OfStats)
    assert int(out[2]) == _abi.OfParams.rho_couple.offset
    assert int(out[3]) == _abi.OfParams.lambda_.offset
    assert int(out[4]) == _abi.OfParams.filters.offset
    assert int(out[5]) == ctypes.sizeof(_abi.OfFilterSet)


def test_no_cpu_fallback_without_library(monkeypatch):
    from optical_flow import _native
    monkeypatch.setattr(_native, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _native.load_library("/nonexistent/liboptflow.so")


# ---- registry (reference tests/test_classic_nl.py:7-41) -------------------
def test_registry_names_and_overrides():
    from optical_flow.methods.config import load_of_method, METHOD_NAMES
    for m in METHOD_NAMES:
        assert hasattr(load_of_method(m), "compute_flow")
    o = load_of_method("classic+nl-fast")
    assert (o.max_iters, o.gnc_iters, o.display, o.lambda_, o.area_hsz, o.sigma_i) == (3, 2, True, 3, 7, 7)
    assert o.interpolation_method == "bi-cubic" and o.texture is True and o.median_filter_size == [5, 5]
    assert load_of_method("classic-c").texture is True and load_of_method("classic-c").lambda_ == 5
    assert load_of_method("classic++").interpolation_method == "bi-cubic"
    assert load_of_method("classic+nl-full").fullVersion is True
    hs = load_of_method("hs-brightness")
    assert (hs.lambda_, hs.max_warping_iters, hs.solver) == (10, 10, "backslash")
    ba = load_of_method("ba")
    assert ba.rho_data.method == "lorentzian" and float(ba.rho_data.param[0]) == 1.5 and ba.lambda_ == 0.06
    a = load_of_method("classic-c-a")
    assert (a.lambda2, a.itersLO, a.weightRatio) == (1e2, 5, 100.0)
    with pytest.raises(ValueError, match="Unknown"):
        load_of_method("nonexistent_method")


def test_parse_input_parameter():
    from optical_flow.methods.config import load_of_method
    o = load_of_method("hs")
    o.parse_input_parameter({"lambda": 7, "max_iters": 2, "not_an_attr": 1})
    assert o.lambda_ == 7 and o.max_iters == 2 and not hasattr(o, "not_an_attr")
    o.parse_input_parameter(["lambda", 9, "solver", "pcg", "dangling"])
    assert o.lambda_ == 9 and o.solver == "pcg"


def test_params_flattening():
    from optical_flow.methods.config import load_of_method
    from optical_flow import _abi
    P = load_of_method("classic+nl-fast").to_params()
    assert P.method == _abi.METHOD["classic_nl"] and P.interp == _abi.INTERP["bi-cubic"]
    assert P.rho_data.kind == _abi.PENALTY["generalized_charbonnier"] and P.rho_data.p1 == 0.45
    assert P.qua_data.kind == _abi.PENALTY["quadratic"] and P.qua_data.p0 == 1e-3   # classic_nl.py:224-226
    assert P.use_wmf == 1 and P.median_filter_size == 5 and P.guide_mode == 1 and P.gnc_iters == 2
    P = load_of_method("classic-c").to_params()
    assert P.qua_data.p0 == 1.0 and P.qua_spatial_u[0].p0 == 1.0                     # ba.py:152-163 (ta = 1)
    P = load_of_method("ba").to_params()
    assert abs(P.qua_data.p0 - 50.0) < 1e-12                                          # ta = 1.5 / 0.03
    P = load_of_method("hs").to_params()
    assert P.rho_data.kind == _abi.PENALTY["const"] and P.rho_data.p0 == 1.0
    o = load_of_method("hs")
    o.solver = "cholesky"
    with pytest.raises(ValueError, match="Unknown solver"):
        o.to_params()
    o = load_of_method("ba")
    o.spatial_filters = [np.array([[1, -2, 1]])]  # general lists run (kernels_gen.hip)
    P = o.to_params()
    assert P.filters.general == 1 and P.filters.n == 1 and (P.filters.fh[0], P.filters.fw[0]) == (1, 3)
    o.spatial_filters = [np.ones((1, 6))]  # beyond 5 x 5 taps
    with pytest.raises(NotImplementedError):
        o.to_params()


# ---- penalties (reference tests/test_robust_functions.py) ------------------
def test_penalties_match_golden(golden):
    from optical_flow.robust import penalties as pen
    from optical_flow.robust.robust_function import RobustFunction
    from test_oracle_golden import PEN_CASES
    d = golden("penalties.npz")
    for k, (name, p) in enumerate(PEN_CASES):
        rf = RobustFunction(name, *p)
        for dt in range(3):
            np.testing.assert_allclose(getattr(pen, name)(d["x"], rf.param, dt), d[f"c{k}_d{dt}"], rtol=1e-13)
    assert np.allclose(RobustFunction("quadratic", 1.0).deriv_over_x(np.array([2.0])), [2.0])
    with pytest.raises(ValueError, match="Unknown penalty"):
        RobustFunction("invalid_method", 1.0)
    with pytest.raises(ValueError):
        pen.quadratic(np.array([1.0]), 1.0, 99)
    assert "lorentzian" in repr(RobustFunction("lorentzian", 0.5))
    rf = RobustFunction("lorentzian", 0.5)
    x = np.array([0.3])
    num = (rf.evaluate(x + 1e-7) - rf.evaluate(x - 1e-7)) / 2e-7
    np.testing.assert_allclose(rf.deriv(x), num, rtol=1e-5)


# ---- io / metrics / colour --------------------------------------------------
def test_flo_roundtrip_and_rubberwhale(tmp_path):
    from optical_flow import read_flo, write_flo
    f = np.random.default_rng(0).normal(size=(100, 200, 2)).astype(np.float32)
    write_flo(f, str(tmp_path / "a.flo"))
    np.testing.assert_array_equal(read_flo(str(tmp_path / "a.flo")), f)
    gt = read_flo(os.path.join(ROOT, "tests", "golden", "flow10.flo"))
    assert gt.shape == (388, 584, 2) and gt.dtype == np.float32
    with pytest.raises(ValueError):
        write_flo(np.zeros((10, 10)), str(tmp_path / "b.flo"))
    (tmp_path / "bad.flo").write_bytes(np.array([1.0, 0, 0], np.float32).tobytes())
    with pytest.raises(ValueError):
        read_flo(str(tmp_path / "bad.flo"))


def test_metrics_known_answers():
    from optical_flow import flow_angular_error
    z = np.zeros((10, 10))
    assert flow_angular_error(z, z, z, z) == (0.0, 0.0, 0.0)
    aae, _, aepe = flow_angular_error(np.array([[3.0]]), np.array([[0.0]]), np.array([[0.0]]), np.array([[0.0]]))
    assert aepe == 3.0
    tu = z.copy()
    tu[0, 0] = 1e10
    assert flow_angular_error(tu, z, z, z)[2] == 0.0
    rng = np.random.default_rng(1)
    a = rng.normal(size=(20, 20))
    assert flow_angular_error(a, a, a, a, border=5)[0] < 1e-5


def test_flow_to_color():
    from oracle_viz import flow_to_color  # the HIP path's checker (tests/test_gpu_viz.py)
    f = np.random.default_rng(2).normal(size=(20, 30, 2)) * 3
    f[0, 0, 0] = 2e9
    img = flow_to_color(f)
    assert img.dtype == np.uint8 and img.shape == (20, 30, 3) and (img[0, 0] == 0).all()


def test_flow_to_color_vs_reference(golden):
    """The oracle's flow_to_color (oracle/oracle_viz.py, the checker of the
    HIP path; viz/flow_color.py:43-107) bit-exact against the reference's
    images (tests/golden/gen_golden.py viz_metrics): RubberWhale GT with 7244
    unknown entries (auto and fixed max_flow), the reference's own RubberWhale
    uv in float32 (coloured in float32) and float64, a synthetic field with
    unknown rows/entries and rad > 1 saturation, and an all-zero field."""
    from oracle_viz import flow_to_color
    from optical_flow import read_flo
    d = golden("viz_metrics.npz")
    gt = read_flo(os.path.join(ROOT, "tests", "golden", "flow10.flo"))
    rw = golden("rubberwhale_ref.npz")
    cases = {"color_gt": flow_to_color(gt), "color_gt_max5": flow_to_color(gt, max_flow=5.0),
             "color_syn": flow_to_color(d["syn"]), "color_syn_max2": flow_to_color(d["syn"], max_flow=2.0),
             "color_syn_f32": flow_to_color(d["syn"].astype(np.float32)),
             "color_zero": flow_to_color(np.zeros((4, 5, 2)))}
    for name in ("classic+nl-fast", "hs-brightness"):
        cases[f"color_{name}"] = flow_to_color(rw[name])
        cases[f"color_{name}_f64"] = flow_to_color(rw[name].astype(np.float64))
    for k, img in cases.items():
        np.testing.assert_array_equal(img, d[k], err_msg=k)


def test_flow_angular_error_vs_reference(golden):
    """flow_angular_error (metrics.py:5-53) against the reference on
    RubberWhale (GT with unknown entries, borders 0 and 10) and a synthetic
    field whose GT has unknown entries in one component only (borders 0, 3)."""
    from optical_flow import flow_angular_error, read_flo
    d = golden("viz_metrics.npz")
    gt = read_flo(os.path.join(ROOT, "tests", "golden", "flow10.flo"))
    rw = golden("rubberwhale_ref.npz")
    for name in ("classic+nl-fast", "hs-brightness"):
        uv = rw[name]
        for border in (0, 10):
            got = flow_angular_error(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1], border)
            np.testing.assert_allclose(got, d[f"err_{name}_b{border}"], rtol=1e-12, err_msg=f"{name} b{border}")
    syn, est = d["syn"], d["syn_est"]
    for border in (0, 3):
        got = flow_angular_error(syn[..., 0], syn[..., 1], est[..., 0], est[..., 1], border)
        np.testing.assert_allclose(got, d[f"err_syn_b{border}"], rtol=1e-12, err_msg=f"syn b{border}")


# ---- sparse <-> planes (the narrow seam, base.py:87-114) --------------------
def test_planes_sparse_roundtrip(golden):
    from scipy import sparse
    from optical_flow.methods.base import planes_to_sparse, sparse_to_planes
    d = golden("operator.npz")
    H, W = d["uv"].shape[:2]
    N = H * W
    for tag in ("nl_robust", "ba_charb", "hs"):
        A = sparse.coo_matrix((d[tag + "_val"], (d[tag + "_row"], d[tag + "_col"])), shape=(2 * N, 2 * N)).tocsc()
        P = sparse_to_planes(A, H, W)
        assert abs(planes_to_sparse(P) - A).max() <= 1e-12 * abs(A).max()
    with pytest.raises(NotImplementedError):
        sparse_to_planes(sparse.random(2 * N, 2 * N, density=1e-3, random_state=0).tocsc(), H, W)


def test_synthetic_pair_deterministic():
    from optical_flow.utils.synthetic import synth_pair
    a1, a2, g = synth_pair(24, 40, seed=7)
    b1, b2, _ = synth_pair(24, 40, seed=7)
    assert np.array_equal(a1, b1) and np.array_equal(a2, b2)
    assert a1.shape == (24, 40, 3) and g.shape == (24, 40, 2)
    assert a1.min() >= 0 and a1.max() <= 255 and np.all(a1 == np.round(a1))


def test_solver_geometry_bounds():
    """of_solver_geometry (no device): every CG grid fits the partial-sum
    slots, the loop that sizes k_cg's bands terminates for very wide levels,
    and levels wider than the slots allow are refused, not mis-sized."""
    from optical_flow import _native
    for H, W in [(1080, 1920), (540, 960), (17, 30), (4096, 100), (64, 30000), (1, 1), (7, 57344)]:
        for solver in ("backslash", "pcg"):
            g = _native.solver_geometry(H, W, solver)
            assert 1 <= g["blocks"] == g["grid_x"] * g["grid_y"] <= 512, (H, W, solver, g)
            assert g["grid_x"] * g["strip_cols"] >= W
            per_block = 1 if solver == "backslash" else 4
            assert g["bands"] * g["rows"] >= H and g["grid_y"] * per_block >= g["bands"]
    for solver in ("backslash", "pcg"):
        with pytest.raises(NotImplementedError):
            _native.solver_geometry(64, 124 * 513, solver)
    g = _native.solver_geometry(480, 640, "sor")
    assert g["blocks"] == 2 * 8 and g["rows"] == 64
    with pytest.raises(NotImplementedError):
        _native.solver_geometry(64 * 257, 100, "sor")
    with pytest.raises(ValueError):
        _native.solver_geometry(0, 10, "pcg")


def test_estimate_flow_batch_rejects_mixed_channels():
    """Every frame of both lists is checked before the [:, :, :3] slice (a 1-
    or 2-channel frame would otherwise pass as 3 and be over-read); raised
    before any library call."""
    from optical_flow import estimate_flow_batch
    rgb = np.zeros((8, 10, 3), np.uint8)
    for bad in (np.zeros((8, 10, 2), np.uint8), np.zeros((8, 10, 1), np.uint8), np.zeros((8, 10), np.uint8),
                np.zeros((8, 11, 3), np.uint8), np.zeros((8, 10, 3, 1), np.uint8)):
        with pytest.raises(ValueError):
            estimate_flow_batch([rgb, bad], [rgb, rgb])
        with pytest.raises(ValueError):
            estimate_flow_batch([rgb, rgb], [rgb, bad])
    with pytest.raises(ValueError):
        estimate_flow_batch([], [])
    with pytest.raises(ValueError):
        estimate_flow_batch([np.full((8, 10, 3), 300.0)], [rgb])
