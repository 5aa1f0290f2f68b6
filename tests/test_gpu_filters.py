"""General spatial_filters on the GPU (kernels_gen.hip) vs the reference's own
outputs (tests/golden/filters.npz, gen_golden.py gen_filters):
flow_operator A, b for three filter lists (first differences in four
directions, second differences, one horizontal filter), the three linear
solvers on the reference's diag4 operator, and estimate_flow end to end on
the RubberWhale crop.  The float64 oracle covers the default pair only, so
these are pinned by the reference's fixtures directly."""
import numpy as np
import pytest
from scipy import sparse
from scipy.sparse.linalg import LinearOperator, cg

from conftest import epe_stats

pytestmark = pytest.mark.gpu

SETS = {
    "diag4": [np.array([[1, -1]]), np.array([[1], [-1]]), np.array([[1, 0], [0, -1]]), np.array([[0, 1], [-1, 0]])],
    "wide": [np.array([[1, -2, 1]]), np.array([[1], [-2], [1]])],
    "one": [np.array([[1, -1]])],
}
METH = {"diag4": "classic+nl-fast", "wide": "classic-c", "one": "classic+nl-fast"}
OP_METH = {"diag4": "classic+nl-fast", "wide": "ba", "one": "classic+nl-fast"}  # gen_golden.py gen_filters


def _method(tag, op=False):
    from optical_flow.methods.config import load_of_method
    o = load_of_method((OP_METH if op else METH)[tag])
    n = len(SETS[tag])
    o.spatial_filters = SETS[tag]
    o.rho_spatial_u = [o.rho_spatial_u[i % 2] for i in range(n)]
    o.rho_spatial_v = [o.rho_spatial_v[i % 2] for i in range(n)]
    return o


def _ref_A(d, key):
    H, W = d["uv"].shape[:2]
    n = 2 * H * W
    return sparse.coo_matrix((d[key + "_val"], (d[key + "_row"], d[key + "_col"])), shape=(n, n)).tocsr()


@pytest.mark.parametrize("tag", ["diag4", "wide", "one"])
@pytest.mark.parametrize("with_duv", [False, True])
def test_flow_operator_general(golden, tag, with_duv):
    """classic_nl.py:279-378 / ba.py:208-302 with a general filter list:
    the GPU's DIA planes rebuilt as scipy A equal the reference's A (and b) to
    float32 rounding (the default pair's gates, tests/test_gpu_stages.py::
    test_flow_operator: 5e-5 max|A|, 1e-4 max|b|; inputs are float32-exact)."""
    d = golden("filters.npz")
    key = f"op_{tag}" + ("_duv" if with_duv else "")
    o = _method(tag, op=True)
    A, b, _, _ = o.flow_operator(d["uv"], d["duv"] if with_duv else None, d["It"], d["Ix"], d["Iy"])
    R = _ref_A(d, key)
    scale = abs(R).max()
    err = abs(A - R).max() / scale
    berr = np.abs(b - d[key + "_b"]).max() / np.abs(d[key + "_b"]).max()
    print(f"{key}: A rel {err:.2e}  b rel {berr:.2e}  nnz {A.nnz} vs {R.nnz}")
    assert err <= 5e-5 and berr <= 1e-4


def test_solvers_general_operator(golden):
    """_solve_linear_system (base.py:87-172) on the reference's diag4
    operator: 'backslash' vs spsolve, 'sor' vs the reference's lexicographic
    SOR (same sweep count), 'pcg' vs scipy cg with the Jacobi preconditioner."""
    d = golden("filters.npz")
    A = _ref_A(d, "op_diag4")
    b = d["op_diag4_b"]
    H, W = d["uv"].shape[:2]
    o = _method("diag4", op=True)
    o.solver = "backslash"
    x = o._solve_linear_system(A, b, (H, W, 2)).ravel(order="F")
    ref = d["spsolve_diag4_x"]
    e = np.abs(x - ref).max() / np.abs(ref).max()
    rres = np.linalg.norm(A @ x - b) / np.linalg.norm(b)
    print(f"backslash: max rel err {e:.2e}, residual {rres:.2e}, iters {o.last_solve}")
    # a float32 x of this operator cannot go below ~2e-6 (its own solve log:
    # the refinement stops at the fp32 floor); measured 1.5e-5 / 4.2e-6
    assert e < 1e-4 and rres < 1e-5
    o.solver = "sor"
    x = o._solve_linear_system(A, b, (H, W, 2)).ravel(order="F")
    ref = d["sor_diag4_x"]
    e = np.abs(x - ref).max() / np.abs(ref).max()
    print(f"sor: sweeps {o.last_solve['iters']} vs {int(d['sor_diag4_sweeps'])}, max rel err {e:.2e}")
    assert abs(o.last_solve["iters"] - int(d["sor_diag4_sweeps"])) <= 1 and e < 1e-3
    o.solver = "pcg"
    x = o._solve_linear_system(A, b, (H, W, 2)).ravel(order="F")
    dg = A.diagonal()
    M = LinearOperator(A.shape, matvec=lambda v: np.where(np.abs(dg) > 1e-12, 1.0 / dg, 0.0) * v)
    xs, _ = cg(A, b, M=M, maxiter=o.pcg_maxiter, rtol=o.pcg_rtol)
    e = np.abs(x - xs).max() / np.abs(xs).max()
    print(f"pcg: max rel err vs scipy cg {e:.2e}, iters {o.last_solve}")
    assert e < 2e-2


# measured (round 3): diag4 1.25e-5 / 9.0e-6 px mean / median; wide
# (classic-c, Charbonnier 1e-3, 'pcg' at rtol 1e-3: the chaotic family of
# test_gpu_e2e.py) 6.6e-3 / 3.4e-3
@pytest.mark.parametrize("tag,tol", [("diag4", (1e-4, 5e-5)), ("wide", (2e-2, 1e-2))])
def test_e2e_general_filters(golden, tag, tol):
    """estimate_flow with a general spatial_filters list (classic+nl-fast with
    four first-difference filters; classic-c with second differences and
    'pcg') on the RubberWhale crop vs the reference."""
    import optical_flow
    d = golden("filters.npz")
    o = _method(tag)
    prm = {"spatial_filters": o.spatial_filters, "rho_spatial_u": o.rho_spatial_u, "rho_spatial_v": o.rho_spatial_v}
    if tag == "wide":
        prm["solver"] = "pcg"
    uv = optical_flow.estimate_flow(d["im1"], d["im2"], METH[tag], prm)
    s = epe_stats(uv, d[f"e2e_{tag}"])
    print(tag, s)
    assert np.all(np.isfinite(uv))
    assert s["mean"] <= tol[0] and s["median"] <= tol[1], s


def test_general_filter_solves_logged(golden):
    """Solves of a general spatial_filters list go through the DIA path
    (gen_solve) and are recorded by the solve log like the 5-point ones, with
    their fp64 true residual: 'backslash' meets its 1e-6 goal (iterative
    refinement on that residual)."""
    import optical_flow
    from optical_flow import _native
    d = golden("filters.npz")
    o = _method("diag4")
    prm = {"spatial_filters": o.spatial_filters, "rho_spatial_u": o.rho_spatial_u, "rho_spatial_v": o.rho_spatial_v}
    ctx = _native.context()
    ctx.set_solve_log(True)
    try:
        optical_flow.estimate_flow(d["im1"], d["im2"], METH["diag4"], prm)
        recs = ctx.solve_log()
    finally:
        ctx.set_solve_log(False)
    assert len(recs) > 0
    for r in recs:
        print(r)
    assert all(r["solver"] == 0 and r["done"] in (1, 3) for r in recs)
    assert max(r["true_rel"] for r in recs) <= 1.5e-6
    assert all(r["true_rel_out"] == r["true_rel"] for r in recs)
