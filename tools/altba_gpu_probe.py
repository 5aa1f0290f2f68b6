"""GPU probe: AltBA compute_flow_base at alpha = 0 on the
tests/golden/altba.npz level with the 'backslash' surrogate's tolerance and
iteration cap varied; EPE to the reference's (uv, uvhat) and the solve log
(iterations, done, fp64 true residual).  The float32-system floor after the
same 4 warps (reference with every solve on its system rounded to float32,
spsolve) is 1.46e-3 / 2.31e-3 px mean (replacement / not).
usage: python tools/altba_gpu_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
from optical_flow import _native  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "altba.npz"))
ctx = _native.context()
for rep in (True, False):
    key = f"base_a0_r{int(rep)}"
    for rtol, mx, solver in ((1e-6, 2000, "backslash"), (1e-9, 2000, "backslash"), (1e-9, 20000, "backslash"),
                             (1e-12, 20000, "backslash")):
        o = load_of_method("classic-c-a")
        o.images = d["base_images"]
        o.lambda2 = 0.01
        o.max_iters = 4
        o.alpha = 0.0
        o.replacement = rep
        o.solver = solver
        o.backslash_rtol = rtol
        o.backslash_maxiter = mx
        ctx.set_solve_log(True)
        uv, uvhat = o.compute_flow_base(d["base_uv"], d["base_uvhat"])
        recs = ctx.solve_log()
        ctx.set_solve_log(False)
        e = np.sqrt(((uv - d[key + "_uv"]) ** 2).sum(-1))
        print(f"rep {rep} rtol {rtol:g} maxiter {mx}: EPE mean {e.mean():.3e} median {np.median(e):.3e}; solves "
              + ", ".join(f"{r['iters']}it d{r['done']} true {r['true_rel']:.1e}" for r in recs), flush=True)

# the reference's own first-warp systems (tests/golden/altba_sys.npz): the
# GPU solver on them (solver error) and the GPU's robust assembly vs the
# reference's A, b (assembly error)
from scipy import sparse  # noqa: E402

s = np.load(os.path.join(ROOT, "tests", "golden", "altba_sys.npz"))
H, W = s["uv"].shape[:2]
n = 2 * H * W


def epe(x, y):
    dd = (x - y).reshape(2, -1)
    return float(np.sqrt((dd ** 2).sum(0)).mean())


for alpha in (0.0, 1.0):
    t = f"a{int(alpha)}_"
    A = sparse.coo_matrix((s[t + "val"], (s[t + "row"], s[t + "col"])), shape=(n, n)).tocsr()
    Af = (A + sparse.diags(s[t + "couple"])).tocsr()
    print(f"alpha {alpha}: float32 floor of the solve {epe(s[t + 'x32'], s[t + 'x64']):.3e}", flush=True)
    for rtol, mx in ((1e-6, 2000), (1e-9, 20000)):
        o = load_of_method("classic-c-a")
        o.backslash_rtol, o.backslash_maxiter = rtol, mx
        x = o._solve_linear_system(Af, s[t + "bfull"], (H, W, 2))
        xf = np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])
        print(f"  GPU solve of the reference system rtol {rtol:g} maxiter {mx}: {o.last_solve} "
              f"EPE to spsolve {epe(xf, s[t + 'x64']):.3e}", flush=True)
    if alpha == 0.0:
        o = load_of_method("classic-c-a")
        Ag, bg, _, _ = o.flow_operator(s["uv"], np.zeros_like(s["uv"]), s[t + "It"], s[t + "Ix"], s[t + "Iy"])
        dA = abs(Ag - A)
        print(f"  GPU assembly vs reference: max |dA| {dA.max():.3e} (max |A| {abs(A).max():.3e}), "
              f"rel {dA.max() / abs(A).max():.2e}; |db| {np.abs(bg - s[t + 'b']).max():.3e} "
              f"(|b| {np.abs(s[t + 'b']).max():.3e})", flush=True)
        x = o._solve_linear_system((Ag + sparse.diags(s[t + "couple"])).tocsr(),
                                   bg + (s[t + "bfull"] - s[t + "b"]), (H, W, 2))
        xf = np.concatenate([x[..., 0].ravel(order="F"), x[..., 1].ravel(order="F")])
        print(f"  GPU assembly + GPU solve: EPE to spsolve {epe(xf, s[t + 'x64']):.3e}", flush=True)
