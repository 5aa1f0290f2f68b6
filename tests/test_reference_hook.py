"""The reference-side binding (tools/reference_hook.py)
against the reference's OWN method objects.

tests/golden/ref_bags.json holds the reference's attribute bags (class name +
instance attributes, RobustFunction as .method / .sigma) for the 12 registry
names and four parse_input_parameter overrides (dict, flat list with a
dangling key, the 'lambda' alias, unknown keys, penalty objects), written by
`gen_golden.py bags` by importing the reference.  Here each bag is rebuilt as
a plain object of a class with the reference's class name, so the hook sees
exactly the attributes the reference defines and nothing of this package:

  - CPU: of_params_from(bag) equals this package's to_params() field by field;
  - CPU, when /root/reference is importable: of_params_from on the LIVE
    reference objects (in a subprocess with the reference on sys.path and the
    hook loaded as optical_flow._mi355x) is byte-identical to the fixture's;
  - GPU: the hook's estimate_flow through the C ABI on the golden crop.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, epe_stats

sys.path.insert(0, os.path.join(ROOT, "tools"))
import reference_hook as hook  # noqa: E402

REF = "/root/reference"


def _bags():
    with open(os.path.join(GOLDEN, "ref_bags.json")) as f:
        return json.load(f)


class _RF:
    """Stand-in for the reference's RobustFunction: only .method / .sigma."""

    def __init__(self, method, sigma):
        self.method, self.sigma = method, np.asarray(sigma, dtype=float)


def _dec(v, robust):
    if isinstance(v, dict) and "__robust__" in v:
        return robust(v["__robust__"], v["sigma"])
    if isinstance(v, dict) and "__ndarray__" in v:
        return np.asarray(v["__ndarray__"], dtype=float).reshape(v["shape"])
    if isinstance(v, list):
        return [_dec(x, robust) for x in v]
    return v


def _ref_object(bag):
    """A plain object of a class named like the reference's, carrying the
    reference's attributes only."""
    cls = type(bag["class"], (), {})
    o = cls()
    for k, v in bag["attrs"].items():
        setattr(o, k, _dec(v, _RF))
    return o


def _our_params(bag):
    from optical_flow.methods.config import load_of_method
    from optical_flow.robust.robust_function import RobustFunction
    ope = load_of_method(bag["method"])
    prm = bag["params"]
    if prm is not None:
        ours = lambda m, s: RobustFunction(m, *s)  # noqa: E731
        prm = {k: _dec(v, ours) for k, v in prm.items()} if isinstance(prm, dict) else _dec(prm, ours)
        ope.parse_input_parameter(prm)
    return ope.to_params()


def _diff(a, b, path=""):
    """Field-by-field comparison of two ctypes structures of the same layout."""
    out = []
    if isinstance(a, C.Structure):
        for name, _ in a._fields_:
            out += _diff(getattr(a, name), getattr(b, name), f"{path}.{name}")
    elif isinstance(a, C.Array):
        for i in range(len(a)):
            out += _diff(a[i], b[i], f"{path}[{i}]")
    elif a != b:
        out.append((path, a, b))
    return out


def test_hook_is_standalone():
    """The hook imports nothing from this repository's package at module level."""
    src = open(os.path.join(ROOT, "tools", "reference_hook.py")).read()
    code = [ln for ln in src.splitlines() if ln.startswith(("import ", "from "))]
    assert all("optical_flow" not in ln for ln in code), code
    from optical_flow import _abi
    assert C.sizeof(hook.OfParams) == C.sizeof(_abi.OfParams)
    assert [f[0] for f in hook.OfParams._fields_] == [f[0] for f in _abi.OfParams._fields_]


@pytest.mark.parametrize("tag", sorted(_bags()))
def test_of_params_from_reference_bag(tag):
    bag = _bags()[tag]
    P_hook = hook.of_params_from(_ref_object(bag))
    P_ours = _our_params(bag)
    d = _diff(P_hook, P_ours)
    assert not d, d[:10]
    assert bytes(P_hook) == bytes(P_ours)


def test_override_fixture_content():
    """The overrides took the reference's route (base.py:65-85)."""
    b = _bags()
    a = b["classic+nl-fast|dict"]["attrs"]
    assert a["lambda_"] == 5.0 and a["solver"] == "pcg" and "bogus_key" not in a
    a = b["classic-c|flat"]["attrs"]
    assert a["lambda_"] == 2.5 and a["pcg_rtol"] == 1e-4 and a["max_iters"] == 4 and "dangling" not in a
    a = b["classic++|robust"]["attrs"]
    assert a["rho_data"] == {"__robust__": "charbonnier", "sigma": [0.01]} and a["median_filter_size"] is None
    assert b["hs|dict"]["class"] == "HSOpticalFlow" and b["hs|dict"]["attrs"]["sigmaD2"] == 2.0


def test_hook_rejects_like_the_reference():
    bag = _ref_object(_bags()["classic+nl-fast"])
    bag.solver = "lu"
    with pytest.raises(ValueError):
        hook.of_params_from(bag)
    bag = _ref_object(_bags()["classic-c"])
    bag.rho_data = _RF("no_such_penalty", [1.0])
    with pytest.raises(ValueError):
        hook.of_params_from(bag)
    with pytest.raises(ValueError):
        hook.of_params_from(object())
    # a general filter list with one filter and unequal penalty lists
    bag = _ref_object(_bags()["classic-c"])
    bag.spatial_filters = [np.array([[1, -1]])]
    bag.rho_spatial_v = bag.rho_spatial_v[:1]
    P = hook.of_params_from(bag)
    assert P.filters.general == 1 and P.filters.n == 1


_LIVE = r"""
import importlib.util, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import optical_flow
from optical_flow.methods.config import load_of_method
from optical_flow.robust.robust_function import RobustFunction
assert optical_flow.__file__.startswith(sys.argv[1]), optical_flow.__file__
spec = importlib.util.spec_from_file_location("optical_flow._mi355x", sys.argv[2])
hook = importlib.util.module_from_spec(spec); spec.loader.exec_module(hook)
def dec(v):
    if isinstance(v, dict) and "__robust__" in v:
        return RobustFunction(v["__robust__"], *v["sigma"])
    if isinstance(v, dict) and "__ndarray__" in v:
        return np.asarray(v["__ndarray__"], dtype=float).reshape(v["shape"])
    if isinstance(v, list):
        return [dec(x) for x in v]
    return v
out = {}
for tag, bag in json.load(open(sys.argv[3])).items():
    ope = load_of_method(bag["method"])
    prm = bag["params"]
    if prm is not None:
        ope.parse_input_parameter({k: dec(v) for k, v in prm.items()} if isinstance(prm, dict) else dec(prm))
    out[tag] = [type(ope).__name__, bytes(hook.of_params_from(ope)).hex()]
print(json.dumps(out))
"""


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "optical_flow")), reason="reference not mounted here")
def test_of_params_from_live_reference():
    """The hook inside the reference package (loaded as optical_flow._mi355x
    next to the reference's own optical_flow) flattens the reference's live
    objects to the same bytes as the fixture's bags."""
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONPATH="")
    r = subprocess.run([sys.executable, "-c", _LIVE, REF, os.path.join(ROOT, "tools", "reference_hook.py"),
                        os.path.join(GOLDEN, "ref_bags.json")], capture_output=True, text=True, env=env,
                       cwd="/tmp", timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    live = json.loads(r.stdout.strip().splitlines()[-1])
    bags = _bags()
    assert set(live) == set(bags)
    for tag, (cls, hexbytes) in live.items():
        assert cls == bags[tag]["class"]
        assert hexbytes == bytes(hook.of_params_from(_ref_object(bags[tag]))).hex(), tag


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["classic+nl-fast", "hs|dict", "classic-c|flat", "classic+nl-fast|dict"])
def test_hook_estimate_flow_gpu(golden, tag):
    """The hook's estimate_flow body on the reference's bag, through the C ABI
    (its own ctypes binding of liboptflow.so), on the golden RubberWhale crop:
    bitwise equal to this package's estimate_flow with the same parameters,
    and for the plain registry name within the e2e gates of the golden flow."""
    import optical_flow
    bag = _bags()[tag]
    d = golden("e2e_small.npz")
    uv = hook.estimate_flow_ope(_ref_object(bag), d["im1"], d["im2"])
    prm = bag["params"]
    prm = _dec(prm, None) if not isinstance(prm, dict) else {k: _dec(v, None) for k, v in prm.items()}
    ours = optical_flow.estimate_flow(d["im1"], d["im2"], bag["method"], prm)
    assert uv.dtype == np.float64 and uv.shape == d["im1"].shape[:2] + (2,)
    np.testing.assert_array_equal(uv, ours)
    if prm is None:
        s = epe_stats(uv, d[bag["method"]])
        assert s["mean"] < 5e-4 and s["median"] < 4e-5, s  # test_gpu_e2e.py TOL["nlfast"]
    # gray input: (H, W) frames, the gray guide of interface.py:62-63
    g = hook.estimate_flow_ope(_ref_object(_bags()["classic+nl-fast"]), d["gray1"], d["gray2"])
    np.testing.assert_array_equal(g, optical_flow.estimate_flow(d["gray1"], d["gray2"], "classic+nl-fast"))
