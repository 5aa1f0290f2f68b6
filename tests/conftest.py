"""Shared test setup.

`gpu` tests call the HIP library through the C ABI and compare with the
golden fixtures (tests/golden/, generated from the reference) and with the
float64 CPU oracle (oracle/).  Everything else runs on CPU.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "optical-flow-python_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and liboptflow.so")
    config.addinivalue_line("markers", "slow: long-running (full-size images)")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name)))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def rubberwhale():
    from PIL import Image
    im1 = np.array(Image.open(os.path.join(GOLDEN, "frame10.png"))).astype(np.float64)
    im2 = np.array(Image.open(os.path.join(GOLDEN, "frame11.png"))).astype(np.float64)
    from optical_flow.io.flo_io import read_flo
    gt = read_flo(os.path.join(GOLDEN, "flow10.flo"))
    return im1, im2, gt


@pytest.fixture(scope="session")
def synthetic_pair():
    """The reference's own fixture (tests/conftest.py:44-54 there): seed 42,
    64x64 noise, 1-px horizontal shift."""
    rs = np.random.RandomState(42)
    im1 = rs.rand(64, 64) * 255
    im2 = np.zeros_like(im1)
    im2[:, 1:] = im1[:, :-1]
    im2[:, 0] = im1[:, 0]
    return im1, im2


def epe_stats(a, b):
    e = np.sqrt(((np.asarray(a) - np.asarray(b)) ** 2).sum(-1))
    return {"mean": float(e.mean()), "median": float(np.median(e)), "p99": float(np.percentile(e, 99)),
            "max": float(e.max())}
