"""CPU sanitizer run of the oracle ("-fsanitize=address on a
CPU build"): oracle/asan/asan_driver links optflow_oracle.c under
-fsanitize=address,undefined and runs ofr_estimate_flow for every registry
method (the same of_params records the product receives, from
BaseOpticalFlow.to_params) on a 24x32 RGB pair.  Test infrastructure only:
it checks the checker's memory safety, not the GPU path."""
import os
import shutil
import subprocess

import pytest

from optical_flow.methods.config import METHOD_NAMES, load_of_method

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_asan_all_methods(tmp_path):
    r = subprocess.run(["make", "-s", "-C", ORACLE, "asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    blob = b""
    names = sorted(METHOD_NAMES)
    for name in names:
        ope = load_of_method(name)
        P = ope.to_params()
        P.guide_mode = int(ope._METHOD == "classic_nl" and ope.color_images is not None)
        blob += bytes(P)
    pfile = tmp_path / "params.bin"
    pfile.write_bytes(blob)
    env = dict(os.environ, OMP_NUM_THREADS="1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "asan", "asan_driver"), str(pfile), "24", "32"],
                       capture_output=True, text=True, env=env, timeout=600)
    log = r.stdout + r.stderr
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert r.returncode == 0, log[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("method ")]
    assert len(lines) == len(names)
