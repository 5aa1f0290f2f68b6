"""ISA-level guards on the shipped weighted-median kernel (k_wmf<3,8,7>, the
1080p instance), read from liboptflow.so's gfx950 code object by
tools/isa_census.py (CPU only: llvm-objdump, no GPU).  They pin the two round-5
restructurings that the timing depends on, so a compiler or source change that
undoes one fails here rather than as a slower bench:
  - the region load issues every global read before the first vmcnt wait
    (was one round trip per sample: profiles/r5x_wmf_load_ab.log);
  - the sort's cross-lane stages compare without v_cmp_*_f64 + SALU mask
    arithmetic (profiles/r5y_wmf_sort_ab.log).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_census as ic  # noqa: E402

pytestmark = pytest.mark.skipif(not (os.path.exists(ic.LIB) and os.path.exists(f"{ic.LLVM}/llvm-objdump")),
                                reason="needs the built library and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def wmf():
    ins = ic.parse(ic.kernel_lines(ic.disassemble(ic.LIB), ic.KERNEL))
    return ins, ic.phases(ins)


def test_phases_in_order(wmf):
    ins, ph = wmf
    names = list(ph)
    assert names == ["load", "sort", "scatter", "window", "chunk", "walk", "epilogue"]
    starts = [ph[n][0][0] for n in names if ph[n][0]]
    assert starts == sorted(starts)
    assert ph["walk"][1] == 8
    ops = [o for _, o, _ in ins]
    assert sum(1 for i in ph["window"][0] if ops[i] in ("ds_add_u64", "ds_add_f64")) == 2 * 15 * 15


def test_region_reads_before_first_wait(wmf):
    ins, ph = wmf
    load = ph["load"][0]
    ops = [ins[i][1] for i in load]
    reads = [k for k, o in enumerate(ops) if o.startswith("global_load")]
    waits = [k for k, (o, t) in enumerate(zip(ops, (ins[i][2] for i in load)))
             if o == "s_waitcnt" and "vmcnt" in t]
    # 8 samples per lane: uv (dwordx2) + 3 guide + occ dwords each
    assert len(reads) == 8 * 5
    assert waits and max(reads) < min(waits)


def test_sort_has_no_f64_compares_or_salu_masks(wmf):
    ins, ph = wmf
    ops = [ins[i][1] for i in ph["sort"][0]]
    assert not [o for o in ops if o.startswith("v_cmp") and "f64" in o]
    assert sum(o.startswith("s_xor") for o in ops) <= 4
    # 18 of the 21 cross-lane stages (DPP partners) are one min(own, -partner)
    # per key (8 keys x 2 lists)
    assert sum(o == "v_min_f64" for o in ops) >= 18 * 16
