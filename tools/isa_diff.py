"""Compare the device ISA of two liboptflow.so builds, kernel by kernel.

A source cleanup (a removed A/B knob, a renamed helper) should leave the
default build's code object instruction-identical; this prints every kernel
whose instruction stream differs (addresses stripped) and exits 1 if any do.

    python tools/isa_diff.py old.so new.so
"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_census import disassemble  # noqa: E402


def _canon(lines):
    # --symbolize-operands numbers branch labels across the whole object:
    # renumber them per kernel in order of first use
    ids = {}
    sub = lambda m: "L%d" % ids.setdefault(m.group(0), len(ids))
    return [re.sub(r"\bL\d+\b", sub, ln) for ln in lines]


def kernels(lib):
    out, name = {}, None
    for ln in disassemble(lib).splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m and re.fullmatch(r"L\d+", m.group(1)) and name:
            out[name].append(m.group(1) + ":")  # a branch label inside the kernel
            continue
        if m:
            name = m.group(1)
            out[name] = []
            continue
        if name and ln.startswith("\t"):
            # drop the address / encoding comment, keep the instruction text
            out[name].append(ln.split("//")[0].strip())
    return {k: _canon(v) for k, v in out.items()}


def main(a, b):
    ka, kb = kernels(a), kernels(b)
    bad = sorted(n for n in set(ka) | set(kb) if ka.get(n) != kb.get(n))
    for n in bad:
        print(f"differs: {n} ({len(ka.get(n, []))} vs {len(kb.get(n, []))} instructions)")
    print(f"{len(set(ka) | set(kb))} symbols, {len(bad)} differ")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
