#!/usr/bin/env python3
"""Per-phase instruction census of the weighted-median kernel (k_wmf<3,8,7>,
the 1080p Lab-guided 15x15 instance) from the gfx950 code object the library
ships, priced with measured issue costs.

  1. the code object: `.hip_fatbin` of liboptflow.so -> clang-offload-bundler
     -> llvm-objdump (the exact ISA the bench runs);
  2. phases by landmarks in the ISA, in program order: load (region reads,
     keys, records; the general-mirror arm, only taken on planes smaller than
     the tile + window, is left out), sort (up to the first ds_write_b16 of
     the sorted positions), scatter (positions and chunk ids), window (to the
     last chunk-sum atomic, ds_add_u64 / ds_add_f64), chunk (prefix sums), walk (the loop body x its trip
     count CH / 8 = 8), epilogue;
  3. each VALU opcode priced by tools/micro/valu_cost.hip's measurement
     (profiles/r5w_valu_cost.json, column w2: wave-cycles per instruction with
     two waves per SIMD -- the kernel's occupancy; a SIMD-cycle is half of
     that), opcodes it did not measure at the cost of the nearest measured
     class (listed in the output).

Output: JSON (per phase: counts by class, priced VALU cycles, top opcodes) and
a text table; with --phases FILE (tools/micro/wmf_phases output) the measured
cycles per wave beside the priced ones.

    python tools/isa_census.py --out profiles/r5_wmf_census
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "optical-flow-python_amd", "optical_flow", "_lib", "liboptflow.so")
KERNEL = "_Z5k_wmfILi3ELi8ELi7E"
WALK_TRIPS = 8  # CH / 8 = (8 * 64 / WMF_NC) / 8 sorted positions per 16-B read


def disassemble(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib,
                        os.path.join(d, "stripped")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], check=True,
                              capture_output=True, text=True).stdout


def kernel_lines(asm, prefix):
    out, on = [], False
    for ln in asm.splitlines():
        if re.match(r"^[0-9a-f]+ <_Z", ln):
            if on:
                break
            on = ln.split("<", 1)[1].startswith(prefix)
            continue
        if on:
            out.append(ln)
    if not out:
        sys.exit(f"kernel {prefix} not found")
    return out


def parse(lines):
    """[(label or None, opcode, text)] in program order"""
    ins, label = [], None
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(L\d+)>:", ln)
        if m:
            label = m.group(1)
            continue
        t = ln.strip()
        if not t or t.startswith("//"):
            continue
        op = t.split()[0]
        ins.append((label, op, t))
        label = None
    return ins


def klass(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_load") or op.startswith("s_memtime"):
        return "smem"
    return "salu"


# opcode -> measured case of tools/micro/valu_cost.hip (exact name or nearest
# class); the second field says which (exact / class)
def price_key(op):
    o = re.sub(r"_e(32|64)$", "", op)
    o = re.sub(r"_(sdwa|dpp)$", "", o)
    exact = {"v_add_f32": "v_add_f32", "v_mul_f32": "v_mul_f32", "v_fmac_f32": "v_fmac_f32",
             "v_exp_f32": "v_exp_f32", "v_max_f32": "v_max_f32", "v_and_b32": "v_and_b32",
             "v_bfe_u32": "v_bfe_u32", "v_lshl_add_u32": "v_lshl_add_u32", "v_xor_b32": "v_xor_b32",
             "v_cvt_f64_f32": "v_cvt_f64_f32", "v_mul_lo_u32": "v_mul_lo_u32", "v_min_f64": "v_min_f64",
             "v_max_f64": "v_min_f64", "v_add_f64": "v_add_f64", "v_lshl_add_u64": "v_lshl_add_u64",
             "v_mov_b64": "v_mov_b64", "v_pk_add_f32": "v_pk_add_f32", "v_pk_mul_f32": "v_pk_mul_f32",
             "v_pk_fma_f32": "v_pk_fma_f32", "v_permlane32_swap_b32": "v_permlane32_swap",
             "v_permlane16_swap_b32": "v_permlane32_swap"}
    if op.startswith("v_mov_b32_dpp") or op.endswith("_dpp"):
        return "v_mov_b32_dpp row_ror", "class"
    if o.startswith("v_cndmask_b32"):
        return ("v_cndmask_b32_e64", "exact") if op.endswith("_e64") else ("v_cndmask_b32(vcc)", "exact")
    if o in exact:
        return exact[o], "exact"
    if op.endswith("_sdwa"):
        return "v_sub_u32_sdwa", "class"
    if re.match(r"v_cmp\w*_f64", o):
        return "v_cmp_nlt_f64_e64", "class"
    if re.search(r"_f64$", o) or o.startswith("v_cvt_f64"):
        return "v_add_f64", "class"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)", o):
        return "v_exp_f32", "class"
    if re.search(r"(mul_hi|mul_lo|mad_u64|mad_i64)", o):
        return "v_mul_lo_u32", "class"
    if re.search(r"_(b64|u64|i64)$", o):
        return "v_lshl_add_u64", "class"
    if o.startswith("v_pk_"):
        return "v_pk_add_f32", "class"
    if o.startswith(("v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_and_", "v_or_", "v_xor_",
                     "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32")):
        return "v_add_f32", "class"
    return "v_lshl_add_u32", "class"  # other VOP3 integer / compare / cvt: the 3-operand ALU rate


def phases(ins):
    ops = [o for _, o, _ in ins]

    def first(pred, start=0):
        for i in range(start, len(ins)):
            if pred(i):
                return i
        sys.exit("landmark not found")

    def last(pred):
        for i in range(len(ins) - 1, -1, -1):
            if pred(i):
                return i
        sys.exit("landmark not found")

    zero = last(lambda i: ops[i].startswith("ds_write2st64_b64"))  # chunk sums cleared: end of load
    scat = first(lambda i: ops[i] == "ds_write_b16", zero)
    win = first(lambda i: ops[i].startswith("ds_read_b") and ops[i] != "ds_read_b16", scat)
    wend = last(lambda i: ops[i] in ("ds_add_f64", "ds_add_u64"))
    # the walk: the backward branch after the window pass
    back = None
    for i in range(wend, len(ins)):
        if ops[i].startswith("s_cbranch"):
            tgt = ins[i][2].split()[1]
            lab = [j for j in range(len(ins)) if ins[j][0] == tgt]
            if lab and lab[0] <= i and lab[0] > wend:
                back = (lab[0], i)
    if back is None:
        sys.exit("walk loop not found")
    # load phase: drop the basic blocks of the general-mirror arm (integer
    # division: v_rcp_iflag_f32), not taken when the plane holds tile + window
    load = list(range(0, zero + 1))
    blocks, cur = [], []
    for i in load:
        if ins[i][0] and cur:
            blocks.append(cur)
            cur = []
        cur.append(i)
    if cur:
        blocks.append(cur)
    load_kept = [i for b in blocks if not any(ops[j] == "v_rcp_iflag_f32_e32" for j in b) for i in b]
    return {"load": (load_kept, 1), "sort": (list(range(zero + 1, scat)), 1),
            "scatter": (list(range(scat, win)), 1), "window": (list(range(win, wend + 1)), 1),
            "chunk": (list(range(wend + 1, back[0])), 1),
            "walk": (list(range(back[0], back[1] + 1)), WALK_TRIPS),
            "epilogue": (list(range(back[1] + 1, len(ins))), 1)}


def read_phases(path):
    """mean cycles per wave per phase, last line of tools/micro/wmf_phases"""
    ln = [l for l in open(path) if "mean cycles per wave" in l][-1]
    d = dict(re.findall(r"(load|sort|window|chunk|walk) (\d+)", ln))
    return {k: int(v) for k, v in d.items()}, float(re.search(r"launch ([\d.]+) ms", ln).group(1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--kernel", default=KERNEL)
    ap.add_argument("--costs", default=os.path.join(ROOT, "profiles", "r5w_valu_cost.json"))
    ap.add_argument("--phases", default=None, help="tools/micro/wmf_phases output (measured cycles)")
    ap.add_argument("--out", default=None, help="write OUT.json and OUT.txt")
    a = ap.parse_args()
    costs = {c["op"]: c for c in json.load(open(a.costs))["cases"]}
    ins = parse(kernel_lines(disassemble(a.lib), a.kernel))
    ph = phases(ins)
    meas, launch_ms = read_phases(a.phases) if a.phases else ({}, None)
    res, approx = {}, collections.Counter()
    tot = collections.Counter()
    for name, (idx, trips) in ph.items():
        cls, ops = collections.Counter(), collections.Counter()
        cyc2 = cyc1 = 0.0
        for i in idx:
            op = ins[i][1]
            k = klass(op)
            cls[k] += trips
            if k == "valu":
                ops[op] += trips
                key, how = price_key(op)
                if how != "exact":
                    approx[f"{op} -> {key}"] += trips
                cyc2 += trips * costs[key]["w2"]
                cyc1 += trips * costs[key]["w1"]
        r = {"trips": trips, "static_instructions": len(idx), "dynamic": dict(cls),
             "valu_wave_cycles_2w": round(cyc2), "valu_wave_cycles_1w": round(cyc1),
             "valu_simd_cycles": round(cyc2 / 2), "top_valu": ops.most_common(12)}
        if name in meas:
            r["measured_wave_cycles"] = meas[name]
        res[name] = r
        for k, v in cls.items():
            tot[k] += v
        tot["valu_simd_cycles"] += cyc2 / 2
        tot["valu_wave_cycles_2w"] += cyc2
    out = {"kernel": a.kernel, "lib": os.path.relpath(a.lib, ROOT), "costs": os.path.relpath(a.costs, ROOT),
           "price": "VALU opcode x tools/micro/valu_cost.hip w2 (wave-cycles per instruction at 2 waves "
                    "per SIMD); SIMD-cycles = half of that",
           "phases": res, "total": {k: round(v) for k, v in tot.items()},
           "approximated_opcodes": dict(approx.most_common())}
    if launch_ms:
        out["measured_launch_ms"] = launch_ms
    lines = [f"{a.kernel}  ({out['lib']}; prices {out['costs']}, w2 column)",
             f"{'phase':9s} {'VALU':>6s} {'SALU':>5s} {'LDS':>5s} {'VMEM':>5s} {'wait':>5s}"
             f" {'VALU cyc (2w)':>13s} {'measured':>9s}  top VALU"]
    for name, r in res.items():
        d = r["dynamic"]
        lines.append(f"{name:9s} {d.get('valu', 0):6d} {d.get('salu', 0):5d} {d.get('lds', 0):5d}"
                     f" {d.get('vmem', 0):5d} {d.get('wait', 0):5d} {r['valu_wave_cycles_2w']:13d}"
                     f" {r.get('measured_wave_cycles', ''):>9}  "
                     + ", ".join(f"{o.replace('_e32', '').replace('_e64', '')} {n}" for o, n in r["top_valu"][:5]))
    t = out["total"]
    lines.append(f"{'total':9s} {t.get('valu', 0):6d} {t.get('salu', 0):5d} {t.get('lds', 0):5d}"
                 f" {t.get('vmem', 0):5d} {t.get('wait', 0):5d} {t['valu_wave_cycles_2w']:13d}"
                 f" {sum(meas.values()) if meas else '':>9}")
    lines.append("approximated (no exact measurement): " +
                 ", ".join(f"{k} x{v}" for k, v in list(approx.most_common())[:10]))
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        json.dump(out, open(a.out + ".json", "w"), indent=1)
        open(a.out + ".txt", "w").write(txt + "\n")


if __name__ == "__main__":
    main()
