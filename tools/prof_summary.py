"""Summarise a tools/profile.sh run: per kernel at the finest level, mean
dispatch duration, HBM bytes (FETCH_SIZE, WRITE_SIZE; KB units), L2 hit rate,
and the algorithmic-bytes roofline.  Writes <dir>/summary.json and, with
--traffic, profiles/pmc_traffic.json (read by bench.py).

usage: python tools/prof_summary.py gpurun_out/prof_TAG [--H 1080 --W 1920] [--traffic]
       [--workload classic+nl-fast@1080x1920/backslash]
The traffic file is keyed by workload (bench.py's method@HxW/solver), then
by bench kernel name, each record naming the kernel symbol it measured.
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(name):
    """kernel family: template variants of the CG / weighted-median kernels
    (first launch, odd width; guide channels) are one kernel here"""
    n = name.split("(")[0].replace("void ", "")
    # the assembly kernels' penalty-mode instances are one kernel; the fused
    # warp + assembly keeps its interpolation (different bytes per pixel)
    if n.startswith("k_flow_operator<"):
        return "k_flow_operator"
    if n.startswith("k_warp_operator<"):
        return "k_warp_operator<" + n[len("k_warp_operator<"):].split(",")[0].strip() + ">"
    for fam in ("k_cgs", "k_cgp", "k_cgn", "k_cg_small", "k_cg<", "k_wmf"):
        if n.startswith(fam):
            return fam.rstrip("<")
    return n


def grid_key(r):
    """total threads of the dispatch (kernel-trace rows carry X/Y/Z, counter rows the product)"""
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def load_counters(path, counter):
    """dispatch id -> summed counter value"""
    out = collections.defaultdict(float)
    meta = {}
    if not os.path.exists(path):
        return out, meta
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        out[d] += float(r["Counter_Value"])
        meta[d] = (short(r["Kernel_Name"]), grid_key(r))
    return out, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--traffic", action="store_true")
    ap.add_argument("--workload", default="classic+nl-fast@1080x1920/backslash")
    ap.add_argument("--source", default=None, help="note stored with the records (e.g. the profile tag)")
    a = ap.parse_args()
    import bench  # noqa: E402  (KERNEL_BYTES_PER_PX, profiler names)
    d = a.dir
    # durations from the isolated (lanes = 1) trace when present: a kernel's
    # own duration, not stretched by another lane's kernels (bench roofline)
    tname = "trace1_kernel_trace.csv" if os.path.exists(os.path.join(d, "trace1_kernel_trace.csv")) else \
        "trace_kernel_trace.csv"
    trace = list(csv.DictReader(open(os.path.join(d, tname))))
    dur = collections.defaultdict(list)
    for r in trace:
        dur[(short(r["Kernel_Name"]), grid_key(r))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fetch, fmeta = load_counters(os.path.join(d, "fetch_counter_collection.csv"), "FETCH_SIZE")
    write, wmeta = load_counters(os.path.join(d, "write_counter_collection.csv"), "WRITE_SIZE")
    hit, hmeta = load_counters(os.path.join(d, "l2_counter_collection.csv"), "TCC_HIT_sum")
    miss, _ = load_counters(os.path.join(d, "l2_counter_collection.csv"), "TCC_MISS_sum")
    valu, vmeta = load_counters(os.path.join(d, "valu_counter_collection.csv"), "SQ_INSTS_VALU")

    def per_key(vals, meta):
        acc = collections.defaultdict(list)
        for disp, v in vals.items():
            acc[meta[disp]].append(v)
        return acc

    F, Wr, Hh, M = per_key(fetch, fmeta), per_key(write, wmeta), per_key(hit, hmeta), per_key(miss, hmeta)
    V = per_key(valu, vmeta)
    # finest-level dispatches: the grid with the most pixels per kernel name
    rows = []
    names = {}
    for (n, g), v in dur.items():
        tot = sum(v)
        names.setdefault(n, []).append((g, v))
    out = {}
    H, W = a.H, a.W

    for n, lst in names.items():
        tot_ms = sum(sum(v) for _, v in lst) / 1e6
        g, v = max(lst, key=lambda gv: gv[0])  # finest level: the largest grid
        vs = sorted(v)
        # active (non early-exit) dispatches: at least half the median
        # duration; the median is robust to dispatches slowed by a concurrent
        # lane's kernels
        med = vs[len(vs) // 2]
        act = [x for x in vs if x >= 0.5 * med]
        mean_us = act[len(act) // 2] / 1e3
        rec = {"total_ms": round(tot_ms, 3), "finest_grid": g, "finest_calls": len(v), "finest_active_calls": len(act),
               "finest_median_us": round(mean_us, 2), "all_mean_us": round(tot_ms * 1e3 / sum(len(x) for _, x in lst), 2)}
        fk = [x for x in F.get((n, g), []) if x > 0]
        wk = [x for x in Wr.get((n, g), []) if x > 0]
        if fk:
            fk = sorted(fk)[len(fk) // 2:]  # active dispatches (no-op CG launches fetch ~nothing)
            rec["fetch_MB"] = round(sum(fk) / len(fk) * 1024 / 1e6, 3)
        if wk:
            wk = sorted(wk)[len(wk) // 2:]
            rec["write_MB"] = round(sum(wk) / len(wk) * 1024 / 1e6, 3)
        vk = V.get((n, g), [])
        if vk:  # VALU wave-instructions per finest-level dispatch (median)
            rec["valu_insts_per_launch"] = int(sorted(vk)[len(vk) // 2])
        hk, mk = Hh.get((n, g), []), M.get((n, g), [])
        if hk and mk and sum(hk) + sum(mk) > 0:
            rec["l2_hit"] = round(sum(hk) / (sum(hk) + sum(mk)), 3)
        key = {"k_cgs": "pcg_iter", "k_cgp": "pcg_iter", "k_cg": "pcg_iter", "k_flow_operator": "flow_operator",
               "k_wmf": "wmf", "k_rof_iters": "rof_iters", "k_update_occ": "update_occ",
               "k_partial_deriv<1>": "partial_deriv_hermite", "k_sor_pipe": "sor_pipe", "k_sor_lex": "sor_sweep",
               "k_warp_operator<1>": "warp_operator_hermite", "k_warp_operator<0>": "warp_operator_bspline",
               "k_warp_operator<2>": "warp_operator_bilinear"}.get(n)
        if key in bench.KERNEL_BYTES_PER_PX:
            px = a.H * a.W * (2 if key == "rof_iters" else 1)
            alg = bench.KERNEL_BYTES_PER_PX[key] * px
            rec["alg_MB"] = round(alg / 1e6, 3)
            rec["alg_GBps"] = round(alg / (mean_us * 1e-6) / 1e9, 1)
            if "fetch_MB" in rec and "write_MB" in rec:
                # FETCH_SIZE counts 64 B per 128-B request on gfx950
                # (MI355X_MICROARCH.md HBM section; re-checked on k_rof_iter's
                # known byte count): double it, WRITE_SIZE is exact
                rec["hbm_bytes_per_launch"] = int((2 * rec["fetch_MB"] + rec["write_MB"]) * 1e6)
            rec["bench_name"] = key
            # every dispatch of the kernel (all levels, incl. converged no-op
            # CG launches): comparable with bench.py's all-launch roofline
            fa = [v for disp, v in fetch.items() if fmeta[disp][0] == n]
            wa = [v for disp, v in write.items() if wmeta[disp][0] == n]
            if fa and wa:
                rec["hbm_bytes_per_launch_all"] = int((2 * sum(fa) / len(fa) + sum(wa) / len(wa)) * 1024)
        out[n] = rec
    out = dict(sorted(out.items(), key=lambda kv: -kv[1]["total_ms"]))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    for n, r in list(out.items())[:14]:
        print(f"{n[:34]:34s} {json.dumps(r)}")
    if a.traffic:
        recs = {r["bench_name"]: {"symbol": n, "source": a.source or os.path.basename(os.path.normpath(d)),
                                  "hbm_bytes_per_launch": r.get("hbm_bytes_per_launch"),
                                  "hbm_bytes_per_launch_all": r.get("hbm_bytes_per_launch_all"),
                                  "fetch_MB": r.get("fetch_MB"),
                                  "write_MB": r.get("write_MB"), "grid": r["finest_grid"],
                                  "l2_hit": r.get("l2_hit"),
                                  "valu_insts_per_launch": r.get("valu_insts_per_launch"),
                                  "note": "2*FETCH_SIZE + WRITE_SIZE (KB->B) per dispatch at the finest level "
                                          "(FETCH_SIZE x2: gfx950 tallies 128-B requests at 64 B); "
                                          "Infinity-Cache (MALL) hits are included in FETCH_SIZE"}
                for n, r in out.items() if "bench_name" in r}
        p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
        traffic = json.load(open(p)) if os.path.exists(p) else {}
        traffic[a.workload] = recs
        json.dump(traffic, open(p, "w"), indent=1)


if __name__ == "__main__":
    main()
