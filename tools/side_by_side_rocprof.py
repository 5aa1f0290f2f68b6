"""Aggregate HBM roofline of the fine CG solves as the timed lanes run them
(two solves side by side, each with CGS_LANES_BLOCKS = 252 k_cgs blocks),
from a rocprofv3 kernel trace of the default bench (tools/profile.sh, pass 1):
the 1080p k_cgs launches with the 252-block geometry (18 x 14 blocks of
64 x 4), 76 B per pixel per active launch (launches shorter
than 15 us returned after the prologue), over the union of their execution
intervals — the wall time during which at least one fine 1080p CG launch
runs.  Also the share of that time with two launches overlapping.

usage: python tools/side_by_side_rocprof.py gpurun_out/prof_TAG/trace_kernel_trace.csv [out.json]
"""
import csv
import json
import sys

PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md
N = 1080 * 1920
BYTES = 76 * N


def main():
    path = sys.argv[1]
    iv = []
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].replace("void ", "").startswith("k_cgs"):
            continue
        if (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])) != (18 * 64, 14 * 4):
            continue
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    active = [(s, e) for s, e in iv if e - s >= 15000]
    # union and 2-overlap time by a sweep over start / end events
    ev = sorted([(s, 1) for s, e in iv] + [(e, -1) for s, e in iv])
    depth, last, union, two = 0, None, 0, 0
    for t, d in ev:
        if last is not None and depth > 0:
            union += t - last
            if depth >= 2:
                two += t - last
        depth += d
        last = t
    dur = sum(e - s for s, e in active) / max(1, len(active))
    out = {
        "launches": len(iv), "active_launches": len(active),
        "mean_active_launch_us": dur / 1e3,
        "union_ms": union / 1e6, "two_overlapping_frac": two / max(1, union),
        "bytes_per_active_launch": BYTES,
        "achieved_GBps": len(active) * BYTES / union if union else 0.0,
        "peak_GBps": PEAK,
    }
    out["frac"] = out["achieved_GBps"] / PEAK
    out["per_launch_GBps"] = BYTES / dur if dur else 0.0
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
