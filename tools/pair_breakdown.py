"""Kernel time of one serial pair by kernel and grid (= pyramid level), from
a rocprofv3 kernel trace of `bench.py --lanes 1` (tools/profile.sh's
trace1_kernel_trace.csv).  Pairs are delimited by their k_rgb_max dispatch;
the PAIR-th one (default 5: past the warm-up) is reported.
usage: python tools/pair_breakdown.py TRACE_CSV [PAIR] > breakdown.txt"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void k_rgb_max")]
    pair = rows[starts[k]:starts[k + 1]]
    t0, t1 = int(pair[0]["Start_Timestamp"]), int(pair[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in pair) / 1e6
    print(f"pair {k}: span {(t1 - t0) / 1e6:.3f} ms, kernel time {busy:.3f} ms, {len(pair)} dispatches")
    g = collections.defaultdict(lambda: [0, 0.0])
    for r in pair:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (n, f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}")
        g[key][0] += 1
        g[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{'kernel':32s} {'grid (threads)':>16s} {'calls':>6s} {'total us':>10s} {'mean us':>9s}")
    for (n, grid), (c, t) in sorted(g.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:32s} {grid:>16s} {c:6d} {t:10.1f} {t / c:9.1f}")


if __name__ == "__main__":
    main()
