"""GPU occupancy of a rocprofv3 --kernel-trace run: in consecutive windows,
the fraction of time at least one kernel runs (busy), the mean number of
kernels in flight, and the largest idle gaps with the kernels around them.

usage: python tools/timeline.py <kernel_trace.csv> [--win-ms 100]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--win-ms", type=float, default=100.0)
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    ev = []
    for r in csv.DictReader(open(a.trace)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
    ev.sort()
    t0 = ev[0][0]
    # union of busy intervals, gaps between them
    busy = []
    cs, ce = ev[0][0], ev[0][1]
    gaps = []
    prev_name = ev[0][2]
    last_end_name = ev[0][2]
    for s, e, n in ev[1:]:
        if s > ce:
            busy.append((cs, ce))
            gaps.append((s - ce, (ce - t0) / 1e6, last_end_name, n))
            cs, ce = s, e
            last_end_name = n
        elif e > ce:
            ce = e
            last_end_name = n
    busy.append((cs, ce))
    win = a.win_ms * 1e6
    tend = max(e for _, e, _ in ev)
    print(f"span {(tend - t0) / 1e6:.1f} ms, {len(ev)} kernels")
    w = t0
    while w < tend:
        we = w + win
        b = sum(max(0, min(e, we) - max(s, w)) for s, e in busy)
        k = sum(max(0, min(e, we) - max(s, w)) for s, e, _ in ev)
        print(f"  [{(w - t0) / 1e6:8.1f} ms] busy {b / win:5.3f}  kernels in flight {k / max(b, 1):4.2f}")
        w = we
    gaps.sort(reverse=True)
    print("largest gaps (us, at ms, before -> after):")
    for g, at, n0, n1 in gaps[:a.gaps]:
        print(f"  {g / 1e3:8.1f}  {at:9.2f}  {n0} -> {n1}")
    tot_gap = sum(g for g, *_ in gaps)
    print(f"total idle {tot_gap / 1e6:.2f} ms in {len(gaps)} gaps")


if __name__ == "__main__":
    main()
