"""Which hardware queue did each batch lane's kernels run on?  From a
rocprofv3 kernel trace (--kernel-trace -f csv) of tools/order_probe.py: per
host thread that launched > 50 kernels (a lane of one of_pairs_run call, or
a pool lane), its HIP stream id(s), hardware Queue_Id(s) and time span.  Two
lanes of one call on one Queue_Id serialise.
usage: python tools/queue_map.py TRACE_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    T = defaultdict(lambda: {"n": 0, "q": set(), "s": set(), "t0": float("inf"), "t1": 0})
    for r in csv.DictReader(open(sys.argv[1])):
        d = T[r["Thread_Id"]]
        d["n"] += 1
        d["q"].add(r["Queue_Id"])
        d["s"].add(r["Stream_Id"])
        d["t0"] = min(d["t0"], int(r["Start_Timestamp"]))
        d["t1"] = max(d["t1"], int(r["End_Timestamp"]))
    t00 = min(d["t0"] for d in T.values())
    for th, d in sorted(T.items(), key=lambda kv: kv[1]["t0"]):
        if d["n"] > 50:
            print(f"thread {th}: {d['n']} kernels, streams {sorted(d['s'])}, queues {sorted(d['q'])}, "
                  f"{(d['t0'] - t00) / 1e6:.0f}-{(d['t1'] - t00) / 1e6:.0f} ms")


if __name__ == "__main__":
    main()
