"""How busy the lanes' fine-solve token is in a rocprofv3 kernel trace of the
default bench (tools/profile.sh's trace_kernel_trace.csv): over the lanes-mode
steps (from the first side-by-side fine k_cgs launch to the serial pair that
follows them) (the 252-block lanes geometry: grid
1152x56 at 1080p, 896x72 at 864x1536), the fraction of time with 0, 1 and 2
of them in flight, and the GPU's overall busy fraction over that span.
usage: python tools/token_util.py TRACE_CSV"""
import csv
import sys

FINE = {("1152", "56"), ("896", "72")}


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    fine, allk = [], []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        allk.append((s, e))
        if "k_cgs" in r["Kernel_Name"] and (r["Grid_Size_X"], r["Grid_Size_Y"]) in FINE:
            fine.append((s, e))
    t0 = min(s for s, _ in fine)
    # the lanes-mode steps (timed, host to host, streamed) end where the
    # serial per-level pair starts: the first single-solve (504-block)
    # 1080p launch after them
    single = sorted(int(r["Start_Timestamp"]) for r in rows
                    if "k_cgs" in r["Kernel_Name"] and (r["Grid_Size_X"], r["Grid_Size_Y"]) == ("1152", "112")
                    and int(r["Start_Timestamp"]) > t0)
    t1 = single[0] if single else max(e for _, e in fine)
    fine = [(s, min(e, t1)) for s, e in fine if s < t1]
    ev = sorted([(s, 1) for s, _ in fine] + [(e, -1) for _, e in fine])
    occ = {0: 0, 1: 0, 2: 0}
    level, last = 0, t0
    for t, d in ev:
        if t > last:
            occ[min(level, 2)] += t - last
        level += d
        last = t
    span = t1 - t0
    busy = union_len([(max(s, t0), min(e, t1)) for s, e in allk if e > t0 and s < t1])
    print(f"span {span / 1e6:.1f} ms over {len(fine)} side-by-side fine k_cgs launches")
    for k in (0, 1, 2):
        print(f"  {k} in flight: {occ[k] / span:.3f}")
    print(f"  GPU busy (any kernel): {busy / span:.3f}")


if __name__ == "__main__":
    main()
