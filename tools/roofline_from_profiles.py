"""Recompute the round's roofline figures from the committed profiles (no
GPU): for every kernel of a PMC summary (tools/prof_summary.py output,
e.g. profiles/r4y_pmc_summary.json) the algorithmic bytes per 1080p launch
over the rocprofv3 median duration, against the 8 TB/s peak, and the HBM
bytes (2 FETCH_SIZE + WRITE_SIZE) over the algorithmic bytes; then the bench
line's roofline block beside it (bench.py's HIP-event figures, which add
≈ 4 us of event overhead per launch).
usage: python tools/roofline_from_profiles.py profiles/r4y_pmc_summary.json [profiles/r4y_bench.json]"""
import json
import sys

PEAK_GBS = 8000.0


def main():
    summ = json.load(open(sys.argv[1]))
    print(f"{'kernel':24s} {'median us':>10s} {'alg MB':>8s} {'alg GB/s':>9s} {'frac':>6s} {'HBM MB':>8s} {'HBM/alg':>8s}")
    for k, r in summ.items():
        if "alg_MB" not in r:
            continue
        gbs = r["alg_MB"] * 1e6 / (r["finest_median_us"] * 1e-6) / 1e9
        hbm = r.get("hbm_bytes_per_launch")
        print(f"{k[:24]:24s} {r['finest_median_us']:10.2f} {r['alg_MB']:8.1f} {gbs:9.1f} {gbs / PEAK_GBS:6.3f} "
              f"{(hbm or 0) / 1e6:8.1f} {(hbm / (r['alg_MB'] * 1e6)) if hbm else float('nan'):8.2f}")
    if len(sys.argv) > 2:
        line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
        rf = line["roofline"]
        f = rf["finest"]
        print(f"bench line ({sys.argv[2]}): {rf['kernel']} all levels {rf['achieved']} GB/s = {rf['frac']}; "
              f"1080p {f['achieved']} GB/s = {f['frac']} (mean active launch {f['mean_active_launch_ms'] * 1e3:.2f} us, "
              f"HIP events); traffic {rf['traffic']} B per launch over all levels (profiles/pmc_traffic.json); "
              f"as timed {rf.get('as_timed', {}).get('frac')}")


if __name__ == "__main__":
    main()
