"""Cost model for a multilevel (aggregation V-cycle) preconditioner in the
fine-level 'backslash' CG, against the production degree-5 polynomial one
(VERDICT r4 item 1).  Iteration counts: tools/twolevel_iters.py at 1080p
(profiles/r5_twolevel_1080.txt, robust stage alpha = 0, CG to 1e-6);
kernel figures: the measured k_cgs (profiles/r4y_*).

Per CG iteration with a V-cycle M^-1 the fine level needs two passes, since
the coarse correction depends on the whole restricted residual:
  down: p = z + beta p, s = w + beta s, x += alpha p, r -= alpha s
        (Chronopoulos-Gear CG, one global reduction per iteration), then
        pre-smoothing e1 = S(r), r1 = r - A e1, restriction r_c = P^T r1
        reads z, w, p, s, x, r (48 B) + 7 coefficient planes (28 B);
        writes p, s, x, r, e1 (40 B) + r_c (2 B)            = 118 B/px
  up:   e = e1 + P e_c, z = e + S(r - A e), w = A z, dots r.z, w.z
        reads r, e1 (16 B) + e_c (2 B) + coefficients (28 B);
        writes z, w (16 B)                                   =  62 B/px
i.e. 180 B/px per iteration against k_cgs's 76 (which fuses its whole
iteration, degree-5 preconditioner included, into one pass by the rho
recurrence -- a recurrence that needs M^-1 q in closed form, which a
V-cycle does not give).  Each coarse level (540x960 ... 68x120) costs a down
and an up launch; the coarsest (<= 2048 px) one single-workgroup solve.
usage: python tools/mg_cost_model.py  -> table + JSON"""
import json

N = 1080 * 1920
PEAK = 8.0e12
# measured (profiles/r4y_kernel_stats_lanes1.csv)
KCGS_US = 45.6             # isolated 1080p k_cgs launch, 76 B/px -> 3.46 TB/s
KCGS_BW = 76 * N / (KCGS_US * 1e-6)
COARSE_LAUNCH_US = {"540x960": 21.9, "270x480": 17.1, "135x240": 17.1, "68x120": 17.1}
CG_REG_US = 47.0           # k_cg_reg whole solve at <= 2048 px
ITERS = {"poly5": 52, "vc-s2": 18, "vc-s3": 15, "2lv-s3 (exact coarse)": 12}


def vcycle_iter_us(bw, coarse_us, coarsest_us):
    fine = 180 * N / bw * 1e6
    coarse = 2 * sum(coarse_us.values())
    return fine + coarse + coarsest_us, fine, coarse


def main():
    rows = []
    base = ITERS["poly5"] * KCGS_US
    rows.append({"scheme": "poly5 (production)", "iters": ITERS["poly5"], "us_per_iter": KCGS_US,
                 "solve_ms": base / 1e3, "vs_poly5": 1.0})
    cases = {
        "measured latencies, k_cgs bandwidth": (KCGS_BW, COARSE_LAUNCH_US, CG_REG_US),
        "optimistic: 0.7 of HBM peak, 8 us coarse launches, 20 us coarsest": (0.7 * PEAK, {k: 8.0 for k in COARSE_LAUNCH_US}, 20.0),
        "bound: fine bytes only (HBM peak, free coarse levels)": (PEAK, {k: 0.0 for k in COARSE_LAUNCH_US}, 0.0),
    }
    for name, (bw, cu, cc) in cases.items():
        for sch in ("vc-s2", "vc-s3"):
            it, fine, coarse = vcycle_iter_us(bw, cu, cc)
            ms = ITERS[sch] * it / 1e3
            rows.append({"scheme": f"{sch}: {name}", "iters": ITERS[sch], "us_per_iter": round(it, 1),
                         "fine_us": round(fine, 1), "coarse_us": round(coarse + cc, 1), "solve_ms": round(ms, 3),
                         "vs_poly5": round(ms * 1e3 / base, 2)})
    for r in rows:
        print(f"{r['scheme']:<80} {r['iters']:>3} it  {r['us_per_iter']:>7} us/it  {r['solve_ms']:.3f} ms  "
              f"x{r['vs_poly5']}")
    print(json.dumps({"N": N, "kcgs_bw_TBps": KCGS_BW / 1e12, "rows": rows}))


if __name__ == "__main__":
    main()
