"""SURVEY.md §8d inner-loop roofline at the finest level from a rocprofv3
kernel trace (bench.py --lanes 1 pass of tools/profile.sh): per warping
iteration N*(48 + 56 + 24) B for warp + assembly + update (fused warp +
assembly, k_warp_operator, round 5: N*(72 + 24)) and 76*N B per active CG
launch, over the mean durations of those kernels' finest-level dispatches.
CG launches that returned after the prologue (solve already converged;
< 15 us) are counted apart, as bench.py does with its per-launch activity
flags.

usage: python tools/inner_loop_rocprof.py gpurun_out/prof_TAG/trace1_kernel_trace.csv [H W]
"""
import csv
import json
import sys

path = sys.argv[1]
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1080, 1920)
N = H * W
rows = list(csv.DictReader(open(path)))
fam = {"warp": "k_partial_deriv<1>", "assembly": "k_flow_operator", "warp_operator": "k_warp_operator<1",
       "update": "k_update_occ", "cg": "k_cgs"}
grid = {}
for r in rows:
    name = r["Kernel_Name"].replace("void ", "")
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])
    for k, pre in fam.items():
        if name.startswith(pre):
            grid.setdefault(k, {}).setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
# finest level = largest grid of the kernel; the fused kernel or the pair
dur = {k: grid[k][max(grid[k])] for k in grid}
fused = "warp_operator" in dur and "warp" not in dur
warps = len(dur["warp_operator" if fused else "warp"])
cg_all = dur["cg"]
cg_act = [d for d in cg_all if d >= 15.0]
mean = lambda v: sum(v) / len(v)
K = len(cg_act) / warps  # active CG launches per warping iteration (one solve each)
t_other = (mean(dur["warp_operator"]) if fused else mean(dur["warp"]) + mean(dur["assembly"])) + mean(dur["update"])
t_cg = K * mean(cg_act)
t_idle_launches = (len(cg_all) - len(cg_act)) / warps * (mean([d for d in cg_all if d < 15.0]) if len(cg_all) > len(cg_act) else 0.0)
B = N * ((72 if fused else 48 + 56) + 24) + 76 * N * K
out = {
    "source": path, "H": H, "W": W, "warping_iterations": warps, "fused_warp_operator": fused,
    "mean_us": {k: round(mean(v), 2) for k, v in dur.items() if k != "cg"},
    "cg_active_mean_us": round(mean(cg_act), 2), "cg_active_per_warp": round(K, 2),
    "cg_noop_us_per_warp": round(t_idle_launches, 2),
    "bytes_per_warp": B, "us_per_warp": round(t_other + t_cg, 1),
    "achieved_GBps": round(B / ((t_other + t_cg) * 1e-6) / 1e9, 1),
}
out["frac"] = round(out["achieved_GBps"] / 8000.0, 4)
out["frac_incl_noop_launches"] = round(B / ((t_other + t_cg + t_idle_launches) * 1e-6) / 1e9 / 8000.0, 4)
print(json.dumps(out, indent=1))
