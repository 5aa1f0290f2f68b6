"""Benchmark: image pairs/s for Classic+NL-fast on 1920x1080 synthetic pairs
(BASELINE.json metric; SURVEY.md §8d config 4, and config 5 across GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--lanes L]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU.  `--gpus N` with N > 1 and no launcher around it
(WORLD_SIZE unset) starts `python -m torch.distributed.run --nproc-per-node N
bench.py <same arguments>` as a child process before anything touches the GPU,
relays rank 0's JSON line and exits with the child's status; under a launcher
WORLD_SIZE must equal --gpus.  `--rccl-self` (N = 1) runs the timed loop with
a one-rank RCCL communicator and the per-step gather: the one-GPU proxy of the
N > 1 timed path.  A step = every rank runs estimate_flow on its P
pairs (default 8 = config 5's 64 pairs over 8 GPUs) with the frames already
resident in HBM (uploaded to device slots before the timed region) and the
flows left there (RGB -> gray/Lab, ROF, pyramids, GNC x levels x IRLS, L
pairs in flight on concurrent streams), through the persistent pair pool
(of_pairs_open + of_pairs_submit_slots: step s+1 is queued before step s is
waited for, so the lanes do not drain between steps; the steps alternate
between two sets of P slots); for N > 1 each step's flows are also gathered
to rank 0 with RCCL over xGMI (of_rccl_gather_slots).  Timed region: barrier
+ device sync on both sides, max over ranks.  value = pairs processed by all
ranks / time (weak scaling: P pairs per GPU).  Reported beside it:
`device_resident_drained` (the same steps as one of_pairs_run call each:
the lanes drain at every step end), `host_to_host` (SURVEY.md §8d's form:
uint8 frames in host memory -> H2D -> ... -> D2H of the fp32 flow,
of_pairs_run_host, copies overlapped with compute; the PCIe-inclusive rate,
never `value` -- the task's measurement contract puts the inputs in HBM)
and `streamed` (host-to-host through the pool, of_pairs_submit /
of_pairs_wait); all over the same K steps.

Also reported (one JSON line on rank 0):
  roofline      dominant HBM kernel: algorithmic bytes per launch / mean
                HIP-event duration of that kernel over a profiled replay of
                the step's pairs one at a time (lanes = 1; the lanes replay
                beside it as `concurrent`); inner_loop = SURVEY.md §8d's
                "SOR/PCG + warp" figure; peak 8 TB/s; traffic from profiles/
                PMC if present (else null)
  cpu_baseline  the float64 C oracle (oracle/, OpenMP) on a bounded crop of
                the same pair, scaled by pixel count to pairs/s
  ms_per_level  GPU time of each compute_flow_base (coarse -> fine, per stage)
  aepe_gt       accuracy against the analytic ground truth
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))

import numpy as np  # noqa: E402

from optical_flow.utils.synthetic import synth_pair  # noqa: E402

# the library (liboptflow.so, loaded before torch) and the method registry are
# imported in main() once the launch decision is made: a process that spawns
# the ranks never touches the GPU (import_native)
_abi = _native = load_of_method = None


def import_native():
    global _abi, _native, load_of_method
    from optical_flow import _abi as a, _native as n
    from optical_flow.methods.config import load_of_method as lm
    _abi, _native, load_of_method = a, n, lm

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

# algorithmic bytes per pixel of each kernel's compulsory I/O (DESIGN.md
# "Kernels and rooflines"); fp32 = 4 B, float2 = 8 B, planes counted once
KERNEL_BYTES_PER_PX = {
    "pcg_iter": 8 + 8 + 8 + 28 + 3 * 8,    # fused CG iteration: r, x, p_old + 7 coef planes -> r, x, p_new
    "flow_operator": 8 + 12 + 28 + 8,      # uv, It/Ix/Iy -> 7 coef + rhs
    # warp + derivatives + assembly fused (nc = 1): uv, I1, I2/DX/DY/DXY (Hermite;
    # 3 planes for the B-spline / bilinear forms), I1x, I1y -> 7 coef + rhs
    "warp_operator_hermite": 8 + 4 + 4 * 4 + 8 + 36,
    "warp_operator_bspline": 8 + 4 + 3 * 4 + 8 + 36,
    "warp_operator_bilinear": 8 + 4 + 3 * 4 + 8 + 36,
    "partial_deriv_hermite": 8 + 4 * 4 + 3 * 4 + 12,  # uv, I2/DX/DY/DXY, I1/I1x/I1y -> It/Ix/Iy
    "update_occ": 16 + 8 + 8 + 4,          # uv, x, I1, I2 -> uv1, occ
    "wmf": 8 + 4 + 12 + 8,                 # uv, occ, Lab -> uv
    "rof_iters": 4 + 8 + 8,                # im, p -> p per channel, ROF_K iterations per launch
    "sor_sweep": 36 + 8 + 8,               # 7 coef + 2 rhs planes, x read + write (52 B/px/sweep)
    # the pipelined SOR: one launch per solve, bytes counted per sweep done
    # ("sor_pipe.active" = sweeps x level pixels)
    "sor_pipe": 36 + 8 + 8,
    "sor_wg": 36 + 8 + 8,  # the one-workgroup form of small levels (LDS ring), per sweep done
}
# VALU issue peak (MI355X_MICROARCH.md: a wave issues one VALU instruction per
# 2 cycles per SIMD; 256 CUs x 4 SIMDs at 2.4 GHz): wave-instructions / s
CLOCK_HZ = 2.4e9
VALU_ISSUE_PEAK = 256 * 4 * 0.5 * CLOCK_HZ
# the weighted median's per-phase ISA census priced by measured issue costs
WMF_CENSUS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r6_wmf_census.json")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=8, help="pairs per GPU per step (config 5: 64 pairs / 8 GPUs)")
    ap.add_argument("--lanes", type=int, default=4, help="concurrent pair pipelines per GPU (of_pairs_run_host)")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--method", default="classic+nl-fast")
    ap.add_argument("--solver", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the streamed (pair pool) rate")
    ap.add_argument("--cpu-sample", type=int, default=360, help="crop height of the CPU-baseline sample")
    ap.add_argument("--sor-pipeline", type=int, default=None,
                    help="OF_OPT_SOR_PIPELINE for 'sor' (0 per sweep, 1 pipelined, 2 + one-workgroup small levels)")
    ap.add_argument("--rccl-self", action="store_true",
                    help="N = 1: one-rank RCCL communicator + the per-step gather in the timed loop "
                         "(the one-GPU proxy of the N > 1 timed path)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only (no library, no GPU): rank 0 prints the line's "
                         "n_gpus and the ranks seen (the CPU test of the --gpus N launch)")
    return ap.parse_args(argv)


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv):
    """--gpus N > 1 with no launcher around bench.py: run `python -m
    torch.distributed.run --nproc-per-node N bench.py <argv>` as a child (the
    contract's N-rank launch; never an exec from this process), pass its
    stderr and non-JSON stdout through, print rank 0's JSON line once with
    the launch recorded in it, and return the child's exit status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    line = None
    for out in proc.stdout:
        if out.startswith('{"metric"'):
            line = out
        else:
            sys.stderr.write(out)
            sys.stderr.flush()
    rc = proc.wait()
    if line is not None:
        rec = json.loads(line)
        rec["launch"] = (f"bench.py --gpus {args.gpus}: torch.distributed.run child, "
                         f"{args.gpus} processes (one per GPU), rc {rc}")
        print(json.dumps(rec), flush=True)
    elif rc == 0:
        sys.stderr.write("bench.py: the ranks exited without a result line\n")
        rc = 1
    return rc


def launch_check(args):
    """WORLD_SIZE from a launcher must match --gpus (a mismatch would time a
    different job than the one asked for)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}\n")
        return 2
    return 0


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist  # gloo only: barrier, max-reduce, RCCL id exchange
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return dist, world, rank, local
    return None, 1, 0, 0


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_seeds(rank, pairs):
    """Pair k of the global batch uses seed k; rank r owns [r*P, (r+1)*P)."""
    return [rank * pairs + k for k in range(pairs)]


def make_params(args):
    ope = load_of_method(args.method)
    if args.solver:
        ope.solver = args.solver
    P = ope.to_params()
    P.guide_mode = int(ope._METHOD == "classic_nl" and ope.color_images is not None)
    P.display = 0
    return P


def run_step(ctx, P0, nslots, lanes):
    """estimate_flow on device slots 0..nslots-1, `lanes` pairs in flight
    (each lane its own HIP stream + host thread inside the library)."""
    ctx.check(ctx.lib.of_pairs_run(ctx.handle, nslots, C.byref(P0), lanes, None))


def flow_digests(outs):
    import hashlib
    return [hashlib.sha1(o.tobytes()).hexdigest() for o in outs]


def verify_gather(buf, every, world, pairs):
    """True iff pair s of rank src sits at offset src * pairs + s of the
    gathered buffer (of_rccl_gather_flows' layout = shard_seeds' global pair
    order), by the sha1 digests every rank published for its own flows."""
    import hashlib
    return all(hashlib.sha1(buf[src * pairs + s].tobytes()).hexdigest() == every[src][s]
               for src in range(world) for s in range(pairs))


def gather_check(dist, ctx, lib, world, rank, pairs, H, W, outs):
    """One untimed RCCL gather into a host buffer on rank 0, checked against
    the digests every rank publishes over gloo; raises on a layout mismatch."""
    every = [None] * world
    dist.all_gather_object(every, flow_digests(outs))
    buf = np.empty((world * pairs, 2, H, W), dtype=np.float32) if rank == 0 else None
    ctx.check(lib.of_rccl_gather_flows(ctx.handle, pairs, _native.ptr(buf) if rank == 0 else None))
    flag = [verify_gather(buf, every, world, pairs) if rank == 0 else None]
    dist.broadcast_object_list(flag, src=0)
    if not flag[0]:
        raise RuntimeError("RCCL gather layout check failed")
    return {"pairs": world * pairs, "layout": "rank r pair s at r*P+s", "ok": True}


def cpu_baseline(args):
    """float64 oracle on a bounded crop of pair 0, scaled by pixel count."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / baseline only
    h = min(args.cpu_sample, args.height)
    w = int(round(h * args.width / args.height))
    im1, im2, _ = synth_pair(args.height, args.width, 0)
    y0, x0 = (args.height - h) // 2, (args.width - w) // 2
    a, b = im1[y0:y0 + h, x0:x0 + w], im2[y0:y0 + h, x0:x0 + w]
    t0 = time.perf_counter()
    oracle.estimate_flow(a, b, args.method, solver=args.solver)
    dt = time.perf_counter() - t0
    scale = (args.height * args.width) / (h * w)
    return {"value": 1.0 / (dt * scale), "unit": "pairs/s", "cores": oracle.num_threads(), "kind": "port",
            "sample": f"float64 C oracle (OpenMP) estimate_flow('{args.method}') on a {h}x{w} centre crop of "
                      f"synth_pair({args.height},{args.width},0): {dt:.2f} s, scaled x{scale:.1f} by pixel count"}


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


WORKLOAD = None  # method@HxW/solver of this run (main)


def workload_key(args):
    return f"{args.method}@{args.height}x{args.width}/{args.solver or 'backslash'}"


def load_pmc(kernel):
    """The kernel's record for THIS run's workload in the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json, keyed by workload then kernel,
    written by tools/prof_summary.py --traffic from tools/profile.sh's counter
    passes; shipped to the GPU box), or {} when that workload was not
    profiled (then `traffic` is null rather than another kernel's figure)."""
    try:
        return (json.load(open(PMC_FILE)).get(WORKLOAD, {}) or {}).get(kernel, {}) or {}
    except (OSError, ValueError):
        return {}


def load_pmc_traffic(kernel, which="finest"):
    """HBM bytes per launch of `kernel` (2*FETCH_SIZE + WRITE_SIZE, profiles/
    pmc_traffic.json): averaged over all launches ("all") or over the finest
    level's launches ("finest")."""
    return load_pmc(kernel).get("hbm_bytes_per_launch_all" if which == "all" else "hbm_bytes_per_launch")


def pmc_symbol(kernel):
    return load_pmc(kernel).get("symbol")


# the reference's own run of each BASELINE.json config on synth_pair(H, W, 0)
# (tests/golden/gen_golden.py full*): its AEPE against the analytic GT
REF_FIXTURE = {"classic+nl-fast@1080x1920/backslash": "ref1080_backslash_sub4.npz",
               "classic+nl-fast@1080x1920/pcg": "ref1080_pcg_sub4.npz",
               "classic-c@720x1280/pcg": "ref720_classic_c_pcg_sub4.npz",
               "hs@480x640/sor": "ref480_hs_sor_sub2.npz"}


def ref_aepe():
    f = REF_FIXTURE.get(WORKLOAD)
    if not f:
        return None, None
    try:
        return float(np.load(os.path.join(ROOT, "tests", "golden", f))["aepe_gt"]), f
    except (OSError, KeyError, ValueError):
        return None, f


def wmf_compute_roofline(per_level):
    """The weighted median is not HBM bound: `frac` = the
    VALU SIMD-cycles its instructions occupy (tools/isa_census.py: the
    shipped ISA per phase, each opcode at its measured issue cost,
    profiles/r6_wmf_census.json) over the finest-level launch's mean duration
    in the isolated replay x 1024 SIMDs x clock.  Beside it the PMC
    instruction rate against a 2-cycle issue (`insts_frac_2cyc`, which
    understates fp64 / transcendental / DPP instructions) and `hbm_frac`."""
    rec = load_pmc("wmf")
    lv = [(px, r) for (n, px), r in per_level.items() if n == "wmf"]
    if not lv:
        return None
    px, r = max(lv, key=lambda t: t[0])
    ms = r["ms_total"] / r["launches"]
    out = {"bound": "valu-issue", "px_per_launch": px, "mean_launch_ms": round(ms, 4),
           "mpx_per_ms": round(px / 1e6 / ms, 3), "alg_bytes_per_px": KERNEL_BYTES_PER_PX["wmf"],
           "hbm_frac": round(KERNEL_BYTES_PER_PX["wmf"] * px / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    vi = rec.get("valu_insts_per_launch")
    if vi and rec.get("grid") == px:
        ach = vi / (ms * 1e-3)
        out.update({"valu_insts_per_launch": vi, "valu_insts_per_px": round(vi * 64 / px, 1),
                    "achieved": round(ach / 1e9, 1), "peak": round(VALU_ISSUE_PEAK / 1e9, 1),
                    "unit": "G wave-instr/s", "insts_frac_2cyc": round(ach / VALU_ISSUE_PEAK, 4)})
    if rec.get("valu_pipe_busy") is not None:
        # issue counts price every instruction at 2 cycles; the SQ's active
        # cycles (fp64, transcendental, 64-bit ops take longer) give the pipe
        out.update({"valu_pipe_busy": rec["valu_pipe_busy"], "valu_pipe_busy_source": rec.get("sq_source")})
    try:
        cen = json.load(open(WMF_CENSUS))
    except (OSError, ValueError):
        cen = None
    if cen:
        # the headline figure: VALU SIMD-cycles per wave from the ISA census
        # (tools/isa_census.py: every opcode priced by its measured issue cost
        # at the kernel's 2 waves per SIMD, tools/micro/valu_cost.hip) x one
        # wave per 8x8 tile / (1024 SIMDs x clock x launch time)
        waves = -(-px // 64)
        simd_s = cen["total"]["valu_simd_cycles"] * waves / (256 * 4) / CLOCK_HZ
        out.update({"valu_simd_cycles_per_wave": cen["total"]["valu_simd_cycles"],
                    "valu_insts_per_wave_isa": cen["total"]["valu"],
                    "frac": round(simd_s / (ms * 1e-3), 4),
                    "frac_basis": "VALU SIMD-cycles at measured issue costs / launch time "
                                  "(" + os.path.relpath(WMF_CENSUS, ROOT) + ")"})
    return out


def roofline_of(ktimes, per_level):
    """Roofline of the dominant HBM kernel.  Algorithmic bytes = bytes/px x
    the level pixels of every launch that did work ("<name>.active" entries
    from the library: CG launches enqueued after convergence return after
    the prologue and move no data); time = HIP events on the ctx stream
    around EVERY launch of the kernel, no-op ones included, so the figure is
    conservative.  Top level: all levels (what the rocprofv3 --stats average
    of the kernel covers); `finest`: the largest level only."""
    hbm = {k: v for k, v in ktimes.items() if k in KERNEL_BYTES_PER_PX}
    if not hbm:
        return None
    dom = max(hbm, key=lambda k: hbm[k]["ms_total"])
    act = dom + ".active"

    def fig(rec, arec):
        """achieved = algorithmic bytes of the launches that did work / time
        of all launches; mean_launch_ms = time / all launches (what the
        rocprofv3 --stats average of the kernel measures)"""
        work = arec if arec and arec["launches"] else rec
        ach = KERNEL_BYTES_PER_PX[dom] * work["px"] / (rec["ms_total"] * 1e-3) / 1e9
        return (round(ach, 1), round(rec["ms_total"] / rec["launches"], 5), int(work["px"] / work["launches"]),
                work["launches"], round(rec["ms_total"] / work["launches"], 5))

    ach, avg_ms, ppl, nact, act_ms = fig(hbm[dom], ktimes.get(act))
    out = {"kernel": dom, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_pmc_traffic(dom, "all"),
           "bytes_per_px": KERNEL_BYTES_PER_PX[dom], "mean_launch_ms": avg_ms, "mean_active_launch_ms": act_ms,
           "px_per_active_launch": ppl, "launches_per_step": hbm[dom]["launches"], "active_launches_per_step": nact}
    lv = [(px, rec) for (n, px), rec in per_level.items() if n == dom]
    if lv:
        px, rec = max(lv, key=lambda t: t[0])
        a2, m2, p2, n2, am2 = fig(rec, per_level.get((act, px)))
        out["finest"] = {"px_per_launch": p2, "achieved": a2, "frac": round(a2 / HBM_PEAK_GBS, 4),
                         "mean_launch_ms": m2, "mean_active_launch_ms": am2, "launches_per_step": rec["launches"],
                         "active_launches_per_step": n2, "traffic": load_pmc_traffic(dom, "finest")}
    return out


def profiled_replay(ctx, lib, P0, pairs, lanes, timeline=None):
    """One step of of_pairs_run with per-launch HIP-event timing keyed by
    kernel and level size; returns (per-kernel totals, per-(kernel, px)).
    With a `timeline` list, every launch's (name, px, t0_ms, t1_ms) on the
    lanes' common time axis is appended to it (profiling mode 3)."""
    ctx.check(lib.of_set_profiling(ctx.handle, 3 if timeline is not None else 2))
    run_step(ctx, P0, pairs, lanes)
    if timeline is not None:
        m = C.c_int(0)
        ctx.check(lib.of_kernel_timeline(ctx.handle, 0, None, None, None, None, C.byref(m)))
        k = m.value
        nm = (C.c_char_p * k)()
        px, t0, t1 = (C.c_double * k)(), (C.c_double * k)(), (C.c_double * k)()
        ctx.check(lib.of_kernel_timeline(ctx.handle, k, nm, px, t0, t1, C.byref(m)))
        timeline.extend((nm[i].decode(), px[i], t0[i], t1[i]) for i in range(min(k, m.value)))
    n = C.c_int(0)
    names = (C.c_char_p * 1024)()
    ms = (C.c_double * 1024)()
    cnt = (C.c_int64 * 1024)()
    pxs = (C.c_double * 1024)()
    ctx.check(lib.of_kernel_times(ctx.handle, 1024, names, ms, cnt, pxs, C.byref(n)))
    ctx.check(lib.of_set_profiling(ctx.handle, 0))
    per_level, ktimes = {}, {}
    for i in range(min(n.value, 1024)):
        name, lvl = names[i].decode().rsplit("@", 1)
        rec = {"ms_total": ms[i], "launches": int(cnt[i]), "px": pxs[i]}
        per_level[(name, int(lvl))] = rec
        agg = ktimes.setdefault(name, {"ms_total": 0.0, "launches": 0.0, "px": 0.0})
        for k in agg:
            agg[k] += rec[k]
    return ktimes, per_level


# SURVEY.md §8d inner-loop figure ("SOR/PCG + warp"): per warping iteration
# N (48 warp+derivatives + 56 weights/assembly + 24 update/clip) + 76 N K_pcg
# bytes, over the time of every kernel of the loop
INNER_BYTES = {"partial_deriv_hermite": 48, "partial_deriv_bspline": 44, "partial_deriv_bilinear": 44,
               "flow_operator": 56, "update_occ": 24,
               # the fused warp + assembly: its compulsory I/O (the It/Ix/Iy
               # round trip of the two-kernel form is gone)
               "warp_operator_hermite": 72, "warp_operator_bspline": 68, "warp_operator_bilinear": 68}
INNER_TIME_ONLY = ("pcg_small", "pcg_check", "cg_update", "cg_finalize", "axpy_diff", "add_update", "sor_init",
                   "sor_final")


def inner_loop_of(ktimes, per_level):
    """bytes: the per-px figures above x the pixels of every launch, 76 B x
    the pixels of every CG launch that did work (pcg_iter.active) and 52 B x
    the pixels of every SOR sweep; the one-workgroup coarse-level solves
    (pcg_small) and the 'backslash' residual replacement / finalisation
    count time but no bytes (conservative); time: HIP events of all those
    kernels."""
    byt, ms = 0.0, 0.0
    for name, rec in ktimes.items():
        if name in INNER_BYTES:
            byt += INNER_BYTES[name] * rec["px"]
            ms += rec["ms_total"]
        elif name == "sor_sweep":
            byt += KERNEL_BYTES_PER_PX["sor_sweep"] * rec["px"]
            ms += rec["ms_total"]
        elif name in ("pcg_iter", "sor_pipe", "sor_wg"):
            ms += rec["ms_total"]
        elif name in INNER_TIME_ONLY:
            ms += rec["ms_total"]
    for it in ("pcg_iter", "sor_pipe", "sor_wg"):
        act = ktimes.get(it + ".active")
        if act:
            byt += KERNEL_BYTES_PER_PX[it] * act["px"]
    if ms <= 0:
        return None
    ach = byt / (ms * 1e-3) / 1e9
    fine = max((px for (n, px) in per_level if n in ("pcg_iter", "sor_sweep", "sor_pipe")), default=None)
    out = {"bytes_per_step": round(byt), "kernel_ms_per_step": round(ms, 3), "achieved": round(ach, 1),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
           "formula": "sum N*(48|44 + 56 + 24) per warp (fused warp + assembly: N*(72|68 + 24)) + 76*N*K_pcg | "
                      "52*N*K_sor; time of warp, assembly, update, solver kernels"}
    if fine:
        b2 = sum(INNER_BYTES[n] * r["px"] for (n, px), r in per_level.items() if px == fine and n in INNER_BYTES)
        b2 += KERNEL_BYTES_PER_PX["pcg_iter"] * per_level.get(("pcg_iter.active", fine), {"px": 0})["px"]
        b2 += KERNEL_BYTES_PER_PX["sor_sweep"] * per_level.get(("sor_sweep", fine), {"px": 0})["px"]
        b2 += KERNEL_BYTES_PER_PX["sor_pipe"] * per_level.get(("sor_pipe.active", fine), {"px": 0})["px"]
        m2 = sum(r["ms_total"] for (n, px), r in per_level.items() if px == fine and
                 (n in INNER_BYTES or n in ("pcg_iter", "sor_sweep", "sor_pipe") or n in INNER_TIME_ONLY))
        if m2 > 0:
            a2 = b2 / (m2 * 1e-3) / 1e9
            out["finest"] = {"px": fine, "achieved": round(a2, 1), "frac": round(a2 / HBM_PEAK_GBS, 4)}
    return out


def as_timed_of(timeline, per_level, dom, fine):
    """The dominant kernel's finest-level launches AS TIMED (the lanes replay:
    several pairs in flight, two fine CG solves side by side): algorithmic
    bytes of their active launches / the UNION of their [start, end]
    intervals on the common time axis, i.e. the aggregate rate while any of
    them runs; `overlap` = share of that union with >= 2 of them running."""
    iv = sorted((t0, t1) for (n, px, t0, t1) in timeline if n == dom and px == fine)
    if not iv:
        return None
    ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
    union = over = 0.0
    depth, last = 0, ev[0][0]
    for t, d in ev:
        if depth >= 1:
            union += t - last
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    act = per_level.get((dom + ".active", fine)) or per_level.get((dom, fine))
    byt = KERNEL_BYTES_PER_PX[dom] * act["px"]
    ach = byt / (union * 1e-3) / 1e9
    return {"kernel": dom, "px_per_launch": int(fine), "launches": len(iv), "active_launches": act["launches"],
            "union_ms": round(union, 3), "overlap": round(over / union, 3) if union > 0 else None,
            "mean_launch_ms": round(sum(b - a for a, b in iv) / len(iv), 5), "achieved": round(ach, 1),
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "method": "lanes replay as timed; HIP events on each lane's stream; bytes of the active launches / "
                      "union of the launches' intervals (tools/side_by_side_rocprof.py's method)"}


# kernels that run before the level loop (preprocessing, ROF, pyramids):
# keyed by a level's pixel count too, but outside its compute_flow_base time
PRE_LEVEL = ("rof_iters", "correlate", "resize", "minmax", "mm_init", "scale", "rgb_max", "rgb_prep", "sub_scaled")


def level_breakdown(levels, per_level, pairs):
    """Per pyramid level of one serial pair: the wall time of resample +
    compute_flow_base (HIP events around the level, of_stats.level_ms) beside
    the HIP-event kernel time of the same level in the lanes = 1 replay
    (per pair); `gap_ms` = wall - kernels = launch gaps + host syncs (e.g. HS's
    ||x|| < 1e-3 exit read, hs.py:127-128).  For SOR: sweeps and us per sweep
    of the pipelined solve (sor_pipe.active = sweeps x level pixels)."""
    out = []
    for px in sorted({l["h"] * l["w"] for l in levels}):
        wall = sum(l["ms"] for l in levels if l["h"] * l["w"] == px)
        ks = {n: r["ms_total"] / pairs for (n, p), r in per_level.items()
              if p == px and not n.endswith(".active") and n not in PRE_LEVEL}
        kern = sum(ks.values())
        lv = next(l for l in levels if l["h"] * l["w"] == px)
        rec = {"h": lv["h"], "w": lv["w"], "wall_ms": round(wall, 3), "kernel_ms": round(kern, 3),
               "gap_ms": round(wall - kern, 3), "gap_share": round((wall - kern) / wall, 4) if wall > 0 else None,
               "top": {n: round(v, 3) for n, v in sorted(ks.items(), key=lambda kv: -kv[1])[:4]}}
        for solver in ("sor_wg", "sor_pipe", "sor_sweep"):
            if (solver, px) in per_level:
                sw = per_level.get((solver + ".active", px), per_level[(solver, px)])["px"] / px / pairs
                ms = per_level[(solver, px)]["ms_total"] / pairs
                rec.update({"solver": solver, "solver_ms": round(ms, 3), "sweeps": round(sw, 2),
                            "solves": per_level[(solver, px)]["launches"] / pairs,
                            "us_per_sweep": round(1e3 * ms / sw, 2) if sw else None})
        out.append(rec)
    return out


def kms(kt, pairs, top=14):
    return {k: round(v["ms_total"] / pairs, 3) for k, v in
            sorted(kt.items(), key=lambda kv: -kv[1]["ms_total"])[:top] if not k.endswith(".active")}


def metric_name(args):
    tag = {"classic+nl-fast": "Classic+NL-fast", "hs": "HS", "classic-c": "Classic-C"}.get(args.method, args.method)
    solver = f" ({args.solver})" if args.solver else ""
    return f"image-pairs/sec at {args.width}x{args.height} {tag}{solver} (+ ms/pyramid-level, AEPE)"


def dry_run(args, dist, world, rank, local):
    """The launch and rendezvous of an N-rank run without the library: every
    rank reports (rank, local rank, world); rank 0 prints the line."""
    seen = [None] * world
    if dist is not None:
        dist.all_gather_object(seen, [rank, local, world])
    else:
        seen = [[rank, local, world]]
    barrier(dist)
    t = max_over_ranks(dist, 0.001 * (1 + rank))
    if rank == 0:
        print(json.dumps({"metric": metric_name(args), "value": None, "unit": "pairs/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True, "ranks": seen,
                          "max_over_ranks": t, "rccl_nranks": None}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = launch_check(args)
    if rc:
        return rc
    if args.gpus > 1 and os.environ.get("WORLD_SIZE") is None:
        return spawn_ranks(args, argv)
    if args.rccl_self and args.gpus != 1:
        sys.stderr.write("bench.py: --rccl-self is the N = 1 proxy\n")
        return 2
    global WORKLOAD
    WORKLOAD = workload_key(args)
    dist, world, rank, local = dist_setup(args)
    if args.dry_run:
        dry_run(args, dist, world, rank, local)
        return 0
    import_native()
    ctx = _native.Context(local)
    if args.sor_pipeline is not None:
        ctx.set_option(_abi.OF_OPT_SOR_PIPELINE, args.sor_pipeline)
    lib = ctx.lib
    H, W = args.height, args.width
    P0 = make_params(args)

    # host frames (uint8, what a caller holds) and host flow buffers; the
    # same pairs also uploaded once to device slots for the device-resident rate
    seeds = shard_seeds(rank, args.pairs)
    gts, f1, f2 = [], [], []
    for seed in seeds:
        im1, im2, gt = synth_pair(H, W, seed)
        gts.append(gt)
        f1.append(np.ascontiguousarray(im1.astype(np.uint8)))
        f2.append(np.ascontiguousarray(im2.astype(np.uint8)))
    outs = [np.empty((2, H, W), dtype=np.float32) for _ in seeds]
    vp = C.c_void_p
    p1 = (vp * args.pairs)(*[x.ctypes.data for x in f1])
    p2 = (vp * args.pairs)(*[x.ctypes.data for x in f2])
    po = (vp * args.pairs)(*[o.ctypes.data for o in outs])
    # the RCCL communicator: N ranks, or one rank for the --rccl-self proxy
    gathering = world > 1 or args.rccl_self
    if gathering:
        uid = C.create_string_buffer(128)
        if rank == 0:
            ctx.check(lib.of_rccl_unique_id(uid))
        obj = [bytes(uid.raw)]
        if dist is not None:
            dist.broadcast_object_list(obj, src=0)
        ctx.check(lib.of_rccl_init(ctx.handle, obj[0], world, rank))
    nr = C.c_int64(0)
    ctx.check(lib.of_get_option(ctx.handle, _abi.OF_OPT_RCCL_NRANKS, C.byref(nr)))
    rccl_nranks = int(nr.value)
    if gathering and rccl_nranks != world:
        raise RuntimeError(f"RCCL communicator has {rccl_nranks} ranks, expected {world}")

    # the timed steps: frames resident in HBM (two sets of device slots,
    # uploaded here, outside the timed region), flows left in HBM (+ the RCCL
    # gather), queued through the pair pool back to back
    NP = args.pairs
    sets = [(C.c_int * NP)(*range(k * NP, (k + 1) * NP)) for k in range(2)]

    def upload_all(nsets=2):
        for k in range(nsets):
            for s, (a, b) in enumerate(zip(f1, f2)):
                ctx.check(lib.of_pair_upload(ctx.handle, k * NP + s, _native.ptr(_native.f32(a)),
                                             _native.ptr(_native.f32(b)), H, W, 3))
    upload_all()
    ctx.check(lib.of_pairs_open(ctx.handle, H, W, 3, C.byref(P0), args.lanes))

    def psubmit(s):
        t = C.c_int64(0)
        ctx.check(lib.of_pairs_submit_slots(ctx.handle, NP, sets[s % 2], C.byref(t)))
        return t.value

    def pwait(s, t0_):
        for t in range(t0_, t0_ + NP):
            ctx.check(lib.of_pairs_wait(ctx.handle, t))
        if gathering:
            ctx.check(lib.of_rccl_gather_slots(ctx.handle, (s % 2) * NP, NP, None))

    def pool_steps(k):
        prev = psubmit(0)
        for s in range(1, k):
            cur = psubmit(s)
            pwait(s - 1, prev)
            prev = cur
        pwait(k - 1, prev)

    if args.warmup:
        pool_steps(args.warmup)
    barrier(dist)
    ctx.check(lib.of_synchronize(ctx.handle))
    t0 = time.perf_counter()
    pool_steps(args.steps)
    ctx.check(lib.of_synchronize(ctx.handle))
    barrier(dist)
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    value = world * NP * args.steps / elapsed
    ctx.check(lib.of_pairs_close(ctx.handle))
    dev_uv = np.empty((2, H, W), dtype=np.float32)  # the timed flow of pair 0 (last step's slot set)
    ctx.check(lib.of_pair_download(ctx.handle, ((args.steps - 1) % 2) * NP, _native.ptr(dev_uv)))

    # the same steps as one of_pairs_run call each (lanes drain at step end)
    def step():
        run_step(ctx, P0, NP, args.lanes)
        if gathering:
            ctx.check(lib.of_rccl_gather_flows(ctx.handle, NP, None))
    step()
    barrier(dist)
    ctx.check(lib.of_synchronize(ctx.handle))
    td = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.check(lib.of_synchronize(ctx.handle))
    barrier(dist)
    d_elapsed = max_over_ranks(dist, time.perf_counter() - td)
    drained_uv = np.empty((2, H, W), dtype=np.float32)
    ctx.check(lib.of_pair_download(ctx.handle, 0, _native.ptr(drained_uv)))

    # host to host (PCIe-inclusive): uint8 frames in host memory -> flows in
    # host memory, copies overlapped inside the library
    def hstep():
        ctx.check(lib.of_pairs_run_host(ctx.handle, args.pairs, p1, p2, H, W, 3, C.byref(P0), args.lanes, po, None))
        if gathering:
            ctx.check(lib.of_rccl_gather_flows(ctx.handle, args.pairs, None))
    hsteps = args.steps
    hstep()  # warm-up (pinned staging buffers)
    barrier(dist)
    ctx.check(lib.of_synchronize(ctx.handle))
    t1 = time.perf_counter()
    for _ in range(hsteps):
        hstep()
    ctx.check(lib.of_synchronize(ctx.handle))
    barrier(dist)
    h_elapsed = max_over_ranks(dist, time.perf_counter() - t1)
    host_eq_dev = bool(np.array_equal(dev_uv, outs[0]))
    gather = gather_check(dist, ctx, lib, world, rank, args.pairs, H, W, outs) if world > 1 else None

    # streamed rate: the same steps through the persistent pair pool
    # (of_pairs_open / submit / wait, include/optflow.h), step s+1 submitted
    # before step s is waited for, so the lanes do not drain between steps
    streamed = None
    if not args.no_stream:
        sctx = _native.Context(local)
        if args.sor_pipeline is not None:
            sctx.set_option(_abi.OF_OPT_SOR_PIPELINE, args.sor_pipeline)
        slib = sctx.lib
        sctx.check(slib.of_pairs_open(sctx.handle, H, W, 3, C.byref(P0), args.lanes))
        souts = [[np.empty((2, H, W), dtype=np.float32) for _ in seeds] for _ in range(2)]
        spo = [(vp * args.pairs)(*[o.ctypes.data for o in so]) for so in souts]

        def ssubmit(s):
            t = C.c_int64(0)
            sctx.check(slib.of_pairs_submit(sctx.handle, args.pairs, p1, p2, spo[s % 2], C.byref(t)))
            return t.value

        def swait(t0_):
            for t in range(t0_, t0_ + args.pairs):
                sctx.check(slib.of_pairs_wait(sctx.handle, t))
        for s in range(args.warmup):
            swait(ssubmit(s))
        barrier(dist)
        ts = time.perf_counter()
        prev = ssubmit(0)
        for s in range(1, args.steps):
            cur = ssubmit(s)
            swait(prev)
            prev = cur
        swait(prev)
        barrier(dist)
        s_elapsed = max_over_ranks(dist, time.perf_counter() - ts)
        sctx.check(slib.of_pairs_close(sctx.handle))
        sctx.close()
        streamed = {"value": round(world * args.pairs * args.steps / s_elapsed, 4),
                    "ms_per_step": round(1e3 * s_elapsed / args.steps, 3), "steps": args.steps,
                    "flows_equal_host_to_host": bool(all(np.array_equal(a, b) for a, b in
                                                 zip(souts[(args.steps - 1) % 2], outs))),
                    "api": "of_pairs_open/submit/wait, step s+1 queued before step s is waited for"}

    # the host steps reused the device slots: upload the frames again for
    # the per-level pair and the profiled replays
    upload_all(1)
    # per-level times + accuracy from one more (untimed) pair
    st = _abi.OfStats()
    P = _abi.OfParams()
    C.memmove(C.byref(P), C.byref(P0), C.sizeof(P0))
    ctx.check(lib.of_pair_run(ctx.handle, 0, C.byref(P), C.byref(st)))
    uv = np.empty((2, H, W), dtype=np.float32)
    ctx.check(lib.of_pair_download(ctx.handle, 0, _native.ptr(uv)))
    uv = np.moveaxis(uv, 0, 2)
    aepe_single = float(np.sqrt(((uv - gts[0]) ** 2).sum(-1)).mean())
    # the timed (lanes) flow of pair 0 = synth_pair(H, W, 0) on rank 0,
    # against the analytic GT and against the reference's own AEPE
    aepe = float(np.sqrt(((np.moveaxis(dev_uv, 0, 2) - gts[0]) ** 2).sum(-1)).mean())
    a_ref, ref_fix = ref_aepe()
    sd = st.as_dict()

    roofline = None
    ktimes, kt_iso = {}, {}
    pl_iso = {}
    pcg_levels = None
    inner = None
    if not args.no_profile:
        # profiled replay of one step, same pairs and lanes as the timed
        # steps: HIP events around every launch on the stream it runs on
        tline = []
        ktimes, per_level = profiled_replay(ctx, lib, P0, args.pairs, args.lanes, timeline=tline)
        pcg_levels = [{"px": px, "ms": round(rec["ms_total"] / args.pairs, 3), "launches": rec["launches"] / args.pairs,
                       "active": per_level.get(("pcg_iter.active", px), {}).get("launches", 0) / args.pairs}
                      for (n, px), rec in sorted(per_level.items(), key=lambda kv: -kv[0][1]) if n == "pcg_iter"]
        # the roofline proper: the same pairs one at a time (lanes = 1), so a
        # kernel's duration is its own, not stretched by another lane's
        # kernels sharing the CUs (profiles/: rocprofv3 of bench.py --lanes 1)
        kt1, pl1 = profiled_replay(ctx, lib, P0, args.pairs, 1)
        kt_iso, pl_iso = kt1, pl1
        roofline = roofline_of(kt1, pl1)
        if roofline is not None:
            roofline["replay"] = "isolated: lanes=1 over the step's pairs"
            inner = inner_loop_of(kt1, pl1)
            rc = roofline_of(ktimes, per_level)
            conc = inner_loop_of(ktimes, per_level)
            roofline["concurrent"] = {
                "replay": f"lanes={args.lanes} as timed; durations include co-running kernels of other lanes",
                "achieved": rc["achieved"], "frac": rc["frac"], "mean_launch_ms": rc["mean_launch_ms"],
                "inner_loop_frac": conc["frac"] if conc else None}
            roofline["inner_loop"] = inner
            roofline["wmf"] = wmf_compute_roofline(pl1)
            roofline["symbol"] = pmc_symbol(roofline["kernel"])
            roofline["pmc_workload"] = WORKLOAD if load_pmc(roofline["kernel"]) else None
            lv = [px for (n, px) in per_level if n == roofline["kernel"]]
            if lv:
                roofline["as_timed"] = as_timed_of(tline, per_level, roofline["kernel"], max(lv))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": metric_name(args),
            "value": round(value, 4), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.method} on synth_pair({H},{W},seed) RGB, {args.pairs} pair(s)/GPU/step, "
                                   f"{min(args.lanes, args.pairs)} in flight",
                       "method": args.method, "height": H, "width": W, "pairs_per_gpu": args.pairs,
                       "lanes": min(args.lanes, args.pairs),
                       "solver": args.solver or "backslash (GPU block-Jacobi PCG surrogate)",
                       "parallelism": f"pairs sharded 1/GPU x {world}, RCCL gather"
                                      + (" (one-rank proxy, --rccl-self)" if args.rccl_self else "")},
            "rccl_nranks": rccl_nranks if gathering else None,
            "rccl_gather_per_step": bool(gathering),
            "timed_region": "frames resident in HBM (device slots, uploaded before the timed region) -> "
                            "flows (fp32) left in HBM; K steps queued back to back through the pair pool "
                            "(of_pairs_submit_slots), each step's flows gathered to rank 0 over RCCL when "
                            "rccl_gather_per_step (N > 1, or --rccl-self); round 5 on: the steps overlap (before "
                            "round 5 each step drained its lanes -- compare those rounds with "
                            "device_resident_drained)",
            "device_resident_drained": {"value": round(world * NP * args.steps / d_elapsed, 4),
                                        "ms_per_step": round(1e3 * d_elapsed / args.steps, 3),
                                        "steps": args.steps,
                                        "flow_equals_timed_flow": bool(np.array_equal(drained_uv, dev_uv)),
                                        "note": "one of_pairs_run per step: the lanes drain at every step end "
                                                "(rounds 1-4's device-resident form)"},
            "host_to_host": {"value": round(world * args.pairs * hsteps / h_elapsed, 4),
                             "ms_per_step": round(1e3 * h_elapsed / hsteps, 3), "steps": hsteps,
                             "host_flow_equals_timed_flow": host_eq_dev,
                             "note": "PCIe-inclusive: uint8 frames in host memory -> flows in host memory "
                                     "(of_pairs_run_host)"},
            "streamed": streamed,
            "gather_check": gather,
            "roofline": roofline, "cpu_baseline": cpu,
            "ms_per_level": [{"stage": l["stage"], "h": l["h"], "w": l["w"], "ms": round(l["ms"], 3)}
                             for l in sd["levels"]],
            "aepe_gt": round(aepe, 6),
            "flow_sha1": __import__("hashlib").sha1(dev_uv.tobytes()).hexdigest()[:16],
            "aepe_ref": None if a_ref is None or seeds[0] != 0 else {
                "ref_aepe_gt": round(a_ref, 6), "aepe_ref_delta": round(aepe - a_ref, 7),
                "fixture": f"tests/golden/{ref_fix}",
                "note": "timed flow of synth_pair(H, W, 0) vs the reference's own estimate_flow on the same pair"},
            "aepe_gt_single_pair": round(aepe_single, 6),
            "solver_iters_total": sd["solver_iters_total"],
            "solver_iters_max": sd["solver_iters_max"], "solves": sd["solves"],
            "pcg_per_level": pcg_levels,
            "level_breakdown": level_breakdown(
                [{"h": l["h"], "w": l["w"], "ms": l["ms"]} for l in sd["levels"]], pl_iso, args.pairs)
            if pl_iso else None,
            # HIP-event kernel time per pair: isolated = the lanes=1 replay
            # (sums to <= the serial pair time); concurrent = the lanes replay
            # as timed, where durations include co-running lanes' kernels
            "kernel_ms_per_pair_isolated": kms(kt_iso, args.pairs),
            "kernel_ms_per_pair_concurrent": kms(ktimes, args.pairs),
        }
        print(json.dumps(line), flush=True)
    if gathering:
        lib.of_rccl_finalize(ctx.handle)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
