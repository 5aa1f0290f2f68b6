"""Multi-GPU bench path on CPU: world size 2 over gloo.

bench.py shards pairs one process per GPU (pair k of the global batch on
rank k // P), times each rank between barriers and reports the max over
ranks; gloo carries only the barrier, the max-reduce and the RCCL unique-id
broadcast.  These tests run exactly those functions in two CPU processes.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, pairs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    dist, w, r, local = bench.dist_setup(None)
    assert (w, r, local) == (world, rank, rank)
    seeds = bench.shard_seeds(r, pairs)
    # every rank's seeds, gathered on every rank (test-side only)
    allseeds = [None] * w
    dist.all_gather_object(allseeds, seeds)
    bench.barrier(dist)
    t = bench.max_over_ranks(dist, 1.0 + rank)  # rank r "took" 1+r seconds
    # RCCL unique-id broadcast as bench.main does it (bytes object from rank 0)
    obj = [bytes([7] * 128) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    q.put((rank, seeds, allseeds, t, obj[0]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pairs", [1, 3])
def test_bench_sharding_world2(pairs):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pairs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    flat = sorted(s for _, _, allseeds, _, _ in res[:1] for ss in allseeds for s in ss)
    # the global batch is covered exactly once: seeds 0 .. world*pairs-1
    assert flat == list(range(world * pairs))
    for rank, seeds, allseeds, t, uid in res:
        assert seeds == list(range(rank * pairs, (rank + 1) * pairs))
        assert allseeds == res[0][2]
        assert t == pytest.approx(float(world))  # max over ranks
        assert uid == bytes([7] * 128)


def test_bench_single_process_defaults(monkeypatch):
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    dist, w, r, local = bench.dist_setup(None)
    assert dist is None and (w, r, local) == (1, 0, 0)
    assert bench.max_over_ranks(None, 3.5) == 3.5
    assert bench.shard_seeds(0, 2) == [0, 1]


def test_roofline_of_all_and_finest():
    import bench
    per_level = {("pcg_iter", 1000): {"ms_total": 2.0, "launches": 10, "px": 1e10},
                 ("pcg_iter.active", 1000): {"ms_total": 0.0, "launches": 8, "px": 8e9},
                 ("pcg_iter", 100): {"ms_total": 1.0, "launches": 10, "px": 1e9},
                 ("wmf", 1000): {"ms_total": 0.5, "launches": 1, "px": 1000.0}}
    kt = {}
    for (n, _), rec in per_level.items():
        a = kt.setdefault(n, {"ms_total": 0.0, "launches": 0.0, "px": 0.0})
        for k in a:
            a[k] += rec[k]
    r = bench.roofline_of(kt, per_level)
    bpp = bench.KERNEL_BYTES_PER_PX["pcg_iter"]
    assert r["kernel"] == "pcg_iter"
    # all levels: only the finest level reports active launches -> 8 launches
    # of 1e9 px priced against the 3 ms of all 20 launches
    assert r["achieved"] == pytest.approx(bpp * 1e9 / (3.0 / 8 * 1e-3) / 1e9, rel=1e-3)
    # finest: 8 active launches of 1e9 px in 2 ms
    assert r["finest"]["achieved"] == pytest.approx(bpp * 1e9 / (2.0 / 8 * 1e-3) / 1e9, rel=1e-3)
    assert r["finest"]["active_launches_per_step"] == 8
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS, rel=1e-3)
    # mean per launch over every launch (the rocprofv3 --stats average)
    assert r["mean_launch_ms"] == pytest.approx(3.0 / 20, rel=1e-3)
    assert r["finest"]["mean_launch_ms"] == pytest.approx(2.0 / 10, rel=1e-3)
    assert r["finest"]["mean_active_launch_ms"] == pytest.approx(2.0 / 8, rel=1e-3)


def _gather_worker(rank, world, port, pairs, q):
    """bench.gather_check's digest exchange and layout verification over
    gloo; the device gather itself (of_rccl_gather_flows: rank 0 receives
    rank src's slot s at src * P + s) is emulated with gather_object."""
    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    dist, w, r, _ = bench.dist_setup(None)
    outs = [np.random.default_rng(k).random((2, 6, 5)).astype(np.float32) for k in bench.shard_seeds(r, pairs)]
    every = [None] * w
    dist.all_gather_object(every, bench.flow_digests(outs))
    got = [None] * w if r == 0 else None
    dist.gather_object(outs, got, dst=0)
    res = None
    if r == 0:
        buf = np.stack([got[src][s] for src in range(w) for s in range(pairs)])
        ok = bench.verify_gather(buf, every, w, pairs)
        bad = buf.copy()
        bad[[0, -1]] = bad[[-1, 0]]  # two pairs swapped: must be caught
        res = (ok, bench.verify_gather(bad, every, w, pairs))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_layout_check_world2():
    world, pairs = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, pairs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == (True, False)


def test_inner_loop_figure():
    """SURVEY.md §8d inner-loop bytes: N*(48+56+24) per warp + 76*N*K over
    the warp / assembly / update / CG kernel time."""
    import bench
    kt = {"pcg_iter": {"ms_total": 10.0, "launches": 100, "px": 2e8},
          "pcg_iter.active": {"ms_total": 0.0, "launches": 90, "px": 1.8e8},
          "partial_deriv_hermite": {"ms_total": 1.0, "launches": 6, "px": 1.2e7},
          "flow_operator": {"ms_total": 1.0, "launches": 6, "px": 1.2e7},
          "update_occ": {"ms_total": 0.5, "launches": 6, "px": 1.2e7},
          "pcg_small": {"ms_total": 0.5, "launches": 6, "px": 1e4},
          "wmf": {"ms_total": 5.0, "launches": 6, "px": 1.2e7}}
    pl = {(n, 2000000): r for n, r in kt.items() if n != "pcg_small"}
    r = bench.inner_loop_of(kt, pl)
    byt = 1.2e7 * (48 + 56 + 24) + 76 * 1.8e8
    assert r["bytes_per_step"] == round(byt)
    assert r["kernel_ms_per_step"] == 13.0  # wmf excluded, pcg_small counted
    assert r["frac"] == pytest.approx(byt / 13e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["finest"]["frac"] == pytest.approx(byt / 12.5e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def _run_bench(args, env, timeout=240):
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher around it starts
    torch.distributed.run with two processes (a child, no exec), each rank
    rendezvouses over gloo, and rank 0's line -- relayed once by the parent --
    reports n_gpus 2 and both ranks (--dry-run stops before the library)."""
    r, recs = _run_bench(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "0"], _bench_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    assert sorted(map(tuple, rec["ranks"])) == [(0, 0, 2), (1, 1, 2)]
    assert rec["max_over_ranks"] == pytest.approx(0.002)
    assert "torch.distributed.run child, 2 processes" in rec["launch"]


def test_bench_gpus1_runs_in_process():
    r, recs = _run_bench(["--gpus", "1", "--dry-run"], _bench_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(recs) == 1 and recs[0]["n_gpus"] == 1 and recs[0]["ranks"] == [[0, 0, 1]]
    assert "launch" not in recs[0]


def test_bench_world_size_mismatch_refused():
    r, recs = _run_bench(["--gpus", "1", "--dry-run"], _bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and not recs
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
    r, recs = _run_bench(["--gpus", "2", "--rccl-self", "--dry-run"], _bench_env(WORLD_SIZE="2"))
    assert r.returncode == 2 and not recs
