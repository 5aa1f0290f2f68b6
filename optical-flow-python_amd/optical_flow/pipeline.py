"""Batch file pipeline around the hot path.

The steps either side of `estimate_flow` in a benchmark run of the reference
(its notebooks loop over them one pair at a time): PNG decode in
`read_flow_file`'s layout (`flo_io.py:66-113`) -> flow -> `write_flo`
(`flo_io.py:46-63`) + `flow_angular_error` against the ground truth when one
exists (`metrics.py:5-53`).  Here the flows of a chunk of same-size pairs come
from ONE `of_pairs_run_host` call (`estimate_flow_batch`: `lanes` pairs in
flight, H2D/D2H overlapped inside the library), and the host file work is
overlapped with the GPU:

    decode pool   : chunk j+1's PNGs (+ GT .flo)                  \
    this thread   : chunk j on the GPU (ctypes releases the GIL)   } at once
    writer pool   : chunk j-1's .flo files + AAE/AEPE              /

Pairs are grouped by frame shape (Middlebury sequences differ in size) and
results come back in job order.  Each flow equals `estimate_flow(im1, im2,
method, params)` on the decoded frames: bitwise below 2^20 px, and to CG
rounding at >= 2^20 px with lanes >= 2, where two pairs' fine solves run side
by side in another block geometry (include/optflow.h, of_pairs_run).
"""
import os
import threading
import time
from collections import namedtuple
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from optical_flow.evaluation.metrics import flow_angular_error
from optical_flow.io.flo_io import read_flo, write_flo

PairJob = namedtuple("PairJob", "name im1 im2 gt out")
PairJob.__new__.__defaults__ = (None, None)
PairJob.__doc__ = """One pair: frame paths im1/im2, optional ground-truth .flo path `gt`
and output .flo path `out` (None: the flow is returned, not written)."""


def middlebury_jobs(data_dir, seqs=None, i_seq=10, out_dir=None):
    """Jobs for Middlebury sequences in `read_flow_file`'s layout
    (data_dir/other-data/<seq>/frame{i:02d}.png, frame{i+1:02d}.png and
    data_dir/other-gt-flow/<seq>/flow{i:02d}.flo when present).  seqs=None:
    every sequence directory under other-data.  Outputs go to
    out_dir/<seq>/flow{i:02d}.flo when out_dir is given."""
    img_root = os.path.join(data_dir, "other-data")
    if seqs is None:
        seqs = sorted(d for d in os.listdir(img_root) if os.path.isdir(os.path.join(img_root, d)))
    jobs = []
    for s in seqs:
        d = os.path.join(img_root, s)
        gt = os.path.join(data_dir, "other-gt-flow", s, f"flow{i_seq:02d}.flo")
        out = os.path.join(out_dir, s, f"flow{i_seq:02d}.flo") if out_dir else None
        jobs.append(PairJob(s, os.path.join(d, f"frame{i_seq:02d}.png"), os.path.join(d, f"frame{i_seq + 1:02d}.png"),
                            gt if os.path.exists(gt) else None, out))
    return jobs


def decode_pair(job):
    """(uint8 frame 1, uint8 frame 2, ground truth (H, W, 2) float32 or None).
    RGB(A) PNGs keep their first 3 channels (estimate_flow uses im[:, :, :3])."""
    from PIL import Image

    def load(p):
        a = np.asarray(Image.open(p))
        if a.dtype != np.uint8:
            raise ValueError(f"{p}: {a.dtype} frames are not supported (8-bit PNGs only)")
        if a.ndim == 3:
            if a.shape[2] < 3:
                raise ValueError(f"{p}: {a.shape[2]}-channel frames are not supported")
            a = a[:, :, :3]
        return np.ascontiguousarray(a)

    a, b = load(job.im1), load(job.im2)
    if a.shape != b.shape:
        raise ValueError(f"{job.name}: frame shapes differ {a.shape} vs {b.shape}")
    return a, b, (read_flo(job.gt) if job.gt else None)


def _finish(job, uv, gt, border):
    """Write the .flo and evaluate one pair (writer thread)."""
    res = {"name": job.name, "shape": uv.shape[:2], "out": job.out}
    if job.out:
        os.makedirs(os.path.dirname(os.path.abspath(job.out)), exist_ok=True)
        write_flo(uv, job.out)
    if gt is not None:
        aae, std, aepe = flow_angular_error(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1], border)
        res.update(aae=float(aae), std_ae=float(std), aepe=float(aepe))
    return res


def run_pipeline(jobs, method="classic+nl-fast", params=None, lanes=4, chunk=8, workers=4, writers=2, border=0,
                 keep_flows=False, flow_fn=None, stream=True):
    """Run `jobs` (PairJob list) through decode -> flow -> write + metrics
    with the three stages overlapped.  Returns (results, stats): one dict
    per job in job order ({name, shape, out, [aae, std_ae, aepe], [uv]}) and
    wall-clock stats {pairs, wall_s, pairs_per_s, decode_s, gpu_s, write_s}
    (decode_s / write_s are busy times summed over their `workers` /
    `writers` threads, so overlap shows as gpu_s ~ wall_s).  `flow_fn(im1s, im2s)` replaces the GPU batch
    call (host-logic tests); by default estimate_flow_batch(..., method,
    params, lanes) per chunk, or with `stream` (the default when no flow_fn
    is given) every decoded pair goes straight into a PairStream of its
    shape (of_pairs_submit), at most 2 lanes + 2 pairs per stream in flight,
    so the GPU lanes never drain between chunks; gpu_s is then the time this
    thread waited for flows."""
    if not jobs:
        return [], {"pairs": 0, "wall_s": 0.0, "pairs_per_s": 0.0, "decode_s": 0.0, "gpu_s": 0.0, "write_s": 0.0}
    if chunk < 1 or workers < 1 or writers < 1:
        raise ValueError("chunk, workers and writers must be >= 1")
    if flow_fn is None and stream:
        return _run_streaming(jobs, method, params, lanes, chunk, workers, writers, border, keep_flows)
    if flow_fn is None:
        from optical_flow.interface import estimate_flow_batch

        def flow_fn(a, b):
            return estimate_flow_batch(a, b, method, params, lanes=lanes)

    t_start = time.perf_counter()
    lock = threading.Lock()
    busy = {"decode_s": 0.0, "write_s": 0.0, "gpu_s": 0.0}

    def timed(key, fn, *a):
        t0 = time.perf_counter()
        try:
            return fn(*a)
        finally:
            with lock:
                busy[key] += time.perf_counter() - t0

    with ThreadPoolExecutor(workers) as dec, ThreadPoolExecutor(writers) as wr:
        # decode runs ahead of the GPU by up to 2 chunks (bounded host
        # memory); chunks are consecutive decoded pairs of one shape, at most
        # `chunk` long (shapes are known only after decoding)
        futs = [None] * len(jobs)
        ahead = 2 * chunk
        nsub = 0

        def submit_upto(n):
            nonlocal nsub
            while nsub < min(n, len(jobs)):
                futs[nsub] = dec.submit(timed, "decode_s", decode_pair, jobs[nsub])
                nsub += 1

        results = [None] * len(jobs)
        writes = []
        pending = {}  # shape -> [(index, decoded pair)]

        def flush(shape):
            items = pending.pop(shape)
            flows = timed("gpu_s", flow_fn, [p[0] for _, p in items], [p[1] for _, p in items])
            for (i, p), uv in zip(items, flows):
                writes.append((i, wr.submit(timed, "write_s", _finish, jobs[i], uv, p[2], border),
                               uv if keep_flows else None))

        for i in range(len(jobs)):
            submit_upto(i + ahead)
            pair = futs[i].result()
            futs[i] = None
            pending.setdefault(pair[0].shape, []).append((i, pair))
            if len(pending[pair[0].shape]) == chunk:
                flush(pair[0].shape)
        for shape in list(pending):
            flush(shape)
        for i, f, uv in writes:
            results[i] = f.result()
            if keep_flows:
                results[i]["uv"] = uv
    wall = time.perf_counter() - t_start
    stats = {"pairs": len(jobs), "wall_s": wall, "pairs_per_s": len(jobs) / wall if wall > 0 else 0.0}
    stats.update(busy)
    return results, stats


def _run_streaming(jobs, method, params, lanes, ahead_chunks, workers, writers, border, keep_flows, max_streams=2):
    """run_pipeline's streaming form: decode pool -> PairStream per frame
    shape (at most `max_streams` open; the least recently used one is drained
    and closed) -> writer pool, results in job order."""
    from optical_flow.interface import PairStream
    t_start = time.perf_counter()
    lock = threading.Lock()
    busy = {"decode_s": 0.0, "write_s": 0.0, "gpu_s": 0.0}

    def timed(key, fn, *a):
        t0 = time.perf_counter()
        try:
            return fn(*a)
        finally:
            with lock:
                busy[key] += time.perf_counter() - t0

    streams = {}    # shape -> PairStream, in least-recently-used order
    inflight = {}   # shape -> [(job index, ticket, ground truth)]
    window = 2 * lanes + 2
    results = [None] * len(jobs)
    writes = []
    with ThreadPoolExecutor(workers) as dec, ThreadPoolExecutor(writers) as wr:
        futs = [None] * len(jobs)
        nsub = 0
        ahead = 2 * max(1, ahead_chunks)

        def submit_upto(n):
            nonlocal nsub
            while nsub < min(n, len(jobs)):
                futs[nsub] = dec.submit(timed, "decode_s", decode_pair, jobs[nsub])
                nsub += 1

        def retire(shape):
            i, t, gt = inflight[shape].pop(0)
            uv = timed("gpu_s", streams[shape].wait, t)
            writes.append((i, wr.submit(timed, "write_s", _finish, jobs[i], uv, gt, border), uv if keep_flows else None))

        def close(shape):
            while inflight[shape]:
                retire(shape)
            streams.pop(shape).close()
            del inflight[shape]

        try:
            for i in range(len(jobs)):
                submit_upto(i + ahead)
                a, b, gt = futs[i].result()
                futs[i] = None
                shape = a.shape
                if shape not in streams:
                    if len(streams) >= max_streams:
                        close(next(iter(streams)))
                    streams[shape] = PairStream(shape[0], shape[1], 3 if a.ndim == 3 else 1, method, params, lanes)
                    inflight[shape] = []
                else:
                    streams[shape] = streams.pop(shape)  # most recently used last
                inflight[shape].append((i, streams[shape].submit(a, b), gt))
                while len(inflight[shape]) > window:
                    retire(shape)
            for shape in list(streams):
                close(shape)
        finally:
            for st in streams.values():
                st.close()
        for i, f, uv in writes:
            results[i] = f.result()
            if keep_flows:
                results[i]["uv"] = uv
    wall = time.perf_counter() - t_start
    stats = {"pairs": len(jobs), "wall_s": wall, "pairs_per_s": len(jobs) / wall if wall > 0 else 0.0,
             "stream": True}
    stats.update(busy)
    return results, stats
