"""Batch file pipeline around the hot path.

The steps either side of `estimate_flow` in a benchmark run of the reference
(its notebooks loop over them one pair at a time): PNG decode in
`read_flow_file`'s layout (`flo_io.py:66-113`) -> flow -> `write_flo`
(`flo_io.py:46-63`) + `flow_angular_error` against the ground truth when one
exists (`metrics.py:5-53`).  Here every decoded pair goes into a PairStream
(`of_pairs_open` / `of_pairs_submit` / `of_pairs_wait`: `lanes` GPU pipelines
fed from a queue, H2D/D2H overlapped inside the library), kept open between
calls, and the host file work is overlapped with the GPU:

    decode pool   : the next pairs' PNGs (+ GT .flo)              \
    this thread   : submits decoded pairs, waits for the oldest    } at once
    writer pool   : .flo files + AAE/AEPE from the flow planes      /

(`stream=False`: the round-3 form, chunks of same-size pairs per
`of_pairs_run_host` call, which drains the lanes at every chunk boundary.)
Pairs are grouped by frame shape (Middlebury sequences differ in size) and
results come back in job order.  Each flow equals `estimate_flow(im1, im2,
method, params)` on the decoded frames: bitwise below 2^20 px, and to CG
rounding at >= 2^20 px with lanes >= 2, where two pairs' fine solves run side
by side in another block geometry (include/optflow.h, of_pairs_run).
"""
import atexit
import os
import threading
import time
from collections import OrderedDict, namedtuple
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


def load_frame(p):
    """One 8-bit PNG frame as uint8; RGB(A) keeps its first 3 channels
    (estimate_flow uses im[:, :, :3])."""
    from PIL import Image
    a = np.asarray(Image.open(p))
    if a.dtype != np.uint8:
        raise ValueError(f"{p}: {a.dtype} frames are not supported (8-bit PNGs only)")
    if a.ndim == 3:
        if a.shape[2] < 3:
            raise ValueError(f"{p}: {a.shape[2]}-channel frames are not supported")
        a = a[:, :, :3]
    return np.ascontiguousarray(a)


def _pair_of(job, a, b, gt):
    if a.shape != b.shape:
        raise ValueError(f"{job.name}: frame shapes differ {a.shape} vs {b.shape}")
    return a, b, gt


def decode_pair(job):
    """(uint8 frame 1, uint8 frame 2, ground truth (H, W, 2) float32 or None)."""
    return _pair_of(job, load_frame(job.im1), load_frame(job.im2), read_flo(job.gt) if job.gt else None)


def _finish(job, uv, gt, border, keep=False, planar=False):
    """Write the .flo and evaluate one pair (writer thread).  `uv` (H, W, 2),
    or with `planar` the library's (2, H, W) float32 planes
    (PairStream.wait(planar=True)): then the .flo is written from the planes
    and the metrics take them as they are (flow_angular_error computes in
    float64 either way, so the numbers are the same), and only `keep` builds
    the (H, W, 2) float64 flow.  The caller says which layout it passes (a
    (2, W, 2) flow is both shapes)."""
    u, v = (uv[0], uv[1]) if planar else (uv[..., 0], uv[..., 1])
    res = {"name": job.name, "shape": u.shape, "out": job.out}
    if job.out:
        os.makedirs(os.path.dirname(os.path.abspath(job.out)), exist_ok=True)
        write_flo(np.moveaxis(uv, 0, 2) if planar else uv, job.out)
    if gt is not None:
        aae, std, aepe = flow_angular_error(gt[..., 0], gt[..., 1], u, v, border)
        res.update(aae=float(aae), std_ae=float(std), aepe=float(aepe))
    if keep:
        if planar:
            from optical_flow import _native as nat
            uv = nat.interleaved(uv)
        res["uv"] = uv
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


# Open PairStreams kept between run_pipeline calls (a server's pool: lane
# threads, contexts and arenas stay warm), keyed by (frame shape, method,
# params, lanes); at most _MAX_STREAMS, the least recently used closed first.
# One by default: a stream's lanes hold GPU_MAX_HW_QUEUES-sized stream sets
# and their own fine-solve token, so two open pools would oversubscribe the
# hardware queues and run their fine solves uncoordinated; a shape change
# drains and closes the open pool.
_STREAMS = OrderedDict()
_MAX_STREAMS = 1
_STREAMS_LOCK = threading.Lock()


def close_streams():
    """Close every PairStream run_pipeline keeps open (frees their lanes'
    device memory); the next run_pipeline call opens new ones."""
    with _STREAMS_LOCK:
        while _STREAMS:
            _STREAMS.popitem(last=False)[1].close()


atexit.register(close_streams)


def _stream_key(shape, method, params, lanes):
    return (shape, method, repr(sorted(params.items())) if isinstance(params, dict) else repr(params), lanes)


def _run_streaming(jobs, method, params, lanes, ahead_chunks, workers, writers, border, keep_flows,
                   max_streams=_MAX_STREAMS):
    """run_pipeline's streaming form: decode pool -> PairStream per frame
    shape (kept open in _STREAMS for later calls; at most `max_streams`, the
    least recently used one drained and closed) -> writer pool, results in job
    order."""
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

    streams = _STREAMS   # key -> PairStream, least recently used first
    inflight = {}   # key -> [(job index, ticket, ground truth)]
    window = 2 * lanes + 2
    results = [None] * len(jobs)
    writes = []
    with ThreadPoolExecutor(workers) as dec, ThreadPoolExecutor(writers) as wr:
        futs = [None] * len(jobs)
        nsub = 0
        ahead = 2 * max(1, ahead_chunks)

        def submit_upto(n):
            # the two frames and the GT of a pair decode on separate workers
            # (the first pair's decode is the pipeline's start-up latency)
            nonlocal nsub
            while nsub < min(n, len(jobs)):
                j = jobs[nsub]
                futs[nsub] = (dec.submit(timed, "decode_s", load_frame, j.im1),
                              dec.submit(timed, "decode_s", load_frame, j.im2),
                              dec.submit(timed, "decode_s", read_flo, j.gt) if j.gt else None)
                nsub += 1

        def retire(key):
            i, t, gt = inflight[key].pop(0)
            uv = timed("gpu_s", streams[key].wait, t, True)  # planar: converted by the writer
            writes.append((i, wr.submit(timed, "write_s", _finish, jobs[i], uv, gt, border, keep_flows, True)))

        def drain(key):
            while inflight.get(key):
                retire(key)
            inflight.pop(key, None)

        with _STREAMS_LOCK:
            try:
                for i in range(len(jobs)):
                    submit_upto(i + ahead)
                    fa, fb, fg = futs[i]
                    futs[i] = None
                    a, b, gt = _pair_of(jobs[i], fa.result(), fb.result(), fg.result() if fg else None)
                    key = _stream_key(a.shape, method, params, lanes)
                    if key not in streams:
                        while len(streams) >= max_streams:
                            old = next(iter(streams))
                            drain(old)
                            streams.pop(old).close()
                        streams[key] = PairStream(a.shape[0], a.shape[1], 3 if a.ndim == 3 else 1, method,
                                                  params, lanes)
                    streams.move_to_end(key)  # most recently used last
                    inflight.setdefault(key, []).append((i, streams[key].submit(a, b), gt))
                    while len(inflight[key]) > window:
                        retire(key)
                for key in list(inflight):
                    drain(key)
            except BaseException:
                # a failed run leaves no half-drained stream behind
                for key in list(inflight):
                    if key in streams:
                        streams.pop(key).close()
                raise
        for i, f in writes:
            results[i] = f.result()
    wall = time.perf_counter() - t_start
    stats = {"pairs": len(jobs), "wall_s": wall, "pairs_per_s": len(jobs) / wall if wall > 0 else 0.0,
             "stream": True}
    stats.update(busy)
    return results, stats
