"""File-to-file throughput of the batch pipeline (optical_flow/pipeline.py,
SURVEY.md §8f row 2) next to the in-memory host-to-host rate of the same
pairs: N synth_pair(H, W, k) pairs written as PNG (+ GT .flo) to a scratch
directory, then decode -> estimate_flow_batch -> write_flo + AAE/AEPE with
host I/O overlapped.  One JSON line.
usage: python tools/pipeline_bench.py [--pairs 16] [--height 1080] [--width 1920] [--out DIR]"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

from optical_flow import estimate_flow_batch, write_flo  # noqa: E402
from optical_flow.pipeline import PairJob, run_pipeline  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=16)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--writers", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tmp = a.out or tempfile.mkdtemp(prefix="ofpipe_")
    jobs, f1, f2 = [], [], []
    for k in range(a.pairs):
        im1, im2, gt = synth_pair(a.height, a.width, k)
        d = os.path.join(tmp, f"p{k:03d}")
        os.makedirs(d, exist_ok=True)
        Image.fromarray(im1.astype(np.uint8)).save(os.path.join(d, "frame10.png"))
        Image.fromarray(im2.astype(np.uint8)).save(os.path.join(d, "frame11.png"))
        write_flo(gt, os.path.join(d, "gt.flo"))
        f1.append(im1.astype(np.uint8))
        f2.append(im2.astype(np.uint8))
        jobs.append(PairJob(f"p{k:03d}", os.path.join(d, "frame10.png"), os.path.join(d, "frame11.png"),
                            os.path.join(d, "gt.flo"), os.path.join(d, "out.flo")))
        if k % 8 == 7:
            print(f"wrote {k + 1} pairs", flush=True)
    estimate_flow_batch(f1[:a.lanes], f2[:a.lanes], lanes=a.lanes)  # warm-up: arenas, lanes, code objects
    t0 = time.perf_counter()
    for s in range(0, a.pairs, a.chunk):
        estimate_flow_batch(f1[s:s + a.chunk], f2[s:s + a.chunk], lanes=a.lanes)
    mem = a.pairs / (time.perf_counter() - t0)
    # warm-up of the streaming path: its PairStream (lanes, arenas) stays open
    # in optical_flow.pipeline for the timed run, as in a long-running server
    run_pipeline(jobs[:2 * a.lanes], lanes=a.lanes, chunk=a.chunk, workers=a.workers, writers=a.writers)
    res, st = run_pipeline(jobs, lanes=a.lanes, chunk=a.chunk, workers=a.workers, writers=a.writers)
    aepe = float(np.mean([r["aepe"] for r in res]))
    # the round-3 form: chunks of `chunk` pairs per of_pairs_run_host call
    res_c, st_c = run_pipeline(jobs, lanes=a.lanes, chunk=a.chunk, workers=a.workers, writers=a.writers,
                               stream=False)
    assert all(np.array_equal(r.get("aepe"), q.get("aepe")) for r, q in zip(res, res_c))
    print(json.dumps({"metric": "file-to-file pairs/s (PNG decode -> flow -> .flo + AAE/AEPE)",
                      "value": round(st["pairs_per_s"], 3), "in_memory_pairs_per_s": round(mem, 3),
                      "pairs": a.pairs, "height": a.height, "width": a.width, "lanes": a.lanes, "chunk": a.chunk,
                      "workers": a.workers, "writers": a.writers,
                      "wall_s": round(st["wall_s"], 3), "gpu_busy_s": round(st["gpu_s"], 3),
                      "decode_busy_s": round(st["decode_s"], 3), "write_busy_s": round(st["write_s"], 3),
                      "mean_aepe_gt": round(aepe, 5),
                      "mode": "stream (of_pairs_submit / of_pairs_wait), stream opened by a warm-up run",
                      "chunked": {"value": round(st_c["pairs_per_s"], 3), "wall_s": round(st_c["wall_s"], 3),
                                  "gpu_busy_s": round(st_c["gpu_s"], 3)}}), flush=True)
    if not a.out:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
