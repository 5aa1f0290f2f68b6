"""Batch file pipeline (optical_flow/pipeline.py):
PNG decode -> flows -> write_flo + flow_angular_error, host I/O overlapped
with the GPU.  CPU tests drive the host logic with a stand-in flow function;
the gpu test runs the real path and checks every written .flo and metric
against per-pair estimate_flow + flow_angular_error, and RubberWhale's AEPE
against the reference's known answer."""
import os
import shutil

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN


def _write_pairs(tmp, shapes, seed=0):
    """Synthetic PNG pairs (uint8, RGB or gray) + GT .flo files; returns jobs."""
    from optical_flow.io.flo_io import write_flo
    from optical_flow.pipeline import PairJob
    from optical_flow.utils.synthetic import synth_pair
    jobs = []
    for k, (h, w, c) in enumerate(shapes):
        im1, im2, gt = synth_pair(h, w, seed + k)
        a, b = im1.astype(np.uint8), im2.astype(np.uint8)
        if c == 1:
            a, b = a[:, :, 1], b[:, :, 1]
        d = tmp / f"p{k}"
        d.mkdir()
        Image.fromarray(a).save(d / "f0.png")
        Image.fromarray(b).save(d / "f1.png")
        write_flo(gt, str(d / "gt.flo"))
        jobs.append(PairJob(f"p{k}", str(d / "f0.png"), str(d / "f1.png"), str(d / "gt.flo"), str(d / "out.flo")))
    return jobs


def test_pipeline_host_logic(tmp_path):
    """Order, shape grouping, chunking, .flo output and metrics with a
    stand-in flow function (no GPU): flow = (mean of frame 1 / 100, index)."""
    from optical_flow import flow_angular_error, read_flo
    from optical_flow.pipeline import run_pipeline
    shapes = [(20, 30, 3), (24, 18, 3), (20, 30, 3), (20, 30, 1), (20, 30, 3), (24, 18, 3), (20, 30, 3)]
    jobs = _write_pairs(tmp_path, shapes)
    jobs[3] = jobs[3]._replace(gt=None)
    calls = []

    def fake(a, b):
        calls.append([x.shape for x in a])
        assert all(x.dtype == np.uint8 for x in a + b)
        return [np.stack([np.full(x.shape[:2], x.mean() / 100.0), np.full(x.shape[:2], float(x.shape[1]))], 2)
                for x in a]

    res, st = run_pipeline(jobs, chunk=2, workers=3, flow_fn=fake, keep_flows=True, border=2)
    assert st["pairs"] == len(jobs) and st["wall_s"] > 0
    assert [r["name"] for r in res] == [j.name for j in jobs]
    # every chunk is one shape, at most 2 long, and every pair ran once
    assert all(len(set(c)) == 1 and len(c) <= 2 for c in calls)
    assert sum(len(c) for c in calls) == len(jobs)
    for j, r, (h, w, c) in zip(jobs, res, shapes):
        assert r["shape"] == (h, w)
        uv = read_flo(j.out)
        np.testing.assert_array_equal(uv, r["uv"].astype(np.float32))
        if j.gt is None:
            assert "aepe" not in r
        else:
            gt = read_flo(j.gt)
            want = flow_angular_error(gt[..., 0], gt[..., 1], r["uv"][..., 0], r["uv"][..., 1], 2)
            np.testing.assert_allclose((r["aae"], r["std_ae"], r["aepe"]), want, rtol=1e-12)


def test_pipeline_errors(tmp_path):
    from optical_flow.pipeline import PairJob, run_pipeline
    assert run_pipeline([], flow_fn=lambda a, b: [])[0] == []
    jobs = _write_pairs(tmp_path, [(16, 16, 3), (16, 20, 3)])
    bad = PairJob("bad", jobs[0].im1, jobs[1].im2)
    with pytest.raises(ValueError):
        run_pipeline([bad], flow_fn=lambda a, b: [np.zeros(a[0].shape[:2] + (2,))])
    with pytest.raises(ValueError):
        run_pipeline(jobs, chunk=0, flow_fn=lambda a, b: [])


def test_finish_layout_is_explicit(tmp_path):
    """_finish takes the layout from its caller: a (2, W, 2) float32 flow in
    (H, W, 2) layout (H == 2) is written and evaluated as such, not read as
    planes."""
    from optical_flow import flow_angular_error, read_flo
    from optical_flow.pipeline import PairJob, _finish
    rng = np.random.default_rng(3)
    uv = rng.standard_normal((2, 7, 2)).astype(np.float32)
    gt = rng.standard_normal((2, 7, 2)).astype(np.float32)
    out = str(tmp_path / "a.flo")
    r = _finish(PairJob("a", None, None, out=out), uv, gt, 0, keep=True)
    np.testing.assert_array_equal(read_flo(out), uv)
    assert r["shape"] == (2, 7)
    want = flow_angular_error(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1], 0)
    np.testing.assert_allclose((r["aae"], r["std_ae"], r["aepe"]), want, rtol=1e-12)
    # the same flow as planes, said so
    out2 = str(tmp_path / "b.flo")
    r2 = _finish(PairJob("b", None, None, out=out2), np.ascontiguousarray(np.moveaxis(uv, 2, 0)), gt, 0,
                 keep=True, planar=True)
    np.testing.assert_array_equal(read_flo(out2), uv)
    np.testing.assert_allclose((r2["aae"], r2["std_ae"], r2["aepe"]), want, rtol=1e-12)


def test_middlebury_jobs_layout(tmp_path):
    from optical_flow.pipeline import middlebury_jobs
    root = tmp_path / "data"
    for s, gt in (("RubberWhale", True), ("Beanbags", False)):
        (root / "other-data" / s).mkdir(parents=True)
        if gt:
            (root / "other-gt-flow" / s).mkdir(parents=True)
            shutil.copy(os.path.join(GOLDEN, "flow10.flo"), root / "other-gt-flow" / s / "flow10.flo")
    jobs = middlebury_jobs(str(root), out_dir=str(tmp_path / "out"))
    assert [j.name for j in jobs] == ["Beanbags", "RubberWhale"]
    assert jobs[0].gt is None and jobs[1].gt.endswith("RubberWhale/flow10.flo")
    assert jobs[1].im2.endswith("RubberWhale/frame11.png") and jobs[1].out.endswith("RubberWhale/flow10.flo")


@pytest.mark.gpu
@pytest.mark.parametrize("stream", [True, False])
def test_pipeline_gpu_matches_estimate_flow(tmp_path, stream):
    """Real path: RubberWhale (Middlebury layout built from the committed
    frames + GT) and synthetic pairs of two other sizes, RGB and gray, chunk
    2, 3 lanes.  Every written .flo equals estimate_flow on the decoded
    frames (fp32), every metric equals flow_angular_error of it, and
    RubberWhale's AEPE is within 1e-3 of the reference's 0.080250 (AAE
    2.46298 within 0.02 deg)."""
    import optical_flow
    from optical_flow import flow_angular_error, read_flo
    from optical_flow.pipeline import middlebury_jobs, run_pipeline
    root = tmp_path / "data"
    (root / "other-data" / "RubberWhale").mkdir(parents=True)
    (root / "other-gt-flow" / "RubberWhale").mkdir(parents=True)
    for f in ("frame10.png", "frame11.png"):
        shutil.copy(os.path.join(GOLDEN, f), root / "other-data" / "RubberWhale" / f)
    shutil.copy(os.path.join(GOLDEN, "flow10.flo"), root / "other-gt-flow" / "RubberWhale" / "flow10.flo")
    jobs = middlebury_jobs(str(root), out_dir=str(tmp_path / "out"))
    syn = tmp_path / "syn"
    syn.mkdir()
    jobs += _write_pairs(syn, [(40, 56, 3), (48, 64, 1), (40, 56, 3), (40, 56, 3)], seed=5)
    # three frame shapes: the streaming form keeps one PairStream open (the
    # default _MAX_STREAMS) and drains and closes it when the shape changes
    res, st = run_pipeline(jobs, lanes=3, chunk=2, keep_flows=True, stream=stream)
    print(f"pipeline: {st}")
    for j, r in zip(jobs, res):
        im1 = np.array(Image.open(j.im1)).astype(np.float64)
        im2 = np.array(Image.open(j.im2)).astype(np.float64)
        uv = optical_flow.estimate_flow(im1, im2)
        np.testing.assert_array_equal(read_flo(j.out), uv.astype(np.float32), err_msg=j.name)
        gt = read_flo(j.gt)
        want = flow_angular_error(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1])
        np.testing.assert_allclose((r["aae"], r["std_ae"], r["aepe"]), want, rtol=1e-12, err_msg=j.name)
    rw = res[0]
    print(f"RubberWhale AAE {rw['aae']:.5f} AEPE {rw['aepe']:.6f} (reference 2.46298 / 0.080250)")
    assert abs(rw["aepe"] - 0.080250) <= 1e-3 and abs(rw["aae"] - 2.46298) <= 0.02
    if stream:
        # the last stream stays open for the next call, which gives the same
        # flows; close_streams releases it
        from optical_flow import pipeline as pl
        assert len(pl._STREAMS) == pl._MAX_STREAMS == 1
        res2, _ = run_pipeline(jobs, lanes=3, chunk=2, keep_flows=True)
        for r, q in zip(res, res2):
            np.testing.assert_array_equal(r["uv"], q["uv"])
        pl.close_streams()
        assert not pl._STREAMS


@pytest.mark.gpu
def test_pair_stream_matches_batch():
    """PairStream (of_pairs_open / submit / wait / close): pairs submitted one
    by one and waited out of order give bitwise the flows of
    estimate_flow_batch with the same lanes; bad frames and tickets raise."""
    import optical_flow
    from optical_flow.utils.synthetic import synth_pair
    pairs = [synth_pair(60, 88, 30 + k) for k in range(5)]
    a = [p[0].astype(np.uint8) for p in pairs]
    b = [p[1].astype(np.uint8) for p in pairs]
    want = optical_flow.estimate_flow_batch(a, b, "classic+nl-fast", lanes=2)
    with optical_flow.PairStream(60, 88, 3, "classic+nl-fast", lanes=2) as s:
        t = [s.submit(x, y) for x, y in zip(a, b)]
        got = {k: s.wait(t[k]) for k in (3, 0, 4, 1, 2)}
        with pytest.raises(ValueError):
            s.submit(a[0][:, :-1], b[0][:, :-1])
        with pytest.raises(ValueError):
            s.wait(t[0])  # already waited
        t5 = s.submit(a[2], b[2])
        late = s.wait(t5)
    for k in range(5):
        np.testing.assert_array_equal(got[k], want[k])
    np.testing.assert_array_equal(late, want[2])
    # gray frames, one lane: bitwise estimate_flow
    g1 = [np.round(x.mean(-1)).astype(np.uint8) for x in a[:2]]
    g2 = [np.round(x.mean(-1)).astype(np.uint8) for x in b[:2]]
    with optical_flow.PairStream(60, 88, 1, "hs", lanes=1) as s:
        uv = [s.wait(s.submit(x, y)) for x, y in zip(g1, g2)]
    for k in range(2):
        np.testing.assert_array_equal(uv[k], optical_flow.estimate_flow(g1[k].astype(float), g2[k].astype(float), "hs"))
