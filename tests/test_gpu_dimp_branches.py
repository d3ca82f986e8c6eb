"""The device DiMP tracker (csrc/dimptrack.hip via mmtrack_amd.dimp_tracker) against the REFERENCE DeT tracker
where it makes decisions and where it is benchmarked.

* tests/golden/tracker_dimp_branches.npz (tests/golden/make_golden_dimp.py): the reference tracker
  (pytracking/tracker/dimp/dimp.py, DeT_DiMP50_Max parameters, use_iou_net False) on sequences that reach every
  branch of localize_advanced (dimp.py:239-302: not_found, uncertain from the threshold and from the distractor
  test, hard_negative from hard_sample_threshold, from the masked second peak and from the displacement test)
  and of update_classifier (dimp.py:607-650: no update for not_found / uncertain, the hard-negative learning
  rate and net_opt_hn_iter steps, net_opt_low_iter under low_score_opt_threshold, the memory filling up and
  replacing samples at the minimum weight).
* the benchmarked launch shape: tracker_dimp.npz's sequence in slots 0, 15, 16 and 31 of a 32-slot DimpPool
  driven by PipelinedBatch (bench.py's mfdimp_rgbt step), other sequences in the remaining slots.

Bar, per frame: the reference's flag, box IoU >= 0.999, confidence within 1 %; per sequence the filter after the
first hard-negative update and at the end within 1e-2 of its scale, the memory's sample weights within 1e-5
(relative) and its boxes, sample count and last replaced index as the reference's.  Both precisions."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def iou(b, r):
    ix = max(0.0, min(b[0] + b[2], r[0] + r[2]) - max(b[0], r[0]))
    iy = max(0.0, min(b[1] + b[3], r[1] + r[3]) - max(b[1], r[1]))
    return ix * iy / (b[2] * b[3] + r[2] * r[3] - ix * iy)


def close(got, ref, rel):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-12)
    assert err < rel, f"max |d| / max |ref| = {err:.2e}"


@pytest.fixture(scope="module")
def nets():
    from mmtrack_amd import synth
    from mmtrack_amd.dimpnet import DiMPNet
    sd = synth.make_dimp_state_dict(0)
    return {p: DiMPNet(sd, precision=p) for p in ("f16x3", "fp32")}


def _check_frame(tag, t, out, flag, gbox, gconf):
    assert flag == gconf[1], (tag, t, flag, gconf[1])
    assert iou(out["target_bbox"], gbox) >= 0.999, (tag, t, out["target_bbox"], gbox.tolist())
    d = abs(out["confidence"] - gconf[0]) / gconf[0]
    assert d < 1e-2, (tag, t, out["confidence"], gconf[0])
    return d


BRANCHES = ("occlusion", "distractor", "distractor_far", "distractor_branch", "uncertain_threshold",
            "hard_sample_threshold", "low_score", "long")


@pytest.mark.parametrize("name", BRANCHES)
@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_dimp_branches_match_reference(nets, precision, name):
    from mmtrack_amd import _lib, synth
    from mmtrack_amd.dimp_tracker import DiMP, parameters
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    assert name in list(gd["names"])
    seed, H, W, C, tseed = [int(v) for v in gd["meta"]]
    p = f"{name}/"
    flags, boxes, conf, ms2 = gd[p + "flags"], gd[p + "boxes"], gd[p + "confidence"], gd[p + "max_score2"]
    n = len(flags)
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(gd["init_box"]), **json.loads(str(gd[p + "events"])))
    params = parameters()
    for k, v in json.loads(str(gd[p + "params"])).items():
        setattr(params, k, v)
    tr = DiMP(params, net=nets[precision])
    torch.manual_seed(tseed)
    tr.initialize(frames[0], {"init_bbox": list(gd["init_box"])})
    hn_frame = int(gd[p + "hn_frame"]) if p + "hn_frame" in gd.files else -1
    dconf = []
    for t in range(1, n):
        out = tr.track(frames[t])
        dconf.append(_check_frame(name, t, out, tr.debug_info["flag"], boxes[t], (conf[t], str(flags[t]))))
        if t == hn_frame:
            close(tr.target_filter.cpu(), gd[p + "hn_filter"], 1e-2)
    close(tr.target_filter.cpu(), gd[p + "final_filter"], 1e-2)
    # the memory bookkeeping (update_memory / update_sample_weights, dimp.py:432-487) in the device state
    raw = tr.pool.states[tr.slot * tr.pool.sbytes:(tr.slot + 1) * tr.pool.sbytes].cpu().numpy().tobytes()
    st = _lib.MmtDimpState.from_buffer_copy(raw)
    np.testing.assert_allclose(np.array(st.sample_weights), gd[p + "sample_weights"], rtol=1e-5, atol=1e-7)
    assert st.num_stored == int(gd[p + "num_stored"]) and st.prev_replace == int(gd[p + "prev_replace"])
    np.testing.assert_allclose(np.array([list(b) for b in st.target_boxes]), gd[p + "target_boxes"], rtol=0, atol=0.05)
    # how close the reference's decisions were: the smallest relative margin of a threshold test it made
    ratio = ms2 / conf
    print(f"{name} [{precision}]: flags {dict(zip(*np.unique(flags[1:], return_counts=True)))}, "
          f"max confidence rel. diff {max(dconf):.2e}, smallest second-peak ratio margin to 0.8 / 0.5: "
          f"{np.nanmin(np.abs(ratio[1:] - 0.8)):.3f} / {np.nanmin(np.abs(ratio[1:] - 0.5)):.3f}")


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_dimp_pool32_bench_launch_matches_reference(nets, precision):
    """The benchmarked launch (bench.py dimp_main: one DimpPool of 32 slots, PipelinedBatch over the whole batch,
    so every conv is the 32-image grouped split-K launch) with the reference golden sequence
    (tracker_dimp.npz) in slots 0, 15, 16 and 31 and other synthetic sequences elsewhere: every golden slot gives
    the reference's flags, boxes and confidences."""
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, PipelinedBatch, parameters
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp.npz"))
    seed, n, H, W, C, tseed = [int(v) for v in gd["meta"]]
    gframes, _ = synth.make_frames(seed, n, H, W, C, box=tuple(gd["init_box"]))
    gframes = torch.from_numpy(gframes).cuda()
    net = nets[precision]
    B, golden = 32, (0, 15, 16, 31)
    pool = DimpPool(net, B, parameters())
    trackers, videos = [], []
    for i in range(B):
        tr = DiMP(parameters(), net=net, pool=pool)
        if i in golden:
            video, box = gframes, list(gd["init_box"])
            torch.manual_seed(tseed)
        else:
            box = [60.0 + (37 * i) % 320, 40.0 + (23 * i) % 240, 40.0 + (i % 5) * 6, 32.0 + (i % 3) * 8]
            video = torch.from_numpy(synth.make_frames(300 + i, n, H, W, C, box=tuple(box))[0]).cuda()
            torch.manual_seed(1000 + i)
        tr.initialize(video[0], {"init_bbox": box})
        trackers.append(tr)
        videos.append(video)
    pipe = PipelinedBatch(trackers)
    got = {i: [] for i in golden}

    def take(outs):
        for i in golden:
            got[i].append((outs[i], trackers[i].debug_info["flag"]))
    for t in range(1, n):
        outs = pipe.step([videos[i][t] for i in range(B)])
        if outs is not None:
            take(outs)
    take(pipe.flush())
    for i in golden:
        assert len(got[i]) == n - 1
        for t, (out, flag) in enumerate(got[i], start=1):
            _check_frame(f"slot {i}", t, out, flag, gd["boxes"][t], (gd["confidence"][t], str(gd["flags"][t])))


def test_pool_launch_does_not_block_the_host(nets):
    """DimpPool.launch queues a frame without waiting for the device (the frame descriptors and host
    frames go through pinned buffers with asynchronous copies): with a long GPU job queued ahead on the stream,
    launch() returns while that job is still running, for device frames and for numpy host frames alike."""
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, parameters
    net = nets["f16x3"]
    pool = DimpPool(net, 2, parameters())
    frames, gts = synth.make_frames(91, 4, 360, 480, 6, box=(200.0, 140.0, 48.0, 40.0))
    trs = [DiMP(parameters(), net=net, pool=pool) for _ in range(2)]
    for tr in trs:
        tr.initialize(frames[0], {"init_bbox": list(gts[0])})
    dev = torch.from_numpy(frames).cuda()
    a = torch.randn(8192, 8192, device="cuda")
    for k, fr in enumerate(([dev[1], dev[1]], [frames[2], frames[2]], [frames[3], dev[3]])):
        torch.cuda.synchronize()
        for _ in range(40):   # ~0.3 s of matrix work queued ahead of the launch
            a = torch.tanh(a @ a * 1e-4)
        busy = torch.cuda.Event()
        busy.record()
        ticket = pool.launch(trs, fr, 0)
        assert not busy.query(), f"launch {k} waited for the queued GPU work"
        outs = pool.finish(trs, 0, ticket)
        assert all(np.isfinite(o["target_bbox"]).all() for o in outs)
