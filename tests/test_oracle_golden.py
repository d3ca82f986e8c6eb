"""The CPU oracle against the reference's own outputs (tests/golden/, made by make_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from mmtrack_amd import synth
from oracle import crop as ocrop
from oracle import tracker as otracker
from oracle import vipt as ov

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

NETS = {
    "deep_rgbt": dict(shape=dict(kind="vipt", prompt_type="vipt_deep"), cfg=ov.NetCfg(), C=6),
    "deep_rgbd": dict(shape=dict(kind="vipt", prompt_type="vipt_deep"), cfg=ov.NetCfg(), C=6),
    "shaw_rgbt": dict(shape=dict(kind="vipt", prompt_type="vipt_shaw"), cfg=ov.NetCfg(prompt_type="vipt_shaw"), C=6),
    "ostrack384": dict(shape=dict(kind="ostrack", search_size=384, template_size=192),
                       cfg=ov.NetCfg(kind="ostrack", search_size=384, template_size=192), C=3),
}


@pytest.mark.parametrize("name", list(NETS))
def test_state_dict_layout_matches_reference(name):
    mani = json.load(open(os.path.join(GOLDEN, "manifest.json")))[name]
    ours = synth.model_shapes(**NETS[name]["shape"])
    assert {k: list(v) for k, v in ours.items()} == {k: v for k, v in mani}


@pytest.mark.parametrize("name", list(NETS))
def test_oracle_network_matches_reference(name):
    spec = NETS[name]
    torch.set_num_threads(min(8, os.cpu_count()))
    g = np.load(os.path.join(GOLDEN, f"net_{name}.npz"))
    sd = synth.make_state_dict(0, **spec["shape"])
    cfg = spec["cfg"]
    for j, (sz, ss) in enumerate(g["seeds"]):
        z = ocrop.preprocess(synth.make_patch(int(sz), cfg.template_size, spec["C"]))
        x = ocrop.preprocess(synth.make_patch(int(ss), cfg.search_size, spec["C"]))
        tr = {}
        out = ov.forward(sd, z, x, cfg, ov.ce_template_mask(cfg), trace=tr)
        removed = torch.cat(out["removed_indexes_s"], dim=1).numpy()
        np.testing.assert_array_equal(removed, g[f"removed_{j}"])
        for k in ("score_map", "size_map", "offset_map", "pred_boxes"):
            np.testing.assert_allclose(out[k].numpy(), g[f"{k}_{j}"], rtol=1e-4, atol=1e-5)
        if f"feat_rows_{j}" in g.files:
            np.testing.assert_allclose(out["backbone_feat"][0, ::8].numpy(), g[f"feat_rows_{j}"], rtol=1e-4,
                                       atol=1e-4)
        # the CE scores of every slot and the boundary margins the reference recorded
        np.testing.assert_allclose(np.stack([k.numpy() for k in tr["ce_keys"]]), g[f"ce_keys_{j}"], rtol=1e-4,
                                   atol=1e-8)
        np.testing.assert_allclose(tr["ce_margin"], g[f"ce_margin_{j}"], rtol=2e-2, atol=2e-6)
        resp = (ov.hann2d(cfg.feat_sz) * out["score_map"]).flatten()
        assert int(torch.argmax(resp)) == int(g[f"resp_argmax_{j}"][0])


def test_crop_geometry_matches_reference():
    g = np.load(os.path.join(GOLDEN, "crop_geometry.npz"))
    im = g["image"]
    for j, (x, y, w, h, f, o) in enumerate(g["cases"]):
        patch, rf = ocrop.sample_target(im, [x, y, w, h], f, int(o))
        np.testing.assert_array_equal(patch, g[f"patch_{j}"])
        assert rf == g[f"rf_{j}"][0]


@pytest.mark.parametrize("name", ["deep_rgbt", "deep_rgbd"])
def test_oracle_tracker_matches_reference(name):
    g = np.load(os.path.join(GOLDEN, f"tracker_{name}.npz"))
    seed, n, H, W, C = [int(v) for v in g["meta"]]
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(g["init_box"]))
    sd = synth.make_state_dict(0, kind="vipt", prompt_type="vipt_deep")
    tr = otracker.OracleTracker(sd, ov.NetCfg())
    boxes, scores = otracker.run_sequence(tr, frames, g["init_box"])
    np.testing.assert_allclose(boxes, g["boxes"], rtol=1e-4, atol=2e-2)
    np.testing.assert_allclose(scores, g["scores"], rtol=1e-3, atol=1e-5)


def test_oracle_ostrack384_tracker_matches_reference():
    """C4 at search factor 5.0: the oracle tracker (the ViPTTrack state machine, oracle/tracker.py) with the
    OSTrack-384 network against the reference build_ostrack network in the reference ViPTTrack
    (tracker_ostrack384.npz, make_golden.py ostrack_tracker_fixture)."""
    g = np.load(os.path.join(GOLDEN, "tracker_ostrack384.npz"))
    seed, n, H, W, C = [int(v) for v in g["meta"]]
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(g["init_box"]))
    sd = synth.make_state_dict(0, kind="ostrack", search_size=384, template_size=192)
    cfg = ov.NetCfg(kind="ostrack", search_size=384, template_size=192)
    tr = otracker.OracleTracker(sd, cfg, search_factor=float(g["search_factor"][0]))
    boxes, scores = otracker.run_sequence(tr, frames, g["init_box"])
    np.testing.assert_allclose(boxes, g["boxes"], rtol=1e-4, atol=2e-2)
    np.testing.assert_allclose(scores, g["scores"], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("name", ["deep_rgbd", "ostrack384"])
def test_oracle_tracker_steps_match_reference(name):
    """The oracle tracker on the teacher-forced one-step goldens (make_golden.py --steps: the reference's state
    set to the ground-truth box of frame t - 1 before frame t), every third frame to keep the CPU suite short."""
    g = np.load(os.path.join(GOLDEN, f"tracker_steps_{name}.npz"))
    seed, n, H, W, C = [int(v) for v in g["meta"]]
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(g["init_box"]))
    if name == "ostrack384":
        sd = synth.make_state_dict(0, kind="ostrack", search_size=384, template_size=192)
        tr = otracker.OracleTracker(sd, ov.NetCfg(kind="ostrack", search_size=384, template_size=192),
                                    search_factor=float(g["search_factor"][0]))
    else:
        tr = otracker.OracleTracker(synth.make_state_dict(0, kind="vipt", prompt_type="vipt_deep"), ov.NetCfg())
    tr.initialize(frames[0], {"init_bbox": list(g["init_box"])})
    for t in range(1, n, 3):
        tr.state = [float(v) for v in g["states"][t]]
        o = tr.track(frames[t])
        np.testing.assert_allclose(o["target_bbox"], g["boxes"][t], rtol=1e-4, atol=2e-2)
        np.testing.assert_allclose(o["best_score"], g["scores"][t], rtol=1e-3, atol=1e-5)


def test_dimp_branch_golden_covers_every_flag():
    """tracker_dimp_branches.npz (make_golden_dimp.py branch_fixture) reaches every localize_advanced outcome,
    a hard-negative filter update, and a full sample memory with replacements; its frames are the plain
    sequence's wherever no event is active (synth.make_frames draws the same numbers with events)."""
    import json
    g = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    flags = set()
    for name in g["names"]:
        flags |= set(str(f) for f in g[f"{name}/flags"][1:])
    assert flags == {"normal", "not_found", "uncertain", "hard_negative"}
    assert any(f"{n}/hn_filter" in g.files for n in g["names"])
    assert int(g["long/num_stored"]) > 50 and int(g["long/prev_replace"]) >= 17
    seed, H, W, C, _ = [int(v) for v in g["meta"]]
    plain, _ = synth.make_frames(seed, 12, H, W, C, box=tuple(g["init_box"]))
    ev, _ = synth.make_frames(seed, 12, H, W, C, box=tuple(g["init_box"]),
                              **json.loads(str(g["occlusion/events"])))
    np.testing.assert_array_equal(ev[:8], plain[:8])
    assert not np.array_equal(ev[8], plain[8])


def test_oracle_dimp_decisions_match_reference():
    """oracle/dimp_decide.py (localize_advanced, update_state, update_memory / update_sample_weights and the
    Gauss-Newton iteration choice of DeT's DiMP tracker) on the decision records of tracker_dimp_branches.npz:
    from the reference's state before every frame and its score map, the reference's flag, iteration count,
    replaced slot, sample count and -- bit for bit -- its position, size, scale, sample weights and boxes after it
    (the same float32 tensor arithmetic), over every branch sequence (261 frames)."""
    import json
    from types import SimpleNamespace

    import torch

    from oracle import dimp_decide as odd
    g = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    base = dict(target_not_found_threshold=0.25, distractor_threshold=0.8, hard_negative_threshold=0.5,
                target_neighborhood_scale=2.2, dispalcement_scale=0.8, hard_negative_learning_rate=0.02,
                learning_rate=0.01, init_samples_minimum_weight=0.25, train_skipping=20, update_classifier=True,
                net_opt_update_iter=2, net_opt_hn_iter=1)
    n_dec = 0
    for name in g["names"]:
        p = f"{name}/"
        prm = SimpleNamespace(**{**base, **json.loads(str(g[p + "params"]))})
        bt0, bt1, ih, iw, smin, smax, ninit = g[p + "const"]
        flags = g[p + "flags"]
        T = lambda a: torch.from_numpy(np.array(a, dtype=np.float32))
        for i in range(len(flags) - 1):
            prev = int(g[p + "dec_pre_prev"][i])
            st = dict(pos=T(g[p + "dec_pre_pos"][i]), target_sz=T(g[p + "dec_pre_sz"][i]), base_target_sz=T([bt0, bt1]),
                      image_sz=T([ih, iw]), target_scale=T(g[p + "dec_pre_scale"][i]), min_scale_factor=T(smin),
                      max_scale_factor=T(smax), frame_num=int(g[p + "dec_pre_frame"][i]), num_init=int(ninit),
                      num_stored=int(g[p + "dec_pre_nstored"][i]), prev_replace=None if prev < 0 else prev,
                      sample_weights=T(g[p + "dec_pre_sw"][i]), target_boxes=T(g[p + "dec_pre_tb"][i]))
            flag, num_iter, r_ind, box = odd.decide(st, T(g[p + "dec_scores"][i]), T(g[p + "dec_coords"][i]), prm)
            t = i + 1
            assert flag == str(flags[t]), (name, t, flag, flags[t])
            assert num_iter == int(g[p + "dec_num_iter"][i]), (name, t)
            assert st["num_stored"] == int(g[p + "dec_post_nstored"][i])
            assert (-1 if st["prev_replace"] is None else st["prev_replace"]) == int(g[p + "dec_post_prev"][i])
            for key, gk in (("pos", "dec_post_pos"), ("target_sz", "dec_post_sz"), ("sample_weights", "dec_post_sw"),
                            ("target_boxes", "dec_post_tb")):
                np.testing.assert_array_equal(st[key].numpy(), g[p + gk][i], err_msg=f"{name} {t} {key}")
            assert float(st["target_scale"]) == float(g[p + "dec_post_scale"][i])
            np.testing.assert_allclose(box.numpy(), g[p + "boxes"][t], rtol=0, atol=1e-4)
            n_dec += 1
    assert n_dec == 261


def test_cv2_resize_restatement_properties():
    """Unpinned piece: self-consistency of the INTER_LINEAR restatement."""
    rng = np.random.Generator(np.random.PCG64(3))
    im = rng.integers(0, 256, size=(70, 70, 6), dtype=np.uint8)
    same = ocrop.cv2_resize_linear_u8(im, 70, 70)          # identity scale reproduces the input
    np.testing.assert_array_equal(same, im)
    const = np.full((37, 53, 3), 117, np.uint8)
    np.testing.assert_array_equal(ocrop.cv2_resize_linear_u8(const, 256, 256), 117)
    half = ocrop.cv2_resize_linear_u8(im[:64, :64], 32, 32)  # exact 2x -> area average
    ref = (im[:64:2, :64:2].astype(int) + im[1:64:2, :64:2] + im[:64:2, 1:64:2] + im[1:64:2, 1:64:2] + 2) >> 2
    np.testing.assert_array_equal(half, ref)


def test_gelu_erfc_form_accuracy():
    """The kernels' GELU (common.h gelu_erf: NR erfcc form, log2-scaled, fp32) vs exact erf GELU (timm Mlp act)."""
    import math
    x = np.concatenate([np.linspace(-12, 12, 20001), np.random.default_rng(0).normal(0, 3, 20000)]).astype(np.float32)
    f = np.float32
    u = np.abs(x) * f(0.70710678118654752440)
    t = f(1) / (f(0.5) * u + f(1))
    q = f(0.246517298)
    for c in (-1.18611495, 2.14747446, -1.63775315, 0.402321582, -0.26875686, 0.139630057, 0.539700616,
              1.4427292, -2.82574822):
        q = q * t + f(c)
    h = t * np.exp2(f(-1.44269504) * u * u + q).astype(np.float32)
    xh = x * h
    y = np.where(x >= 0, x - xh, xh)
    ref = np.array([0.5 * v * (1 + math.erf(v / math.sqrt(2))) for v in x.astype(np.float64)])
    err = np.abs(y - ref)
    assert (err <= 2e-7 * np.maximum(1.0, np.abs(x))).all()       # absolute, everywhere
    big = np.abs(ref) > 1e-4
    assert (err[big] / np.abs(ref[big])).max() < 5e-6            # relative, where it matters


def test_gelu_bf16out_accuracy():
    """common.h gelu_erf_bf16out (A&S 7.1.26 erfc, used by the bf16 GEMM epilogue) vs exact erf GELU:
    abs error < 5e-7 * max(1, |x|), and after bf16 rounding < 0.5 % of activation-like outputs move
    (by one ulp)."""
    import math
    f = np.float32
    x = np.concatenate([np.linspace(-12, 12, 20001), np.random.default_rng(1).normal(0, 1.5, 50000)]).astype(np.float32)
    a = np.abs(x)
    t = f(1) / (f(0.2316418917) * a + f(1))
    p = f(0.5307027145)
    for c in (-0.7265760135, 0.7107068705, -0.142248368, 0.127414796):
        p = p * t + f(c)
    e = np.exp2((x * f(-0.7213475204)) * x).astype(np.float32)
    y = (np.maximum(x, f(0)).astype(np.float64) - a.astype(np.float64) * ((p * t) * e)).astype(np.float32)  # fma
    ref = np.array([0.5 * v * (1 + math.erf(v / math.sqrt(2))) for v in x.astype(np.float64)])
    assert (np.abs(y - ref) <= 5e-7 * np.maximum(1.0, np.abs(x))).all()

    def bf16(v):
        b = v.astype(np.float32).view(np.uint32).astype(np.uint64)
        return ((((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16).astype(np.uint32)).view(np.float32)
    act = slice(20001, None)   # the N(0, 1.5) samples: activation-like inputs
    assert (bf16(y[act]) != bf16(ref[act].astype(np.float32))).mean() < 5e-3


def test_oracle_dimp_matches_reference():
    """DiMP filter / transposed filter / steepest-descent GN iterates vs the DeT reference (golden)."""
    from oracle import dimp as od
    g = np.load(os.path.join(GOLDEN, "dimp.npz"))
    feat, filt, bb = (torch.from_numpy(g[k]) for k in ("feat", "filt", "bb"))
    np.testing.assert_allclose(od.apply_filter(feat, filt).numpy(), g["scores"], rtol=1e-5, atol=1e-5)
    ft = od.apply_feat_transpose(feat, torch.from_numpy(g["resid"]), (4, 4)).numpy()
    np.testing.assert_allclose(ft, g["feat_t"], rtol=1e-4, atol=1e-3)
    sd = {k[4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("opt.")}
    w, iters, losses = od.steepest_descent_gn(filt, feat, bb, sd, num_iter=5)
    np.testing.assert_allclose(torch.stack(iters).numpy(), g["iterates"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(torch.stack(losses).numpy().ravel(), g["losses"], rtol=1e-4)


def test_cubic_resize_oracle_properties():
    """cv2 INTER_CUBIC restatement (oracle/siamfc.py): constants stay constant (the A = -0.75 kernel is a
    partition of unity) and the float32 result
    matches an independent float64 evaluation of the same separable kernel."""
    from oracle import siamfc as osf
    c = np.full((17, 17), 3.25, np.float32)
    np.testing.assert_allclose(osf.cv2_resize_cubic_f32(c, 272), 3.25, rtol=1e-6)
    rng = np.random.default_rng(0)
    src = rng.standard_normal((17, 17)).astype(np.float32)

    def kern(t):
        a = -0.75
        t = abs(t)
        return ((a + 2) * t - (a + 3)) * t * t + 1 if t <= 1 else (((t - 5) * t + 8) * t - 4) * a if t < 2 else 0.0

    ref = np.zeros((272, 272))
    for oy in range(0, 272, 7):
        fy = (oy + 0.5) / 16 - 0.5
        sy = int(np.floor(fy))
        for ox in range(0, 272, 5):
            fx = (ox + 0.5) / 16 - 0.5
            sx = int(np.floor(fx))
            v = 0.0
            for i in range(4):
                for j in range(4):
                    yy, xx = min(max(sy + i - 1, 0), 16), min(max(sx + j - 1, 0), 16)
                    v += src[yy, xx] * kern(fy - (sy + i - 1)) * kern(fx - (sx + j - 1))
            ref[oy, ox] = v
    got = osf.cv2_resize_cubic_f32(src, 272)
    np.testing.assert_allclose(got[::7, ::5], ref[::7, ::5], atol=2e-5)


def test_frames_oracle_properties():
    """oracle/frames.py: NORM_MINMAX spans 0..255, the clip replaces values above 3x the median,
    the JET table runs blue -> red, and the merged frame keeps the RGB half untouched."""
    from oracle import frames as ofr
    rng = np.random.default_rng(0)
    dp = rng.integers(100, 1000, (40, 50)).astype(np.uint16)
    d8 = ofr.normalize_minmax_u8(dp)
    assert d8.min() == 0 and d8.max() == 255
    lut = ofr.jet_bgr()
    assert tuple(lut[0]) == (128, 0, 0) and tuple(lut[255]) == (0, 0, 128)   # dark blue .. dark red (BGR)
    far = dp.copy()
    far[:5] = 60000
    rgb = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    fr = ofr.rgbd_frame(rgb, far, depth_clip=True)
    np.testing.assert_array_equal(fr[..., :3], rgb)
    # after the clip the far rows share the top code with the 3x-median clip value
    assert (fr[:5, :, 3:] == lut[255]).all()


def test_dimpnet_oracle_matches_reference_golden():
    """oracle/dimpnet.py (backbones + max merge, clf features, FilterInitializerLinear) == the reference
    DiMPnet_DeT on the seeded weights (tests/golden/dimpnet_det.npz, make_golden_dimp.py)."""
    import torch

    from mmtrack_amd import synth
    from oracle import dimpnet as odn
    gd = np.load(os.path.join(GOLDEN, "dimpnet_det.npz"))
    sd = synth.make_dimp_state_dict(0)
    ims = torch.stack([torch.from_numpy(synth.make_patch(int(s), 288, 6)).float().permute(2, 0, 1)
                       for s in gd["seeds"]])
    with torch.no_grad():
        l3 = odn.backbone(odn.preprocess(ims), sd)
        clf = odn.clf_features(l3, sd)
        filt = odn.init_filter(clf, torch.from_numpy(gd["boxes"]), sd)
    np.testing.assert_allclose(l3.double().sum(dim=(1, 2, 3)).numpy(), gd["layer3_sum"], rtol=1e-5)
    np.testing.assert_allclose(l3[:, ::32].numpy(), gd["layer3_ch"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(clf[:, ::8].numpy(), gd["clf_ch"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(filt.numpy(), gd["init_filter"], rtol=1e-4, atol=1e-7)
