"""Generate tests/golden/dimpnet_det.npz and tracker_dimp.npz by running the REFERENCE DeT DiMP-50
(RGBD/models/DeT: ltr/models/tracking/dimpnet.py dimp50_DeT, pytracking/tracker/dimp/dimp.py DiMP) on
seeded synthetic weights (mmtrack_amd.synth.make_dimp_state_dict) and frames, on the CPU.

Build container only (needs /root/reference).  No bytecode is written into the reference tree
(sys.dont_write_bytecode).  Stand-ins beyond make_golden.install_shims():
* ``torch._six`` (removed from torch 2.x; ``string_classes`` / ``int_classes`` only);
* third-party packages the reference imports but never calls on this path (pycocotools, lvis,
  torchvision.models.resnet model_urls / BasicBlock -- clf_feat_blocks = 0, backbone_pretrained = False):
  empty modules;
* ``PrRoIPool2D`` (a CUDA extension, ltr/external/PreciseRoIPooling): oracle/dimpnet.py's restatement of
  its forward kernel -- the initial filter is pinned only to that restatement;
* ``cv2.warpAffine`` (Rotate init augmentation): oracle/dimpnet.py's restatement of OpenCV -- unpinned.
The tracker runs with use_iou_net = False (IoU-Net refinement is not on the MI355X path) and
torch.manual_seed(SEED) right before initialize, so the init shifts / dropout masks are reproducible.

tracker_dimp_branches.npz drives the same reference tracker through every decision branch of
localize_advanced / update_classifier (dimp.py:94-176, 239-302, 432-487, 607-650) on sequences with a full
occlusion, a pasted distractor near and far from the target, and DeT parameters with the optional thresholds
(uncertain_threshold, hard_sample_threshold, low_score_opt_threshold) set, plus a 52-frame sequence that
fills the 50-sample memory and replaces samples.  Per frame it records the flag, box, confidence and the
masked second maximum (max_score2, NaN where the branch returns before computing it); per sequence the filter
after the first hard-negative update and at the end, and the memory bookkeeping (sample weights, boxes,
num_stored, previous replace index).
dimp_stages.npz (``stages``, not in the default set) records every stage of the tracker_dimp.npz run (stages_fixture).
Usage:  python tests/golden/make_golden_dimp.py [net] [tracker] [branches] [stages]   (default: the first three)
"""
import importlib
import json
import math
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd"))

import make_golden as mg  # noqa: E402
from mmtrack_amd import synth  # noqa: E402
from oracle import dimpnet as odn  # noqa: E402

NET_SEEDS = (501, 502)
SEQ = dict(seed=61, n=24, H=360, W=480, C=6, box=(200.0, 140.0, 48.0, 40.0))
TRACK_SEED = 7


class _Any:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Any()


def _stub(name):
    m = types.ModuleType(name)
    m.__getattr__ = lambda n: _Any
    m.__path__ = []
    sys.modules[name] = m


def install():
    mg.install_shims()
    mg._mod("torch._six", string_classes=(str, bytes), int_classes=int)
    sys.modules["torchvision"].__version__ = "0.13.1"
    for n in ("pycocotools", "pycocotools.coco", "pycocotools.mask", "lvis", "lvis.lvis", "torchvision.models",
              "torchvision.models.resnet"):
        _stub(n)
    cv2 = sys.modules["cv2"]
    cv2.warpAffine = lambda img, M, dsize, borderMode=None, flags=None: odn.warp_affine_replicate(img, M, dsize)
    sys.path.insert(0, os.path.join(REF, "RGBD/models/DeT"))


class PrRoIPoolStandIn(torch.nn.Module):
    def __init__(self, ph, pw, scale):
        super().__init__()
        self.ph, self.pw, self.scale = ph, pw, scale

    def forward(self, feat, rois):
        return odn.prroi_pool(feat, rois, self.scale, self.ph, self.pw)


def build_net(sd):
    dn = importlib.import_module("ltr.models.tracking.dimpnet")
    net = dn.dimp50_DeT(filter_size=4, backbone_pretrained=False, optim_iter=5, clf_feat_norm=True, clf_feat_blocks=0,
                        final_conv=True, out_feature_dim=512, optim_init_step=0.9, optim_init_reg=0.1,
                        init_gauss_sigma=0.9, num_dist_bins=100, bin_displacement=0.1, mask_init_factor=3.0,
                        target_mask_act='sigmoid', score_act='relu', merge_type='max')
    missing, unexpected = net.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith(("bb_regressor.", "feature_extractor.layer4", "feature_extractor_depth.layer4",
                             "feature_extractor.fc", "feature_extractor_depth.fc")) for k in missing), missing
    net.classifier.filter_initializer.filter_pool.prroi_pool = PrRoIPoolStandIn(4, 4, 1 / 16)
    return net.eval()


def wrap(net):
    from pytracking.features.net_wrappers import NetWithBackbone
    w = NetWithBackbone(net_path=None, use_gpu=False)
    w.net = net
    return w


def net_fixture(net, wnet):
    res = {"seeds": np.array(NET_SEEDS)}
    ims = torch.stack([torch.from_numpy(synth.make_patch(s, 288, 6)).float().permute(2, 0, 1) for s in NET_SEEDS])
    with torch.no_grad():
        feats = wnet.extract_backbone(ims.clone())
        l3 = feats["layer3"]
        clf = net.extract_classification_feat(feats)
        boxes = torch.tensor([[120.0, 110.0, 50.0, 64.0], [90.5, 140.25, 80.0, 36.0]])
        filt = net.classifier.filter_initializer(clf, boxes)
        scores = net.classifier.classify(filt, clf)
    res["layer3_sum"] = l3.double().sum(dim=(1, 2, 3)).numpy()
    res["layer3_ch"] = l3[:, ::32].numpy()               # every 32nd channel, full maps
    res["clf_ch"] = clf[:, ::8].numpy()                  # every 8th channel
    res["clf_sum"] = clf.double().sum(dim=(1, 2, 3)).numpy()
    res["boxes"] = boxes.numpy()
    res["init_filter"] = filt.numpy()
    res["scores"] = scores.numpy()
    np.savez_compressed(os.path.join(HERE, "dimpnet_det.npz"), **res)
    print("wrote dimpnet_det: layer3 sums", res["layer3_sum"], "score max", float(scores.max()))


def tracker_fixture(wnet):
    from pytracking.parameter.dimp import DeT_DiMP50_Max as P
    from pytracking.tracker.dimp.dimp import DiMP
    params = P.parameters()   # its NetWithBackbone(net_path=...) loads nothing until initialize(); replaced below
    params.use_gpu = False
    params.device = "cpu"
    params.use_iou_net = False
    params.net = wnet
    tr = DiMP(params)
    tr.features_initialized = True
    frames, gts = synth.make_frames(SEQ["seed"], SEQ["n"], SEQ["H"], SEQ["W"], SEQ["C"], box=SEQ["box"])
    torch.manual_seed(TRACK_SEED)
    tr.initialize(frames[0], {"init_bbox": list(SEQ["box"])})
    init_filter = tr.target_filter.clone()
    boxes, conf, flags = [list(SEQ["box"])], [1.0], ["init"]
    for t in range(1, SEQ["n"]):
        o = tr.track(frames[t])
        boxes.append([float(v) for v in o["target_bbox"]])
        conf.append(float(o["confidence"]))
        flags.append(tr.debug_info["flag"])
    meta = np.array([SEQ["seed"], SEQ["n"], SEQ["H"], SEQ["W"], SEQ["C"], TRACK_SEED])
    np.savez_compressed(os.path.join(HERE, "tracker_dimp.npz"), boxes=np.array(boxes), confidence=np.array(conf),
                        flags=np.array(flags), init_box=np.array(SEQ["box"]), meta=meta,
                        init_filter=init_filter.numpy())
    print("wrote tracker_dimp", np.round(np.array(boxes), 2).tolist(), flags, np.round(conf, 4).tolist())


# name -> (frame events for synth.make_frames, DeT parameter overrides, number of frames); frames, seed and box
# otherwise those of SEQ.  Distractors are blended at alpha < 1: an identical copy of the target ties with it on
# the score map, and an argmax decided by fp32 summation order pins nothing.
BRANCH_SEQS = {
    "occlusion": (dict(occlude=(8, 14)), {}, 24),                              # not_found x 6, recovery
    "distractor": (dict(distractor=(10, 30, -60, 20)), {}, 24),               # uncertain, hard_negative (2nd peak)
    "distractor_far": (dict(distractor=(10, 30, -85, -50)), {}, 27),          # hard_negative by displacement
    "distractor_branch": (dict(distractor=(10, 30, -60, 20)), {"distractor_threshold": 0.5}, 24),  # uncertain
    "distractor_97": (dict(distractor=(10, 30, -60, 20, 0.97)), {}, 24),       # hard_negative (2nd peak)
    "distractor_above": (dict(distractor=(10, 30, 0, -55)), {}, 24),          # hard_negative, uncertain
    "uncertain_threshold": ({}, {"uncertain_threshold": 0.33}, 24),
    "hard_sample_threshold": ({}, {"hard_sample_threshold": 0.34}, 24),
    "low_score": ({}, {"low_score_opt_threshold": 0.36, "net_opt_low_iter": 1}, 24),
    "long": ({}, {}, 52),                                                     # memory full at ~36, replacements
}


def _margin(ms1, ms2, disp, params):
    """Smallest relative distance of one of localize_advanced's threshold tests (dimp.py:260-301) from flipping
    on this frame, counting only the tests that decide the outcome: ms1 against the not-found / uncertain /
    hard-sample thresholds, then the distractor ratio, then (no distractor) the hard-negative pair, or (distractor)
    the two displacement tests against their threshold."""
    g = params.get
    m = [abs(ms1 - g("target_not_found_threshold")) / g("target_not_found_threshold")]
    for k in ("uncertain_threshold", "hard_sample_threshold"):
        if g(k, None) is not None:
            m.append(abs(ms1 - g(k)) / g(k))
    if ms2 is None or ms1 < max(g("target_not_found_threshold"), g("uncertain_threshold", -1), g("hard_sample_threshold", -1)):
        return min(m)
    r = ms2 / ms1
    m.append(abs(r - g("distractor_threshold")) / g("distractor_threshold"))
    if r > g("distractor_threshold"):
        n1, n2, thr = disp
        m.extend([abs(n1 - thr) / thr, abs(n2 - thr) / thr])
    else:
        a = (r - g("hard_negative_threshold")) / g("hard_negative_threshold")
        b = (ms2 - g("target_not_found_threshold")) / g("target_not_found_threshold")
        m.append(min(abs(a), abs(b)) if (a > 0 and b > 0) else (max(abs(a), abs(b)) if (a <= 0 and b <= 0)
                                                                else abs(a if a <= 0 else b)))
    return min(m)


def _runner_up(s):
    """The score map's best value outside the 3 x 3 cells around its maximum, relative to the maximum: how near
    the argmax is to jumping to another peak."""
    s = s.reshape(s.shape[-2], s.shape[-1]).clone()
    r, c = divmod(int(s.argmax()), s.shape[1])
    m1 = float(s[r, c])
    s[max(r - 1, 0):r + 2, max(c - 1, 0):c + 2] = -1
    return float(s.max()) / m1


def branch_fixture(wnet, seqs=None, path=None):
    """Per sequence: the end-to-end record (flags, boxes, confidences, filters, memory) and, per frame, the
    decision record -- the tracker state before track() (position, size, scale, frame number, sample memory
    bookkeeping), the sample coordinates and the raw score map it localised on, and the state after it, with
    the Gauss-Newton iteration count update_classifier chose -- so the device state machine can be run on the
    reference's own score maps, independent of the network's arithmetic."""
    from pytracking.parameter.dimp import DeT_DiMP50_Max as P
    from pytracking.tracker.dimp import dimp as dm
    seen = []
    max2d = dm.dcf.max2d

    def rec_max2d(x):   # localize_advanced's two maxima (scores, then the masked scores)
        r = max2d(x)
        seen.append(float(r[0].max()))
        return r
    dm.dcf.max2d = rec_max2d
    seqs = BRANCH_SEQS if seqs is None else seqs
    out = {"names": np.array(list(seqs))}
    try:
        for name, (events, over, n) in seqs.items():
            params = P.parameters()
            params.use_gpu, params.device, params.use_iou_net, params.net = False, "cpu", False, wnet
            for k, v in over.items():
                setattr(params, k, v)
            tr = dm.DiMP(params)
            tr.features_initialized = True
            cap = {}
            ebf, ct = tr.extract_backbone_features, tr.classify_target

            def extract(*a, **k):
                r = ebf(*a, **k)
                cap["coords"] = r[1][0].float().clone()
                return r

            def classify(x):
                r = ct(x)
                cap["scores"] = r[0, 0].clone()
                return r
            tr.extract_backbone_features, tr.classify_target = extract, classify
            opt = wnet.net.classifier.filter_optimizer
            opt_fwd = opt.forward

            def opt_forward(*a, **k):
                cap["num_iter"] = k.get("num_iter")
                return opt_fwd(*a, **k)
            frames, _ = synth.make_frames(SEQ["seed"], n, SEQ["H"], SEQ["W"], SEQ["C"], box=SEQ["box"], **events)
            torch.manual_seed(TRACK_SEED)
            tr.initialize(frames[0], {"init_bbox": list(SEQ["box"])})
            opt.forward = opt_forward
            boxes, conf, ms2, flags, margin, runner = [list(SEQ["box"])], [1.0], [np.nan], ["init"], [np.nan], [np.nan]
            dec = {k: [] for k in ("pre_pos", "pre_sz", "pre_scale", "pre_frame", "pre_nstored", "pre_prev", "pre_sw",
                                   "pre_tb", "coords", "scores", "post_pos", "post_sz", "post_scale", "post_sw",
                                   "post_tb", "post_nstored", "post_prev", "num_iter")}

            def snap(pre):
                p = "pre_" if pre else "post_"
                dec[p + "pos"].append(tr.pos.numpy().copy())
                dec[p + "sz"].append(tr.target_sz.numpy().copy())
                dec[p + "scale"].append(float(tr.target_scale))
                dec[p + "sw"].append(tr.sample_weights[0].numpy().copy())
                dec[p + "tb"].append(tr.target_boxes.numpy().copy())
                dec[p + "nstored"].append(int(tr.num_stored_samples[0]))
                prev = tr.previous_replace_ind[0]
                dec[p + "prev"].append(-1 if prev is None else int(prev))
            hn_filter = None
            for t in range(1, n):
                seen.clear()
                cap.clear()
                snap(True)
                dec["pre_frame"].append(tr.frame_num)
                pos_before = tr.pos.clone()
                o = tr.track(frames[t])
                snap(False)
                dec["coords"].append(cap["coords"].numpy())
                dec["scores"].append(cap["scores"].numpy())
                dec["num_iter"].append(int(cap.get("num_iter") or 0))
                boxes.append([float(v) for v in o["target_bbox"]])
                conf.append(float(o["confidence"]))
                flags.append(tr.debug_info["flag"])
                ms2.append(seen[1] if len(seen) > 1 else np.nan)
                # the displacement test's operands (dimp.py:280-292), for the margin
                sc = cap["coords"]
                spos = 0.5 * (sc[:2] + sc[2:] - 1)
                sscale = ((sc[2:] - sc[:2]) / tr.img_sample_sz).prod().sqrt()
                sz = torch.Tensor(list(cap["scores"].shape))
                osz = sz - (tr.kernel_size + 1) % 2
                ctr = (sz - 1) / 2
                s = cap["scores"]
                d1 = torch.Tensor(divmod(int(s.argmax()), s.shape[1])) - ctr
                prev_vec = (pos_before - spos) / ((tr.img_support_sz / osz) * sscale)
                n1 = float(torch.sqrt(((d1 - prev_vec) ** 2).sum()))
                thr = params.dispalcement_scale * math.sqrt(sz[0] * sz[1]) / 2
                n2 = np.nan
                if len(seen) > 1:
                    # the masked second peak's position: recompute as localize_advanced does
                    tns = params.target_neighborhood_scale * (tr.target_sz / sscale) * (osz / tr.img_support_sz)
                    md = d1 + ctr
                    t0 = max(round(md[0].item() - tns[0].item() / 2), 0)
                    t1 = min(round(md[0].item() + tns[0].item() / 2 + 1), int(sz[0]))
                    l0 = max(round(md[1].item() - tns[1].item() / 2), 0)
                    l1 = min(round(md[1].item() + tns[1].item() / 2 + 1), int(sz[1]))
                    sm = s.clone()
                    sm[t0:t1, l0:l1] = 0
                    d2 = torch.Tensor(divmod(int(sm.argmax()), sm.shape[1])) - ctr
                    n2 = float(torch.sqrt(((d2 - prev_vec) ** 2).sum()))
                margin.append(_margin(seen[0], seen[1] if len(seen) > 1 else None, (n1, n2, thr), params))
                runner.append(_runner_up(s))
                if flags[-1] == "hard_negative" and hn_filter is None:
                    hn_filter = (t, tr.target_filter.clone())
            opt.forward = opt_fwd
            p = f"{name}/"
            out[p + "boxes"], out[p + "confidence"], out[p + "flags"] = np.array(boxes), np.array(conf), np.array(flags)
            out[p + "max_score2"], out[p + "margin"], out[p + "runner_up"] = np.array(ms2), np.array(margin), np.array(runner)
            out[p + "events"] = np.array(json.dumps(events))
            out[p + "params"] = np.array(json.dumps(over))
            out[p + "final_filter"] = tr.target_filter.numpy()
            if hn_filter is not None:
                out[p + "hn_frame"], out[p + "hn_filter"] = np.array(hn_filter[0]), hn_filter[1].numpy()
            out[p + "sample_weights"] = tr.sample_weights[0].numpy()
            out[p + "target_boxes"] = tr.target_boxes.numpy()
            out[p + "num_stored"] = np.array(int(tr.num_stored_samples[0]))
            prev = tr.previous_replace_ind[0]
            out[p + "prev_replace"] = np.array(-1 if prev is None else int(prev))
            for k, v in dec.items():
                out[p + "dec_" + k] = np.array(v)
            out[p + "const"] = np.array([*tr.base_target_sz.tolist(), *tr.image_sz.tolist(), float(tr.min_scale_factor),
                                         float(tr.max_scale_factor), int(tr.num_init_samples[0])], dtype=np.float64)
            counts = {f: flags.count(f) for f in ("normal", "not_found", "uncertain", "hard_negative")}
            print(f"{name}: {counts} num_stored {int(tr.num_stored_samples[0])} prev_replace {prev} "
                  f"min decision margin {np.nanmin(margin):.4f} max runner-up {np.nanmax(runner):.3f}")
    finally:
        dm.dcf.max2d = max2d
    meta = np.array([SEQ["seed"], SEQ["H"], SEQ["W"], SEQ["C"], TRACK_SEED])
    np.savez_compressed(path or os.path.join(HERE, "tracker_dimp_branches.npz"), meta=meta,
                        init_box=np.array(SEQ["box"]), **out)


def _summ(t, step):
    """A stage tensor [n, C, H, W] as (per-sample channel sums in float64, every step-th channel's full maps)."""
    t = t.detach().float()
    return t.double().sum(dim=(2, 3)).numpy(), t[:, ::step].numpy()


def stages_fixture(wnet, n_frames=6):
    """dimp_stages.npz: the tracker_dimp.npz run (same sequence, seed and parameters) with every stage of
    initialize() and of the first frames recorded, so the HIP path can be compared stage by stage (VERDICT r4
    item 3): the 15 augmented init patches (every 8th pixel of every channel) and their sums, the backbone
    layer3 and the classification features (per-channel sums + every 64th / 32nd channel), the dropout-augmented
    feature stack's sums, the initial filter and all Gauss-Newton iterates, the target boxes; per frame the
    sampled patch (every 8th pixel), its sample coordinates, the clf features' sums, the raw score map and the
    filter the frame's scores used."""
    from pytracking.parameter.dimp import DeT_DiMP50_Max as P
    from pytracking.tracker.dimp.dimp import DiMP
    net = wnet.net
    params = P.parameters()
    params.use_gpu, params.device, params.use_iou_net, params.net = False, "cpu", False, wnet
    tr = DiMP(params)
    tr.features_initialized = True
    cap = {"bb_in": [], "bb_out": [], "clf": [], "scores": []}
    eb, gcf, ct = wnet.extract_backbone, tr.get_classification_features, tr.classify_target
    ebf = tr.extract_backbone_features
    fi = net.classifier.filter_initializer
    fo = net.classifier.filter_optimizer
    fi_fwd, fo_fwd = fi.forward, fo.forward

    def extract(im):
        r = eb(im)
        cap["bb_in"].append(im.clone())
        cap["bb_out"].append(r["layer3"].clone())
        return r

    def clf_feat(f):
        r = gcf(f)
        cap["clf"].append(r.clone())
        return r

    def backbone_feat(*a, **k):
        r = ebf(*a, **k)
        cap.setdefault("coords", []).append(r[1][0].float().clone())
        return r

    def classify(x):
        cap["filter_used"] = tr.target_filter.clone()
        r = ct(x)
        cap["scores"].append((r.clone(), cap["filter_used"]))
        return r

    def init_fwd(feat, bb):
        r = fi_fwd(feat, bb)
        cap["init_in_sums"] = feat.double().sum(dim=tuple(range(2, feat.dim()))).numpy()
        cap["init_bb"] = bb.clone()
        cap["init_filter"] = r.clone()
        return r

    def opt_fwd(w, *a, **k):
        r = fo_fwd(w, *a, **k)
        if "iterates" not in cap:
            cap["iterates"] = [x.clone() for x in r[1]]
        return r
    wnet.extract_backbone = extract
    tr.get_classification_features, tr.classify_target = clf_feat, classify
    tr.extract_backbone_features = backbone_feat
    fi.forward, fo.forward = init_fwd, opt_fwd
    try:
        frames, _ = synth.make_frames(SEQ["seed"], SEQ["n"], SEQ["H"], SEQ["W"], SEQ["C"], box=SEQ["box"])
        torch.manual_seed(TRACK_SEED)
        tr.initialize(frames[0], {"init_bbox": list(SEQ["box"])})
        res = {}
        p = cap["bb_in"][0]
        res["init_patch_sums"] = p.double().sum(dim=(1, 2, 3)).numpy()
        res["init_patch_sub"] = p[:, :, ::8, ::8].numpy()
        res["init_l3_sums"], res["init_l3_ch"] = _summ(cap["bb_out"][0], 64)
        res["init_clf_sums"], res["init_clf_ch"] = _summ(cap["clf"][0], 32)
        res["init_stack_sums"] = cap["init_in_sums"]
        res["init_target_boxes"] = cap["init_bb"].reshape(-1, 4).numpy()
        res["init_filter"] = cap["init_filter"].numpy()
        res["iterates"] = torch.stack(cap["iterates"]).numpy()
        conf = []
        for t in range(1, n_frames + 1):
            o = tr.track(frames[t])
            conf.append(float(o["confidence"]))
            k = t   # capture index: bb_in[0] / clf[0] are the init ones
            pf = cap["bb_in"][k]
            res[f"f{t}_patch_sums"] = pf.double().sum(dim=(1, 2, 3)).numpy()
            res[f"f{t}_patch_sub"] = pf[:, :, ::8, ::8].numpy()
            res[f"f{t}_l3_sums"] = cap["bb_out"][k].double().sum(dim=(2, 3)).numpy()
            res[f"f{t}_clf_sums"] = cap["clf"][k].double().sum(dim=(2, 3)).numpy()
            sc, fu = cap["scores"][t - 1]
            res[f"f{t}_scores"] = sc.numpy()
            res[f"f{t}_filter"] = fu.numpy()
            # the sample the frame localised in and the state after it (dimp.py:107-131)
            res[f"f{t}_coords"] = cap["coords"][t - 1].numpy()
            res[f"f{t}_state"] = np.array([*tr.pos.tolist(), *tr.target_sz.tolist(), float(tr.target_scale)],
                                          dtype=np.float64)
            res[f"f{t}_flag"] = np.array(tr.debug_info["flag"])
        res["confidence"] = np.array(conf)
        gold = np.load(os.path.join(HERE, "tracker_dimp.npz"))
        assert np.array_equal(res["confidence"], gold["confidence"][1:n_frames + 1]), "stage run != tracker golden"
        np.savez_compressed(os.path.join(HERE, "dimp_stages.npz"), **res)
        print("wrote dimp_stages:", {k: v.shape for k, v in res.items() if k.startswith("init")}, conf)
    finally:
        wnet.extract_backbone = eb
        fi.forward, fo.forward = fi_fwd, fo_fwd


def main():
    what = set(sys.argv[1:]) or {"net", "tracker", "branches"}
    install()
    torch.set_num_threads(8)
    sd = synth.make_dimp_state_dict(0)
    net = build_net(sd)
    wnet = wrap(net)
    if "net" in what:
        net_fixture(net, wnet)
    if "tracker" in what:
        tracker_fixture(wnet)
    if "branches" in what:
        branch_fixture(wnet)
    if "stages" in what:
        stages_fixture(wnet)


if __name__ == "__main__":
    main()
