"""Stage-by-stage comparison of the HIP DiMP tracker with the reference DeT tracker (dimp_stages.npz,
make_golden_dimp.py stages_fixture): the tracker_dimp.npz run with every stage of initialize() and of the first
six frames recorded.  Each stage's relative error against the reference is printed in run order, so a drift that
the end-to-end confidences show is located at the stage where it appears, not only at the end."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def run_stages(precision, n_frames=6):
    """The HIP tracker on the golden sequence with its stages captured (monkeypatched hooks, same call order)."""
    from mmtrack_amd import _lib
    from mmtrack_amd import dimp as mdimp
    from mmtrack_amd import dimp_tracker as mdt
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, parameters
    # frames through the NCHW patch + extract_backbone (the hooked entry point); the normalising sampler the pools
    # use by default gives the same bits (test_gpu_dimpnet.py test_fused_sampler_bits)
    mdt.FUSED_SAMPLE = False
    from mmtrack_amd.dimpnet import DiMPNet
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp.npz"))
    seed, n, H, W, C, tseed = [int(v) for v in gd["meta"]]
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(gd["init_box"]))
    net = DiMPNet(synth.make_dimp_state_dict(0), precision=precision)
    tr = DiMP(parameters(), net=net)
    cap = {"bb_in": [], "l3": [], "clf": [], "scores": []}
    eb, ecf, initf, opt = net.extract_backbone, net.extract_classification_feat, net.init_filter, tr.optimizer.optimize
    af = mdimp.apply_filter

    def extract(p):
        r = eb(p)
        cap["bb_in"].append(p.detach().cpu())
        cap["l3"].append(r.detach().permute(0, 3, 1, 2).float().cpu())   # NHWC merged layer3
        return r

    def clf(f, **k):
        r = ecf(f, **k)
        cap["clf"].append((r[0] if isinstance(r, tuple) else r).detach().cpu())
        return r

    def init_filter(x, bb):
        r = initf(x, bb)
        cap["stack"] = x.detach().cpu()
        cap["init_bb"] = bb.detach().cpu()
        cap["init_filter"] = r.detach().cpu()
        return r

    def optimize(w, feat, bb, num_iter=None, **k):
        its = [w.detach().cpu()]
        cap["opt_in"] = (feat.detach().cpu(), torch.as_tensor(bb).detach().cpu(),
                         {kk: (v.detach().cpu() if torch.is_tensor(v) else v) for kk, v in k.items()})
        cur = w
        for _ in range(num_iter):
            cur = opt(cur, feat, bb, num_iter=1, **k)
            its.append(cur.detach().cpu())
        cap["iterates"] = its
        return cur

    def apply_filter(x, filt):
        r = af(x, filt)
        cap["scores"].append((r.detach().cpu(), filt.detach().cpu()))
        return r
    net.extract_backbone, net.extract_classification_feat, net.init_filter = extract, clf, init_filter
    tr.optimizer.optimize = optimize
    mdimp.apply_filter = apply_filter
    try:
        torch.manual_seed(tseed)
        tr.initialize(frames[0], {"init_bbox": list(gd["init_box"])})
        conf = []
        for t in range(1, n_frames + 1):
            conf.append(tr.track(frames[t])["confidence"])
            pool = tr.pool
            st = _lib.MmtDimpState.from_buffer_copy(bytes(
                pool.states[tr.slot * pool.sbytes:(tr.slot + 1) * pool.sbytes].cpu().numpy()))
            rr = _lib.MmtDimpResult.from_buffer_copy(bytes(
                pool.results[tr.slot * pool.rbytes:(tr.slot + 1) * pool.rbytes].cpu().numpy()))
            cap.setdefault("state", []).append([st.pos[0], st.pos[1], st.target_sz[0], st.target_sz[1],
                                                st.target_scale])
            cap.setdefault("sample", []).append([rr.sample_pos[0], rr.sample_pos[1], rr.sample_scale])
    finally:
        mdimp.apply_filter = af
        mdt.FUSED_SAMPLE = True
    return cap, conf


def stage_errors(cap, conf, g, n_frames=6):
    """(stage, relative error) in run order."""
    out = []
    p = cap["bb_in"][0]
    out.append(("init patches (every 8th pixel)", rel(p[:, :, ::8, ::8], g["init_patch_sub"])))
    out.append(("init patch sums", rel(p.double().sum(dim=(1, 2, 3)), g["init_patch_sums"])))
    l3 = cap["l3"][0]
    out.append(("init layer3 (every 64th channel)", rel(l3[:, ::64], g["init_l3_ch"])))
    out.append(("init layer3 channel sums", rel(l3.double().sum(dim=(2, 3)), g["init_l3_sums"])))
    x = cap["clf"][0]
    out.append(("init clf features (every 32nd channel)", rel(x[:, ::32], g["init_clf_ch"])))
    out.append(("init clf channel sums", rel(x.double().sum(dim=(2, 3)), g["init_clf_sums"])))
    st = cap["stack"]
    st = st.permute(0, 3, 1, 2) if st.shape[-1] == g["init_stack_sums"].shape[-1] else st
    out.append(("init stack (+ dropout) channel sums", rel(st.double().sum(dim=(2, 3)), g["init_stack_sums"])))
    out.append(("init target boxes", rel(cap["init_bb"].reshape(-1, 4), g["init_target_boxes"])))
    out.append(("initial filter (PrRoIPool init)", rel(cap["init_filter"], g["init_filter"])))
    for k, w in enumerate(cap["iterates"]):
        out.append((f"filter after {k} GN steps", rel(w, g["iterates"][k])))
    for t in range(1, n_frames + 1):
        pf = cap["bb_in"][t]
        out.append((f"frame {t} patch (every 8th pixel)", rel(pf[:, :, ::8, ::8], g[f"f{t}_patch_sub"])))
        out.append((f"frame {t} layer3 channel sums", rel(cap["l3"][t].double().sum(dim=(2, 3)), g[f"f{t}_l3_sums"])))
        out.append((f"frame {t} clf channel sums", rel(cap["clf"][t].double().sum(dim=(2, 3)), g[f"f{t}_clf_sums"])))
        sc, fu = cap["scores"][t - 1]
        out.append((f"frame {t} filter used", rel(fu, g[f"f{t}_filter"])))
        out.append((f"frame {t} scores", rel(sc.reshape(g[f"f{t}_scores"].shape), g[f"f{t}_scores"])))
        out.append((f"frame {t} confidence", rel(conf[t - 1], g["confidence"][t - 1])))
        if f"f{t}_state" in g:
            c = g[f"f{t}_coords"]   # the reference's sample: coords (y0, x0, y1, x1) -> centre and scale
            ref_sp = [0.5 * (c[0] + c[2] - 1), 0.5 * (c[1] + c[3] - 1)]
            out.append((f"frame {t} sample centre (px, abs)", float(np.abs(np.array(cap["sample"][t - 1][:2]) -
                                                                            np.array(ref_sp)).max())))
            out.append((f"frame {t} state pos (px, abs)", float(np.abs(np.array(cap["state"][t - 1][:2]) -
                                                                        g[f"f{t}_state"][:2]).max())))
            out.append((f"frame {t} state size / scale", rel(cap["state"][t - 1][2:], g[f"f{t}_state"][2:])))
    return out


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_dimp_stages_vs_reference(precision):
    g = np.load(os.path.join(GOLDEN, "dimp_stages.npz"))
    cap, conf = run_stages(precision)
    errs = stage_errors(cap, conf, g)
    for name, e in errs:
        print(f"[{precision}] {name:42s} {e:.3e}")
    d = dict(errs)
    # the stages up to the sampled patches are integer geometry + bilinear resampling of uint8 pixels
    assert d["init patches (every 8th pixel)"] < 1e-5
    assert d["initial filter (PrRoIPool init)"] < 1e-3
