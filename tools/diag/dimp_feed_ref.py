"""The REFERENCE DeT classifier on the HIP tracker's own classifier inputs (build-container diagnostic, not a test;
needs /root/reference and gpurun_out/dimp_init_dump_<prec>.npz from tools/diag/dimp_init_dump.py).

Separates where the HIP DiMP confidence drift comes from:
* initialiser error   -- reference filter_initializer on the HIP feature stack vs the HIP initial filter;
* optimiser step error -- ONE reference Gauss-Newton step from the HIP iterate k on the HIP features vs the HIP
                          iterate k+1 (same inputs: the optimiser's own arithmetic difference, per step);
* trajectory          -- the reference optimiser's ten steps from the HIP initial filter on the HIP features
                          (fp32 and float64) vs the HIP iterates, and vs the golden's iterates (reference features);
* sign margins        -- per step, the score elements closest to 0 (LeakyReluPar's |x| kink, activation.py): a
                          score within the features' error of 0 flips the score mask and the gradient discontinuously.
Usage:  python tools/diag/dimp_feed_ref.py [f16x3|fp32 ...]"""
import copy
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden_dimp as mgd  # noqa: E402
from mmtrack_amd import synth  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def reference_init_inputs(net):
    """The reference tracker's own optimiser inputs at initialize() on the golden sequence (feat, bb)."""
    from pytracking.parameter.dimp import DeT_DiMP50_Max as P
    from pytracking.tracker.dimp.dimp import DiMP
    wnet = mgd.wrap(net)
    params = P.parameters()
    params.use_gpu, params.device, params.use_iou_net, params.net = False, "cpu", False, wnet
    tr = DiMP(params)
    tr.features_initialized = True
    fo = net.classifier.filter_optimizer
    fwd = fo.forward
    cap = {}

    def hook(w, feat=None, bb=None, *a, **k):
        cap.setdefault("in", (feat.clone(), bb.clone()))
        return fwd(w, feat, bb, *a, **k)
    fo.forward = hook
    try:
        S = mgd.SEQ
        frames, _ = synth.make_frames(S["seed"], 1, S["H"], S["W"], S["C"], box=S["box"])
        torch.manual_seed(mgd.TRACK_SEED)
        tr.initialize(frames[0], {"init_bbox": list(S["box"])})
    finally:
        fo.forward = fwd
    return cap["in"]


def main():
    mgd.install()
    torch.set_num_threads(8)
    net = mgd.build_net(synth.make_dimp_state_dict(0))
    clf = net.classifier
    fi, fo = clf.filter_initializer, clf.filter_optimizer
    with torch.no_grad():
        rfeat, rbb = reference_init_inputs(net)
    fo64 = copy.deepcopy(fo).double()
    from ltr.models.layers import filter as filter_layer
    g = np.load(os.path.join(REPO, "tests", "golden", "dimp_stages.npz"))
    for prec in sys.argv[1:] or ["f16x3", "fp32"]:
        d = np.load(os.path.join(REPO, "gpurun_out", f"dimp_init_dump_{prec}.npz"))
        feat = torch.from_numpy(d["opt_feat"])
        bb = torch.from_numpy(d["opt_bb"]).reshape(feat.shape[0], feat.shape[1], 4)
        its = d["iterates"]
        n = its.shape[0] - 1
        print(f"== {prec}: feat {tuple(feat.shape)}, {n} steps", flush=True)
        x = torch.from_numpy(d["init_stack_nhwc"]).permute(0, 3, 1, 2).unsqueeze(1).contiguous()
        with torch.no_grad():
            w0 = fi(x, torch.from_numpy(d["init_bb"]).reshape(x.shape[0], 1, 4))
            print(f"initialiser: ref(HIP stack) vs HIP initial filter {rel(w0, d['init_filter']):.3e}; "
                  f"HIP initial filter vs golden {rel(d['init_filter'], g['init_filter']):.3e}")
            w = torch.from_numpy(its[0])
            _, traj, _ = fo(w, feat=feat, bb=bb, num_iter=n, compute_losses=False)
            _, traj64, _ = fo64(w.double(), feat=feat.double(), bb=bb.double(), num_iter=n, compute_losses=False)
            print(" k  step(HIP k -> k+1)  traj ref32 vs HIP  traj ref64 vs HIP  ref32 vs ref64  HIP vs golden  "
                  "ref32 vs golden  min|score|/max  #|s|<1e-5max")
            for k in range(n + 1):
                if k < n:
                    _, st, _ = fo(torch.from_numpy(its[k]), feat=feat, bb=bb, num_iter=1, compute_losses=False)
                    e_step = rel(st[1], its[k + 1])
                else:
                    e_step = float("nan")
                s = filter_layer.apply_filter(feat, traj[k]).abs()
                smax = float(s.max())
                print(f"{k:2d}  {e_step:.3e}           {rel(traj[k], its[k]):.3e}          "
                      f"{rel(traj64[k], its[k]):.3e}          {rel(traj[k], traj64[k]):.3e}      "
                      f"{rel(its[k], g['iterates'][k]):.3e}      {rel(traj[k], g['iterates'][k]):.3e}       "
                      f"{float(s.min()) / smax:.2e}        {int((s < 1e-5 * smax).sum())}", flush=True)
            # sign of every score element (the LeakyReluPar kink): reference features + golden iterate k vs HIP
            # features + HIP iterate k; the elements whose sign differs and their magnitudes
            print(" k  sign flips HIP vs reference run: (image, y, x, reference score / max, HIP score / max)")
            rf = rfeat.reshape(feat.shape)
            print(f"    reference features vs HIP features: {rel(feat, rf):.3e} of max")
            for k in range(n + 1):
                sr = filter_layer.apply_filter(rf, torch.from_numpy(g["iterates"][k]))
                sh = filter_layer.apply_filter(feat, torch.from_numpy(its[k]))
                m = float(sr.abs().max())
                diff = (torch.sign(sr) != torch.sign(sh)).nonzero().tolist()
                print(f"{k:2d}  {len(diff)}  " + "  ".join(
                    f"({i[0]}, {i[-2]}, {i[-1]}, {float(sr[tuple(i)]) / m:+.2e}, {float(sh[tuple(i)]) / m:+.2e})"
                    for i in diff[:6]), flush=True)


if __name__ == "__main__":
    main()
