"""DiMP classifier inner loop on the HIP path vs the reference golden (tests/golden/dimp.npz,
generated from RGBD/models/DeT/ltr) and vs oracle/dimp.py on seeded shapes (fp32, tolerances inline)."""
import os

import numpy as np
import pytest
import torch

from oracle import dimp as od

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dimp.npz")


@pytest.fixture(scope="module")
def gold():
    g = np.load(GOLDEN)
    return {k: g[k] for k in g.files}


def _opt_sd(g):
    return {k[4:]: torch.from_numpy(g[k]) for k in g if k.startswith("opt.")}


def test_apply_filter_golden(gold):
    from mmtrack_amd import dimp
    feat, filt = (torch.from_numpy(gold[k]).cuda() for k in ("feat", "filt"))
    sc = dimp.apply_filter(feat, filt).cpu().numpy()
    np.testing.assert_allclose(sc, gold["scores"], rtol=1e-5, atol=2e-5)


def test_feat_transpose_golden(gold):
    from mmtrack_amd import dimp
    feat, r = (torch.from_numpy(gold[k]).cuda() for k in ("feat", "resid"))
    ft = dimp.apply_feat_transpose(feat, r, (4, 4)).cpu().numpy()
    np.testing.assert_allclose(ft, gold["feat_t"], rtol=1e-4, atol=1e-3)


def test_steepest_descent_golden(gold):
    from mmtrack_amd import dimp
    opt = dimp.DiMPSteepestDescentGN(_opt_sd(gold), num_iter=5)
    feat, filt = (torch.from_numpy(gold[k]).cuda() for k in ("feat", "filt"))
    w, iters, losses = opt(filt, feat, torch.from_numpy(gold["bb"]))
    assert len(iters) == 6 and len(losses) == 6
    np.testing.assert_allclose(torch.stack([i.cpu() for i in iters]).numpy(), gold["iterates"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(torch.stack(losses).numpy(), gold["losses"], rtol=1e-4)
    # single-call path (no per-iterate copies) lands on the same filter
    w2 = opt.optimize(filt, feat, torch.from_numpy(gold["bb"]))
    torch.testing.assert_close(w2, w, rtol=0, atol=0)


@pytest.mark.parametrize("I,S,C,H,W,fk", [(1, 1, 8, 9, 9, 1), (2, 3, 64, 18, 18, 4), (4, 2, 512, 22, 22, 4),
                                          (3, 1, 128, 15, 20, 5), (1, 5, 256, 18, 18, 3)])
def test_vs_oracle_shapes(I, S, C, H, W, fk):
    from mmtrack_amd import dimp
    g = torch.Generator().manual_seed(I * 1000 + C + fk)
    feat = torch.randn(I, S, C, H, W, generator=g) * 0.5
    filt = torch.randn(S, C, fk, fk, generator=g) * 0.02
    bb = torch.rand(I, S, 4, generator=g) * torch.tensor([H * 10.0, W * 10.0, 60, 60]) + 8.0
    sd = {"log_step_length": torch.tensor([0.3]), "filter_reg": torch.tensor([0.05]),
          "label_map_predictor.weight": torch.linspace(1.0, -0.2, 10).view(1, 10, 1, 1),
          "target_mask_predictor.0.weight": torch.linspace(3.0, -3.0, 10).view(1, 10, 1, 1),
          "spatial_weight_predictor.weight": torch.ones(1, 10, 1, 1)}
    sw = torch.rand(I, S, generator=g) + 0.1
    fc = feat.cuda()
    sc = dimp.apply_filter(fc, filt.cuda()).cpu()
    torch.testing.assert_close(sc, od.apply_filter(feat, filt), rtol=1e-4, atol=1e-4)
    r = torch.randn(sc.shape, generator=g)
    gt = dimp.apply_feat_transpose(fc, r.cuda(), (fk, fk)).cpu()
    torch.testing.assert_close(gt, od.apply_feat_transpose(feat, r, (fk, fk)), rtol=1e-4, atol=1e-3)
    for swt in (None, sw):
        w_ref, it_ref, l_ref = od.steepest_descent_gn(filt, feat, bb, sd, num_iter=3, sample_weight=swt)
        w, its, ls = dimp.DiMPSteepestDescentGN(sd, num_iter=3)(filt.cuda(), fc, bb, sample_weight=swt)
        torch.testing.assert_close(w.cpu(), w_ref, rtol=1e-3, atol=1e-5)
        np.testing.assert_allclose(torch.stack(ls).numpy(), torch.stack(l_ref).numpy().ravel(), rtol=1e-3)


def test_errors():
    from mmtrack_amd import dimp
    with pytest.raises(ValueError):
        dimp.apply_filter(torch.zeros(1, 1, 4, 8, 8), torch.zeros(1, 4, 3, 3))        # host tensors
    with pytest.raises(ValueError):
        dimp.apply_filter(torch.zeros(1, 2, 4, 8, 8).cuda(), torch.zeros(1, 4, 3, 3).cuda())   # S mismatch
    with pytest.raises(ValueError):
        dimp.apply_filter(torch.zeros(1, 1, 4, 8, 8).cuda(), torch.zeros(1, 4, 7, 7).cuda())   # > 25 taps
