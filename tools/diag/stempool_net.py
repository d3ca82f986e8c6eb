"""Diagnostic (tuning tool): the DiMP feature net's layer3 with the fused stem + max-pool against the separate
max-pool (bitwise), the pooled stem maps of both, and layer3 sums against the reference golden
(tests/golden/dimpnet_det.npz).  Conv kernel knobs come from the environment (MMT_CONV_*)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmtrack_amd import dimpnet, synth  # noqa: E402

gd = np.load(os.path.join(REPO, "tests", "golden", "dimpnet_det.npz"))
net = dimpnet.DiMPNet(synth.make_dimp_state_dict(0), precision="f16x3")
ims = torch.stack([torch.from_numpy(synth.make_patch(int(s), 288, 6)).float().permute(2, 0, 1)
                   for s in gd["seeds"]]).cuda()
res = {}
for pool in (False, True):
    dimpnet.STEM_POOL = pool
    l3 = net.extract_backbone(ims).clone()
    torch.cuda.synchronize()
    res[pool] = l3
    rel = np.abs(l3.permute(0, 3, 1, 2).double().sum(dim=(1, 2, 3)).cpu().numpy() / gd["layer3_sum"] - 1)
    print(f"stem_pool={pool}: layer3 sum rel err vs golden {rel}")
d = (res[True] - res[False]).abs()
print("fused vs separate layer3: equal" if torch.equal(res[True], res[False]) else
      f"fused vs separate layer3 differ: max |d| {float(d.max())}, n {int((d > 0).sum())} of {d.numel()}")
