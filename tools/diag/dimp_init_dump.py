"""Dump the HIP DiMP tracker's classifier inputs and iterates at initialisation (GPU diagnostic, not a test): the
tracker_dimp.npz run's feature stack as the filter initialiser and the Gauss-Newton optimiser received it, the
target boxes, the initial filter and all ten iterates, per precision, to gpurun_out/dimp_init_dump_<prec>.npz.
tools/diag/dimp_feed_ref.py then runs the REFERENCE classifier on exactly these inputs in the build container, which
separates the optimiser's own error (same inputs, one step at a time) from the error the features carry in."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.test_gpu_dimp_stages import run_stages  # noqa: E402

os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
for prec in sys.argv[1:] or ["f16x3", "fp32"]:
    cap, conf = run_stages(prec, n_frames=1)
    feat, bb, kw = cap["opt_in"]
    out = {"opt_feat": feat.numpy(), "opt_bb": bb.numpy(), "iterates": torch.stack(cap["iterates"]).numpy(),
           "init_stack_nhwc": cap["stack"].numpy(), "init_bb": cap["init_bb"].numpy(),
           "init_filter": cap["init_filter"].numpy(), "f1_clf": cap["clf"][1].numpy(),
           "f1_scores": cap["scores"][0][0].numpy(), "confidence": np.array(conf)}
    if kw.get("sample_weight") is not None:
        out["opt_sw"] = np.asarray(kw["sample_weight"])
    np.savez_compressed(os.path.join(REPO, "gpurun_out", f"dimp_init_dump_{prec}.npz"), **out)
    print(prec, {k: v.shape for k, v in out.items()}, flush=True)
