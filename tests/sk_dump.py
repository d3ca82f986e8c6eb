"""Helper of test_gpu_kernels.py::test_ring_copy_bitwise (run as a child process, GPU only): split-K
GEMM outputs through mmt_op_gemm (bf16 operands) and one parity-mode sequence tracked by the engine (its
few-tile f16x3 GEMMs split K), saved to an .npz.  The test runs it with the ring hand-off and with copy launches
(MMT_RING_COPY=1) and compares the files bit for bit.

usage: python tests/sk_dump.py <out.npz>"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-trakcing-bechmark_amd"))
from mmtrack_amd import _lib, synth  # noqa: E402
from mmtrack_amd.engine import Engine, EngineConfig  # noqa: E402

out = {}
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
for (M, N, K, epi) in [(306, 768, 3072, 0), (306, 768, 3072, 2), (64, 128, 768, 1), (200, 768, 3072, 4)]:
    g = torch.Generator(device="cuda").manual_seed(M + N + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    R = torch.randn(M, N, device="cuda", generator=g)
    C = R.clone() if epi == 2 else torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if epi in (0, 1) else torch.float32)
    rc = lib.mmt_op_gemm(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), C.data_ptr(), N,
                         C.data_ptr() if epi == 2 else None, N if epi == 2 else 0, M, N, K, epi, 0, 0, 0, s)
    assert rc == 0
    torch.cuda.synchronize()
    out[f"gemm_{M}_{N}_{K}_{epi}"] = C.float().cpu().numpy()

sd = synth.make_state_dict(0, kind="vipt", prompt_type="vipt_deep")
eng = Engine(EngineConfig(max_batch=1, use_graphs=True, precision="fp32"), sd)
frames, gts = synth.make_frames(21, 5, 360, 480, 6)
eng.initialize(0, frames[0], list(gts[0]))
out["boxes"] = np.array([eng.track(0, frames[t])[0] for t in range(1, 5)])
# device frames whose size and address change between launches that reuse a ring entry (the ring hand-off
# reads each launch's frame parameters from pinned memory: a stale entry would show against the copy path)
big, _ = synth.make_frames(22, 6, 360, 480, 6)
small, _ = synth.make_frames(23, 6, 300, 400, 6)
seq = []
for t in range(20):   # > 2 x the ring depth (MMT_PIPELINE_DEPTH = 8)
    src = big if (t // 3) % 2 == 0 else small
    f = torch.from_numpy(np.ascontiguousarray(src[1 + t % 5])).cuda()   # a fresh device buffer per launch
    if t % 4 == 1:
        f = torch.cat([f, f[:1]]).contiguous()[:-1]                       # another address, same contents
    seq.append(eng.track(0, f)[0])
    del f
out["boxes_device_frames"] = np.array(seq)
eng.close()
np.savez(sys.argv[1], **out)
print("sk_dump ok", sorted(out))
