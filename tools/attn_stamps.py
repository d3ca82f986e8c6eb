"""Per-part cycles of the f16x3 attention kernel's key-tile loop (GPU tuning tool, not a test): run with
MMTRACK_LIB pointing at an ATTN_STAMPS build (tools/build_variant.sh attnst -DATTN_STAMPS), it launches
mmt_op_attention_f16x3 at the benchmarked shapes (B sequences x 12 heads, N tokens) and the kernel's first workgroups
print wave 0's cycles per loop part (wait = tile landed + barrier + next issue, S = K Q^T issue, softmax incl. the S
results, PV issue), summed over the key tiles.  usage: python tools/attn_stamps.py [B] [N ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
for N in [int(v) for v in sys.argv[2:]] or [320]:
    heads, C = 12, 768
    hi = (torch.randn(B, N, 3 * C, device="cuda") * 100).half()
    lo = (torch.randn(B, N, 3 * C, device="cuda") * 1e-2).half()
    out = torch.empty(B, N, C, device="cuda", dtype=torch.float16)
    out_lo = torch.empty_like(out)
    lens_t = 64
    prob = torch.empty(B, heads, N - lens_t, device="cuda")
    for rep in range(3):   # the last launch's prints are the warm ones
        print(f"## B {B} N {N} launch {rep}", flush=True)
        lib.mmt_op_attention_f16x3(hi.data_ptr(), lo.data_ptr(), out.data_ptr(), out_lo.data_ptr(), B, N, heads, 27,
                                   lens_t, prob.data_ptr(), 2.0 ** -7, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
