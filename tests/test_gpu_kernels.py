"""Operator-level parity of the gfx950 kernels against fp32 PyTorch references (GPU only).

Each kernel consumes bf16 operands; the reference is the same math in fp32 on the same
(bf16-rounded) inputs, so the tolerance only has to cover fp32 accumulation order and the bf16
rounding of outputs.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from mmtrack_amd import _lib
    return _lib.load()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _gemm(lib, A, W, bias, C, R=None, epi=0, conv_hw=0, conv_cin=0, pos_rows=0, lda=None, ldc=None, M=None):
    M = M if M is not None else (A.shape[0] if conv_hw == 0 else A.shape[0])
    N, K = W.shape
    rc = lib.mmt_op_gemm(A.data_ptr(), lda or A.shape[-1], W.data_ptr(), K, bias.data_ptr() if bias is not None else None,
                         C.data_ptr(), ldc or C.shape[-1], R.data_ptr() if R is not None else None,
                         R.shape[-1] if R is not None else 0, M, N, K, epi, conv_hw, conv_cin, pos_rows, _stream())
    assert rc == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K", [(320, 2304, 768), (306, 768, 3072), (64, 128, 768), (5120, 3072, 768),
                                   (153, 768, 768), (1, 32, 64), (4896, 768, 3072), (4896, 768, 768)])
@pytest.mark.parametrize("epi", [0, 1, 2, 4])
def test_gemm_dense(lib, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.float() @ W.float().t() + bias
    if epi in (0, 1):
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        _gemm(lib, A, W, bias, C, epi=epi)
        if epi == 1:
            ref = F.gelu(ref)
        torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=1e-2)
    elif epi == 2:
        R = torch.randn(M, N, device="cuda", generator=g)
        C = R.clone()
        _gemm(lib, A, W, bias, C, R=C, epi=2)   # in place, as the residual stream is updated
        torch.testing.assert_close(C, R + ref, rtol=1e-4, atol=1e-3)
    else:
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        _gemm(lib, A, W, bias, C, epi=4)
        torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-3)


def test_ring_copy_bitwise(tmp_path):
    """The engine with copy launches for the frame parameters and results (MMT_RING_COPY=1) instead of the ring
    hand-off gives the same bits, including device frames whose size and address change between launches that reuse a
    ring entry: op-level GEMMs and a parity-mode sequence whose few-tile GEMMs split K (tests/sk_dump.py, one child
    process each)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for mode, extra in (("ring", {}), ("ringcopy", {"MMT_RING_COPY": "1"})):
        env = {k: v for k, v in os.environ.items() if k != "MMT_RING_COPY"}
        env.update(extra)
        path = str(tmp_path / f"{mode}.npz")
        r = subprocess.run([sys.executable, os.path.join(here, "sk_dump.py"), path], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        res[mode] = np.load(path)
    assert sorted(res["ringcopy"].files) == sorted(res["ring"].files)
    for k in res["ring"].files:
        np.testing.assert_array_equal(res["ringcopy"][k], res["ring"][k], err_msg=f"ringcopy {k}")


@pytest.mark.parametrize("M,N,K", [(4896, 3072, 768), (10240, 2304, 768), (300, 256, 128), (7808, 768, 3072),
                                   (256, 512, 64)])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("cfg", [9, 11, 12, 13])
def test_gemm_forced_configs(lib, M, N, K, epi, cfg):
    """Forced tile configurations on the path's shapes, M tails and K = 64 / 128: 9 = the 256x256
    eight-phase kernel, 11-13 = 32-deep K-tiles (BK 32) with 3-4 deep LDS rings."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 100 * epi)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.float() @ W.float().t() + bias
    if cfg == 9 and N % 256:
        pytest.skip("256 x 256 tiles need N % 256 == 0")
    lib.mmt_gemm_force_config(cfg)
    try:
        if epi in (0, 1):
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            _gemm(lib, A, W, bias, C, epi=epi)
            torch.testing.assert_close(C.float(), F.gelu(ref) if epi == 1 else ref, rtol=1e-2, atol=1e-2)
        else:
            R = torch.randn(M, N, device="cuda", generator=g)
            C = R.clone()
            _gemm(lib, A, W, bias, C, R=C, epi=2)
            torch.testing.assert_close(C, R + ref, rtol=1e-4, atol=1e-3)
    finally:
        lib.mmt_gemm_force_config(-1)


@pytest.mark.parametrize("M,N,K,epi", [(10240, 3072, 768, 1), (10240, 2304, 768, 0), (7808, 2304, 768, 0),
                                       (4899, 3072, 768, 1), (70000, 256, 64, 0), (9000, 384, 128, 1)])
def test_gemm_persistent_forced(lib, M, N, K, epi):
    """The persistent bf16-output kernel (forced): several tiles per workgroup, the next tile's first
    K-tile in flight across the epilogue, M tails (full/partial tiles mixed), K = 64 / 128."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 7 * epi)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.float() @ W.float().t() + bias
    C0 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _gemm(lib, A, W, bias, C0, epi=epi)   # default dispatch: the non-persistent kernels
    lib.mmt_gemm_force_config(10)
    try:
        C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _gemm(lib, A, W, bias, C, epi=epi)
    finally:
        lib.mmt_gemm_force_config(-1)
    torch.testing.assert_close(C.float(), F.gelu(ref) if epi == 1 else ref, rtol=1e-2, atol=1e-2)
    assert torch.equal(C, C0)   # same K order per output: bit-identical to the per-tile kernels


@pytest.mark.parametrize("M,N,K,epi", [(10240, 3072, 768, 1), (10240, 2304, 768, 0), (7808, 2304, 768, 0),
                                       (4899, 3072, 768, 1), (60000, 256, 128, 0), (9000, 512, 128, 1),
                                       (300, 256, 256, 1)])
@pytest.mark.parametrize("cfg", [16, 17, 18, 19, 20])
def test_gemm_ring_forced(lib, M, N, K, epi, cfg):
    """The persistent ring kernel (forced): one K-tile stream across a workgroup's output tiles, the
    permlane-transposed register epilogue, bias through LDS, M tails dropped by the C resource, small
    grids; bit-identical to the per-tile kernels (same K order per output)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 11 * epi)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.float() @ W.float().t() + bias
    C0 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.mmt_gemm_force_config(3)   # a per-tile kernel (128 x 128, 4 waves) as the bitwise reference
    try:
        _gemm(lib, A, W, bias, C0, epi=epi)
        lib.mmt_gemm_force_config(cfg)
        C = torch.full((M + 1, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _gemm(lib, A, W, bias, C[:M], epi=epi)
    finally:
        lib.mmt_gemm_force_config(-1)
    torch.testing.assert_close(C[:M].float(), F.gelu(ref) if epi == 1 else ref, rtol=1e-2, atol=1e-2)
    assert torch.equal(C[:M], C0)
    assert torch.isnan(C[M].float()).all(), "a store past row M"


def test_gemm_pos_epilogue(lib):
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K, L = 2 * 720, 768, 768, 720
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    pos = torch.randn(L, N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    _gemm(lib, A, W, bias, C, R=pos, epi=6, pos_rows=L)
    ref = A.float() @ W.float().t() + bias + pos.repeat(2, 1)
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("B,hw,cin,cout,epi", [(2, 16, 768, 768, 3), (3, 16, 256, 128, 3), (1, 24, 128, 64, 3),
                                               (2, 16, 64, 32, 5)])
def test_gemm_conv3x3(lib, B, hw, cin, cout, epi):
    """head.py:8-21 conv3x3 (pad 1) as an implicit GEMM over the NHWC token map."""
    g = torch.Generator(device="cuda").manual_seed(cin + cout)
    x = torch.randn(B, cin, hw, hw, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(cout, device="cuda", generator=g)
    ref = F.relu(F.conv2d(x.float(), w.float(), bias, padding=1))       # [B, cout, hw, hw]
    A = x.permute(0, 2, 3, 1).contiguous().view(B * hw * hw, cin)      # NHWC rows
    Wk = w.permute(0, 2, 3, 1).contiguous().view(cout, 9 * cin)        # [out][ky][kx][in]
    if epi == 3:
        C = torch.empty(B * hw * hw, cout, device="cuda", dtype=torch.bfloat16)
    else:
        C = torch.empty(B * hw * hw, cout, device="cuda", dtype=torch.float32)
    _gemm(lib, A, Wk, bias, C, epi=epi, conv_hw=hw, conv_cin=cin)
    out = C.float().view(B, hw, hw, cout).permute(0, 3, 1, 2)
    torch.testing.assert_close(out, ref, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("B,N", [(1, 320), (3, 244), (2, 153), (1, 720), (5, 190), (1, 17),
                                 (12, 320), (16, 244), (11, 190), (12, 153), (16, 64), (11, 17), (11, 720),
                                 (12, 548)])
def test_attention(lib, B, N):
    """attn.py:33-59 with the CE probability row of template token 27 (attn_blocks.py:44-53).
    B * heads >= 128 with N > 320 takes the 8-wave workgroups, the others 1-4 waves."""
    heads, C = 12, 768
    g = torch.Generator(device="cuda").manual_seed(N + B)
    qkv = (torch.randn(B, N, 3 * C, device="cuda", generator=g) * 2.0).bfloat16()
    out = torch.empty(B, N, C, device="cuda", dtype=torch.bfloat16)
    lens_t = min(64, N - 1)
    ceq = min(27, lens_t - 1)
    prob = torch.empty(B, heads, N - lens_t, device="cuda")
    rc = lib.mmt_op_attention(qkv.data_ptr(), out.data_ptr(), B, N, heads, ceq, lens_t, prob.data_ptr(), _stream())
    assert rc == 0
    torch.cuda.synchronize()
    q, k, v = qkv.float().view(B, N, 3, heads, 64).permute(2, 0, 3, 1, 4)
    attn = ((q @ k.transpose(-2, -1)) * 0.125).softmax(-1)
    ref = (attn @ v).transpose(1, 2).reshape(B, N, C)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(prob, attn[:, :, ceq, lens_t:], rtol=1e-4, atol=1e-6)


def test_xlane_reductions_bitwise():
    """common.h's permlane / DPP wave reductions equal the __shfl_xor butterfly bit for bit (built by build())."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "bin", "xlane_check")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_layernorm(lib):
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(333, 768, device="cuda", generator=g) * 3 + 1
    w = torch.randn(768, device="cuda", generator=g)
    b = torch.randn(768, device="cuda", generator=g)
    ob = torch.empty(333, 768, device="cuda", dtype=torch.bfloat16)
    of = torch.empty(333, 768, device="cuda")
    assert lib.mmt_op_layernorm(x.data_ptr(), w.data_ptr(), b.data_ptr(), ob.data_ptr(), of.data_ptr(), 333,
                                _stream()) == 0
    torch.cuda.synchronize()
    ref = F.layer_norm(x, (768,), w, b, 1e-6)
    torch.testing.assert_close(of, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ob.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,C,hz,hx", [(1, 256, 6, 22), (3, 256, 6, 22), (2, 64, 4, 18), (1, 512, 5, 21)])
def test_xcorr(lib, B, C, hz, hx):
    """SiamFC xcorr / DiMP apply_filter as per-sequence grouped conv (filter.py:51-52)."""
    from mmtrack_amd import xcorr
    g = torch.Generator(device="cuda").manual_seed(C + hz)
    z = torch.randn(B, C, hz, hz, device="cuda", generator=g)
    x = torch.randn(B, C, hx, hx, device="cuda", generator=g)
    out = xcorr(z, x, scale=0.001, bias=0.5)
    torch.cuda.synchronize()
    ref = F.conv2d(x.reshape(1, B * C, hx, hx), z, groups=B).view(B, 1, hx - hz + 1, hx - hz + 1) * 0.001 + 0.5
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
