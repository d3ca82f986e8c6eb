"""Operator-level parity of the parity-mode ("f16x3") kernels against fp32/fp64 PyTorch (GPU only).

The engine's default precision carries every MFMA operand as the fp16 pair hi = f16(v s), lo = f16(v s - hi)
of a power-of-two range scale s (csrc/common.h) and accumulates Wh*Ah + Wl*Ah + Wh*Al in fp32.  These tests
drive the exact kernels of the benchmarked 32-sequence launch through mmt_op_gemm_f16x3 /
mmt_op_attention_f16x3 (include/mmtrack.h) on the path's shapes:

* M = 10240 (32 sequences x 320 tokens), N = 2304 / 3072, K = 768: the 256 x 256 eight-phase kernel
  gemm256s_kernel<EPI> (qkv EPI 0, fc1 EPI 1);
* N = 768, K = 768 (proj, EPI 2) and K = 3072 (fc2, EPI 2): the 128 x 128 / 128 x 192 f16x3 gemm_kernel (32- and
  64-deep K-tiles) and, where its tiles fill one round, the 128 x 256 two-group gemm128w_kernel; EPI 4 (patch embed);
* one sequence's few-tile shapes (M = 320 / 153): the 64 x 64 kernels and the split-K path;
* attention at B * heads >= 128: attn_kernel<8, true>; one sequence: the key-split attn_kernel<4, true, 1, true>.

The reference is float64 on the reconstructed operands (hi + lo) / s, so the tolerance only has to cover the
dropped lo*lo term (2^-22 relative per product) and fp32 accumulation: 1e-5 of the output scale
(the bf16 tests in test_gpu_kernels.py use 1e-2).  Reference: attn.py:17-19 / 33-59, timm Mlp (fc1 GELU-erf,
fc2), attn_blocks.py:44-53 (the CE probability row).
"""
import math

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


def range_scale(t):
    """engine.cpp range_scale: the power of two s with max|t| * s <= 2^14."""
    m = float(t.abs().max())
    return 2.0 ** (14 - math.ceil(math.log2(m))) if m > 0 else 1.0


def split(t, s):
    """fp16 hi / lo halves of t * s (fp32 arithmetic, RNE) and the exact value they carry, in float64."""
    v = t.float() * s
    hi = v.half()
    lo = (v - hi.float()).half()
    return hi.contiguous(), lo.contiguous(), (hi.double() + lo.double()) / s


def _gemm(lib, Ah, Al, Wh, Wl, bias, C, Cl, inv, out_scale, epi, R=None, M=None):
    M = Ah.shape[0] if M is None else M
    N, K = Wh.shape
    rc = lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh.data_ptr(), Wl.data_ptr(), K, bias.data_ptr(),
                               C.data_ptr(), Cl.data_ptr() if Cl is not None else None, N,
                               R.data_ptr() if R is not None else None, N if R is not None else 0,
                               M, N, K, epi, inv, out_scale, 0, 0, _stream())
    assert rc == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K,epi", [
    (10240, 2304, 768, 0),    # qkv, 32 sequences: gemm256s_kernel<0>
    (10240, 3072, 768, 1),    # fc1, 32 sequences: gemm256s_kernel<1>
    (7808, 3072, 768, 1),     # fc1 after CE (244 tokens), M % 256 != 0
    (4896, 2304, 768, 0),     # qkv after the last CE (153 tokens)
    (10240, 768, 768, 2),     # proj, 32 x 320 rows in one launch: the 128 x 256 two-group tile (240 tiles, one round)
    (4896, 768, 3072, 2),     # fc2 after the last CE: 128 x 128, 64-deep K-tiles
    (7808, 768, 3072, 2),     # fc2 (244 tokens): 128 x 192 tiles (one round of them against two of 128 x 128)
    (6080, 768, 768, 2),      # proj (190 tokens): 128 x 192, the residual chunks loaded in the drain
    (4096, 768, 768, 4),      # patch embed (fp32 output)
    (320, 2304, 768, 0),      # one sequence: 64 x 64 few-tile kernels
    (320, 3072, 768, 1),
    (153, 768, 3072, 2),      # one sequence's fc2: split-K + fixed-order reduce
    (320, 768, 768, 2),
])
def test_gemm_f16x3_vs_fp64(lib, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g) * (3.0 if epi == 4 else 1.0)
    W = torch.randn(N, K, device="cuda", generator=g) * (0.5 / math.sqrt(K))
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    sa, sw = range_scale(A), range_scale(W)
    Ah, Al, A64 = split(A, sa)
    Wh, Wl, W64 = split(W, sw)
    ref = A64 @ W64.t() + bias.double()
    inv = 1.0 / (sa * sw)
    if epi in (0, 1):
        y = F.gelu(ref) if epi == 1 else ref
        so = range_scale(y.float())
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        Cl = torch.empty_like(C)
        _gemm(lib, Ah, Al, Wh, Wl, bias, C, Cl, inv, so, epi)
        out = (C.double() + Cl.double()) / so
        tol = 1e-5 * float(y.abs().max())
    elif epi == 2:
        R = torch.randn(M, N, device="cuda", generator=g)
        C = R.clone()
        _gemm(lib, Ah, Al, Wh, Wl, bias, C, None, inv, 1.0, epi, R=C)   # in place, as the residual stream
        out = C.double()
        y = R.double() + ref
        tol = 1e-5 * float(ref.abs().max()) + 4e-7 * float(y.abs().max())
    else:
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        _gemm(lib, Ah, Al, Wh, Wl, bias, C, None, inv, 1.0, epi)
        out = C.double()
        y = ref
        tol = 1e-5 * float(y.abs().max())
    err = float((out - y).abs().max())
    print(f"f16x3 gemm M={M} N={N} K={K} epi={epi}: max|err| {err:.3e} (tol {tol:.3e})")
    assert err <= tol
    assert torch.isfinite(out).all()


@pytest.mark.parametrize("M,N,K,epi", [
    (7808, 2304, 768, 0),     # qkv after the first CE (244 tokens): the rule picks 320 x 256 (225 tiles, one round)
    (6080, 3072, 768, 1),     # fc1 after the second CE (190 tokens): 320 x 256 by the rule (228 tiles)
    (10240, 3072, 768, 1),    # forced: whole tiles, 32 rows per M tile
    (4896, 2304, 768, 0),     # forced: M % 320 = 96 (the last tile's second half-tile empty)
    (700, 3072, 128, 1),      # forced: K = 128 (four K-steps: the tail-wait path only), M % 320 = 60
    (330, 2304, 64, 0),       # forced: K = 64 (two K-steps), M = 320 + 10
])
def test_gemm_f16x3_t320(lib, M, N, K, epi):
    """The 320 x 256 eight-phase tile (gemm256s_kernel<EPI, 5>) against fp64, and bit-identical to the 256 x 256 tile:
    both accumulate every output over the same K order, so only the tiling differs (attn.py:17-19 qkv, timm Mlp fc1)."""
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * (0.5 / math.sqrt(K))
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    sa, sw = range_scale(A), range_scale(W)
    Ah, Al, A64 = split(A, sa)
    Wh, Wl, W64 = split(W, sw)
    ref = A64 @ W64.t() + bias.double()
    y = F.gelu(ref) if epi == 1 else ref
    so = range_scale(y.float())
    outs = []
    try:
        for cfg in (320, 256):
            lib.mmt_gemm_force_config(cfg)
            C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
            Cl = torch.full_like(C, float("nan"))
            _gemm(lib, Ah, Al, Wh, Wl, bias, C, Cl, 1.0 / (sa * sw), so, epi)
            outs.append((C, Cl))
    finally:
        lib.mmt_gemm_force_config(-1)
    (C, Cl), (C2, Cl2) = outs
    out = (C.double() + Cl.double()) / so
    err = float((out - y).abs().max())
    tol = 1e-5 * float(y.abs().max())
    print(f"f16x3 gemm 320x256 M={M} N={N} K={K} epi={epi}: max|err| {err:.3e} (tol {tol:.3e})")
    assert torch.isfinite(out).all()
    assert err <= tol
    assert torch.equal(C.view(torch.int16), C2.view(torch.int16)) and torch.equal(Cl.view(torch.int16),
                                                                                  Cl2.view(torch.int16))


@pytest.mark.parametrize("M,N,K", [(10240, 768, 3072), (4896, 768, 3072), (11520, 768, 768), (700, 768, 128)])
def test_gemm_f16x3_256s_residual(lib, M, N, K):
    """The eight-phase 256 x 256 tile with the fp32 residual epilogue (gemm256s_kernel<EPI_RESID_F32, 4>: the residual
    chunks requested first, the tile staged through the LDS per 128-row half, whole 16-B row chunks stored), in place
    on the residual stream as fc2 / proj run it at OSTrack-384's long layers (timm Mlp fc2, attn.py proj + the block's
    residual adds, attn_blocks.py:93-104), vs fp64."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 11)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * (0.5 / math.sqrt(K))
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    sa, sw = range_scale(A), range_scale(W)
    Ah, Al, A64 = split(A, sa)
    Wh, Wl, W64 = split(W, sw)
    ref = A64 @ W64.t() + bias.double()
    R = torch.randn(M, N, device="cuda", generator=g)
    C = R.clone()
    lib.mmt_gemm_force_config(256)
    try:
        _gemm(lib, Ah, Al, Wh, Wl, bias, C, None, 1.0 / (sa * sw), 1.0, 2, R=C)
    finally:
        lib.mmt_gemm_force_config(-1)
    y = R.double() + ref
    err = float((C.double() - y).abs().max())
    tol = 1e-5 * float(ref.abs().max()) + 4e-7 * float(y.abs().max())
    print(f"f16x3 gemm 256x256 residual M={M} N={N} K={K}: max|err| {err:.3e} (tol {tol:.3e})")
    assert torch.isfinite(C).all()
    assert err <= tol


@pytest.mark.parametrize("M,N,K,epi", [
    (5120, 768, 768, 2),      # proj, one stream half of 16 x 320 tokens (the default rule's shape)
    (3904, 768, 3072, 2),     # fc2, a half of 16 x 244 tokens
    (3040, 768, 3072, 2),     # fc2, a half of 16 x 190 tokens: M % 128 = 96
    (700, 768, 128, 2),       # forced: K = 128 (four K-tiles: the ring's tail), M % 128 = 60
    (130, 768, 64, 2),        # forced: K = 64 (two K-tiles: the prologue's second load, no steady step), M = 128 + 2
    (4096, 768, 768, 4),      # forced: fp32 output without a residual (patch-embed shape)
    (2048, 768, 768, 6),      # forced: the position epilogue (row m % pos_rows; the op entry fixes pos_rows = 1)
])
def test_gemm_f16x3_w256(lib, M, N, K, epi):
    """The 128 x 256 two-group tile (gemm128w_kernel<EPI>: three half-tiles per 32-deep K-tile in a 3-stage ring, two
    MFMA phases, waves 4-7 one barrier behind) against fp64 and bit for bit against the 256 x 256 eight-phase tile,
    which accumulates every output over the same K order (attn.py proj, timm Mlp fc2 + the block's residual adds,
    attn_blocks.py:93-104; patch_embed.py:20 for the fp32 / position epilogues)."""
    g = torch.Generator(device="cuda").manual_seed(M + 5 * N + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * (0.5 / math.sqrt(K))
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    sa, sw = range_scale(A), range_scale(W)
    Ah, Al, A64 = split(A, sa)
    Wh, Wl, W64 = split(W, sw)
    ref = A64 @ W64.t() + bias.double()
    pos_rows = 1   # mmt_op_gemm_f16x3's position epilogue: every row adds R's row 0
    R = torch.randn(M if epi == 2 else pos_rows, N, device="cuda", generator=g)
    outs = []
    try:
        for cfg in (128, 256):
            lib.mmt_gemm_force_config(cfg)
            if epi == 2:
                C = R.clone()
                _gemm(lib, Ah, Al, Wh, Wl, bias, C, None, 1.0 / (sa * sw), 1.0, epi, R=C)   # in place
            else:
                C = torch.full((M, N), float("nan"), device="cuda")
                rc = lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh.data_ptr(), Wl.data_ptr(), K,
                                           bias.data_ptr(), C.data_ptr(), None, N,
                                           R.data_ptr() if epi == 6 else None, N if epi == 6 else 0,
                                           M, N, K, epi, 1.0 / (sa * sw), 1.0, 0, 0, _stream())
                assert rc == 0
                torch.cuda.synchronize()
            outs.append(C)
    finally:
        lib.mmt_gemm_force_config(-1)
    C, C2 = outs
    if epi == 2:
        y = R.double() + ref
    elif epi == 6:
        y = ref + R.double()[torch.arange(M, device="cuda") % pos_rows]
    else:
        y = ref
    err = float((C.double() - y).abs().max())
    tol = 1e-5 * float(ref.abs().max()) + 4e-7 * float(y.abs().max())
    print(f"f16x3 gemm 128x256 M={M} N={N} K={K} epi={epi}: max|err| {err:.3e} (tol {tol:.3e})")
    assert torch.isfinite(C).all()
    assert err <= tol
    assert torch.equal(C.view(torch.int32), C2.view(torch.int32))


@pytest.mark.parametrize("B,N", [(32, 320), (16, 320), (16, 244), (16, 153), (16, 720), (12, 190), (1, 320),
                                 (1, 153), (2, 244), (1, 720)])
def test_attention_f16x3_vs_fp64(lib, B, N):
    """attn.py:33-59 with the CE probability row of the CTR_POINT template token (attn_blocks.py:44-53)."""
    heads, C = 12, 768
    g = torch.Generator(device="cuda").manual_seed(7 * N + B)
    qkv = torch.randn(B, N, 3 * C, device="cuda", generator=g) * 1.5
    s = range_scale(qkv)
    hi, lo, q64 = split(qkv, s)
    out = torch.empty(B, N, C, device="cuda", dtype=torch.float16)
    out_lo = torch.empty_like(out)
    lens_t = 64 if N > 64 else N - 1
    ceq = 27 if lens_t > 27 else 0
    prob = torch.empty(B, heads, N - lens_t, device="cuda")
    rc = lib.mmt_op_attention_f16x3(hi.data_ptr(), lo.data_ptr(), out.data_ptr(), out_lo.data_ptr(), B, N, heads, ceq,
                                    lens_t, prob.data_ptr(), s, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    q, k, v = q64.view(B, N, 3, heads, 64).permute(2, 0, 3, 1, 4)
    attn = ((q @ k.transpose(-2, -1)) * 0.125).softmax(-1)
    ref = (attn @ v).transpose(1, 2).reshape(B, N, C)
    got = (out.double() + out_lo.double()) / s
    err = float((got - ref).abs().max())
    perr = float((prob.double() - attn[:, :, ceq, lens_t:]).abs().max())
    print(f"f16x3 attention B={B} N={N}: max|dO| {err:.3e}, max|dP| {perr:.3e}")
    assert err <= 1e-5 * float(ref.abs().max())
    assert perr <= 1e-6


def test_split_halves_are_exact():
    """The fp16 pair carries v * s to ~22 bits: |(hi + lo) / s - v| <= 2^-21 |v| wherever lo stays a normal
    fp16 (|v s| >= 2^-3; the range scale puts the largest value at 2^13..2^14)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    v = torch.randn(1 << 16, device="cuda", generator=g)
    s = range_scale(v)
    _, _, v64 = split(v, s)
    rel = ((v64 - v.double()).abs() / v.double().abs().clamp_min(1e-30))
    big = (v.abs() * s) >= 2 ** -3
    assert float(rel[big].max()) <= 2.0 ** -21
    assert np.isfinite(float(rel.max()))
