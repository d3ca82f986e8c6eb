"""mfDiMP / DeT-DiMP feature path and tracker on the HIP kernels (csrc/dimpnet.hip, mmtrack_amd.dimpnet,
mmtrack_amd.dimp_tracker) vs torch fp32 on the CPU, the oracle, and the reference's own outputs
(tests/golden/dimpnet_det.npz, tracker_dimp.npz from tests/golden/make_golden_dimp.py).

Tolerances: the device path computes in fp32 (fp32 MFMA products) with a different summation order and
BatchNorm folded into the convs, so feature maps agree to ~1e-5 relative and are checked at rtol 1e-3 /
atol 1e-3 of the map's scale; integer-geometry and index work (patch crops, flips, max-pool) is exact."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import dimpnet as odn

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def close(got, ref, rel=1e-3):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-12)
    err = np.abs(got - ref).max() / scale
    assert err < rel, f"max |d| / max |ref| = {err:.2e}"


@pytest.mark.parametrize("N,C,H,W,Co,k,s,p", [(2, 3, 37, 41, 64, 7, 2, 3), (1, 64, 18, 18, 256, 1, 1, 0),
                                             (3, 128, 19, 17, 128, 3, 1, 1), (2, 128, 36, 36, 128, 3, 2, 1),
                                             (2, 256, 35, 33, 512, 1, 2, 0), (1, 1024, 18, 18, 512, 3, 1, 1),
                                             (1, 48, 9, 9, 64, 3, 1, 1),
                                             # wide layers with a ragged M
                                             (4, 256, 37, 35, 1024, 1, 1, 0), (16, 128, 48, 48, 512, 3, 2, 1)])
def test_conv2d_vs_torch(N, C, H, W, Co, k, s, p):
    from mmtrack_amd import dimpnet
    g = torch.Generator().manual_seed(N * 100 + C + k)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k)
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x, w, b, stride=s, padding=p)
    got = dimpnet.conv2d(x.cuda(), w, bias=b, stride=s, pad=p).cpu()
    close(got, ref, 1e-4)
    r = torch.randn(ref.shape, generator=g)
    got = dimpnet.conv2d(x.cuda(), w, bias=b, stride=s, pad=p, resid=r.cuda(), relu=True).cpu()
    close(got, F.relu(ref + r), 1e-4)


@pytest.mark.parametrize("N,C,H,W,Co,k,s,p", [(2, 3, 37, 41, 64, 7, 2, 3), (1, 64, 18, 18, 256, 1, 1, 0),
                                             (3, 128, 19, 17, 128, 3, 1, 1), (2, 128, 36, 36, 128, 3, 2, 1),
                                             (2, 256, 35, 33, 512, 1, 2, 0), (1, 1024, 18, 18, 512, 3, 1, 1),
                                             (1, 64, 9, 9, 64, 3, 1, 1), (4, 256, 37, 35, 1024, 1, 1, 0),
                                             (16, 128, 48, 48, 512, 3, 2, 1), (5, 3, 288, 288, 64, 7, 2, 3)])
def test_conv2d_f16x3_vs_fp64(N, C, H, W, Co, k, s, p):
    """The parity-mode conv (mmt_conv2d_f16x3: fp16 hi / lo halves of range-scaled operands, three fp16 MFMAs,
    fp32 accumulation) against float64 on the same fp32 operands: within 1e-5 of the output's scale (measured
    up to 2.3e-6 at K = 9216; the fp32 kernel's test allows 1e-4); the epilogue's sharded max|y| words hold exactly max|y| of its output,
    and a consumer that reads them (x_max) gives the bits of one given the same scale statically."""
    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    g = torch.Generator().manual_seed(N * 100 + C + k + 1)
    x = torch.randn(N, C, H, W, generator=g) * 3.0
    w = torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k)
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=p)
    words = torch.zeros(lib.mmt_conv_max_words(), device="cuda")
    got = dimpnet.conv2d(x.cuda(), w, bias=b, stride=s, pad=p, precision="f16x3", y_max=words).cpu()
    close(got, ref, 1e-5)
    assert float(words.max()) == float(got.abs().max())
    r = torch.randn(ref.shape, generator=g)
    got2 = dimpnet.conv2d(x.cuda(), w, bias=b, stride=s, pad=p, resid=r.cuda(), relu=True, precision="f16x3").cpu()
    close(got2, F.relu(ref + r.double()), 1e-5)
    # a consumer reading the producer's words: the words of max|x| (every shard) give the static scale's bits
    xw = torch.full((lib.mmt_conv_max_words(),), float(x.abs().max()), device="cuda")
    got3 = dimpnet.conv2d(x.cuda(), w, bias=b, stride=s, pad=p, precision="f16x3", x_max=xw).cpu()
    assert torch.equal(got3, got)


def _dimp_layer_inputs():
    """Every convolution of the RGB ResNet-50 to layer3 and the clf conv on the network's own activations: the fp64
    forward of oracle/dimpnet.py (seeded synthetic weights, BN folded as the HIP path folds it) of a 288 x 288 patch
    of a synthetic frame, each conv's fp64 input rounded to fp32.  Yields (name, x32, w32, stride, pad)."""
    from mmtrack_amd import synth
    sd = {k: v.double() for k, v in synth.make_dimp_state_dict(0).items()}
    frames, _ = synth.make_frames(3, 1, 480, 640, 6, box=(300.0, 200.0, 60.0, 45.0))
    im = torch.from_numpy(np.ascontiguousarray(frames[0][96:384, 176:464, :3])).permute(2, 0, 1)[None].double()
    mean = torch.tensor(odn.MEAN, dtype=torch.float64).view(1, -1, 1, 1)
    std = torch.tensor(odn.STD, dtype=torch.float64).view(1, -1, 1, 1)
    x = (im / 255 - mean) / std

    def fold(w, pre):   # conv + BN -> conv weight, bias
        sc = sd[pre + ".weight"] / torch.sqrt(sd[pre + ".running_var"] + 1e-5)
        return w * sc.view(-1, 1, 1, 1), sd[pre + ".bias"] - sd[pre + ".running_mean"] * sc

    def conv(name, x, w, b, stride, pad):
        out = F.conv2d(x, w, b, stride=stride, padding=pad)
        return out, (name, x.float(), w.float(), stride, pad)

    fe = "feature_extractor"
    res = []
    w, b = fold(sd[fe + ".conv1.weight"], fe + ".bn1")
    y, rec = conv("stem", x, w, b, 2, 3)
    res.append(rec)
    x = F.max_pool2d(F.relu(y), 3, 2, 1)
    for li, (planes, blocks, stride) in enumerate(odn.LAYERS):
        for bi in range(blocks):
            pre = f"{fe}.layer{li + 1}.{bi}"
            st = stride if bi == 0 else 1
            w, b = fold(sd[pre + ".conv1.weight"], pre + ".bn1")
            y, rec = conv(pre + ".conv1", x, w, b, 1, 0)
            res.append(rec)
            y = F.relu(y)
            w, b = fold(sd[pre + ".conv2.weight"], pre + ".bn2")
            y, rec = conv(pre + ".conv2", y, w, b, st, 1)
            res.append(rec)
            y = F.relu(y)
            w, b = fold(sd[pre + ".conv3.weight"], pre + ".bn3")
            y, rec = conv(pre + ".conv3", y, w, b, 1, 0)
            res.append(rec)
            if bi == 0:
                w, b = fold(sd[pre + ".downsample.0.weight"], pre + ".downsample.1")
                r, rec = conv(pre + ".downsample", x, w, b, st, 0)
                res.append(rec)
            else:
                r = x
            x = F.relu(y + r)
    _, rec = conv("clf", x, sd["classifier.feature_extractor.0.weight"], None, 1, 1)
    res.append(rec)
    return res


def test_conv2d_fp32_per_layer_vs_fp64():
    """precision="fp32" convolutions (conv_f32_kernel, fp32-input MFMA) layer by layer on the network's own
    activations, against float64 on the same fp32 operands, beside the parity-mode kernel and the CPU's fp32 conv
    (torch, the reference's arithmetic) on the same operands.  An fp32-input MFMA adds its four products to the
    accumulator one rounding at a time, so one accumulator per output is a K-long sequential sum (K = 9 216 for the
    clf conv): the kernel keeps four accumulator sets over interleaved K-tiles and adds them pairwise (dimpnet.hip
    CONV_F32_NACC), which brings it to the CPU's distance from float64 on every layer (DeT dimpnet.py:421-476,
    resnet.py:76-95)."""
    from mmtrack_amd import dimpnet
    rows = []
    for name, x, w, stride, pad in _dimp_layer_inputs():
        ref = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
        scale = float(ref.abs().max())
        err = lambda got: float((got.double() - ref).abs().max()) / scale
        e32 = err(dimpnet.conv2d(x.cuda(), w, stride=stride, pad=pad).cpu())
        e16 = err(dimpnet.conv2d(x.cuda(), w, stride=stride, pad=pad, precision="f16x3").cpu())
        ecpu = err(F.conv2d(x, w, stride=stride, padding=pad))
        rows.append((name, w.shape[1] * w.shape[2] * w.shape[3], e32, e16, ecpu))
    for name, K, e32, e16, ecpu in rows:
        print(f"{name:40s} K {K:5d}  fp32 {e32:.2e}  f16x3 {e16:.2e}  cpu-fp32 {ecpu:.2e}")
    for name, K, e32, e16, ecpu in rows:
        assert e32 < 1e-5, (name, e32)
        assert e16 < 1e-5, (name, e16)
        # (one accumulator set: up to 2.85e-6 on the clf conv and above the parity-mode kernel on 30 of 44 layers;
        # four: 1.33e-6, at or below it on every layer -- profiles/r06_dimp_fp32_per_layer.txt)
        assert e32 <= 1.1 * max(ecpu, e16), (name, e32, ecpu, e16)


def test_conv_kernels_bitwise(tmp_path):
    """The f16x3 conv kernels against each other (tests/conv_dump.py, one child process per setting: the knobs are
    read once per process): the deep-pipelined generic kernel (conv_f16x3_deep_kernel: three or two register sets,
    the default three-set kernel with the next K-tile's split woven into the MFMAs, 256-pixel tiles) gives the bits
    of the two-deep conv_f16x3_kernel (same products, same summation order) -- split-K launches too, except where
    256-pixel tiles pick another K split (within 1e-5 then); the 3 x 3 patch kernel (another summation order)
    agrees with them within 1e-5 of the output scale."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for mode, extra in (("old", {"MMT_CONV_OLD": "1", "MMT_CONV_NOPATCH": "1"}),
                        ("deep3", {"MMT_CONV_NR": "3", "MMT_CONV_OVL": "0", "MMT_CONV_NOPATCH": "1"}),
                        ("deep2", {"MMT_CONV_OVL": "0", "MMT_CONV_NOPATCH": "1"}),
                        ("bm256", {"MMT_CONV_BM": "256", "MMT_CONV_NOPATCH": "1"}),
                        ("ovl", {"MMT_CONV_NOPATCH": "1"}), ("patch", {})):
        env = {k: v for k, v in os.environ.items() if not k.startswith("MMT_CONV_")}
        env.update(extra)
        path = str(tmp_path / f"{mode}.npz")
        r = subprocess.run([sys.executable, os.path.join(here, "conv_dump.py"), path], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        res[mode] = np.load(path)
    for mode in ("deep3", "deep2", "ovl"):
        for key in res["old"].files:
            np.testing.assert_array_equal(res[mode][key], res["old"][key], err_msg=f"{mode} {key}")
    for key in res["old"].files:
        close(res["patch"][key], res["old"][key], 1e-5)
        # 256-pixel tiles: same products and order per output (bit-identical) unless fewer tiles pick another K split
        if key.startswith("y"):
            np.testing.assert_array_equal(res["bm256"][key], res["old"][key], err_msg=f"bm256 {key}")
        else:
            close(res["bm256"][key], res["old"][key], 1e-5)


@pytest.mark.parametrize("N,C,H,W,Co,k,s,p", [(1, 1024, 18, 18, 256, 3, 1, 1), (2, 1024, 18, 18, 512, 3, 1, 1),
                                             (3, 512, 18, 18, 256, 1, 1, 0), (1, 256, 35, 33, 128, 3, 2, 1)])
def test_conv2d_f16x3_groups_and_splitk(N, C, H, W, Co, k, s, p):
    """The grouped launch (the two backbones' twin layers, mmt_conv2d_f16x3_groups) with its K split in slices
    (few output tiles): each group's output against float64 within 1e-5 of its scale, each group's max words
    exactly its max|y|, split vs unsplit within 1e-5 (the slices change the fp32 summation order), and a
    split launch that max-merges into an existing map (MMT_CONV_MAX in the slice-reduce kernel)."""
    import ctypes
    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    assert lib.mmt_conv2d_f16x3_ws_bytes(N, H, W, C, Co, k, k, s, p, 2) > 0, "shape expected to split"
    g = torch.Generator().manual_seed(N * 7 + C + Co + k)
    xs = [torch.randn(N, C, H, W, generator=g) * (1.0 + 2 * i) for i in range(2)]
    ws = [torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k) for _ in range(2)]
    bs = [torch.randn(Co, generator=g) * 0.1 for _ in range(2)]
    convs = [dimpnet._Conv(ws[i], bias=bs[i], stride=s, pad=p, dev="cuda", f16x3=True) for i in range(2)]
    Ho, Wo = convs[0].out_hw(H, W)
    refs = [F.conv2d(xs[i].double(), ws[i].double(), bs[i].double(), stride=s, padding=p) for i in range(2)]
    rs = [torch.randn(refs[0].shape, generator=g) for _ in range(2)]
    xd = [x.permute(0, 2, 3, 1).contiguous().cuda() for x in xs]
    rd = [r.permute(0, 2, 3, 1).contiguous().cuda() for r in rs]
    outs = [torch.empty(N, Ho, Wo, Co, device="cuda") for _ in range(2)]
    words = [torch.zeros(lib.mmt_conv_max_words(), device="cuda") for _ in range(2)]
    groups = [convs[i].group(xd[i], outs[i], relu=True, resid=rd[i], x_scale=dimpnet.range_scale(float(xs[i].abs().max())),
                             y_max=words[i]) for i in range(2)]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    wsf = lambda n: torch.empty((n + 3) // 4, device="cuda")
    dimpnet.run_f16x3(lib, convs[0], groups, N, H, W, wsf, stream)
    for i in range(2):
        got = outs[i].permute(0, 3, 1, 2).cpu()
        close(got, F.relu(refs[i] + rs[i].double()), 1e-5)
        assert float(words[i].max()) == float(got.abs().max())
    # the same conv split and unsplit
    one = dimpnet.conv2d(xs[0].cuda(), ws[0], bias=bs[0], stride=s, pad=p, precision="f16x3").cpu()
    spl = dimpnet.conv2d(xs[0].cuda(), ws[0], bias=bs[0], stride=s, pad=p, precision="f16x3", split=True).cpu()
    close(spl, refs[0], 1e-5)
    close(one, spl, 1e-5)
    # a split launch max-merging into group 0's map
    base = outs[0].clone()
    merged = dimpnet.conv2d(xs[1].cuda(), ws[1], bias=bs[1], stride=s, pad=p, precision="f16x3", split=True,
                            merge_into=base).cpu()
    close(merged, torch.maximum(F.relu(refs[0] + rs[0].double()), refs[1]), 1e-5)
    # twin layers writing the same output, or merging, are refused
    bad = (_lib.MmtConvGroup * 2)(groups[0], groups[0])
    assert lib.mmt_conv2d_f16x3_groups(bad, 2, N, H, W, C, convs[0].kp, Co, k, k, s, p, None, 0, stream) == -1


@pytest.mark.parametrize("N,Cin3,Cin2,H2,W2,Co,s2,G", [(3, 64, 64, 18, 18, 256, 1, 2), (2, 128, 256, 36, 36, 512, 2, 2),
                                                     (1, 256, 512, 35, 33, 1024, 2, 1), (32, 64, 64, 18, 18, 256, 1, 2)])
def test_conv2d_f16x3_fused_downsample(N, Cin3, Cin2, H2, W2, Co, s2, G):
    """conv3 + the block's downsample as one GEMM over concatenated K (mmt_conv2d_f16x3_ds_groups, resnet.py:76-95):
    relu(conv3(b) + b3 + downsample(x2) + b_d) against float64 within 1e-5 of the output's scale for each of G
    groups (their own inputs of different ranges, so the two sources' scales differ), split-K shapes included; the
    max words hold exactly max|y|; a residual operand, a wrong Kp and an inconsistent strided geometry are refused."""
    import ctypes
    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    g = torch.Generator().manual_seed(N + Cin3 + Cin2 + Co + s2)
    H, W = (H2 - 1) // s2 + 1, (W2 - 1) // s2 + 1
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    w3 = torch.randn(Co, Cin3, 1, 1, generator=g) / math.sqrt(Cin3)
    wd = torch.randn(Co, Cin2, 1, 1, generator=g) / math.sqrt(Cin2) * 3.0
    b3, bd = torch.randn(Co, generator=g) * 0.1, torch.randn(Co, generator=g) * 0.1
    fu = dimpnet._ConvDs(dimpnet._Conv(w3, bias=b3, dev="cuda", f16x3=True),
                         dimpnet._Conv(wd, bias=bd, stride=s2, dev="cuda", f16x3=True), "cuda")
    nw = lib.mmt_conv_max_words()
    groups, ds, outs, words, refs, keep = [], [], [], [], [], []
    for i in range(G):
        b = torch.relu(torch.randn(N, Cin3, H, W, generator=g)) * (1.0 + i)
        x2 = torch.relu(torch.randn(N, Cin2, H2, W2, generator=g)) * (4.0 - i)
        refs.append(F.relu(F.conv2d(b.double(), w3.double(), b3.double())
                           + F.conv2d(x2.double(), wd.double(), bd.double(), stride=s2)))
        bdev, xdev = b.permute(0, 2, 3, 1).contiguous().cuda(), x2.permute(0, 2, 3, 1).contiguous().cuda()
        bm = torch.full((nw,), float(b.abs().max()), device="cuda")
        xm = torch.full((nw,), float(x2.abs().max()), device="cuda")
        outs.append(torch.empty(N, H, W, Co, device="cuda"))
        words.append(torch.zeros(nw, device="cuda"))
        groups.append(fu.group(bdev, outs[i], x_max=bm, y_max=words[i]))
        ds.append((xdev, xm))
        keep += [bdev, bm]
    fu.run(lib, groups, ds, N, H, W, H2, W2, lambda n: torch.empty((n + 3) // 4, device="cuda"), stream)
    for i in range(G):
        got = outs[i].permute(0, 3, 1, 2).cpu()
        close(got, refs[i], 1e-5)
        assert float(words[i].max()) == float(got.abs().max())
    arr = (_lib.MmtConvGroup * 1)(groups[0])
    darr = (_lib.MmtConvDs * 1)(_lib.MmtConvDs(ds[0][0].data_ptr(), ds[0][1].data_ptr(), 0.0))
    call = lambda h, kp: lib.mmt_conv2d_f16x3_ds_groups(arr, darr, 1, N, h, W, Cin3, H2, W2, Cin2, s2, kp, Co, None, 0,
                                                        stream)
    assert call(H, fu.kp + 32) == -1 and call(H + 1, fu.kp) == -1
    r = torch.zeros(N, H, W, Co, device="cuda")
    arr[0].resid = r.data_ptr()
    assert call(H, fu.kp) == -1


def test_conv2d_f16x3_stem_padded_input_bitwise():
    """The f16x3 stem over the image padded to 4 channels (mmt_image_normalize4 layout, one 16-B load per tap)
    gives the bits of the stem over the 3-channel image (the same K order, the pad channel's weight is 0)."""
    import ctypes
    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    g = torch.Generator().manual_seed(17)
    x = torch.randn(3, 3, 75, 61, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) / math.sqrt(147)
    b = torch.randn(64, generator=g) * 0.1
    conv = dimpnet._Conv(w, bias=b, stride=2, pad=3, dev="cuda", f16x3=True)
    Ho, Wo = conv.out_hw(75, 61)
    x3 = x.permute(0, 2, 3, 1).contiguous().cuda()
    x4 = torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 1)).contiguous().cuda()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for xi, cin in ((x3, 3), (x4, 4)):
        out = torch.empty(3, Ho, Wo, 64, device="cuda")
        dimpnet.run_f16x3(lib, conv, [conv.group(xi, out, relu=True, x_scale=dimpnet.range_scale(float(x.abs().max())))],
                          3, 75, 61, None, stream, cin=cin)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    close(outs[0].permute(0, 3, 1, 2), F.relu(F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=3)), 1e-5)
    # the padded normalisation: the first three channels of each pixel as mmt_image_normalize, the fourth 0
    im = (torch.rand(2, 6, 20, 24, generator=g) * 255).cuda()
    mean = (ctypes.c_float * 3)(*dimpnet.MEAN)
    std = (ctypes.c_float * 3)(*dimpnet.STD)
    a3, b3 = torch.empty(2, 20, 24, 3, device="cuda"), torch.empty(2, 20, 24, 3, device="cuda")
    a4, b4 = torch.full((2, 20, 24, 4), 7.0, device="cuda"), torch.full((2, 20, 24, 4), 7.0, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    assert lib.mmt_image_normalize(P(im), 2, 6, 20, 24, mean, std, P(a3), P(b3), stream) == 0
    assert lib.mmt_image_normalize4(P(im), 2, 6, 20, 24, mean, std, P(a4), P(b4), stream) == 0
    assert torch.equal(a4[..., :3], a3) and torch.equal(b4[..., :3], b3)
    assert float(a4[..., 3].abs().max()) == 0.0 and float(b4[..., 3].abs().max()) == 0.0


@pytest.mark.parametrize("N,H,W", [(3, 75, 61), (2, 288, 288), (1, 33, 50)])
def test_conv2d_f16x3_stem_pool_bitwise(N, H, W):
    """The stem with the 3 x 3 / stride-2 / pad-1 max-pool fused (MMT_CONV_POOL, conv_stem_pool_f16x3_kernel: 8 x 8
    pooled tiles over 17 x 17 stem tiles) gives the bits of the stem kernel followed by mmt_maxpool2d_f32, for both
    groups of a grouped launch, and the same max|y| (max over the sharded words); launches it does not cover are
    refused."""
    import ctypes
    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    g = torch.Generator().manual_seed(N * 1000 + H)
    convs, xs = [], []
    for k in range(2):
        w = torch.randn(64, 3, 7, 7, generator=g) / math.sqrt(147)
        b = torch.randn(64, generator=g) * 0.1
        convs.append(dimpnet._Conv(w, bias=b, stride=2, pad=3, dev="cuda", f16x3=True))
        x = torch.randn(N, 3, H, W, generator=g) * (1 + k)
        xs.append(torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 1)).contiguous().cuda())
    Ho, Wo = convs[0].out_hw(H, W)
    PHo, PWo = (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    MW = lib.mmt_conv_max_words()
    words = torch.zeros(4, MW, device="cuda")
    scale = dimpnet.range_scale(6.0)
    full = [torch.empty(N, Ho, Wo, 64, device="cuda") for _ in range(2)]
    ref = [torch.empty(N, PHo, PWo, 64, device="cuda") for _ in range(2)]
    dimpnet.run_f16x3(lib, convs[0], [c.group(x, y, relu=True, x_scale=scale, y_max=words[k])
                                      for k, (c, x, y) in enumerate(zip(convs, xs, full))], N, H, W, None, stream, cin=4)
    for y, r in zip(full, ref):
        assert lib.mmt_maxpool2d_f32(ctypes.c_void_p(y.data_ptr()), N, Ho, Wo, 64, 3, 2, 1, ctypes.c_void_p(r.data_ptr()),
                                     stream) == 0
    got = [torch.full((N, PHo, PWo, 64), float("nan"), device="cuda") for _ in range(2)]
    dimpnet.run_f16x3(lib, convs[0], [c.group(x, y, relu=True, x_scale=scale, y_max=words[2 + k], pool=True)
                                      for k, (c, x, y) in enumerate(zip(convs, xs, got))], N, H, W, None, stream, cin=4)
    torch.cuda.synchronize()
    for k in range(2):
        assert torch.equal(got[k], ref[k]), f"group {k}: max |diff| {float((got[k] - ref[k]).abs().max())}"
        assert float(words[2 + k].max()) == float(words[k].max()) == float(full[k].abs().max())
    # refused: the pool with a MAX merge, on another conv shape, or set on one group only
    gr = [c.group(x, y, relu=True, x_scale=scale, pool=True) for c, x, y in zip(convs, xs, got)]
    bad = convs[0].group(xs[0], got[0], relu=True, merge_max=True, x_scale=scale, pool=True)
    arr = (_lib.MmtConvGroup * 1)(bad)
    assert lib.mmt_conv2d_f16x3_groups(arr, 1, N, H, W, 4, convs[0].kp, 64, 7, 7, 2, 3, None, 0, stream) == -1
    arr = (_lib.MmtConvGroup * 2)(gr[0], convs[1].group(xs[1], got[1], relu=True, x_scale=scale))
    assert lib.mmt_conv2d_f16x3_groups(arr, 2, N, H, W, 4, convs[0].kp, 64, 7, 7, 2, 3, None, 0, stream) == -1
    arr = (_lib.MmtConvGroup * 1)(gr[0])
    assert lib.mmt_conv2d_f16x3_groups(arr, 1, N, H, W, 4, convs[0].kp, 64, 7, 7, 1, 3, None, 0, stream) == -1
    # ... and operands the pooled kernel would drop: a MAX merge on the second group only, a residual on either
    bad1 = convs[1].group(xs[1], got[1], relu=True, merge_max=True, x_scale=scale, pool=True)
    arr = (_lib.MmtConvGroup * 2)(gr[0], bad1)
    assert lib.mmt_conv2d_f16x3_groups(arr, 2, N, H, W, 4, convs[0].kp, 64, 7, 7, 2, 3, None, 0, stream) == -1
    for k in range(2):
        pair = list(gr)
        pair[k] = convs[k].group(xs[k], got[k], relu=True, resid=full[k], x_scale=scale, pool=True)
        arr = (_lib.MmtConvGroup * 2)(*pair)
        assert lib.mmt_conv2d_f16x3_groups(arr, 2, N, H, W, 4, convs[0].kp, 64, 7, 7, 2, 3, None, 0, stream) == -1


def test_conv2d_stem_w4():
    """The 3-channel stem through MMT_CONV_W4 (weights padded to 4 channels per tap) and through the generic
    per-element path agree with torch and each other (summation orders differ: fp32 rounding)."""
    from mmtrack_amd import dimpnet
    g = torch.Generator().manual_seed(7)
    x = torch.randn(3, 3, 75, 61, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) / math.sqrt(147)
    b = torch.randn(64, generator=g) * 0.1
    ref = F.conv2d(x, w, b, stride=2, padding=3)
    got4 = dimpnet.conv2d(x.cuda(), w, bias=b, stride=2, pad=3, relu=False, w4=True).cpu()
    gotg = dimpnet.conv2d(x.cuda(), w, bias=b, stride=2, pad=3, relu=False, w4=False).cpu()
    close(got4, ref, 1e-5)
    close(gotg, ref, 1e-5)
    close(got4, gotg, 1e-5)


def test_conv2d_max_merge_and_errors():
    import ctypes

    from mmtrack_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 8, 8, 16, generator=g).cuda()
    w = torch.randn(64, 1, 1, 16, generator=g).cuda()
    y = torch.randn(64, 64, generator=g).cuda()
    y0 = y.clone()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.mmt_conv2d_f32(ctypes.c_void_p(x.data_ptr()), 1, 8, 8, 16, ctypes.c_void_p(w.data_ptr()), None, 64, 1, 1,
                              1, 0, None, ctypes.c_void_p(y.data_ptr()), 2, s) == 0
    conv = (x.reshape(64, 16) @ w.reshape(64, 16).t())
    close(y.cpu(), torch.max(y0, conv).cpu(), 1e-5)
    assert lib.mmt_conv2d_f32(ctypes.c_void_p(x.data_ptr()), 1, 8, 8, 16, ctypes.c_void_p(w.data_ptr()), None, 48, 1, 1,
                              1, 0, None, ctypes.c_void_p(y.data_ptr()), 0, s) == -1   # Cout % 64


def test_maxpool_l2norm_prroi():
    import ctypes

    from mmtrack_amd import _lib, dimpnet
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 64, 37, 29, generator=g)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda()
    y = torch.empty(2, 19, 15, 64, device="cuda")
    assert lib.mmt_maxpool2d_f32(ctypes.c_void_p(xd.data_ptr()), 2, 37, 29, 64, 3, 2, 1, ctypes.c_void_p(y.data_ptr()),
                                 s) == 0
    np.testing.assert_array_equal(y.permute(0, 3, 1, 2).cpu().numpy(), F.max_pool2d(x, 3, 2, 1).numpy())
    # InstanceL2Norm
    f = torch.randn(3, 512, 18, 18, generator=g)
    fd = f.permute(0, 2, 3, 1).contiguous().cuda()
    o_nchw = torch.empty(3, 512, 18, 18, device="cuda")
    o_nhwc = torch.empty(3, 18, 18, 512, device="cuda")
    sc = math.sqrt(1.0 / (512 * 16))
    l2ws = torch.empty(lib.mmt_instance_l2norm_ws_bytes(3, 18, 18) // 4, device="cuda")
    assert lib.mmt_instance_l2norm(ctypes.c_void_p(fd.data_ptr()), 3, 18, 18, 512, sc, 1e-5,
                                   ctypes.c_void_p(o_nhwc.data_ptr()), ctypes.c_void_p(o_nchw.data_ptr()),
                                   ctypes.c_void_p(l2ws.data_ptr()), s) == 0
    ref = odn.instance_l2norm(f, sc)
    close(o_nchw.cpu(), ref, 1e-5)
    close(o_nhwc.permute(0, 3, 1, 2).cpu(), ref, 1e-5)
    # PrRoIPool (restated CUDA forward), boxes inside, across and outside the map
    feat = torch.randn(3, 32, 18, 18, generator=g)
    boxes = torch.tensor([[40.0, 52.5, 130.0, 150.0], [-20.0, 200.0, 90.0, 330.0], [100.0, 100.0, 100.0, 140.0]])
    got = dimpnet.prroi_pool(feat.cuda(), boxes, 1 / 16, 4, 4).cpu()
    rois = torch.cat([torch.arange(3.0).view(-1, 1), boxes], 1)
    close(got, odn.prroi_pool(feat, rois, 1 / 16, 4, 4), 1e-5)


@pytest.mark.parametrize("pos,sample,out,HW", [((180.0, 240.0), (288.0, 288.0), (288, 288), (360, 480)),
                                               ((30.4, 460.9), (700.0, 700.0), (288, 288), (360, 480)),
                                               ((200.0, 100.0), (1100.0, 1100.0), (576, 576), (360, 480)),
                                               ((10.0, 10.0), (130.5, 95.0), (288, 288), (120, 90))])
def test_sample_patch_vs_reference_algorithm(pos, sample, out, HW):
    from mmtrack_amd import dimpnet
    rng = np.random.default_rng(5)
    frame = rng.integers(0, 256, (HW[0], HW[1], 6), dtype=np.uint8)
    pos_t, ss, os_ = torch.Tensor(pos), torch.Tensor(sample), torch.Tensor(out)
    im = torch.from_numpy(frame).float().permute(2, 0, 1)[None]
    ref, coord = odn.sample_patch(im, pos_t, ss, os_)
    geom = odn.patch_geometry(HW, pos_t, ss, os_)
    got = dimpnet.sample_patch_device(torch.from_numpy(frame).cuda(), geom, out).cpu()
    # ATen's CPU bilinear kernel is built with FMA contraction; the device restates it with fmaf at the same
    # places, so pixels agree to a few ulp of 255 (atol 2e-3 leaves room for the vectorised CPU path)
    err = np.abs(got.numpy() - ref.numpy()).max()
    print("sample_patch max |d|", err)
    assert err < 2e-3


def test_patch_transforms_vs_reference_ops():
    from mmtrack_amd import dimpnet
    from mmtrack_amd.dimp_tracker import _Tf
    g = torch.Generator().manual_seed(6)
    img = torch.rand(1, 6, 96, 96, generator=g) * 255
    out = (48, 48)

    def crop(im, shift):
        top, left = math.floor((48 - 96) / 2) + shift[0], math.floor((48 - 96) / 2) + shift[1]
        return F.pad(im, (left, math.ceil((48 - 96) / 2) - shift[1], top, math.ceil((48 - 96) / 2) - shift[0]),
                     'replicate')
    for shift in ((0, 0), (20, -31), (-40, 50)):
        t = _Tf(0, out, shift).c_struct((96, 96))
        np.testing.assert_array_equal(dimpnet.patch_transform_device(img.cuda(), t, out).cpu().numpy(),
                                      crop(img, shift).numpy())
        t = _Tf(1, out, shift).c_struct((96, 96))
        np.testing.assert_array_equal(dimpnet.patch_transform_device(img.cuda(), t, out).cpu().numpy(),
                                      crop(img.flip((3,)), shift).numpy())
    for sig in ((3, 1), (1, 3), (2, 2)):   # augmentation.py Blur: vertical then horizontal zero-padded conv
        fs = [math.ceil(2 * s) for s in sig]
        taps = [torch.exp(-(torch.arange(-z, z + 1, dtype=torch.float32) ** 2) / (2 * s ** 2)) for z, s in zip(fs, sig)]
        f0 = (taps[0] / taps[0].sum()).view(1, 1, -1, 1)
        f1 = (taps[1] / taps[1].sum()).view(1, 1, 1, -1)
        im1 = F.conv2d(img.view(-1, 1, 96, 96), f0, padding=(fs[0], 0))
        ref = crop(F.conv2d(im1, f1, padding=(0, fs[1])).view(1, -1, 96, 96), (3, -2))
        t = _Tf(2, out, (3, -2), sigma=sig).c_struct((96, 96))
        close(dimpnet.patch_transform_device(img.cuda(), t, out).cpu(), ref, 1e-5)
    for ang in (10, -45):   # Rotate: cv2.warpAffine restatement (unpinned: no OpenCV here)
        a = math.pi * ang / 180
        c = (np.array([[96.0], [96.0]]) - 1) / 2
        R = np.array([[math.cos(a), math.sin(a)], [-math.sin(a), math.cos(a)]])
        H = np.concatenate([R, c - R @ c], 1)
        rot = odn.warp_affine_replicate(img[0].permute(1, 2, 0).numpy(), H, (96, 96))
        ref = crop(torch.from_numpy(rot).permute(2, 0, 1)[None], (5, 7))
        t = _Tf(3, out, (5, 7), angle=ang).c_struct((96, 96))
        close(dimpnet.patch_transform_device(img.cuda(), t, out).cpu(), ref, 1e-5)


@pytest.fixture(scope="module")
def nets():
    from mmtrack_amd import synth
    from mmtrack_amd.dimpnet import DiMPNet
    sd = synth.make_dimp_state_dict(0)
    return {p: DiMPNet(sd, precision=p) for p in ("f16x3", "fp32")}


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_dimpnet_matches_reference_golden(nets, precision):
    """Both precisions against the reference DiMPnet_DeT outputs (layer3, clf features, initial filter, scores)
    at 1e-3 of each map's scale."""
    from mmtrack_amd import synth
    net = nets[precision]
    gd = np.load(os.path.join(GOLDEN, "dimpnet_det.npz"))
    ims = torch.stack([torch.from_numpy(synth.make_patch(int(s), 288, 6)).float().permute(2, 0, 1)
                       for s in gd["seeds"]]).cuda()
    l3 = net.extract_backbone(ims)
    l3n = l3.permute(0, 3, 1, 2).cpu()
    np.testing.assert_allclose(l3n.double().sum(dim=(1, 2, 3)).numpy(), gd["layer3_sum"], rtol=1e-4)
    close(l3n[:, ::32], gd["layer3_ch"])
    clf, clf_nhwc = net.extract_classification_feat(l3, nhwc=True)
    close(clf.cpu()[:, ::8], gd["clf_ch"])
    filt = net.init_filter(clf_nhwc, torch.from_numpy(gd["boxes"]))
    close(filt.cpu(), gd["init_filter"])
    close(net.classify(filt, clf).cpu(), gd["scores"])


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_dimp_tracker_matches_reference_sequence(precision):
    """The reference DiMP tracker (DeT_DiMP50_Max parameters, use_iou_net False, torch.manual_seed before
    initialize) on a 24-frame synthetic RGB-D sequence: per-frame boxes IoU >= 0.999, identical
    localisation flags, confidences within the derived bar (tests/dimp_tolerance.py: 2 x the reference's own
    confidence spread under fp32-order feature differences -- a score element of the 10-step Gauss-Newton init
    sits 2e-6 of the maximum from LeakyReluPar's kink, so ~1e-5 feature differences move the filter by ~1e-3);
    24 frames cover init with 15 augmented samples, per-frame memory updates and the frame-21 Gauss-Newton update)."""
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, parameters
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp.npz"))
    seed, n, H, W, C, tseed = [int(v) for v in gd["meta"]]
    frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(gd["init_box"]))
    from mmtrack_amd.dimpnet import DiMPNet
    tr = DiMP(parameters(), net=DiMPNet(synth.make_dimp_state_dict(0), precision=precision))
    torch.manual_seed(tseed)
    tr.initialize(frames[0], {"init_bbox": list(gd["init_box"])})
    close(tr.target_filter.cpu(), gd["init_filter"], 1e-2)
    from tests.dimp_tolerance import confidence_bar, reference_spread
    bar = confidence_bar()
    dconf = []
    for t in range(1, n):
        out = tr.track(frames[t])
        b, r = out["target_bbox"], gd["boxes"][t]
        ix = max(0.0, min(b[0] + b[2], r[0] + r[2]) - max(b[0], r[0]))
        iy = max(0.0, min(b[1] + b[3], r[1] + r[3]) - max(b[1], r[1]))
        iou = ix * iy / (b[2] * b[3] + r[2] * r[3] - ix * iy)
        assert tr.debug_info["flag"] == str(gd["flags"][t]), (t, tr.debug_info["flag"], gd["flags"][t])
        assert iou >= 0.999, (t, b, r.tolist())
        dconf.append(abs(out["confidence"] - gd["confidence"][t]) / gd["confidence"][t])
        assert dconf[-1] < bar, (t, out["confidence"], gd["confidence"][t], bar)
    print("relative confidence differences per frame:", np.round(dconf, 5).tolist(),
          f"bar {bar:.2e} (2 x the reference's fp32-order spread {reference_spread()})")


def test_fused_sampler_bits():
    """The pools' normalising sampler (mmt_dimp_track_sample_norm4: the 6-channel patch written as the two
    normalised 4-channel halves the f16x3 backbones read) against the NCHW patch + mmt_image_normalize4 path: the
    tracker_dimp.npz sequence tracked both ways gives identical boxes, confidences and flags, bit for bit."""
    from mmtrack_amd import dimp_tracker as mdt
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, parameters
    from mmtrack_amd.dimpnet import DiMPNet
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp.npz"))
    seed, n, H, W, C, tseed = [int(v) for v in gd["meta"]]
    frames, _ = synth.make_frames(seed, 8, H, W, C, box=tuple(gd["init_box"]))
    net = DiMPNet(synth.make_dimp_state_dict(0), precision="f16x3")
    runs = []
    try:
        for fused in (True, False):
            mdt.FUSED_SAMPLE = fused
            tr = DiMP(parameters(), net=net)
            torch.manual_seed(tseed)
            tr.initialize(frames[0], {"init_bbox": list(gd["init_box"])})
            out = []
            for t in range(1, 8):
                o = tr.track(frames[t])
                out.append((list(o["target_bbox"]), o["confidence"], tr.debug_info["flag"]))
            runs.append(out)
    finally:
        mdt.FUSED_SAMPLE = True
    assert runs[0] == runs[1]


@pytest.mark.parametrize("groups", [1, 2])
def test_pipelined_batch_equals_sequential(groups):
    """PipelinedBatch (the host one frame behind the device; the filter updates decided on the device) gives
    every sequence the results of tracking it alone with DiMP.track, over enough frames for the scheduled
    Gauss-Newton updates (within 1e-3 px: a batch's convs may split K differently from a single image's)."""
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, PipelinedBatch, parameters
    from mmtrack_amd.dimpnet import DiMPNet
    net = DiMPNet(synth.make_dimp_state_dict(0))
    nf = 24
    seqs = [synth.make_frames(70 + i, nf, 360, 480, 6, box=(150.0 + 20 * i, 120.0, 44.0, 36.0)) for i in range(3)]
    pool = DimpPool(net, 3, parameters())

    def fresh(i, batched=False):
        t = DiMP(parameters(), net=net, pool=pool if batched else None)
        torch.manual_seed(100 + i)
        t.initialize(seqs[i][0][0], {"init_bbox": list(seqs[i][1][0])})
        return t
    ref = []
    for i in range(3):
        t = fresh(i)
        ref.append([t.track(seqs[i][0][k])["target_bbox"] for k in range(1, nf)])
    trs = [fresh(i, batched=True) for i in range(3)]
    pipe = PipelinedBatch(trs, groups=groups)
    got = [[] for _ in range(3)]
    for k in range(1, nf):
        outs = pipe.step([seqs[i][0][k] for i in range(3)])
        if outs is not None:
            for i in range(3):
                got[i].append(outs[i]["target_bbox"])
    for i, o in enumerate(pipe.flush()):
        got[i].append(o["target_bbox"])
    for i in range(3):
        np.testing.assert_allclose(np.array(got[i]), np.array(ref[i]), rtol=0, atol=1e-3)
