"""Seeded synthetic weights and frames for the ViPT / OSTrack tracking path.

No checkpoint of the reference ships (``*.pth`` is git-ignored, reference
``.gitignore:19-20``; ViPT expects ``models/ViPT_<yaml>.pth``,
``ViPT/lib/test/parameter/vipt.py:25``), so every test, the bench and the
golden-fixture generator build weights from the same portable law:

* the key / shape list is the reference ``state_dict`` layout
  (``ViPT/lib/models/vipt/ostrack_prompt.py:94-145`` for ViPT,
  ``ViPT/lib/models/vipt/ostrack.py:95-144`` for OSTrack),
* every tensor is drawn from ``torch.Generator`` (CPU mt19937, identical on
  every host running this image) seeded with ``seed ^ crc32(key)``.

The law is chosen so the random network behaves like a trained one in the
ways the parity tests care about: peaked attention (so candidate elimination
is decided by clear margins), a score map with a distinct peak, and sizes
away from the sigmoid's saturation.

Frames are H x W x C uint8 (RGB + aux), smooth backgrounds plus a bright
moving target, from numpy's PCG64 (portable across hosts).
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import numpy as np
import torch

EMBED = 768
DEPTH = 12
HEADS = 12
MLP = 3072
PATCH = 16


def model_shapes(kind: str = "vipt", prompt_type: str = "vipt_deep", search_size: int = 256,
                 template_size: int = 128, head_channels: int = 256, in_chans: int = 3) -> "OrderedDict[str, tuple]":
    """Reference ``state_dict`` keys and shapes.

    kind == "vipt": ``VisionTransformerCE`` of ``vit_ce_prompt.py:84-182`` (+ the
    leftover ``cls_token`` / 197-row ``pos_embed`` of ``vit.py:137-139``).
    kind == "ostrack": ``VisionTransformerCE`` of ``vit_ce.py:21-100`` with the
    ``pos_embed_z/x`` parameters that ``finetune_track`` adds
    (``base_backbone.py:92-93``).
    """
    s = OrderedDict()
    lz = (template_size // PATCH) ** 2
    lx = (search_size // PATCH) ** 2
    s["backbone.cls_token"] = (1, 1, EMBED)
    s["backbone.pos_embed"] = (1, 197, EMBED)
    if kind == "vipt":
        s["backbone.pos_embed_z"] = (1, lz, EMBED)
        s["backbone.pos_embed_x"] = (1, lx, EMBED)
    s["backbone.patch_embed.proj.weight"] = (EMBED, in_chans, PATCH, PATCH)
    s["backbone.patch_embed.proj.bias"] = (EMBED,)
    if kind == "vipt":
        s["backbone.patch_embed_prompt.proj.weight"] = (EMBED, in_chans, PATCH, PATCH)
        s["backbone.patch_embed_prompt.proj.bias"] = (EMBED,)
        nprompt = DEPTH if prompt_type == "vipt_deep" else 1
        for i in range(nprompt):
            p = f"backbone.prompt_blocks.{i}."
            s[p + "conv0_0.weight"] = (8, EMBED, 1, 1)
            s[p + "conv0_0.bias"] = (8,)
            s[p + "conv0_1.weight"] = (8, EMBED, 1, 1)
            s[p + "conv0_1.bias"] = (8,)
            s[p + "conv1x1.weight"] = (EMBED, 8, 1, 1)
            s[p + "conv1x1.bias"] = (EMBED,)
            s[p + "fovea.smooth"] = (1,)
        for i in range(nprompt):
            s[f"backbone.prompt_norms.{i}.weight"] = (EMBED,)
            s[f"backbone.prompt_norms.{i}.bias"] = (EMBED,)
    for i in range(DEPTH):
        p = f"backbone.blocks.{i}."
        s[p + "norm1.weight"] = (EMBED,)
        s[p + "norm1.bias"] = (EMBED,)
        s[p + "attn.qkv.weight"] = (3 * EMBED, EMBED)
        s[p + "attn.qkv.bias"] = (3 * EMBED,)
        s[p + "attn.proj.weight"] = (EMBED, EMBED)
        s[p + "attn.proj.bias"] = (EMBED,)
        s[p + "norm2.weight"] = (EMBED,)
        s[p + "norm2.bias"] = (EMBED,)
        s[p + "mlp.fc1.weight"] = (MLP, EMBED)
        s[p + "mlp.fc1.bias"] = (MLP,)
        s[p + "mlp.fc2.weight"] = (EMBED, MLP)
        s[p + "mlp.fc2.bias"] = (EMBED,)
    s["backbone.norm.weight"] = (EMBED,)
    s["backbone.norm.bias"] = (EMBED,)
    if kind == "ostrack":
        s["backbone.pos_embed_z"] = (1, lz, EMBED)
        s["backbone.pos_embed_x"] = (1, lx, EMBED)
    ch = [EMBED, head_channels, head_channels // 2, head_channels // 4, head_channels // 8]
    for br in ("ctr", "offset", "size"):
        for j in range(1, 5):
            p = f"box_head.conv{j}_{br}."
            s[p + "0.weight"] = (ch[j], ch[j - 1], 3, 3)
            s[p + "0.bias"] = (ch[j],)
            s[p + "1.weight"] = (ch[j],)
            s[p + "1.bias"] = (ch[j],)
            s[p + "1.running_mean"] = (ch[j],)
            s[p + "1.running_var"] = (ch[j],)
            s[p + "1.num_batches_tracked"] = ()
    # conv5 comes after all conv1..4 of a branch in the module order of head.py:106-124
    out = OrderedDict()
    for k, v in s.items():
        out[k] = v
    ordered = OrderedDict()
    for k, v in out.items():
        if not k.startswith("box_head"):
            ordered[k] = v
    for br, n5 in (("ctr", 1), ("offset", 2), ("size", 2)):
        for j in range(1, 5):
            for k, v in out.items():
                if k.startswith(f"box_head.conv{j}_{br}."):
                    ordered[k] = v
        ordered[f"box_head.conv5_{br}.weight"] = (n5, ch[4], 1, 1)
        ordered[f"box_head.conv5_{br}.bias"] = (n5,)
    return ordered


def _gen(seed: int, key: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((int(seed) ^ zlib.crc32(key.encode())) & 0x7FFFFFFFFFFF)
    return g


def _law(key: str, shape: tuple, g: torch.Generator) -> torch.Tensor:
    if key.endswith("num_batches_tracked"):
        return torch.tensor(0, dtype=torch.int64)

    def normal(std, mean=0.0):
        return torch.randn(shape, generator=g) * std + mean

    def uniform(lo, hi):
        return torch.rand(shape, generator=g) * (hi - lo) + lo

    if key.endswith("fovea.smooth"):
        return uniform(8.0, 12.0)
    if "pos_embed" in key or key.endswith("cls_token"):
        return normal(0.5)
    if "patch_embed" in key:
        return normal(0.05) if key.endswith("weight") else normal(0.05)
    if "prompt_blocks" in key:
        if key.endswith("weight"):
            fan_in, fan_out = shape[1], shape[0]
            bound = math.sqrt(6.0 / (fan_in + fan_out))  # xavier_uniform_, vit_ce_prompt.py:58-60
            return uniform(-bound, bound)
        return normal(0.02)
    if "norm" in key and key.startswith("backbone"):
        return normal(0.1, 1.0) if key.endswith("weight") else normal(0.05)
    if ".attn.qkv." in key:
        return normal(0.07) if key.endswith("weight") else normal(0.05)
    if ".attn.proj." in key:
        return normal(0.025) if key.endswith("weight") else normal(0.02)
    if ".mlp.fc1." in key:
        return normal(0.03) if key.endswith("weight") else normal(0.02)
    if ".mlp.fc2." in key:
        return normal(0.02) if key.endswith("weight") else normal(0.02)
    if key.startswith("box_head"):
        if "conv5_size" in key:   # sizes near 0.25 of the search region keep the box scale stable
            return normal(0.05) if key.endswith("weight") else normal(0.05, -1.1)
        if "conv5_offset" in key:
            return normal(0.05) if key.endswith("weight") else normal(0.05, 0.5)
        if "conv5" in key:
            return normal(0.3)
        if key.endswith(".1.weight"):
            return uniform(0.8, 1.2)
        if key.endswith(".1.bias"):
            return normal(0.1)
        if key.endswith("running_mean"):
            return normal(0.1)
        if key.endswith("running_var"):
            return uniform(0.5, 1.5)
        if key.endswith("weight"):
            fan_in = shape[1] * shape[2] * shape[3]
            return normal(math.sqrt(2.0 / fan_in))  # He-normal keeps ReLU stacks alive
        return normal(0.05)
    raise KeyError(key)


def make_state_dict(seed: int = 0, **shape_kw) -> "OrderedDict[str, torch.Tensor]":
    """Seeded fp32 ``state_dict`` in the reference key layout."""
    sd = OrderedDict()
    for k, shp in model_shapes(**shape_kw).items():
        sd[k] = _law(k, shp, _gen(seed, k)).contiguous()
    return sd


SIAMFC_LAYERS = [  # AlexNetV1 (siamfc backbone): (name, out, in/groups, k, has_bn)
    ("conv1", 96, 3, 11, True), ("conv2", 256, 48, 5, True), ("conv3", 384, 256, 3, True),
    ("conv4", 384, 192, 3, True), ("conv5", 256, 192, 3, False)]


def siamfc_shapes():
    """TrackerSiamFC Net(backbone=AlexNetV1, head=SiamFC) state_dict layout (head has no parameters)."""
    shp = OrderedDict()
    for name, co, ci, k, bn in SIAMFC_LAYERS:
        shp[f"backbone.{name}.0.weight"] = (co, ci, k, k)
        shp[f"backbone.{name}.0.bias"] = (co,)
        if bn:
            for t in ("weight", "bias", "running_mean", "running_var"):
                shp[f"backbone.{name}.1.{t}"] = (co,)
            shp[f"backbone.{name}.1.num_batches_tracked"] = ()
    return shp


def make_siamfc_state_dict(seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict()
    for k, shp in siamfc_shapes().items():
        g = _gen(seed, k)
        if k.endswith("num_batches_tracked"):
            v = torch.tensor(0, dtype=torch.int64)
        elif k.endswith(".0.weight"):
            fan_in = shp[1] * shp[2] * shp[3]
            v = torch.randn(shp, generator=g) * math.sqrt(2.0 / fan_in) * (0.02 if "conv1." in k else 1.0)
        elif k.endswith(".1.weight"):
            v = torch.rand(shp, generator=g) * 0.4 + 0.8
        elif k.endswith("running_var"):
            v = torch.rand(shp, generator=g) + 0.5
        else:
            v = torch.randn(shp, generator=g) * 0.05
        sd[k] = v.contiguous()
    return sd


# ----------------------------------------------------------------------------- frames
def make_frames(seed: int, n: int, H: int = 480, W: int = 640, C: int = 6,
                box=(300.0, 200.0, 40.0, 30.0), drift=(1.5, 0.75), occlude=None, distractor=None):
    """Synthetic RGB+aux video: smooth textured background + bright target.

    Optional events (the same random draws as without them, so a sequence with events shares its background,
    texture and noise with the plain one):
    * ``occlude=(t0, t1)``: the target is not drawn in frames t0 <= t < t1 (full occlusion);
    * ``distractor=(t0, t1, dx, dy[, alpha])``: a second blob of the target's colour and size at the target's
      centre + (dx, dy) in frames t0 <= t < t1, blended over the background with weight alpha (default 1).

    Returns (frames uint8 [n,H,W,C], gt boxes float64 [n,4] in x,y,w,h)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    # low-frequency background: upsampled coarse noise per channel
    coarse = rng.integers(0, 256, size=(H // 32 + 2, W // 32 + 2, C)).astype(np.float32)
    ys = np.linspace(0, coarse.shape[0] - 1.001, H)
    xs = np.linspace(0, coarse.shape[1] - 1.001, W)
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    wy = (ys - y0)[:, None, None]
    wx = (xs - x0)[None, :, None]
    bg = (coarse[y0][:, x0] * (1 - wy) * (1 - wx) + coarse[y0 + 1][:, x0] * wy * (1 - wx)
          + coarse[y0][:, x0 + 1] * (1 - wy) * wx + coarse[y0 + 1][:, x0 + 1] * wy * wx)
    tex = rng.integers(-12, 13, size=(H, W, C)).astype(np.float32)
    target_col = rng.integers(0, 256, size=(C,)).astype(np.float32)
    frames = np.empty((n, H, W, C), dtype=np.uint8)
    gts = np.empty((n, 4), dtype=np.float64)
    yy = np.arange(H, dtype=np.float32)[:, None]
    xx = np.arange(W, dtype=np.float32)[None, :]
    # Python floats: a NumPy float64 box (e.g. read back from a golden .npz) would turn the float32 mask arithmetic
    # below into float64 (NEP 50 promotion) and move a few pixels of some frames by one level -- the goldens were made
    # from Python floats, so every caller must see these frames (round 5: the DiMP tests had compared the tracker on
    # frames that differed from the reference's at a few pixels of frames 2+)
    x, y, w, h = (float(v) for v in box)
    drift = (float(drift[0]), float(drift[1]))
    if distractor is not None:
        distractor = tuple(float(v) for v in distractor)
    for t in range(n):
        cx = x + 0.5 * w + drift[0] * t + 6.0 * math.sin(0.21 * t)
        cy = y + 0.5 * h + drift[1] * t + 4.0 * math.cos(0.17 * t)
        cx = min(max(cx, w), W - w)
        cy = min(max(cy, h), H - h)
        m = np.exp(-(((xx - cx) / (0.5 * w)) ** 4 + ((yy - cy) / (0.5 * h)) ** 4))[..., None]
        if occlude is not None and occlude[0] <= t < occlude[1]:
            m = np.zeros_like(m)
        if distractor is not None and distractor[0] <= t < distractor[1]:
            dx_, dy_ = cx + distractor[2], cy + distractor[3]
            alpha = distractor[4] if len(distractor) > 4 else 1.0
            m = np.maximum(m, alpha * np.exp(-(((xx - dx_) / (0.5 * w)) ** 4 + ((yy - dy_) / (0.5 * h)) ** 4))[..., None])
        noise = rng.integers(-6, 7, size=(H, W, C)).astype(np.float32)
        img = bg * (1 - m) + target_col * m + tex + noise
        frames[t] = np.clip(img, 0, 255).astype(np.uint8)
        gts[t] = (cx - 0.5 * w, cy - 0.5 * h, w, h)
    return frames, gts


def make_patch(seed: int, size: int, C: int = 6) -> np.ndarray:
    """A single synthetic crop (size x size x C uint8) with a centred target."""
    rng = np.random.Generator(np.random.PCG64(seed))
    coarse = rng.integers(0, 256, size=(size // 16 + 2, size // 16 + 2, C)).astype(np.float32)
    idx = np.linspace(0, coarse.shape[0] - 1.001, size)
    i0 = np.floor(idx).astype(int)
    w = (idx - i0)
    bg = (coarse[i0][:, i0] * ((1 - w)[:, None, None] * (1 - w)[None, :, None])
          + coarse[i0 + 1][:, i0] * (w[:, None, None] * (1 - w)[None, :, None])
          + coarse[i0][:, i0 + 1] * ((1 - w)[:, None, None] * w[None, :, None])
          + coarse[i0 + 1][:, i0 + 1] * (w[:, None, None] * w[None, :, None]))
    yy = np.arange(size, dtype=np.float32)[:, None]
    c = size / 2 + rng.uniform(-size / 8, size / 8, size=2)
    r = size / 8
    m = np.exp(-(((yy - c[1]) / r) ** 2 + ((yy.T - c[0]) / r) ** 2))[..., None]
    col = rng.integers(0, 256, size=(C,)).astype(np.float32)
    img = bg * (1 - m) + col * m + rng.integers(-10, 11, size=(size, size, C))
    return np.clip(img, 0, 255).astype(np.uint8)


# ----------------------------------------------------------------------------- DeT / mfDiMP DiMP-50
RESNET50_LAYERS = ((64, 3, 1), (128, 4, 2), (256, 6, 2))   # (planes, blocks, stride) of layer1..layer3


def dimp_shapes(num_dist_bins: int = 100, feature_dim: int = 256, out_dim: int = 512, filter_size: int = 4):
    """The DiMPnet_DeT state_dict keys the classification path reads (dimpnet.py:421-476: two ResNet-50
    backbones to layer3, the clf feature conv, FilterInitializerLinear, DiMPSteepestDescentGN)."""
    shp = OrderedDict()
    for fe in ("feature_extractor", "feature_extractor_depth"):
        shp[f"{fe}.conv1.weight"] = (64, 3, 7, 7)
        for t in ("weight", "bias", "running_mean", "running_var"):
            shp[f"{fe}.bn1.{t}"] = (64,)
        shp[f"{fe}.bn1.num_batches_tracked"] = ()
        inplanes = 64
        for li, (planes, blocks, stride) in enumerate(RESNET50_LAYERS):
            for b in range(blocks):
                pre = f"{fe}.layer{li + 1}.{b}"
                cin = inplanes if b == 0 else planes * 4
                for ci, (co, k, i) in enumerate(((planes, 1, cin), (planes, 3, planes), (planes * 4, 1, planes))):
                    shp[f"{pre}.conv{ci + 1}.weight"] = (co, i, k, k)
                    for t in ("weight", "bias", "running_mean", "running_var"):
                        shp[f"{pre}.bn{ci + 1}.{t}"] = (co,)
                    shp[f"{pre}.bn{ci + 1}.num_batches_tracked"] = ()
                if b == 0:
                    shp[f"{pre}.downsample.0.weight"] = (planes * 4, cin, 1, 1)
                    for t in ("weight", "bias", "running_mean", "running_var"):
                        shp[f"{pre}.downsample.1.{t}"] = (planes * 4,)
                    shp[f"{pre}.downsample.1.num_batches_tracked"] = ()
            inplanes = planes * 4
    shp["classifier.feature_extractor.0.weight"] = (out_dim, 4 * feature_dim, 3, 3)
    shp["classifier.filter_initializer.filter_conv.weight"] = (out_dim, out_dim, 3, 3)
    shp["classifier.filter_initializer.filter_conv.bias"] = (out_dim,)
    shp["classifier.filter_optimizer.log_step_length"] = (1,)
    shp["classifier.filter_optimizer.filter_reg"] = (1,)
    shp["classifier.filter_optimizer.label_map_predictor.weight"] = (1, num_dist_bins, 1, 1)
    shp["classifier.filter_optimizer.target_mask_predictor.0.weight"] = (1, num_dist_bins, 1, 1)
    shp["classifier.filter_optimizer.spatial_weight_predictor.weight"] = (1, num_dist_bins, 1, 1)
    return shp


def make_dimp_state_dict(seed: int = 0, num_dist_bins: int = 100, bin_displacement: float = 0.1,
                         init_gauss_sigma: float = 0.9, mask_init_factor: float = 3.0, init_step_length: float = 0.9,
                         init_filter_reg: float = 0.1) -> "OrderedDict[str, torch.Tensor]":
    """Seeded fp32 DiMP-50 (DeT) weights: He-normal convs as the reference initialises them
    (resnet.py: normal(0, sqrt(2 / (k*k*out)))), non-trivial BatchNorm statistics so the host-side BN
    folding is exercised, and the optimiser's learnt maps at their constructor values for the DeT
    training settings (train_settings/dimp/DeT_DiMP50_Max.py:101-106: 100 bins of 0.1, sigma 0.9,
    mask factor 3, step 0.9, reg 0.1; optimizer.py:37-64).

    A trained ResNet's BatchNorm statistics are its data's statistics; random convs with arbitrary
    statistics give near-constant (all-positive, DC-dominated) layer3 maps that no filter can localise on.
    So the running mean / variance of every BN are calibrated in float64 on a seeded 96 x 96 synthetic
    image (``_calibrate_bn``), which makes each conv's output unit-normalised before its affine, as in a
    trained network; and the clf feature conv's filters are zero-mean (a trained one responds to the
    post-ReLU features' variation, so the 19 x 19 scores of the synthetic tracker peak near 0.3-0.7)."""
    sd = OrderedDict()
    d = torch.arange(num_dist_bins, dtype=torch.float32).reshape(1, -1, 1, 1) * bin_displacement
    gauss = torch.exp(-1 / 2 * (d / init_gauss_sigma) ** 2)
    fixed = {
        "classifier.filter_optimizer.log_step_length": math.log(init_step_length) * torch.ones(1),
        "classifier.filter_optimizer.filter_reg": init_filter_reg * torch.ones(1),
        "classifier.filter_optimizer.label_map_predictor.weight": gauss - gauss.min(),
        "classifier.filter_optimizer.target_mask_predictor.0.weight": mask_init_factor * torch.tanh(2.0 - d),
        "classifier.filter_optimizer.spatial_weight_predictor.weight": torch.ones(1, num_dist_bins, 1, 1),
    }
    for k, shp in dimp_shapes(num_dist_bins).items():
        g = _gen(seed, k)
        if k in fixed:
            v = fixed[k]
        elif k.endswith("num_batches_tracked"):
            v = torch.tensor(0, dtype=torch.int64)
        elif k.endswith("running_var"):
            v = torch.rand(shp, generator=g) + 0.5
        elif k.endswith("running_mean"):
            v = torch.randn(shp, generator=g) * 0.1
        elif ".bn" in k or ".downsample.1." in k:
            v = torch.rand(shp, generator=g) * 0.4 + 0.4 if k.endswith("weight") else torch.randn(shp, generator=g) * 0.1
        elif k.endswith("filter_conv.bias"):
            v = torch.zeros(shp)
        else:   # conv weights
            v = torch.randn(shp, generator=g) * math.sqrt(2.0 / (shp[0] * shp[2] * shp[3]))
            if k == "classifier.feature_extractor.0.weight":   # respond to feature variation, not the DC
                v = v - v.mean(dim=(1, 2, 3), keepdim=True)
        sd[k] = v.float().contiguous() if v.dtype != torch.int64 else v
    _calibrate_bn(sd, seed)
    return sd


def _calibrate_bn(sd, seed, size=96):
    """Set every backbone BN's running_mean / running_var to its conv output's per-channel mean / variance
    (float64, one seeded synthetic 6-channel image, ImageNet normalisation as net_wrappers.py:62-72)."""
    import torch.nn.functional as F
    im = torch.from_numpy(make_patch(seed + 9001, size, 6)).double().permute(2, 0, 1)[None]
    mean = torch.tensor((0.485, 0.456, 0.406), dtype=torch.float64).view(1, -1, 1, 1)
    std = torch.tensor((0.229, 0.224, 0.225), dtype=torch.float64).view(1, -1, 1, 1)

    def bn(x, pre):
        m = x.mean(dim=(0, 2, 3))
        v = x.var(dim=(0, 2, 3), unbiased=False) + 1e-3
        sd[pre + ".running_mean"] = m.float()
        sd[pre + ".running_var"] = v.float()
        g, b = sd[pre + ".weight"].double(), sd[pre + ".bias"].double()
        return (x - m.view(1, -1, 1, 1)) / torch.sqrt(sd[pre + ".running_var"].double().view(1, -1, 1, 1) + 1e-5) * \
            g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)

    def conv(x, key, stride=1, pad=0):
        return F.conv2d(x, sd[key].double(), stride=stride, padding=pad)
    for fe, half in (("feature_extractor", im[:, :3]), ("feature_extractor_depth", im[:, 3:])):
        x = ((half / 255) - mean) / std
        x = F.relu(bn(conv(x, fe + ".conv1.weight", 2, 3), fe + ".bn1"))
        x = F.max_pool2d(x, 3, 2, 1)
        for li, (planes, blocks, stride) in enumerate(RESNET50_LAYERS):
            for b in range(blocks):
                pre = f"{fe}.layer{li + 1}.{b}"
                s = stride if b == 0 else 1
                out = F.relu(bn(conv(x, pre + ".conv1.weight"), pre + ".bn1"))
                out = F.relu(bn(conv(out, pre + ".conv2.weight", s, 1), pre + ".bn2"))
                out = bn(conv(out, pre + ".conv3.weight"), pre + ".bn3")
                res = bn(conv(x, pre + ".downsample.0.weight", s), pre + ".downsample.1") if b == 0 else x
                x = F.relu(out + res)
