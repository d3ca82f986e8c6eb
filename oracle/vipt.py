"""fp32 CPU restatement of the ViPT / OSTrack one-stream network (TEST ORACLE).

Follows, op for op and in the same order, the reference forward so that its
outputs match the reference's to fp32 round-off:

* ``ViPT/lib/models/vipt/vit_ce_prompt.py:184-346``  (ViPT backbone, prompts, CE)
* ``ViPT/lib/models/vipt/vit_ce.py:101-193``         (OSTrack backbone, no prompts)
* ``ViPT/lib/models/layers/attn.py:33-59``           (attention, returns P)
* ``ViPT/lib/models/layers/attn_blocks.py:9-104``    (CE block, candidate elimination)
* ``ViPT/lib/models/layers/head.py:98-201``          (CENTER head, cal_bbox)
* ``ViPT/lib/models/vipt/ostrack_prompt.py:39-91``   (forward / forward_head)

Weights come as a reference-layout ``state_dict`` of fp32 tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn.functional as F

LN_EPS = 1e-6   # vit_ce_prompt.py:121
BN_EPS = 1e-5   # head.py:20 (nn.BatchNorm2d default)


@dataclass
class NetCfg:
    kind: str = "vipt"              # "vipt" | "ostrack"
    prompt_type: str = "vipt_deep"  # "vipt_deep" | "vipt_shaw" (ViPT only)
    search_size: int = 256
    template_size: int = 128
    ce_loc: List[int] = field(default_factory=lambda: [3, 6, 9])
    ce_keep_ratio: List[float] = field(default_factory=lambda: [0.7, 0.7, 0.7])
    ce_template_range: str = "CTR_POINT"
    depth: int = 12
    heads: int = 12

    @property
    def feat_sz(self):
        return self.search_size // 16

    @property
    def lens_z(self):
        return (self.template_size // 16) ** 2

    @property
    def lens_x(self):
        return (self.search_size // 16) ** 2


def ce_template_mask(cfg: NetCfg, bs: int = 1) -> Optional[torch.Tensor]:
    """``generate_mask_cond`` for ALL / CTR_POINT (``ViPT/lib/utils/ce_utils.py:15-35``)."""
    if cfg.ce_template_range == "ALL" or not cfg.ce_loc:
        return None
    tf = cfg.template_size // 16
    idx = {8: 3, 12: 5, 7: 3, 14: 6}[tf]
    m = torch.zeros([bs, tf, tf])
    m[:, idx:idx + 1, idx:idx + 1] = 1
    return m.flatten(1).to(torch.bool)


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], LN_EPS)


def _lin(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def _patch_embed(img, sd, p):
    # PatchEmbed.forward: proj conv k16 s16, flatten(2).transpose(1,2)  (patch_embed.py:28-31)
    y = F.conv2d(img, sd[p + ".proj.weight"], sd[p + ".proj.bias"], stride=16)
    return y.flatten(2).transpose(1, 2)


def token2feature(t):
    B, L, D = t.shape
    H = W = int(L ** 0.5)
    return t.permute(0, 2, 1).view(B, D, W, H).contiguous()   # vipt/utils.py:105-109


def feature2token(x):
    B, C, W, H = x.shape
    return x.view(B, C, W * H).permute(0, 2, 1).contiguous()  # vipt/utils.py:115-119


def prompt_block(feat, sd, i):
    """``Prompt_block.forward`` + ``Fovea.forward`` (vit_ce_prompt.py:62-71, 33-47)."""
    p = f"backbone.prompt_blocks.{i}"
    B, C, W, H = feat.shape
    x0 = feat[:, 0:int(C / 2)].contiguous()
    x0 = F.conv2d(x0, sd[p + ".conv0_0.weight"], sd[p + ".conv0_0.bias"])
    x1 = feat[:, int(C / 2):].contiguous()
    x1 = F.conv2d(x1, sd[p + ".conv0_1.weight"], sd[p + ".conv0_1.bias"])
    b, c, h, w = x0.shape
    v = x0.contiguous().view(b, c, h * w)
    mask = torch.softmax(v * sd[p + ".fovea.smooth"], dim=-1)
    fov = (mask * v).contiguous().view(b, c, h, w)
    x0 = fov + x1
    return F.conv2d(x0, sd[p + ".conv1x1.weight"], sd[p + ".conv1x1.bias"])


def attention(x, sd, p, heads=12):
    """``Attention.forward`` with return_attention=True (attn.py:33-59)."""
    B, N, C = x.shape
    qkv = _lin(x, sd, p + ".qkv").reshape(B, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.unbind(0)
    attn = (q @ k.transpose(-2, -1)) * ((C // heads) ** -0.5)
    attn = attn.softmax(dim=-1)
    o = (attn @ v).transpose(1, 2).reshape(B, N, C)
    return _lin(o, sd, p + ".proj"), attn


def candidate_elimination(attn, tokens, lens_t, keep_ratio, global_index, box_mask_z):
    """attn_blocks.py:21-75."""
    lens_s = attn.shape[-1] - lens_t
    bs, hn, _, _ = attn.shape
    lens_keep = math.ceil(keep_ratio * lens_s)
    if lens_keep == lens_s:
        return tokens, global_index, None, None
    attn_t = attn[:, :, :lens_t, lens_t:]
    if box_mask_z is not None:
        m = box_mask_z.unsqueeze(1).unsqueeze(-1).expand(-1, attn_t.shape[1], -1, attn_t.shape[-1])
        attn_t = attn_t[m].view(bs, hn, -1, lens_s)
        attn_t = attn_t.mean(dim=2).mean(dim=1)
    else:
        attn_t = attn_t.mean(dim=2).mean(dim=1)
    sorted_attn, indices = torch.sort(attn_t, dim=1, descending=True)
    topk_idx, non_topk_idx = indices[:, :lens_keep], indices[:, lens_keep:]
    keep_index = global_index.gather(dim=1, index=topk_idx)
    removed_index = global_index.gather(dim=1, index=non_topk_idx)
    tokens_t = tokens[:, :lens_t]
    tokens_s = tokens[:, lens_t:]
    B, L, C = tokens_s.shape
    attentive = tokens_s.gather(dim=1, index=topk_idx.unsqueeze(-1).expand(B, -1, C))
    return torch.cat([tokens_t, attentive], dim=1), keep_index, removed_index, sorted_attn


def ce_block(x, sd, i, gi_t, gi_s, keep_ratio, box_mask_z, heads, trace=None):
    """``CEBlock.forward`` (attn_blocks.py:93-104); timm 0.5.4 ``Mlp`` = fc1 -> GELU(erf) -> fc2."""
    p = f"backbone.blocks.{i}"
    x_attn, attn = attention(_ln(x, sd, p + ".norm1"), sd, p + ".attn", heads)
    x = x + x_attn
    lens_t = gi_t.shape[1]
    removed = None
    if keep_ratio < 1:
        gi_prev = gi_s
        x, gi_s, removed, sorted_attn = candidate_elimination(attn, x, lens_t, keep_ratio, gi_s, box_mask_z)
        if trace is not None and sorted_attn is not None:
            k = gi_s.shape[1]
            trace.setdefault("ce_margin", []).append(
                float(((sorted_attn[:, k - 1] - sorted_attn[:, k]) / sorted_attn[:, k - 1]).min()))
            trace.setdefault("ce_keep", []).append(gi_s.clone())
            # every surviving slot's score, by slot id (sequence 0): the teacher-forcing keys
            lx = trace.get("lens_x")
            if lx:
                keys = torch.zeros(lx)
                attn_t = attn[:1, :, :lens_t, lens_t:]
                if box_mask_z is not None:
                    m = box_mask_z[:1].unsqueeze(1).unsqueeze(-1).expand(-1, attn_t.shape[1], -1, attn_t.shape[-1])
                    attn_t = attn_t[m].view(1, attn_t.shape[1], -1, attn_t.shape[-1])
                keys[gi_prev[0].long()] = attn_t.mean(dim=2).mean(dim=1)[0]
                trace.setdefault("ce_keys", []).append(keys)
    h = _lin(_ln(x, sd, p + ".norm2"), sd, p + ".mlp.fc1")
    h = F.gelu(h)
    x = x + _lin(h, sd, p + ".mlp.fc2")
    return x, gi_t, gi_s, removed, attn


def _recover(x, gi_s, removed, lens_x):
    # token recovery with zeros at pruned slots (vit_ce_prompt.py:276-285, 325-334)
    B = x.shape[0]
    if removed and removed[0] is not None:
        removed_cat = torch.cat(removed, dim=1)
        pad = torch.zeros([B, lens_x - gi_s.shape[1], x.shape[2]])
        x = torch.cat([x, pad], dim=1)
        index_all = torch.cat([gi_s, removed_cat], dim=1)
        C = x.shape[-1]
        x = torch.zeros_like(x).scatter_(dim=1, index=index_all.unsqueeze(-1).expand(B, -1, C).to(torch.int64),
                                         src=x)
    return x


def backbone(sd, z, x, cfg: NetCfg, box_mask_z=None, trace=None):
    B = x.shape[0]
    lens_z, lens_x = cfg.lens_z, cfg.lens_x
    if trace is not None:
        trace["lens_x"] = lens_x
    prompted = cfg.kind == "vipt" and cfg.prompt_type in ("vipt_shaw", "vipt_deep")
    if cfg.kind == "vipt":
        x_rgb, z_rgb = x[:, :3], z[:, :3]
        x_dte, z_dte = x[:, 3:], z[:, 3:]
        zt = _patch_embed(z_rgb, sd, "backbone.patch_embed")
        xt = _patch_embed(x_rgb, sd, "backbone.patch_embed")
        z_dte = _patch_embed(z_dte, sd, "backbone.patch_embed_prompt")
        x_dte = _patch_embed(x_dte, sd, "backbone.patch_embed_prompt")
        if prompted:   # vit_ce_prompt.py:205-219
            z_feat = token2feature(_ln(zt, sd, "backbone.prompt_norms.0"))
            x_feat = token2feature(_ln(xt, sd, "backbone.prompt_norms.0"))
            z_dte_feat = token2feature(_ln(z_dte, sd, "backbone.prompt_norms.0"))
            x_dte_feat = token2feature(_ln(x_dte, sd, "backbone.prompt_norms.0"))
            z_feat = prompt_block(torch.cat([z_feat, z_dte_feat], dim=1), sd, 0)
            x_feat = prompt_block(torch.cat([x_feat, x_dte_feat], dim=1), sd, 0)
            z_dte, x_dte = feature2token(z_feat), feature2token(x_feat)
            z_prompted, x_prompted = z_dte, x_dte
        zt = zt + z_dte
        xt = xt + x_dte
    else:  # vit_ce.py:104-105
        xt = _patch_embed(x, sd, "backbone.patch_embed")
        zt = _patch_embed(z, sd, "backbone.patch_embed")
    zt = zt + sd["backbone.pos_embed_z"]
    xt = xt + sd["backbone.pos_embed_x"]
    x = torch.cat((zt, xt), dim=1)

    gi_t = torch.arange(lens_z, dtype=torch.int64).repeat(B, 1)
    gi_s = torch.arange(lens_x, dtype=torch.int64).repeat(B, 1)
    removed_s = []
    ce_ratio = {loc: r for loc, r in zip(cfg.ce_loc, cfg.ce_keep_ratio)}
    attn = None
    for i in range(cfg.depth):
        if i >= 1 and cfg.kind == "vipt" and cfg.prompt_type == "vipt_deep":   # vit_ce_prompt.py:268-310
            x_ori = x
            lz_new = gi_t.shape[1]
            zz = x[:, :lz_new]
            xx = _recover(x[:, lz_new:], gi_s, removed_s, lens_x)
            x = torch.cat([zz, xx], dim=1)
            x = _ln(x, sd, f"backbone.prompt_norms.{i - 1}")
            z_feat = token2feature(x[:, :lens_z, :])
            x_feat = token2feature(x[:, lens_z:, :])
            z_prompted = _ln(z_prompted, sd, f"backbone.prompt_norms.{i}")
            x_prompted = _ln(x_prompted, sd, f"backbone.prompt_norms.{i}")
            z_feat = prompt_block(torch.cat([z_feat, token2feature(z_prompted)], dim=1), sd, i)
            x_feat = prompt_block(torch.cat([x_feat, token2feature(x_prompted)], dim=1), sd, i)
            zp, xp = feature2token(z_feat), feature2token(x_feat)
            z_prompted, x_prompted = zp, xp
            # candidate_elimination_prompt (attn_blocks.py:9-18)
            Bq, Lq, Cq = xp.shape
            xp_kept = xp.gather(dim=1, index=gi_s.unsqueeze(-1).expand(Bq, -1, Cq))
            x = x_ori + torch.cat([zp, xp_kept], dim=1)
        x, gi_t, gi_s, removed, attn = ce_block(x, sd, i, gi_t, gi_s, ce_ratio.get(i, 1.0), box_mask_z,
                                                cfg.heads, trace)
        if i in ce_ratio:
            removed_s.append(removed)
    x = _ln(x, sd, "backbone.norm")
    lz_new = gi_t.shape[1]
    zz = x[:, :lz_new]
    xx = _recover(x[:, lz_new:], gi_s, removed_s, lens_x)
    x = torch.cat([zz, xx], dim=1)
    return x, {"attn": attn, "removed_indexes_s": removed_s, "global_index_s": gi_s}


def _conv_bn_relu(x, sd, p):
    y = F.conv2d(x, sd[p + ".0.weight"], sd[p + ".0.bias"], padding=1)
    y = F.batch_norm(y, sd[p + ".1.running_mean"], sd[p + ".1.running_var"], sd[p + ".1.weight"],
                     sd[p + ".1.bias"], False, 0.1, BN_EPS)
    return F.relu(y)


def get_score_map(feat, sd):
    """``CenterPredictor.get_score_map`` (head.py:175-201)."""
    outs = {}
    for br in ("ctr", "offset", "size"):
        h = feat
        for j in range(1, 5):
            h = _conv_bn_relu(h, sd, f"box_head.conv{j}_{br}")
        outs[br] = F.conv2d(h, sd[f"box_head.conv5_{br}.weight"], sd[f"box_head.conv5_{br}.bias"])

    def _sig(t):
        return torch.clamp(t.sigmoid(), min=1e-4, max=1 - 1e-4)
    return _sig(outs["ctr"]), _sig(outs["size"]), outs["offset"]


def cal_bbox(score_map_ctr, size_map, offset_map, feat_sz, return_score=False):
    """head.py:142-160."""
    max_score, idx = torch.max(score_map_ctr.flatten(1), dim=1, keepdim=True)
    idx_y = idx // feat_sz
    idx_x = idx % feat_sz
    idx2 = idx.unsqueeze(1).expand(idx.shape[0], 2, 1)
    size = size_map.flatten(2).gather(dim=2, index=idx2)
    offset = offset_map.flatten(2).gather(dim=2, index=idx2).squeeze(-1)
    bbox = torch.cat([(idx_x.to(torch.float) + offset[:, :1]) / feat_sz,
                      (idx_y.to(torch.float) + offset[:, 1:]) / feat_sz,
                      size.squeeze(-1)], dim=1)
    if return_score:
        return bbox, max_score
    return bbox


def forward(sd, template, search, cfg: NetCfg, box_mask_z=None, trace=None):
    """``ViPTrack.forward`` / ``OSTrack.forward`` with the CENTER head (ostrack_prompt.py:39-91)."""
    with torch.no_grad():
        x, aux = backbone(sd, template, search, cfg, box_mask_z, trace)
        fs = cfg.feat_sz
        enc = x[:, -fs * fs:]
        opt = enc.unsqueeze(-1).permute((0, 3, 2, 1)).contiguous()
        bs, Nq, C, HW = opt.size()
        feat = opt.view(-1, C, fs, fs)
        ctr, size, offset = get_score_map(feat, sd)
        bbox = cal_bbox(ctr, size, offset, fs)
        out = {"pred_boxes": bbox.view(bs, Nq, 4), "score_map": ctr, "size_map": size, "offset_map": offset,
               "backbone_feat": x}
        out.update(aux)
        return out


def hann1d(sz: int, centered=True):
    """``ViPT/lib/test/utils/hann.py:6-11``."""
    if centered:
        return 0.5 * (1 - torch.cos((2 * math.pi / (sz + 1)) * torch.arange(1, sz + 1).float()))
    w = 0.5 * (1 + torch.cos((2 * math.pi / (sz + 2)) * torch.arange(0, sz // 2 + 1).float()))
    return torch.cat([w, w[1:sz - sz // 2].flip((0,))])


def hann2d(sz: int, centered=True):
    """``hann.py:14-16`` for a square map."""
    return hann1d(sz, centered).reshape(1, 1, -1, 1) * hann1d(sz, centered).reshape(1, 1, 1, -1)
