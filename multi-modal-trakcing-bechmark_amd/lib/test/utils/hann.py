"""Cosine windows (ViPT/lib/test/utils/hann.py:6-16), computed with torch fp32 like the reference; the
engine receives hann2d(feat_sz) as its 'output_window' tensor so its windowed argmax sees the same values."""
import math

import torch


def hann1d(sz: int, centered=True) -> torch.Tensor:
    if centered:
        return 0.5 * (1 - torch.cos((2 * math.pi / (sz + 1)) * torch.arange(1, sz + 1).float()))
    w = 0.5 * (1 + torch.cos((2 * math.pi / (sz + 2)) * torch.arange(0, sz // 2 + 1).float()))
    return torch.cat([w, w[1:sz - sz // 2].flip((0,))])


def hann2d(sz: torch.Tensor, centered=True) -> torch.Tensor:
    return hann1d(sz[0].item(), centered).reshape(1, 1, -1, 1) * hann1d(sz[1].item(), centered).reshape(1, 1, 1, -1)
