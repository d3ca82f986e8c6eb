"""CPU restatement of the ViPT / OSTrack per-frame tracker (TEST ORACLE).

``ViPTTrack`` of ``ViPT/lib/test/tracker/vipt.py:17-126`` (initialize / track /
map_box_back) with ``clip_box`` of ``ViPT/lib/utils/box_ops.py:97-106``, on the
CPU in fp32, using :mod:`oracle.vipt` for the network and :mod:`oracle.crop`
for ``sample_target``.  Also the CPU baseline ``bench.py`` times.
"""
from __future__ import annotations

import numpy as np
import torch

from . import crop as ocrop
from . import vipt as ovipt


def clip_box(box, H, W, margin=0):
    """box_ops.py:97-106."""
    x1, y1, w, h = box
    x2, y2 = x1 + w, y1 + h
    x1 = min(max(0, x1), W - margin)
    x2 = min(max(margin, x2), W)
    y1 = min(max(0, y1), H - margin)
    y2 = min(max(margin, y2), H)
    w = max(margin, x2 - x1)
    h = max(margin, y2 - y1)
    return [x1, y1, w, h]


class OracleTracker:
    def __init__(self, sd, cfg: ovipt.NetCfg, template_factor=2.0, search_factor=4.0):
        self.sd = sd
        self.cfg = cfg
        self.template_factor = template_factor
        self.search_factor = search_factor
        self.window = ovipt.hann2d(cfg.feat_sz)   # vipt.py:28-30
        self.state = None
        self.last = None

    def initialize(self, image, info):
        patch, rf = ocrop.sample_target(image, info['init_bbox'], self.template_factor, self.cfg.template_size)
        self.z_tensor = ocrop.preprocess(patch)
        self.box_mask_z = ovipt.ce_template_mask(self.cfg, 1)
        self.state = list(info['init_bbox'])

    def track(self, image, info=None):
        H, W, _ = image.shape
        patch, rf = ocrop.sample_target(image, self.state, self.search_factor, self.cfg.search_size)
        search = ocrop.preprocess(patch)
        out = ovipt.forward(self.sd, self.z_tensor, search, self.cfg, self.box_mask_z)
        response = self.window * out['score_map']
        pred_boxes, best_score = ovipt.cal_bbox(response, out['size_map'], out['offset_map'], self.cfg.feat_sz,
                                                return_score=True)
        max_score = best_score[0][0].item()
        pred_boxes = pred_boxes.view(-1, 4)
        pred_box = (pred_boxes.mean(dim=0) * self.cfg.search_size / rf).tolist()
        self.state = clip_box(self.map_box_back(pred_box, rf), H, W, margin=10)
        self.last = out
        self.last_idx = int(torch.argmax(response.flatten()))
        return {"target_bbox": self.state, "best_score": max_score}

    def map_box_back(self, pred_box, resize_factor):
        """vipt.py:112-118."""
        cx_prev, cy_prev = self.state[0] + 0.5 * self.state[2], self.state[1] + 0.5 * self.state[3]
        cx, cy, w, h = pred_box
        half_side = 0.5 * self.cfg.search_size / resize_factor
        cx_real = cx + (cx_prev - half_side)
        cy_real = cy + (cy_prev - half_side)
        return [cx_real - 0.5 * w, cy_real - 0.5 * h, w, h]


def run_sequence(tracker: OracleTracker, frames: np.ndarray, init_box):
    boxes = [list(init_box)]
    scores = [1.0]
    tracker.initialize(frames[0], {'init_bbox': list(init_box)})
    for t in range(1, len(frames)):
        o = tracker.track(frames[t])
        boxes.append(o['target_bbox'])
        scores.append(o['best_score'])
    return np.array(boxes, dtype=np.float64), np.array(scores)
