"""Sequence (ViPT/lib/test/evaluation/data.py): frames are file paths (read with get_x_frame) or arrays."""
from collections import OrderedDict

import numpy as np


class Sequence:
    def __init__(self, name, frames, dataset, ground_truth_rect, init_data=None, object_ids=None,
                 target_visible=None, aux_frames=None, xtype='rgbrgb'):
        self.name = name
        self.frames = frames                 # list of paths (RGB) or H x W x C uint8 arrays
        self.aux_frames = aux_frames         # list of aux-modality paths when frames are paths
        self.dataset = dataset
        self.ground_truth_rect = np.asarray(ground_truth_rect, dtype=np.float64) \
            if ground_truth_rect is not None else None
        self.object_ids = object_ids
        self.target_visible = target_visible
        self.xtype = xtype
        self.init_data = init_data if init_data is not None else {0: {'bbox': list(self.ground_truth_rect[0])}}

    def init_info(self):
        info = dict(self.init_data[0])
        info['init_bbox'] = list(info['bbox'])
        return info

    def frame_info(self, frame_num):
        return OrderedDict(self.init_data.get(frame_num, {}))

    def image(self, i):
        f = self.frames[i]
        if isinstance(f, np.ndarray) or hasattr(f, 'data_ptr'):
            return f
        from lib.train.dataset.depth_utils import get_x_frame
        return get_x_frame(f, self.aux_frames[i] if self.aux_frames else None, dtype=self.xtype)

    def __len__(self):
        return len(self.frames)
