"""VOT RGB-D per-frame loop (ViPT/lib/test/vot/vipt_class.py:19-101) over the MI355X engine.

Frames come from the handle as paths; an RGB-D [color, depth] pair is assembled on the GPU
(get_rgbd_frame_device: median depth clip, NORM_MINMAX, JET, merge -- vipt_class.py:79, 92 flags) and
the tracker reads the HBM frame in place; a single path is read as RGB.  Visualisation (cv2 drawing) is
not part of the path and is not provided.
"""
import sys

import torch

from lib.test.evaluation import Tracker
from lib.test.vot import vot
from lib.train.dataset.depth_utils import get_rgbd_frame_device, get_x_frame


class vipt(object):
    def __init__(self, tracker_name='', para_name='', params_overrides=None):
        tracker_info = Tracker(tracker_name, para_name, "vot22", None)
        params = tracker_info.get_parameters()
        params.visualization = False
        params.debug = False
        for k, v in (params_overrides or {}).items():
            setattr(params, k, v)
        self.tracker = tracker_info.create_tracker(params)

    def initialize(self, img_rgb, selection):
        x, y, w, h = selection
        self.H, self.W = int(img_rgb.shape[0]), int(img_rgb.shape[1])
        self.tracker.initialize(img_rgb, {'init_bbox': [x, y, w, h]})

    def track(self, img_rgb):
        outputs = self.tracker.track(img_rgb)
        return outputs['target_bbox'], outputs['best_score']


def read_frame(imagefile):
    if isinstance(imagefile, (list, tuple)) and len(imagefile) == 2:
        return get_rgbd_frame_device(imagefile[0], imagefile[1], depth_clip=True)
    return get_x_frame(imagefile, None, dtype='color')


def run_vot_exp(tracker_name, para_name, vis=False, out_conf=False, channel_type='color', handle=None,
                params_overrides=None):
    """vipt_class.py:50-101; ``handle``: a ready vot.VOT (offline runs), else a TraX-backed one."""
    torch.set_num_threads(1)
    if vis:
        raise NotImplementedError('visualisation is not part of the MI355X path')
    tracker = vipt(tracker_name=tracker_name, para_name=para_name, params_overrides=params_overrides)
    if handle is None:
        handle = vot.VOT("rectangle", channels=None if channel_type == 'rgb' else channel_type)
    selection = handle.region()
    imagefile = handle.frame()
    if not imagefile:
        sys.exit(0)
    tracker.initialize(read_frame(imagefile), selection)
    while True:
        imagefile = handle.frame()
        if not imagefile:
            break
        b1, max_score = tracker.track(read_frame(imagefile))
        if out_conf:
            handle.report(vot.Rectangle(*b1), max_score)
        else:
            handle.report(vot.Rectangle(*b1))
    return handle
