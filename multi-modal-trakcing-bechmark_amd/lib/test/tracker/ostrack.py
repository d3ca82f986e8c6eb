"""OSTrack (RGB, 3-channel) drop-in (ViPT/lib/test/tracker/ostrack.py:19-164) over the MI355X engine.

The reference class is broken as shipped (it calls Preprocessor.process with two arguments and
reads .tensors, ostrack.py:56-86); this one implements the intended behaviour: same constructor
signature (params, dataset_name), track() returns {'target_bbox': [x, y, w, h]}.
"""
from lib.test.tracker.basetracker import BaseTracker


class OSTrack(BaseTracker):
    def __init__(self, params, dataset_name=None):
        super(OSTrack, self).__init__(params)
        self.cfg = params.cfg
        self.engine = self.build_engine(in_chans=3)
        self.state = None
        self.feat_sz = self.cfg.TEST.SEARCH_SIZE // self.cfg.MODEL.BACKBONE.STRIDE
        self.frame_id = 0
        self.save_all_boxes = params.save_all_boxes

    def initialize(self, image, info: dict):
        self.engine.initialize(0, image, info['init_bbox'])
        self.state = info['init_bbox']
        self.frame_id = 0

    def track(self, image, info: dict = None):
        self.frame_id += 1
        box, score = self.engine.track(0, image)
        self.state = box
        return {"target_bbox": self.state, "best_score": score}


def get_tracker_class():
    return OSTrack
