"""ViPTTrack drop-in (ViPT/lib/test/tracker/vipt.py:17-130) over the MI355X engine.

Same constructor, initialize(image, info) and track(image, info=None) contract; image is the
H x W x 6 uint8 RGB+aux frame (numpy, or a torch uint8 tensor already on the GPU).  Crop, normalise,
the ViPT network, Hann window, argmax decode, box back-mapping and clip_box all run in the engine.
"""
from lib.test.tracker.basetracker import BaseTracker


class ViPTTrack(BaseTracker):
    def __init__(self, params):
        super(ViPTTrack, self).__init__(params)
        self.cfg = params.cfg
        self.engine = self.build_engine()
        self.state = None
        self.feat_sz = self.cfg.TEST.SEARCH_SIZE // self.cfg.MODEL.BACKBONE.STRIDE
        if getattr(params, 'debug', None) is None:
            setattr(params, 'debug', 0)
        self.debug = params.debug
        self.frame_id = 0
        self.save_all_boxes = params.save_all_boxes

    def initialize(self, image, info: dict):
        self.engine.initialize(0, image, info['init_bbox'])
        self.state = info['init_bbox']
        self.frame_id = 0
        if self.save_all_boxes:
            # the reference reads cfg.MODEL.NUM_OBJECT_QUERIES here (vipt.py:59-62), which its config lacks
            all_boxes_save = info['init_bbox'] * self.cfg.MODEL.NUM_OBJECT_QUERIES
            return {"all_boxes": all_boxes_save}

    def track(self, image, info: dict = None):
        self.frame_id += 1
        box, score = self.engine.track(0, image)
        self.state = box
        return {"target_bbox": self.state, "best_score": score}


def get_tracker_class():
    return ViPTTrack
