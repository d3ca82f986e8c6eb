"""BaseTracker (ViPT/lib/test/tracker/basetracker.py:10-26) + the engine plumbing shared by the trackers."""
from mmtrack_amd import Engine, EngineConfig


def load_net(params):
    """The reference loads torch.load(ckpt)['net'] strictly (vipt.py:20-21).  Here: the safe loader, or a
    state_dict handed over in params.state_dict (synthetic weights in tests / bench)."""
    sd = getattr(params, 'state_dict', None)
    if sd is None:
        import torch
        sd = torch.load(params.checkpoint, map_location='cpu', weights_only=True)['net']
    return sd


def current_device():
    import torch
    return torch.cuda.current_device() if torch.cuda.is_available() else 0


class BaseTracker:
    """Base class for all trackers."""

    def __init__(self, params):
        self.params = params
        self.visdom = None

    def predicts_segmentation_mask(self):
        return False

    def initialize(self, image, info: dict) -> dict:
        raise NotImplementedError

    def track(self, image, info: dict = None) -> dict:
        raise NotImplementedError

    def build_engine(self, in_chans=None):
        ecfg = EngineConfig.from_cfg(self.params.cfg, max_batch=1,
                                     precision=getattr(self.params, 'precision', 'fp32'),
                                     use_graphs=getattr(self.params, 'use_graphs', True),
                                     debug_outputs=bool(getattr(self.params, 'debug_outputs', False)))
        ecfg.template_factor = self.params.template_factor
        ecfg.search_factor = self.params.search_factor
        ecfg.template_size = self.params.template_size
        ecfg.search_size = self.params.search_size
        if in_chans is not None:
            ecfg.in_chans = in_chans
        return Engine(ecfg, load_net(self.params), device=current_device())
