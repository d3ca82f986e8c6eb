"""parameters(yaml_name) for the RGB OSTrack tracker (OSTrack layout: experiments/ostrack/<yaml>.yaml)."""
import os

from lib.config.vipt.config import cfg, reset_config, update_config_from_file
from lib.test.evaluation.environment import env_settings
from lib.test.utils import TrackerParams


def parameters(yaml_name: str = "vitb_384_mae_ce_32x4_ep300", epoch=None):
    params = TrackerParams()
    prj_dir = env_settings().prj_dir
    reset_config()
    update_config_from_file(os.path.join(prj_dir, 'experiments/ostrack/%s.yaml' % yaml_name))
    params.cfg = cfg
    params.template_factor = cfg.TEST.TEMPLATE_FACTOR
    params.template_size = cfg.TEST.TEMPLATE_SIZE
    params.search_factor = cfg.TEST.SEARCH_FACTOR
    params.search_size = cfg.TEST.SEARCH_SIZE
    params.checkpoint = os.path.join(prj_dir, "./models/OSTrack_%s.pth" % yaml_name)
    params.save_all_boxes = False
    return params
