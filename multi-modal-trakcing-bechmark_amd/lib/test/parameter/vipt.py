"""parameters(yaml_name, epoch) -> TrackerParams (ViPT/lib/test/parameter/vipt.py:7-29)."""
import os

from lib.config.vipt.config import cfg, reset_config, update_config_from_file
from lib.test.evaluation.environment import env_settings
from lib.test.utils import TrackerParams


def parameters(yaml_name: str, epoch=None):
    params = TrackerParams()
    prj_dir = env_settings().prj_dir
    reset_config()
    yaml_file = os.path.join(prj_dir, 'experiments/vipt/%s.yaml' % yaml_name)
    update_config_from_file(yaml_file)
    params.cfg = cfg
    params.template_factor = cfg.TEST.TEMPLATE_FACTOR
    params.template_size = cfg.TEST.TEMPLATE_SIZE
    params.search_factor = cfg.TEST.SEARCH_FACTOR
    params.search_size = cfg.TEST.SEARCH_SIZE
    params.checkpoint = os.path.join(prj_dir, "./models/ViPT_%s.pth" % yaml_name)
    params.save_all_boxes = False
    return params
