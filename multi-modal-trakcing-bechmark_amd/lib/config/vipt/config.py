"""Default tracker config + yaml override, same keys and semantics as ViPT/lib/config/vipt/config.py:7-149.

Unknown yaml keys raise ValueError (config.py:128-139), so a yaml accepted here is accepted there.
"""
import yaml


class EasyDict(dict):
    """Attribute-access dict; nested dicts become EasyDicts (the easydict package's behaviour)."""

    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            setattr(self, k, v)

    def __setattr__(self, name, value):
        if isinstance(value, dict) and not isinstance(value, EasyDict):
            value = EasyDict(value)
        elif isinstance(value, (list, tuple)):
            value = [EasyDict(x) if isinstance(x, dict) else x for x in value]
        super().__setattr__(name, value)
        super().__setitem__(name, value)

    __setitem__ = __setattr__


def _defaults():
    return EasyDict({
        "MODEL": {"PRETRAIN_FILE": "", "EXTRA_MERGER": False, "RETURN_INTER": False, "RETURN_STAGES": [],
                  "BACKBONE": {"TYPE": "vit_base_patch16_224", "STRIDE": 16, "MID_PE": False, "SEP_SEG": False,
                               "CAT_MODE": "direct", "MERGE_LAYER": 0, "ADD_CLS_TOKEN": False,
                               "CLS_TOKEN_USE_MODE": "ignore", "CE_LOC": [], "CE_KEEP_RATIO": [],
                               "CE_TEMPLATE_RANGE": "ALL"},
                  "HEAD": {"TYPE": "CENTER", "NUM_CHANNELS": 256}},
        "TRAIN": {"PROMPT": {"TYPE": "vipt_deep"}, "LR": 0.0001, "WEIGHT_DECAY": 0.0001, "EPOCH": 500,
                  "LR_DROP_EPOCH": 400, "BATCH_SIZE": 16, "NUM_WORKER": 8, "OPTIMIZER": "ADAMW",
                  "BACKBONE_MULTIPLIER": 0.1, "GIOU_WEIGHT": 2.0, "L1_WEIGHT": 5.0, "FREEZE_LAYERS": [0],
                  "PRINT_INTERVAL": 50, "VAL_EPOCH_INTERVAL": 20, "GRAD_CLIP_NORM": 0.1, "AMP": False,
                  "FIX_BN": True, "SAVE_EPOCH_INTERVAL": 1, "SAVE_LAST_N_EPOCH": 1, "CE_START_EPOCH": 20,
                  "CE_WARM_EPOCH": 80, "DROP_PATH_RATE": 0.1,
                  "SCHEDULER": {"TYPE": "step", "DECAY_RATE": 0.1}},
        "DATA": {"SAMPLER_MODE": "causal", "MEAN": [0.485, 0.456, 0.406], "STD": [0.229, 0.224, 0.225],
                 "MAX_SAMPLE_INTERVAL": 200,
                 "TRAIN": {"DATASETS_NAME": ["LASOT", "GOT10K_vottrain"], "DATASETS_RATIO": [1, 1],
                           "SAMPLE_PER_EPOCH": 60000},
                 "VAL": {"DATASETS_NAME": [], "DATASETS_RATIO": [1], "SAMPLE_PER_EPOCH": 10000},
                 "SEARCH": {"SIZE": 320, "FACTOR": 5.0, "CENTER_JITTER": 4.5, "SCALE_JITTER": 0.5, "NUMBER": 1},
                 "TEMPLATE": {"NUMBER": 1, "SIZE": 128, "FACTOR": 2.0, "CENTER_JITTER": 0, "SCALE_JITTER": 0}},
        "TEST": {"TEMPLATE_FACTOR": 2.0, "TEMPLATE_SIZE": 128, "SEARCH_FACTOR": 5.0, "SEARCH_SIZE": 320,
                 "EPOCH": 500},
    })


cfg = _defaults()


def _update_config(base_cfg, exp_cfg):
    if isinstance(base_cfg, dict) and isinstance(exp_cfg, dict):
        for k, v in exp_cfg.items():
            if k not in base_cfg:
                raise ValueError("{} not exist in config.py".format(k))
            if isinstance(v, dict):
                _update_config(base_cfg[k], v)
            else:
                base_cfg[k] = v


def update_config_from_file(filename, base_cfg=None):
    with open(filename) as f:
        exp_config = EasyDict(yaml.safe_load(f))
    _update_config(cfg if base_cfg is None else base_cfg, exp_config)


def reset_config():
    """Back to the defaults (the reference mutates a module-level cfg; tests need a clean one)."""
    fresh = _defaults()
    for k in list(cfg.keys()):
        cfg[k] = fresh[k]
