"""Candidate-elimination template mask (ViPT/lib/utils/ce_utils.py:15-35): the engine supports ALL-less
CTR_POINT selection and needs only the selected template token index."""


def ctr_point_index(template_size: int, stride: int = 16) -> int:
    tf = template_size // stride
    idx = {8: 3, 12: 5, 7: 3, 14: 6}.get(tf)
    if idx is None:
        raise NotImplementedError
    return idx * tf + idx


def generate_mask_cond(cfg, bs, device, gt_bbox):
    import torch
    template_size = cfg.DATA.TEMPLATE.SIZE
    stride = cfg.MODEL.BACKBONE.STRIDE
    tf = template_size // stride
    rng = cfg.MODEL.BACKBONE.CE_TEMPLATE_RANGE
    if rng == 'ALL':
        return None
    if rng == 'CTR_POINT':
        i = {8: 3, 12: 5, 7: 3, 14: 6}.get(tf)
        if i is None:
            raise NotImplementedError
        m = torch.zeros([bs, tf, tf], device=device)
        m[:, i:i + 1, i:i + 1] = 1
        return m.flatten(1).to(torch.bool)
    raise NotImplementedError(rng)
