import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'multi-modal-trakcing-bechmark_amd')
import torch, numpy as np
from mmtrack_amd import Engine, EngineConfig, synth
for graphs in (False, True):
    eng = Engine(EngineConfig(max_batch=4, use_graphs=graphs), synth.make_state_dict(0, kind="vipt", prompt_type="vipt_deep"))
    fr, gt = synth.make_frames(3, 4, 480, 640, 6)
    frd = torch.from_numpy(fr).cuda()
    for i in range(4): eng.initialize(i, frd[0], list(gt[0]))
    eng.timing_enable("fc1")
    for k in range(5):
        eng.track_batch(0, [frd[1 + k % 3]] * 4)
    print("graphs", graphs, eng.timing_read())
    eng.close()
