"""Host-side profile of the DiMP tracking step (tuning tool): cProfile of track_batch over B trackers."""
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "multi-modal-trakcing-bechmark_amd"))

import torch  # noqa: E402

from mmtrack_amd import synth  # noqa: E402
from mmtrack_amd.dimp_tracker import DiMP, parameters, track_batch  # noqa: E402
from mmtrack_amd.dimpnet import DiMPNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
net = DiMPNet(synth.make_dimp_state_dict(0))
video_np, _ = synth.make_frames(5, 9, 480, 640, 6)
video = torch.from_numpy(video_np).cuda()
trs = [DiMP(parameters(), net=net) for _ in range(B)]
for i, t in enumerate(trs):
    t.initialize(video[0], {"init_bbox": [60.0 + 13 * i, 40.0 + 7 * i, 40.0, 32.0]})
for k in range(3):
    track_batch(trs, [video[1 + k]] * B)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for k in range(5):
    track_batch(trs, [video[1 + k % 8]] * B)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
