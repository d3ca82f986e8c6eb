"""Per-frame dispatch for whole datasets (the reference's run_sequence loops, batched).

The reference evaluates a dataset by handing sequences to a spawn Pool, one ViPTTrack per sequence,
each worker pinning GPU worker_id % num_gpu (RGBT_workspace/test_rgbt_mgpus.py:66-117, 180-184).
On MI355X one engine per GPU tracks up to ``max_batch`` sequences per launch: every step advances
each active sequence by one frame (mmt_track_batch); a sequence that ends is replaced by the next
one, and the slots stay contiguous by re-homing the last active sequence (initialize from its own
first frame + set_state to its current box), so the batch is always slots [0, n).

Timing follows the reference: per-sequence seconds include reading the frame.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, List

import numpy as np


@dataclass
class SeqJob:
    name: str
    n_frames: int
    get_frame: Callable[[int], object]        # frame index -> H x W x C uint8 (numpy or device tensor)
    init_box: List[float]
    boxes: np.ndarray = None
    scores: np.ndarray = None
    seconds: float = 0.0
    t: int = 0                                # next frame to track
    frame0: object = None
    state: List[float] = field(default_factory=list)


def run_batched(engine, jobs: List[SeqJob], max_batch: int, on_done=None):
    """Track every job to its last frame, max_batch sequences per engine launch."""
    pending = list(jobs)
    active: List[SeqJob] = []

    def start(job, slot):
        tic = time.perf_counter()
        job.frame0 = job.get_frame(0)
        engine.initialize(slot, job.frame0, job.init_box)
        job.seconds += time.perf_counter() - tic
        job.boxes = np.zeros((job.n_frames, 4), dtype=np.float64)
        job.scores = np.zeros(job.n_frames, dtype=np.float32)
        job.boxes[0] = job.init_box
        job.scores[0] = 1.0
        job.t = 1
        job.state = list(job.init_box)

    while pending and len(active) < max_batch:
        job = pending.pop(0)
        start(job, len(active))
        active.append(job)
    while active:
        tic = time.perf_counter()
        frames = [j.get_frame(j.t) for j in active]
        boxes, scores = engine.track_batch(0, frames)
        dt = (time.perf_counter() - tic) / len(active)
        for i, j in enumerate(active):
            j.boxes[j.t] = boxes[i]
            j.scores[j.t] = scores[i]
            j.state = list(boxes[i])
            j.seconds += dt
            j.t += 1
        # retire finished sequences; survivors keep their slot unless a slot above the new count
        # must be compacted down (re-homed from their own first frame + current box)
        finished = [j for j in active if j.t >= j.n_frames]
        for j in finished:
            if on_done:
                on_done(j)
        survivors = [j for j in active if j.t < j.n_frames]
        new_active: List[SeqJob] = [None] * min(max_batch, len(survivors) + len(pending))
        movers = []
        for slot, j in enumerate(active):
            if j.t < j.n_frames:
                if slot < len(new_active):
                    new_active[slot] = j
                else:
                    movers.append(j)
        for slot in range(len(new_active)):
            if new_active[slot] is not None:
                continue
            if movers:
                j = movers.pop(0)
                engine.initialize(slot, j.frame0, j.init_box)
                engine.set_state(slot, j.state)
            else:
                j = pending.pop(0)
                start(j, slot)
            new_active[slot] = j
        active = new_active
    return jobs
