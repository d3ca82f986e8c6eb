"""The benchmarked launch itself against the reference's golden outputs (GPU only).

bench.py's headline line runs 32 sequences per mmt_track_batch launch with the launch sequence captured in a
hipGraph and split into two stream halves of 16 sequences (engine.cpp enqueue_split), which selects a
different kernel set from the one-sequence launches of test_gpu_parity.py: gemm256s_kernel<0/1> for qkv /
fc1, the 128 x 128 f16x3 gemm_kernel for proj / fc2 / patch / head convs, attn_kernel<8, true> and no
split-K.  Here every golden pair of tests/golden/net_*.npz (the reference network's own outputs,
make_golden.py) sits in one slot of such a 32-sequence launch -- the halves' edge slots 0, 15, 16, 31 first --
with random pairs in the other slots; the launch is run once eagerly (the first use of a batch shape, which
also captures it) and then replayed from the captured graph, and each golden slot is read back with
mmt_debug_fetch(..., slot).  Thresholds are test_gpu_parity.py's: identical CE removed sets, exact windowed
argmax, score / size maps within 1e-3, offset maps within 3e-3, feature rows within 5e-3.
Reference: ViPT/lib/models/vipt/ostrack_prompt.py:39-91, ViPT/lib/models/layers/attn_blocks.py:21-75,
ViPT/lib/test/tracker/vipt.py:64-110.
"""
import os

import numpy as np
import pytest

from mmtrack_amd import Engine, EngineConfig, synth

from test_gpu_parity import SHAPES, _cfg, identity_frames

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BATCH = 32
GOLDEN_SLOTS = [0, 15, 16, 31, 7, 8, 23, 24]


def _check_slot(eng, g, j, slot, name):
    maps = eng.debug("maps", slot)
    res = eng.debug("result", slot)
    removed = eng.debug("removed", slot)
    ref_removed = g[f"removed_{j}"][0]
    assert min(g[f"ce_margin_{j}"]) > 1e-5
    np.testing.assert_array_equal(np.sort(removed[:len(ref_removed)]), np.sort(ref_removed),
                                  err_msg=f"{name} golden {j} in slot {slot}: CE removed set")
    keys = eng.debug("ce_keys", slot)
    ref_keys = g[f"ce_keys_{j}"]
    m = ref_keys > 0
    rel = float((np.abs(keys[m] - ref_keys[m]) / ref_keys[m]).max())
    gs = g[f"score_map_{j}"][0, 0]
    ds = float(np.abs(maps[0] - gs).max())
    print(f"{name}[{j}] slot {slot}: CE score rel err {rel:.2e}, max|dscore| {ds:.2e}")
    assert rel < 1e-4
    np.testing.assert_allclose(maps[0], gs, atol=1e-3)
    np.testing.assert_allclose(maps[1:3], g[f"size_map_{j}"][0], atol=1e-3)
    np.testing.assert_allclose(maps[3:5], g[f"offset_map_{j}"][0], atol=3e-3)
    assert int(res[5]) == int(g[f"resp_argmax_{j}"][0]), f"{name} golden {j} slot {slot}: windowed argmax"
    if f"feat_rows_{j}" in g.files:
        np.testing.assert_allclose(eng.debug("feat", slot)[::8], g[f"feat_rows_{j}"], atol=5e-3)


@pytest.mark.parametrize("name", list(SHAPES))
def test_bench_launch_matches_reference_golden(name):
    cfg = _cfg(name, max_batch=BATCH, use_graphs=True)   # debug_outputs, parity mode, default tiles
    assert cfg.precision == "fp32" and cfg.use_graphs
    g = np.load(os.path.join(GOLDEN, f"net_{name}.npz"))
    seeds = [tuple(int(v) for v in s) for s in g["seeds"]]
    slot_of = dict(zip(range(len(seeds)), GOLDEN_SLOTS))
    golden_at = {s: j for j, s in slot_of.items()}
    C = cfg.in_chans
    f0s, f1s, boxes = [], [], []
    for slot in range(BATCH):
        sz, ss = seeds[golden_at[slot]] if slot in golden_at else (7000 + slot, 8000 + slot)
        zp = synth.make_patch(sz, cfg.template_size, C)
        xp = synth.make_patch(ss, cfg.search_size, C)
        f0, f1, box = identity_frames(zp, xp, cfg.search_factor)
        f0s.append(f0)
        f1s.append(f1)
        boxes.append(box)
    eng = Engine(cfg, synth.make_state_dict(0, **SHAPES[name]))
    try:
        results = []
        for rep in range(2):   # rep 0: eager run + capture; rep 1: graph replay
            for slot in range(BATCH):
                eng.initialize(slot, f0s[slot], boxes[slot])
            boxes_out, scores = eng.track_batch(0, f1s)
            results.append((boxes_out, scores))
            for j, slot in slot_of.items():
                _check_slot(eng, g, j, slot, f"{name} rep{rep}")
        # the graph replay reproduces the eager launch bit for bit
        np.testing.assert_array_equal(results[0][0], results[1][0])
        np.testing.assert_array_equal(results[0][1], results[1][1])
    finally:
        eng.close()
