"""One-sequence row-kernel phase stamps (GPU tuning tool, not a test).  Needs the ROW_STAMPS build
(`bash tools/build_variant.sh rowst -DROW_STAMPS`, selected with MMTRACK_LIB=abx/librowst.so): the deep-prompt
kernel, LN1 with the prompt residual and LN2 with the pending proj split-K update write per-block s_memtime stamps
of wave 0 (entry, operands landed, statistics / LayerNorm done, stores drained) and s_memrealtime at entry / end.
The stamps of the last launch of each kind in one replayed frame are printed, one JSON line per kind, as medians
over blocks (cycles), with the launch's span in real time (100 MHz ticks -> us) from the first block's entry to the
last block's end.  usage: MMTRACK_LIB=abx/librowst.so python tools/b1_row_stamps.py [frames]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from mmtrack_amd import Engine, EngineConfig, _lib, synth  # noqa: E402

KINDS = {0: ("ln_kernel<true> (LN2 + proj split-K update)", ("row+slabs landed", "layernorm", "stores drained")),
         1: ("ln_prompt_kernel<2> (prompt residual + LN1)", ("weights/rows landed", "fovea stats", "rows + stores")),
         2: ("prompt_reduce_deep_kernel (deep prompt, fc2 slabs)", ("weights/rows landed", "barrier", "rows + stores")),
         3: ("ln_kernel<false>", ("row landed", "layernorm", "stores drained"))}


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    lib = _lib.load()
    if not hasattr(lib, "mmt_row_stamps"):
        raise SystemExit("not a ROW_STAMPS build: MMTRACK_LIB=abx/librowst.so")
    lib.mmt_row_stamps.argtypes = [ctypes.c_void_p]
    ekw, skw, H, W, C, _ = bench.WORKLOADS["vipt_deep_rgbt"]
    eng = Engine(EngineConfig(max_batch=1, use_graphs=True, precision="fp32", **ekw), synth.make_state_dict(0, **skw),
                 device=0)
    video_np, _ = synth.make_frames(1000, frames + 1, H, W, C)
    video = torch.from_numpy(video_np).cuda()
    eng.initialize(0, video[0], [60.0, 40.0, 30.0, 24.0])
    for t in range(frames):   # warm: graphs captured, caches in their steady state
        eng.track_batch(0, [video[1 + t]])
    torch.cuda.synchronize()
    st = torch.zeros(4 * 4096 * 8, dtype=torch.int64, device="cuda")
    lib.mmt_row_stamps(ctypes.c_void_p(st.data_ptr()))
    eng.track_batch(0, [video[1]])
    torch.cuda.synchronize()
    lib.mmt_row_stamps(None)
    t = st.view(4, 4096, 8).cpu().double()
    for k, (name, phases) in KINDS.items():
        s = t[k]
        s = s[s[:, 0] > 0]
        if not s.shape[0]:
            continue
        # a later launch of the kind with fewer blocks (candidate elimination) overwrites only its own blocks: keep
        # the blocks of the last launch (entries within 30 us of the latest; launches of a kind are a layer apart)
        s = s[s[:, 4] >= s[:, 4].max() - 3000]
        med = lambda v: float(v.median())  # noqa: E731
        rec = {"kind": name, "blocks": int(s.shape[0]),
               "block_cycles": med(s[:, 3] - s[:, 0]),
               phases[0] + "_cyc": med(s[:, 1] - s[:, 0]),
               phases[1] + "_cyc": med(s[:, 2] - s[:, 1]),
               phases[2] + "_cyc": med(s[:, 3] - s[:, 2]),
               "block_us_rt": med(s[:, 5] - s[:, 4]) / 100.0,
               "start_spread_us_rt": float(s[:, 4].max() - s[:, 4].min()) / 100.0,
               "launch_span_us_rt": float(s[:, 5].max() - s[:, 4].min()) / 100.0}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
