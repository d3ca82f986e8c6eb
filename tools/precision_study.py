"""GPU diagnostic: which arithmetic reproduces the fp32 reference's decisions.

For N random template/search crop pairs (identity crops, tests/test_gpu_parity.py) the CPU oracle
(fp32, pinned to the reference by tests/golden) gives the CE kept sets, their boundary margins, the CE
scores of every slot and the windowed argmax; the engine runs the same pair in several arithmetic
modes, each also with teacher-forced CE (the oracle's own CE scores injected, mmt_debug_force_ce), so
a CE flip is told apart from the kernels' own error:

  bf16          plain bf16 MFMA operands
  fp32          f16x3 split products (fp16 halves of range-scaled values, hi*hi + lo*hi + hi*lo; common.h)

python tools/precision_study.py [--n 48] [--net deep_rgbt] [--modes bf16,fp32,...] > report
(on the GPU box; asserts nothing, prints one row per mode and a JSON summary)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "multi-modal-trakcing-bechmark_amd"))
sys.path.insert(0, HERE)

from mmtrack_amd import Engine, EngineConfig, synth  # noqa: E402
from oracle import crop as ocrop  # noqa: E402
from oracle import vipt as ov  # noqa: E402
from test_gpu_parity import SHAPES, _cfg, identity_frames, iou  # noqa: E402

MODES = {"bf16": "bf16", "fp32": "fp32"}


def to_xywh(b):
    return [b[0] - b[2] / 2, b[1] - b[3] / 2, b[2], b[3]]


def oracle_pairs(name, n, seed0):
    shape = SHAPES[name]
    cfg = _cfg(name)
    sd = synth.make_state_dict(0, **shape)
    ocfg = ov.NetCfg(kind=shape["kind"], prompt_type=shape.get("prompt_type", "vipt_deep"),
                     search_size=cfg.search_size, template_size=cfg.template_size)
    pairs = []
    for j in range(n):
        zp = synth.make_patch(seed0 + j, cfg.template_size, cfg.in_chans)
        xp = synth.make_patch(seed0 + 1000 + j, cfg.search_size, cfg.in_chans)
        tr = {}
        out = ov.forward(sd, ocrop.preprocess(zp), ocrop.preprocess(xp), ocfg, ov.ce_template_mask(ocfg), trace=tr)
        resp = (ov.hann2d(ocfg.feat_sz) * out["score_map"]).flatten()
        top = torch.sort(resp, descending=True).values
        pb = ov.cal_bbox(resp.view(1, 1, ocfg.feat_sz, ocfg.feat_sz), out["size_map"], out["offset_map"],
                         ocfg.feat_sz)[0].numpy()
        pairs.append(dict(zp=zp, xp=xp, argmax=int(torch.argmax(resp)), box=pb,
                          score=out["score_map"][0, 0].numpy(), top2=float((top[0] - top[1]) / top[0]),
                          margins=tr.get("ce_margin", []), keep=[k[0].numpy() for k in tr.get("ce_keep", [])],
                          keys=np.stack([k.numpy() for k in tr["ce_keys"]]) if tr.get("ce_keys") else None))
    return sd, cfg, pairs


def run_mode(name, sd, cfg, pairs, precision, forced, batch=1):
    """batch > 1: the pairs go B at a time through one track_batch launch (the bench path's kernels: 8-wave
    attention, 256 x 256 / 128 x 128 f16x3 tiles, two-stream halves from 32 sequences)."""
    eng = Engine(EngineConfig(**{**cfg.__dict__, "precision": precision, "max_batch": max(batch, 1)}), sd)
    rows = []
    for c0 in range(0, len(pairs), batch):
        chunk = pairs[c0:c0 + batch]
        f1s = []
        for i, p in enumerate(chunk):
            f0, f1, box = identity_frames(p["zp"], p["xp"], cfg.search_factor)
            if forced and p["keys"] is not None:
                eng.force_ce(i, p["keys"])
            eng.initialize(i, f0, box)
            f1s.append(f1)
        if batch == 1:
            eng.track(0, f1s[0])
        else:
            eng.track_batch(0, f1s)
        if forced:
            for i in range(len(chunk)):
                eng.force_ce(i, None)
        for i, p in enumerate(chunk):
            rows.append(check_pair(eng, cfg, p, i, forced))
    eng.close()
    return rows


def check_pair(eng, cfg, p, bi, forced):
    res = eng.debug("result", bi)
    maps = eng.debug("maps", bi)
    removed = eng.debug("removed", bi)
    r = {"argmax": int(res[5]) == p["argmax"], "iou": float(iou(to_xywh(res[:4]), to_xywh(p["box"]))),
         "dscore": float(np.abs(maps[0] - p["score"]).max()), "top2": p["top2"]}
    ce_ok, off = [], 0
    Lx = cfg.search_size ** 2 // 256
    for st, keep in enumerate(p["keep"]):
        n_rm = (Lx if st == 0 else len(p["keep"][st - 1])) - len(keep)
        got_rm = set(removed[off:off + n_rm].tolist())
        prev = set(range(Lx)) if st == 0 else set(p["keep"][st - 1].tolist())
        ce_ok.append(got_rm == prev - set(keep.tolist()))
        off += n_rm
    r["ce_ok"] = all(ce_ok)
    r["ce_stage_ok"] = ce_ok
    r["min_margin"] = min(p["margins"]) if p["margins"] else None
    if p["keys"] is not None and not forced:
        ek = eng.debug("ce_keys", bi)
        rel = []
        for st in range(len(p["keep"])):
            m = p["keys"][st] > 0
            rel.append(float(np.max(np.abs(ek[st][m] - p["keys"][st][m]) / p["keys"][st][m])))
        r["key_rel_err"] = max(rel)
    return r


def summarize(label, rows):
    n = len(rows)
    s = {"mode": label, "n": n, "ce_all_match": int(sum(r["ce_ok"] for r in rows)),
         "argmax_match": int(sum(r["argmax"] for r in rows)),
         "iou_min": round(min(r["iou"] for r in rows), 5), "iou_median": round(float(np.median([r["iou"] for r in rows])), 5),
         "iou_ge_0999": int(sum(r["iou"] >= 0.999 for r in rows)),
         "dscore_median": float(np.median([r["dscore"] for r in rows])),
         "dscore_max": float(max(r["dscore"] for r in rows))}
    if rows and "key_rel_err" in rows[0]:
        ke = [r["key_rel_err"] for r in rows]
        s["ce_key_rel_err_median"] = float(np.median(ke))
        s["ce_key_rel_err_max"] = float(max(ke))
        # flips explained by a reference margin below the key error of the same pair
        s["ce_flips_with_margin_below_keyerr"] = int(sum((not r["ce_ok"]) and r["min_margin"] is not None
                                                        and r["min_margin"] < 2 * r["key_rel_err"] for r in rows))
    s["min_ref_margin_of_ce_mismatch"] = min([r["min_margin"] for r in rows if not r["ce_ok"] and r["min_margin"]],
                                             default=None)
    s["min_ref_margin_all"] = min([r["min_margin"] for r in rows if r["min_margin"]], default=None)
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--net", default="deep_rgbt")
    ap.add_argument("--seed0", type=int, default=700)
    ap.add_argument("--modes", default="bf16,fp32")
    ap.add_argument("--forced", default="bf16,fp32", help="modes also run with teacher-forced CE")
    ap.add_argument("--batch", type=int, default=1, help="pairs per track_batch launch (32: the bench path)")
    args = ap.parse_args()
    torch.set_num_threads(16)
    sd, cfg, pairs = oracle_pairs(args.net, args.n, args.seed0)
    print(f"# {args.net}: {args.n} pairs, {args.batch} per launch; reference CE margins min {min(min(p['margins']) for p in pairs):.2e}, "
          f"top-2 score gap min {min(p['top2'] for p in pairs):.2e}", flush=True)
    out = []
    for m in args.modes.split(","):
        precision = MODES[m]
        s = summarize(m, run_mode(args.net, sd, cfg, pairs, precision, False, args.batch))
        print(json.dumps(s), flush=True)
        out.append(s)
        if m in args.forced.split(","):
            s = summarize(m + "+forcedCE", run_mode(args.net, sd, cfg, pairs, precision, True, args.batch))
            print(json.dumps(s), flush=True)
            out.append(s)
    print("SUMMARY " + json.dumps(out))


if __name__ == "__main__":
    main()
