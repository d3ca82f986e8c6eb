"""Dataset-level evaluation driver shared by RGBT_workspace / RGBE_workspace / RGBD (the reference's
test_rgbt_mgpus.py:66-190 and test_rgbe_mgpus.py:30-131, same CLI and result files).

Sequences come from the reference's dataset layouts (LasHeR / RGBT234 / GTOT / VTUAV / VisEvent,
genConfig in the reference scripts) or, with --synthetic N, from seeded synthetic videos.

Parallelism:
  * --mode parallel --threads T: the reference's spawn Pool; worker w uses GPU w % num_gpus and runs
    one ViPTTrack per sequence (reference behaviour);
  * under torchrun (WORLD_SIZE > 1): one process per GPU, sequence i on rank i % world (no collective);
  * --batch B: inside a process, one engine tracks B sequences per launch (mmtrack_amd.runner).
Result formats: RGB-T np.savetxt default ('%.18e', space); RGB-E '%.14f' comma-delimited.
"""
from __future__ import annotations

import argparse
import multiprocessing
import os
import sys
import time
from os.path import isdir, join

import numpy as np

PRJ = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PRJ not in sys.path:
    sys.path.insert(0, PRJ)


# ------------------------------------------------------------------ datasets (reference genConfig layouts)
def gen_config(seq_path, set_type):
    if set_type in ('RGBT234', 'LasHeR', 'lasher'):
        rgb = sorted(join(seq_path, 'visible', p) for p in os.listdir(join(seq_path, 'visible')) if p.endswith('.jpg'))
        aux = sorted(join(seq_path, 'infrared', p) for p in os.listdir(join(seq_path, 'infrared')) if p.endswith('.jpg'))
        gt = np.loadtxt(join(seq_path, 'visible.txt'), delimiter=',', ndmin=2)
    elif set_type == 'GTOT':
        rgb = sorted(join(seq_path, 'v', p) for p in os.listdir(join(seq_path, 'v')) if p.endswith('.png'))
        aux = sorted(join(seq_path, 'i', p) for p in os.listdir(join(seq_path, 'i')) if p.endswith('.png'))
        g = np.loadtxt(join(seq_path, 'groundTruth_v.txt'), delimiter=' ', ndmin=2)
        x0, y0 = g[:, [0, 2]].min(1), g[:, [1, 3]].min(1)
        x1, y1 = g[:, [0, 2]].max(1), g[:, [1, 3]].max(1)
        gt = np.stack([x0, y0, x1 - x0, y1 - y0], axis=1)
    elif 'VTUAV' in set_type:
        rgb = sorted(join(seq_path, 'rgb', p) for p in os.listdir(join(seq_path, 'rgb')) if p.endswith('.jpg'))
        aux = sorted(join(seq_path, 'ir', p) for p in os.listdir(join(seq_path, 'ir')) if p.endswith('.jpg'))
        gt = np.loadtxt(join(seq_path, 'rgb.txt'), delimiter=' ', ndmin=2)
    elif set_type in ('DepthTrack', 'depthtrack', 'CDTB', 'cdtb'):   # VOT-RGBD layout: color/, depth/
        rgb = sorted(join(seq_path, 'color', p) for p in os.listdir(join(seq_path, 'color')) if p.endswith('.jpg'))
        aux = sorted(join(seq_path, 'depth', p) for p in os.listdir(join(seq_path, 'depth')) if p.endswith('.png'))
        gt = np.loadtxt(join(seq_path, 'groundtruth.txt'), delimiter=',', ndmin=2)
    elif set_type in ('VisEvent', 'visevent'):
        rgb = sorted(join(seq_path, 'vis_imgs', p) for p in os.listdir(join(seq_path, 'vis_imgs')) if p.endswith('.bmp'))
        aux = sorted(join(seq_path, 'event_imgs', p) for p in os.listdir(join(seq_path, 'event_imgs'))
                     if p.endswith('.bmp'))
        gt = np.loadtxt(join(seq_path, 'groundtruth.txt'), delimiter=',', ndmin=2)
        absent = np.loadtxt(join(seq_path, 'absent_label.txt'))
        if absent[0] == 0:   # first frame absent (test_rgbe_mgpus.py:56-61)
            k = int(absent.argmax())
            rgb, aux, gt = rgb[k:], aux[k:], gt[k:]
    else:
        raise ValueError("Error dataset!")
    return rgb, aux, gt


def sequence_list(seq_home, dataset_name):
    """Sequence names as the reference lists them (test_rgbt_mgpus.py:155-177): VTUAV reads its split file
    ('group/sequence' entries), the other datasets list the directories under seq_home."""
    if dataset_name in ('VTUAVST', 'VTUAVLT'):
        with open(join(seq_home, 'VTUAV-ST.txt' if dataset_name == 'VTUAVST' else 'VTUAV-LT.txt')) as f:
            return [l for l in f.read().splitlines() if l.strip()]
    return sorted(f for f in os.listdir(seq_home) if isdir(join(seq_home, f)))


def result_name(seq_name, dataset_name):
    """Result-file stem: VTUAV's 'group/sequence' entries save under the sequence part (test_rgbt_mgpus.py:70)."""
    return seq_name.split('/')[-1] if 'VTUAV' in dataset_name else seq_name


def synthetic_sequences(n, frames, H=480, W=640, C=6, seed=0):
    from mmtrack_amd import synth
    out = []
    for i in range(n):
        box = (150.0 + 31 * (i % 9), 100.0 + 17 * (i % 7), 36.0 + 4 * (i % 5), 28.0 + 3 * (i % 4))
        fr, gt = synth.make_frames(seed + i, frames, H, W, C, box=box)
        out.append((f"synthetic_{i:03d}", fr, gt))
    return out


def default_xtype(dataset_name, script_name='vipt'):
    """Frame assembly per modality: RGB-T/E aux read as RGB ('rgbrgb', test_rgbt_mgpus.py:98),
    RGB-D depth JET-colormapped ('rgbcolormap', vipt_class.py:70); the RGB-only OSTrack reads 'color'."""
    if script_name == 'ostrack':
        return 'color'
    return 'rgbcolormap' if dataset_name in ('DepthTrack', 'depthtrack', 'CDTB', 'cdtb') else 'rgbrgb'


def frame_getter(rgb, aux, xtype):
    """Frame i of a dataset sequence as the tracker's input: RGB-D ('rgbcolormap') clip / normalise /
    colormap / merge on the GPU (vipt_class.py:79 flags), RGB-T / RGB-E ('rgbrgb') merged on the GPU
    (test_rgbt_mgpus.py:106), other layouts host-assembled (depth_utils.get_x_frame)."""
    import torch
    from lib.train.dataset.depth_utils import get_rgbd_frame_device, get_x_frame, get_x_frame_device
    if xtype == 'rgbcolormap':
        return lambda i: get_rgbd_frame_device(rgb[i], aux[i], depth_clip=True)
    if xtype == 'rgbrgb' and torch.cuda.is_available():
        return lambda i: get_x_frame_device(rgb[i], aux[i], dtype='rgbrgb')
    if xtype == 'color':
        return lambda i: get_x_frame(rgb[i], None, dtype='color')
    return lambda i: get_x_frame(rgb[i], aux[i], dtype=xtype)


def synthetic_state_dict(script_name, yaml_name):
    from mmtrack_amd import synth
    if script_name == 'ostrack':
        return synth.make_state_dict(0, kind='ostrack', search_size=384, template_size=192)
    return synth.make_state_dict(0, kind='vipt', prompt_type='vipt_' + yaml_name.split('_')[0])


# ------------------------------------------------------------------ one sequence through the reference-shaped tracker
def save_result(path, result, modality):
    if modality == 'rgbe':
        np.savetxt(path, result, fmt='%.14f', delimiter=',')
    else:
        np.savetxt(path, result)


def run_sequence(seq_name, seq_home, dataset_name, yaml_name, num_gpu=1, epoch=60, debug=0, script_name='vipt',
                 modality='rgbt', out_root='.', synthetic=None, params_overrides=None):
    save_folder = join(out_root, f'{modality.upper()}_workspace', 'results', dataset_name, yaml_name)
    save_path = join(save_folder, result_name(seq_name, dataset_name) + '.txt')
    os.makedirs(save_folder, exist_ok=True)
    if os.path.exists(save_path):
        print(f'-1 {seq_name}')
        return
    import torch
    try:
        worker_name = multiprocessing.current_process().name
        worker_id = int(worker_name[worker_name.find('-') + 1:]) - 1
        torch.cuda.set_device(worker_id % num_gpu)
    except Exception:
        pass
    import importlib
    params = importlib.import_module(f'lib.test.parameter.{script_name}').parameters(yaml_name, epoch)
    for k, v in (params_overrides or {}).items():
        setattr(params, k, v)
    tracker = importlib.import_module(f'lib.test.tracker.{script_name}').get_tracker_class()(params)
    if synthetic is not None:
        frames, gt = synthetic
        get = lambda i: frames[i]
        n = len(frames)
    else:
        rgb, aux, gt = gen_config(join(seq_home, seq_name), dataset_name)
        get = frame_getter(rgb, aux, default_xtype(dataset_name, script_name))
        n = len(rgb)
    result = np.zeros((n, 4), dtype=np.float64)
    result[0] = np.copy(gt[0])
    toc = 0.0
    for i in range(n):
        tic = time.perf_counter()
        image = get(i)
        if i == 0:
            tracker.initialize(image, {'init_bbox': list(np.array(gt[0]).astype(np.float32))})
        else:
            out = tracker.track(image)
            result[i] = np.array(out['target_bbox'])
        toc += time.perf_counter() - tic
    if not debug:
        save_result(save_path, result, modality)
    print('{} , fps:{}'.format(seq_name, (n - 1) / toc))


# ------------------------------------------------------------------ batched engine path
def run_batched_dataset(seqs, yaml_name, batch, modality, out_root, dataset_name, params_overrides=None,
                        script_name='vipt'):
    """seqs: list of (name, n_frames, frame getter, gt); one engine, `batch` sequences per launch."""
    import importlib
    from lib.test.tracker.basetracker import current_device, load_net
    from mmtrack_amd import Engine, EngineConfig
    from mmtrack_amd.runner import SeqJob, run_batched
    params = importlib.import_module(f'lib.test.parameter.{script_name}').parameters(yaml_name)
    for k, v in (params_overrides or {}).items():
        setattr(params, k, v)
    ecfg = EngineConfig.from_cfg(params.cfg, max_batch=batch, precision=getattr(params, 'precision', 'fp32'))
    eng = Engine(ecfg, load_net(params), device=current_device())
    save_folder = join(out_root, f'{modality.upper()}_workspace', 'results', dataset_name, yaml_name)
    os.makedirs(save_folder, exist_ok=True)
    jobs = [SeqJob(name, n, get, list(np.array(gt[0], dtype=np.float64))) for name, n, get, gt in seqs]

    def done(job):
        save_result(join(save_folder, result_name(job.name, dataset_name) + '.txt'), job.boxes, modality)
        print('{} , fps:{}'.format(job.name, (job.n_frames - 1) / max(job.seconds, 1e-9)))

    t0 = time.perf_counter()
    run_batched(eng, jobs, batch, on_done=done)
    dt = time.perf_counter() - t0
    frames = sum(j.n_frames - 1 for j in jobs)
    print(f"batched: {len(jobs)} sequences, {frames} tracked frames in {dt:.2f}s -> {frames / dt:.1f} frames/s")
    eng.close()
    return jobs


def main(modality='rgbt', argv=None):
    ap = argparse.ArgumentParser(description=f'Run tracker on {modality.upper()} dataset.')
    ap.add_argument('--script_name', type=str, default='vipt')
    ap.add_argument('--yaml_name', type=str, default=f'deep_{modality}')
    ap.add_argument('--dataset_name', type=str, default={'rgbt': 'LasHeR', 'rgbe': 'VisEvent', 'rgbd': 'DepthTrack'}[modality])
    ap.add_argument('--seq_home', type=str, default='')
    ap.add_argument('--threads', default=0, type=int)
    ap.add_argument('--num_gpus', default=None, type=int)
    ap.add_argument('--epoch', default=60, type=int)
    ap.add_argument('--mode', default='sequential', type=str)
    ap.add_argument('--debug', default=0, type=int)
    ap.add_argument('--video', default='', type=str)
    ap.add_argument('--batch', default=0, type=int, help='sequences per engine launch (0: one tracker per sequence)')
    ap.add_argument('--synthetic', default=0, type=int, help='use N seeded synthetic sequences')
    ap.add_argument('--frames', default=100, type=int, help='frames per synthetic sequence')
    ap.add_argument('--synthetic_weights', action='store_true', help='seeded weights instead of models/ViPT_<yaml>.pth')
    ap.add_argument('--precision', default='fp32', choices=['bf16', 'fp32'],
                    help='fp32: parity mode (f16x3 products, the reference CE decisions and argmax); bf16: faster, not parity')
    ap.add_argument('--out_root', default='.', type=str)
    args = ap.parse_args(argv)
    import torch
    num_gpus = args.num_gpus if args.num_gpus is not None else max(torch.cuda.device_count(), 1)
    overrides = {'precision': args.precision}
    if args.synthetic_weights:
        overrides['state_dict'] = synthetic_state_dict(args.script_name, args.yaml_name)
    # sequences
    if args.synthetic:
        syn = synthetic_sequences(args.synthetic, args.frames, C=3 if args.script_name == 'ostrack' else 6)
        names = [s[0] for s in syn]
    else:
        names = sequence_list(args.seq_home, args.dataset_name)
        if args.video:
            names = [args.video]
    from mmtrack_amd.sharding import rank_world, shard_indices
    rank, world = rank_world()
    if world > 1 and torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', 0)))
    mine = shard_indices(len(names), rank, world)
    start = time.time()
    if args.batch > 0:
        seqs = []
        for i in mine:
            if args.synthetic:
                name, fr, gt = syn[i]
                seqs.append((name, len(fr), (lambda f: (lambda k: f[k]))(fr), gt))
            else:
                rgb, aux, gt = gen_config(join(args.seq_home, names[i]), args.dataset_name)
                seqs.append((names[i], len(rgb), frame_getter(rgb, aux, default_xtype(args.dataset_name,
                                                                                      args.script_name)), gt))
        run_batched_dataset(seqs, args.yaml_name, args.batch, modality, args.out_root, args.dataset_name, overrides,
                            script_name=args.script_name)
    else:
        jobs = [(names[i], args.seq_home, args.dataset_name, args.yaml_name, num_gpus, args.epoch, args.debug,
                 args.script_name, modality, args.out_root, (syn[i][1], syn[i][2]) if args.synthetic else None, overrides)
                for i in mine]
        if args.mode == 'parallel' and args.threads > 0:
            multiprocessing.set_start_method('spawn', force=True)
            with multiprocessing.Pool(processes=args.threads) as pool:
                pool.starmap(run_sequence, jobs)
        else:
            for j in jobs:
                run_sequence(*j)
    print(f"Totally cost {time.time() - start} seconds!")
