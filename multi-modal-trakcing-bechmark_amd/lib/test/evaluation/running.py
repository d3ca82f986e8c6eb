"""Dataset runner and result writers (ViPT/lib/test/evaluation/running.py:11-176).

Result formats are the reference's: boxes '%d' tab-separated, times '%f', scores '%.2f'.
Multi-GPU: the reference's spawn-Pool mapping (worker_id % num_gpu), or, with torch.distributed
initialised (one process per GPU, torchrun), sequence i goes to rank i % world_size -- no collective.
"""
import multiprocessing
import os
import sys
from itertools import product

import numpy as np


def _save_tracker_output(seq, tracker, output: dict):
    os.makedirs(tracker.results_dir, exist_ok=True)
    if seq.dataset in ['trackingnet', 'got10k']:
        os.makedirs(os.path.join(tracker.results_dir, seq.dataset), exist_ok=True)
        base = os.path.join(tracker.results_dir, seq.dataset, seq.name)
    elif seq.dataset in ['vtuav_st', 'vtuav_lt']:
        os.makedirs(os.path.join(tracker.results_dir, seq.dataset), exist_ok=True)
        base = os.path.join(tracker.results_dir, seq.dataset, seq.name.split('/')[1])
    else:
        base = os.path.join(tracker.results_dir, seq.name)
    for key, data in output.items():
        if not data:
            continue
        if key == 'target_bbox':
            np.savetxt('{}.txt'.format(base), np.array(data).astype(int), delimiter='\t', fmt='%d')
        elif key == 'all_scores':
            np.savetxt('{}_all_scores.txt'.format(base), np.array(data).astype(float), delimiter='\t', fmt='%.2f')
        elif key == 'time':
            np.savetxt('{}_time.txt'.format(base), np.array(data).astype(float), delimiter='\t', fmt='%f')


def results_exist(seq, tracker):
    if seq.dataset in ['trackingnet', 'got10k']:
        f = '{}.txt'.format(os.path.join(tracker.results_dir, seq.dataset, seq.name))
    else:
        f = '{}/{}.txt'.format(tracker.results_dir, seq.name)
    return os.path.isfile(f)


def run_sequence(seq, tracker, debug=False, num_gpu=8):
    try:
        import torch
        worker_name = multiprocessing.current_process().name
        worker_id = int(worker_name[worker_name.find('-') + 1:]) - 1
        torch.cuda.set_device(worker_id % num_gpu)
    except Exception:
        pass
    if results_exist(seq, tracker) and not debug:
        print('FPS: {}'.format(-1))
        return None
    print('Tracker: {} {} {} ,  Sequence: {}'.format(tracker.name, tracker.parameter_name, tracker.run_id, seq.name))
    output = tracker.run_sequence(seq, debug=debug)
    sys.stdout.flush()
    exec_time = sum(output['time'])
    print('FPS: {}'.format(len(output['time']) / exec_time))
    if not debug:
        _save_tracker_output(seq, tracker, output)
    return output


def shard(items, rank: int, world: int):
    """Sequence i -> rank i % world (one process per GPU)."""
    return [x for i, x in enumerate(items) if i % world == rank]


def run_dataset(dataset, trackers, debug=False, threads=0, num_gpus=8):
    pairs = list(product(dataset, trackers))
    try:
        import torch.distributed as dist
        distributed = dist.is_available() and dist.is_initialized()
    except Exception:
        distributed = False
    print('Evaluating {:4d} trackers on {:5d} sequences'.format(len(trackers), len(dataset)))
    if distributed:
        rank, world = dist.get_rank(), dist.get_world_size()
        for seq, tr in shard(pairs, rank, world):
            run_sequence(seq, tr, debug=debug, num_gpu=num_gpus)
        dist.barrier()
    elif threads == 0:
        for seq, tr in pairs:
            run_sequence(seq, tr, debug=debug)
    else:
        multiprocessing.set_start_method('spawn', force=True)
        with multiprocessing.Pool(processes=threads) as pool:
            pool.starmap(run_sequence, [(seq, tr, debug, num_gpus) for seq, tr in pairs])
    print('Done')
