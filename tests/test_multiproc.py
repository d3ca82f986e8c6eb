"""The N>1 path on CPU: world-size-2 gloo process groups (one process per 'GPU'), sequence sharding
with no data-path collective, and the max-over-ranks timing reduction bench.py uses."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _FakeTracker:
    def __init__(self, results_dir, rank):
        self.name, self.parameter_name, self.run_id = "fake", "p", None
        self.results_dir = results_dir
        self.rank = rank

    def run_sequence(self, seq, debug=False):
        with open(os.path.join(self.results_dir, f"{seq.name}.rank"), "w") as f:
            f.write(str(self.rank))
        return {"target_bbox": [[1, 2, 3, 4]] * len(seq), "time": [0.01] * len(seq)}


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lib.test.evaluation.data import Sequence
        from lib.test.evaluation.running import run_dataset
        from mmtrack_amd.sharding import max_over_ranks, rank_world, sum_over_ranks
        assert rank_world() == (rank, world)
        seqs = [Sequence(f"seq{i:02d}", [None] * (3 + i), "lasher", [[0, 0, 5, 5]]) for i in range(7)]
        os.makedirs(out_dir, exist_ok=True)
        run_dataset(seqs, [_FakeTracker(out_dir, rank)], threads=0, num_gpus=world)
        m = max_over_ranks(1.5 + rank)
        s = sum_over_ranks(1.0)
        with open(os.path.join(out_dir, f"reduce{rank}.txt"), "w") as f:
            f.write(f"{m} {s}")
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_dataset(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    owners = {}
    for i in range(7):
        name = f"seq{i:02d}"
        owners[name] = int((tmp_path / f"{name}.rank").read_text())
        assert owners[name] == i % world                   # sequence i on rank i % world
        assert (tmp_path / f"{name}.txt").exists()          # result file per sequence, reference format
        assert len((tmp_path / f"{name}.txt").read_text().splitlines()) == 3 + i
    for r in range(world):
        m, s = map(float, (tmp_path / f"reduce{r}.txt").read_text().split())
        assert m == 2.5 and s == 2.0


def _bench_reduce_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        frames = bench.aggregate_throughput(batch=8, steps=10, elapsed=1.0 + rank)
        with open(os.path.join(out_dir, f"b{rank}.txt"), "w") as f:
            f.write(repr(frames))
    finally:
        dist.destroy_process_group()


def test_bench_aggregate_gloo(tmp_path):
    """value = frames over all ranks / max-over-ranks elapsed (weak scaling)."""
    world = 2
    mp.start_processes(_bench_reduce_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        value, elapsed, w = eval((tmp_path / f"b{r}.txt").read_text())
        assert w == world and elapsed == 2.0 and value == pytest.approx(2 * 8 * 10 / 2.0)


def test_bench_spawns_ranks_for_gpus_flag():
    """`bench.py --gpus 2` without a torchrun environment launches its two rank processes itself (before
    any GPU call) and rank 0 reports n_gpus = 2 with the whole-job rate; a torchrun world that disagrees
    with --gpus is refused."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry", "--steps", "20",
                        "--warmup", "2", "--batch", "8"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 16
    assert line["value"] == pytest.approx(2 * 8 * 20 / (line["ms_per_step"] * 20 / 1e3), rel=1e-3)
    # value is the whole-job rate (the driver's contract); the metric's per-GPU rate sits beside it
    assert line["n_gpus"] == 2
    assert line["per_gpu_fps"] == pytest.approx(line["value"] / 2, rel=1e-3)
    env1 = dict(env, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry"], capture_output=True,
                       text=True, env=env1, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
