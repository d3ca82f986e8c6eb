"""RGB-D benchmark dispatch (RGBD/benchmark.py): runs each tracker and records time_cost[name] in seconds.

    python RGBD/benchmark.py [--trackers vipt OSTrack] [-- <args for every tracker>]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from mmtrack_amd.benchmark import run  # noqa: E402

TRACKERS = {
    "vipt": ("../RGBD_workspace", ["python", "test_rgbd_mgpus.py", "--script_name", "vipt",
                                   "--yaml_name", "deep_rgbd", "--dataset_name", "DepthTrack"]),
    "OSTrack": ("../RGBD_workspace", ["python", "test_rgbd_mgpus.py", "--script_name", "ostrack",
                                      "--yaml_name", "vitb_384_mae_ce_32x4_ep300", "--dataset_name", "DepthTrack"]),
}

if __name__ == "__main__":
    run(HERE, TRACKERS)
