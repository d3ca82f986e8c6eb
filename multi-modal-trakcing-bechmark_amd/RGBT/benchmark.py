"""RGB-T benchmark dispatch (RGBT/benchmark.py): runs each tracker and records time_cost[name] in seconds.

    python RGBT/benchmark.py [--trackers mfDiMP vipt] [-- <args for every tracker>]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from mmtrack_amd.benchmark import run  # noqa: E402

TRACKERS = {
    "vipt": ("../RGBT_workspace", ["python", "test_rgbt_mgpus.py", "--script_name", "vipt",
                                   "--yaml_name", "deep_rgbt", "--dataset_name", "LasHeR"]),
    "mfDiMP": ("models/mfDiMP", ["python", "test.py"]),
}

if __name__ == "__main__":
    run(HERE, TRACKERS)
