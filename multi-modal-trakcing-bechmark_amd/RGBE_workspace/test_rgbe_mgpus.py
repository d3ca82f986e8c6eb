"""RGBE dataset evaluation (reference: ViPT/RGBE_workspace/test_rgbe_mgpus.py) over the MI355X engine.

  python RGBE_workspace/test_rgbe_mgpus.py --yaml_name deep_rgbe --dataset_name ... --seq_home ...
  python RGBE_workspace/test_rgbe_mgpus.py --synthetic 8 --frames 100 --synthetic_weights --batch 8
  torchrun --nproc-per-node 8 RGBE_workspace/test_rgbe_mgpus.py ...      (sequence i on rank i % 8)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

from mmtrack_amd.workspace import main  # noqa: E402

if __name__ == '__main__':
    main('rgbe')
