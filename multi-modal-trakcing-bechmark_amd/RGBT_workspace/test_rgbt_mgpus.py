"""RGBT dataset evaluation (reference: ViPT/RGBT_workspace/test_rgbt_mgpus.py) over the MI355X engine.

  python RGBT_workspace/test_rgbt_mgpus.py --yaml_name deep_rgbt --dataset_name ... --seq_home ...
  python RGBT_workspace/test_rgbt_mgpus.py --synthetic 8 --frames 100 --synthetic_weights --batch 8
  torchrun --nproc-per-node 8 RGBT_workspace/test_rgbt_mgpus.py ...      (sequence i on rank i % 8)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

from mmtrack_amd.workspace import main  # noqa: E402

if __name__ == '__main__':
    main('rgbt')
