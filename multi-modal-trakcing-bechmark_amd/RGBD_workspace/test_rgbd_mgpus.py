"""RGB-D (DepthTrack shapes) evaluation over the MI355X engine.  The reference runs RGB-D through the
VOT toolkit (ViPT/lib/test/vot/vipt_class.py:50-101); this driver runs the same per-frame tracker on
dataset folders or synthetic sequences, with the RGB-T/E workspace CLI."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

from mmtrack_amd.workspace import main  # noqa: E402

if __name__ == '__main__':
    main('rgbd')
