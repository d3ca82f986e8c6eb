"""MI355X-native per-frame multi-modal tracking engine (ViPT / OSTrack one-stream trackers).

The compute path is the hand-written gfx950 HIP library ``libmmtrack.so`` behind the C ABI of
``include/mmtrack.h``; this package is its Python host side.  ``lib/`` next to it mirrors the
reference's tracker interface (``lib.test.tracker.vipt.get_tracker_class()`` ...).
"""
from .engine import Engine, EngineConfig, TrackerError, hann_window, xcorr  # noqa: F401

__all__ = ["Engine", "EngineConfig", "TrackerError", "hann_window", "xcorr"]
