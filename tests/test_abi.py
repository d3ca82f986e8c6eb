"""The C-ABI library loads without a GPU and exports every symbol include/mmtrack.h declares."""
import os
import re

from mmtrack_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "mmtrack.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmt_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("mmt_create", "mmt_initialize", "mmt_track", "mmt_track_batch", "mmt_set_tensor", "mmt_finalize",
                 "mmt_xcorr", "mmt_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert set(declared()) == set(_lib.SIGNATURES)


def test_version_without_gpu():
    assert _lib.load().mmt_version().startswith(b"mmtrack-mi355x")


def test_dimp_state_layout_matches_binding():
    """The device DiMP tracker state / record structs of include/mmtrack.h and the ctypes binding agree in size
    (the library reports sizeof(mmt_dimp_state); no GPU needed)."""
    import ctypes
    from mmtrack_amd import _lib
    lib = _lib.load()
    assert lib.mmt_dimp_state_bytes() == ctypes.sizeof(_lib.MmtDimpState)
    assert _lib.MmtDimpState.target_boxes.offset % 16 == 0 or _lib.MmtDimpState.target_boxes.offset % 4 == 0
