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


def test_abi_version_matches_header_and_binding():
    """The library, the header's MMT_ABI_VERSION and the ctypes binding agree; the pre-5 strided optimiser
    (stride 0 = contiguous) is not exported, so a binding written against it fails to resolve the symbol."""
    hdr = open(HDR).read()
    v = int(re.search(r"#define\s+MMT_ABI_VERSION\s+(\d+)", hdr).group(1))
    lib = _lib.load()
    assert lib.mmt_abi_version() == v == _lib.ABI_VERSION
    assert not hasattr(lib, "mmt_dimp_optimize_dev")


def test_dimp_state_layout_matches_binding():
    """The device DiMP tracker state / record structs of include/mmtrack.h and the ctypes binding agree in size
    (the library reports sizeof(mmt_dimp_state); no GPU needed)."""
    import ctypes
    from mmtrack_amd import _lib
    lib = _lib.load()
    assert lib.mmt_dimp_state_bytes() == ctypes.sizeof(_lib.MmtDimpState)
    assert _lib.MmtDimpState.target_boxes.offset % 16 == 0 or _lib.MmtDimpState.target_boxes.offset % 4 == 0


def test_conv_launch_plan_without_gpu():
    """The f16x3 conv's host-side launch plan through mmt_conv2d_f16x3_ws_bytes (no GPU call): split-K slices
    follow the output tiles -- the 3 x 3 stride-1 patch kernel tiles 18 x 18 maps over the flattened batch (32 images:
    81 tiles of 128 pixels instead of 96 per-image ones), the generic kernel's 1 x 1 layers fill the chip unsplit."""
    lib = _lib.load()

    def slices(N, H, W, Cin, Cout, k, s, p, G):
        b = lib.mmt_conv2d_f16x3_ws_bytes(N, H, W, Cin, Cout, k, k, s, p, G)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        return b // (G * N * Ho * Wo * Cout * 4) if b else 1

    # layer3 conv2 (2 backbones): 81 tiles x 2 column tiles x 2 = 324 >= 256 slots -> no split (per-image tiles would
    # be 384); the clf conv (one group, 1 024 -> 512, 288 K-tiles: 512 slots): 81 x 4 = 324 -> 3 slices
    assert lib.mmt_conv2d_f16x3_ws_bytes(32, 18, 18, 256, 256, 3, 3, 1, 1, 2) == 0
    assert slices(32, 18, 18, 1024, 512, 3, 1, 1, 1) == 3
    # 4 images: 11 batch tiles (1 296 pixels) x 2 x 2 = 44 -> split K: 5 slices fill 220 of 256 slots
    assert slices(4, 18, 18, 256, 256, 3, 1, 1, 2) == 5
    assert lib.mmt_conv2d_f16x3_ws_bytes(4, 18, 18, 256, 256, 3, 3, 1, 1, 2) == 5 * 2 * 4 * 324 * 256 * 4
    # layer1 conv3 (1 x 1, 72 x 72): 1 296 x 2 x 2 tiles -- no split
    assert lib.mmt_conv2d_f16x3_ws_bytes(32, 72, 72, 64, 256, 1, 1, 1, 0, 2) == 0
    # one image: per-image tiles (3), few tiles -> split over the chunks (at most Cin / 32)
    assert 1 < slices(1, 18, 18, 256, 256, 3, 1, 1, 2) <= 8
    # invalid shapes report no workspace
    assert lib.mmt_conv2d_f16x3_ws_bytes(0, 18, 18, 256, 256, 3, 3, 1, 1, 2) == 0
