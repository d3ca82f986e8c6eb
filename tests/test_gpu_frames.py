"""RGB-D frame assembly on the GPU (mmt_rgbd_assemble) vs the CPU restatement (oracle/frames.py):
bit-exact, with and without the median depth clip, even and odd pixel counts, a constant depth
map (NORM_MINMAX with max == min) and a caller-supplied colormap.  Parity at the OpenCV boundary
is unpinned (no cv2 in the image)."""
import numpy as np
import pytest
import torch

from oracle import frames as ofr

pytestmark = pytest.mark.gpu


def _case(seed, H, W, kind):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if kind == "const":
        dp = np.full((H, W), 1234, np.uint16)
    elif kind == "far":   # a far background that the clip removes
        dp = rng.integers(500, 3000, (H, W)).astype(np.uint16)
        dp[: H // 3] = 60000
    else:
        dp = rng.integers(0, 65536, (H, W)).astype(np.uint16)
    return rgb, dp


@pytest.mark.parametrize("H,W", [(360, 640), (37, 53), (480, 641)])
@pytest.mark.parametrize("kind", ["rand", "far", "const"])
@pytest.mark.parametrize("clip", [True, False])
def test_rgbd_assemble_bitexact(H, W, kind, clip):
    from mmtrack_amd.frames import assemble_rgbd
    rgb, dp = _case(H * W, H, W, kind)
    got = assemble_rgbd(rgb, dp, depth_clip=clip).cpu().numpy()
    ref = ofr.rgbd_frame(rgb, dp, depth_clip=clip)
    np.testing.assert_array_equal(got, ref)


def test_rgbd_custom_lut_and_device_inputs():
    from mmtrack_amd.frames import assemble_rgbd
    rgb, dp = _case(3, 120, 160, "far")
    lut = np.random.default_rng(0).integers(0, 256, (256, 3), dtype=np.uint8)
    got = assemble_rgbd(torch.from_numpy(rgb).cuda(), torch.from_numpy(dp.view(np.int16)).cuda(), True, lut)
    np.testing.assert_array_equal(got.cpu().numpy(), ofr.rgbd_frame(rgb, dp, True, lut))
    with pytest.raises(ValueError):
        assemble_rgbd(rgb[:, :10], dp)


def test_rgbd_dataset_path_end_to_end(tmp_path):
    """A DepthTrack-layout folder (color/*.jpg, depth/*.png 16-bit, groundtruth.txt) through the RGB-D
    workspace CLI: frames assembled on the GPU, tracked, one result file in the reference format."""
    from PIL import Image

    from mmtrack_amd import synth
    from mmtrack_amd.workspace import main
    frames, gt = synth.make_frames(5, 5, 240, 320, 3, box=(120.0, 90.0, 40.0, 30.0))
    seq = tmp_path / "data" / "seqA"
    (seq / "color").mkdir(parents=True)
    (seq / "depth").mkdir()
    rng = np.random.default_rng(0)
    for i, f in enumerate(frames):
        Image.fromarray(f).save(seq / "color" / f"{i + 1:08d}.jpg", quality=95)
        dp = rng.integers(800, 4000, (240, 320)).astype(np.uint16)
        Image.fromarray(dp).save(seq / "depth" / f"{i + 1:08d}.png")
    np.savetxt(seq / "groundtruth.txt", gt, delimiter=",")
    main("rgbd", ["--seq_home", str(tmp_path / "data"), "--dataset_name", "DepthTrack", "--synthetic_weights",
                  "--out_root", str(tmp_path / "out")])
    res = np.loadtxt(tmp_path / "out" / "RGBD_workspace" / "results" / "DepthTrack" / "deep_rgbd" / "seqA.txt")
    assert res.shape == (5, 4) and np.isfinite(res).all()
    np.testing.assert_allclose(res[0], gt[0])
