import sys, numpy as np, torch
sys.path.insert(0, 'multi-modal-trakcing-bechmark_amd'); sys.path.insert(0, '.')
from mmtrack_amd.frames import assemble_rgbd
from oracle import frames as ofr
rng = np.random.default_rng(360*640)
H, W = 360, 640
rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
dp = rng.integers(500, 3000, (H, W)).astype(np.uint16); dp[: H // 3] = 60000
ident = np.repeat(np.arange(256, dtype=np.uint8)[:, None], 3, 1)
got = assemble_rgbd(rgb, dp, depth_clip=False, lut_bgr=ident).cpu().numpy()[..., 3]
ref = ofr.normalize_minmax_u8(dp)
bad = np.argwhere(got != ref)
print("d8 mismatches", len(bad))
for y, x in bad[:5]:
    d = dp[y, x]; lo, hi = float(dp.min()), float(dp.max()); sc = 255.0/(hi-lo); sh = 0.0 - lo*sc
    f = np.float32(d) * np.float32(sc) + np.float32(sh)
    print(d, got[y, x], ref[y, x], repr(f), repr(np.float32(d) * np.float32(sc)), np.float32(sh))
# JET table check
dp2 = np.tile(np.arange(256, dtype=np.uint16), (4, 1))
rgb2 = np.zeros((4, 256, 3), np.uint8)
got2 = assemble_rgbd(rgb2, dp2, depth_clip=False).cpu().numpy()[0, :, 3:]
print("jet mismatches", (got2 != ofr.jet_bgr()).sum())
