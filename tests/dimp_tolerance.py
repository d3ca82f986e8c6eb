"""The DiMP end-to-end confidence bars, derived from the reference's own fp32-order spread.

tests/golden/dimp_spread.npz (tests/golden/make_dimp_spread.py) holds the REFERENCE DeT tracker's per-frame
confidences on every golden DiMP sequence, run again with its backbone features perturbed at the level the HIP
backbone differs from it (test_gpu_dimp_stages: init layer3 within 1.2e-5 / 1.4e-5 of the map's maximum in f16x3 /
fp32; the ``feat5e-6`` seeds land at 1.1e-5 .. 1.6e-5 in that metric, ``feat1e-5`` at 2.5e-5 .. 3.2e-5) and with its
two backbones in float64 (``bb64``: the reference's own fp32 rounding of its features removed).

Why the spread is this large (tools/diag/dimp_feed_ref.py, profiles/r05_dimp_feed_ref.txt): on the golden
sequence one score element of the 10-step Gauss-Newton initialisation sits 2.2e-6 of the score maximum from
LeakyReluPar's kink at step 6; features that differ by ~1e-5 move it across, the score mask and gradient change
discontinuously and the filter moves by ~1e-3 at step 8.  Run on the HIP path's own features, the reference
optimiser reproduces the HIP filter trajectory to 1e-4 (and each HIP Gauss-Newton step matches the reference step
from the same inputs to 4e-7): the drift is carried in by fp32-order feature differences, not added downstream.

Bar per sequence = 2 x the largest relative confidence difference any of those reference runs shows against the
reference's own run over the frames the test asserts, never looser than the former blanket 1 %."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# fp32-order variants of the reference run (make_dimp_spread.py): exact backbone, seeded feature noise at the HIP
# backbone's error level and at about twice it
FAMILY = ("bb64", "feat3e-6", "feat5e-6_s1234", "feat5e-6_s99", "feat5e-6_s7", "feat5e-6_s11",
          "feat1e-5", "feat1e-5_s2", "feat1e-5_s7", "feat1e-5_s11")
CAP = 1e-2
_cache = {}


def _spread_npz():
    if "d" not in _cache:
        _cache["d"] = np.load(os.path.join(GOLDEN, "dimp_spread.npz"))
    return _cache["d"]


def reference_spread(seq=None, last=None):
    """(largest relative confidence difference of the FAMILY runs vs the reference's own run over frames
    [1, last), the variant that gives it) for the golden sequence (seq None) or a branch sequence."""
    d = _spread_npz()
    p = "" if seq is None else seq + ":"
    base = d[p + "base/confidence"]
    last = len(base) if last is None else last
    best, which = 0.0, None
    for v in FAMILY:
        k = p + v + "/confidence"
        if k not in d.files:
            continue
        c = d[k]
        rel = float(np.max(np.abs(c[1:last] - base[1:last]) / np.abs(base[1:last])))
        if rel > best:
            best, which = rel, v
    return best, which


def confidence_bar(seq=None, last=None):
    """2 x reference_spread, capped at 1 %."""
    return min(2.0 * reference_spread(seq, last)[0], CAP)
