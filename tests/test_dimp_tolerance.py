"""The DiMP tolerance fixture (tests/golden/dimp_spread.npz) pinned on the CPU: its reference runs reproduce the
goldens, its perturbations sit at the level they claim, no perturbed run changes a decision over the frames the
GPU tests assert, and the bars derived from it (tests/dimp_tolerance.py) are what the GPU tests use."""
import os

import numpy as np
import pytest

from tests.dimp_tolerance import CAP, FAMILY, confidence_bar, reference_spread

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MIN_MARGIN, MAX_RUNNER_UP = 5e-3, 0.995   # test_gpu_dimp_branches.py
BRANCHES = ("occlusion", "distractor", "distractor_far", "distractor_branch", "distractor_97", "distractor_above",
            "uncertain_threshold", "hard_sample_threshold", "low_score", "long")


@pytest.fixture(scope="module")
def spread():
    return np.load(os.path.join(GOLDEN, "dimp_spread.npz"))


def _last(gd, name):
    p = name + "/"
    flags, margin, runner = gd[p + "flags"], gd[p + "margin"], gd[p + "runner_up"]
    thin = [t for t in range(1, len(flags)) if margin[t] < MIN_MARGIN or runner[t] > MAX_RUNNER_UP]
    return thin[0] if thin else len(flags)


def test_spread_base_runs_are_the_goldens(spread):
    gd = np.load(os.path.join(GOLDEN, "tracker_dimp.npz"))
    np.testing.assert_array_equal(spread["base/confidence"], gd["confidence"])
    bd = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    for name in BRANCHES:
        np.testing.assert_array_equal(spread[f"{name}:base/confidence"], bd[f"{name}/confidence"])


def test_spread_family_present_at_its_level(spread):
    """Every FAMILY variant exists for every sequence; the seeded noise runs record the perturbation they applied
    in the stage tests' metric (layer3: max |d| / max |ref|), 1e-5 .. 3.5e-5: the HIP backbone's own level
    (1.2e-5 / 1.4e-5, test_gpu_dimp_stages) to about twice it."""
    for seq in [None] + list(BRANCHES):
        p = "" if seq is None else seq + ":"
        for v in FAMILY:
            assert p + v + "/confidence" in spread.files, p + v
            if p + v + "/level" in spread.files:
                assert 1e-5 <= float(spread[p + v + "/level"]) <= 3.5e-5, (p + v, float(spread[p + v + "/level"]))


def test_spread_runs_keep_the_decisions(spread):
    """Over the frames the GPU tests assert, no fp32-order variant of the reference changes a flag: the bars
    compare confidences of the same decisions."""
    bd = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    for seq in [None] + list(BRANCHES):
        p = "" if seq is None else seq + ":"
        last = None if seq is None else _last(bd, seq)
        base = spread[p + "base/flags"][1:last]
        for v in FAMILY:
            np.testing.assert_array_equal(spread[p + v + "/flags"][1:last], base, err_msg=p + v)


def test_derived_bars(spread):
    """The bars the GPU tests apply: 2 x the reference's own fp32-order spread, capped at 1 %.  Printed per
    sequence with the variant that sets it; on the golden sequence the bar is below the former blanket 1 %."""
    bd = np.load(os.path.join(GOLDEN, "tracker_dimp_branches.npz"))
    s, which = reference_spread()
    assert confidence_bar() == pytest.approx(2 * s) and confidence_bar() < CAP
    print(f"tracker_dimp: spread {s:.2e} ({which}) bar {confidence_bar():.2e}")
    for name in BRANCHES:
        last = _last(bd, name)
        s, which = reference_spread(name, last)
        bar = confidence_bar(name, last)
        assert bar == pytest.approx(min(2 * s, CAP)) and bar > 0
        print(f"{name}: frames 1..{last - 1} spread {s:.2e} ({which}) bar {bar:.2e}")
