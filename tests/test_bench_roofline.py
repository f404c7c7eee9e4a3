"""bench.py's roofline bookkeeping on the host (no GPU).

The roofline's kernel is the largest pixel-kernel class by serialised time. The planner's
class ("k_plan": one span over its ~10 kernels, whose bytes are not part of BASELINE.md's B)
is never chosen. Round 6's first final bench line chose it once it grew level with k_plf.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_planner_span_is_never_the_roofline_kernel():
    names = ["k_mc", "k_resid", "k_pred", "k_lf", "k_plf", "k_lfr", "k_plan"]
    # C3-like: the planner span slightly above k_plf
    ksum = {"k_resid": [1.9, 60], "k_lf": [2.6, 81], "k_plf": [4.25, 48], "k_plan": [4.28, 12]}
    assert bench.dominant_kernel(names, ksum) == "k_plf"
    # C2-like: the row LF dominates
    ksum = {"k_mc": [1.6, 30], "k_resid": [1.3, 30], "k_plf": [2.0, 20], "k_lfr": [9.6, 30], "k_plan": [0.9, 4]}
    assert bench.dominant_kernel(names, ksum) == "k_lfr"


def test_kernels_without_time_are_ranked_last():
    names = ["k_mc", "k_plf", "k_plan"]
    assert bench.dominant_kernel(names, {"k_plf": [1.0, 2]}) == "k_plf"
