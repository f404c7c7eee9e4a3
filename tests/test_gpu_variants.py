"""The A/B switches of the inter-frame kernels stay bit-exact: the single-tile row LF
(VP9HIP_LFR_DB=0 instead of k_lfrd), 256-thread high-bit-depth MC (VP9HIP_MC64=0) and one
residual launch per transform size (VP9HIP_RESID_MULTI=0). Each is switched off (read
per launch / per staging) on a key + P chain of the C2 (1080p 8-bit) or C5 (8K 10-bit)
shape, decoded through the bench's batch path and compared with the CPU oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = [
    ("VP9HIP_LFR_DB", "C2", 4),
    ("VP9HIP_LFR_DB", "C5", 2),
    ("VP9HIP_MC64", "C5", 2),
    ("VP9HIP_RESID_MULTI", "C2", 4),
    ("VP9HIP_RESID_MULTI", "C5", 2),
]


@pytest.mark.parametrize("var,config,n", CASES)
def test_switch_off_matches_oracle(v9, orc, var, config, n):
    frames, refs, geom = bench.make_frames(v9, config, n)
    W, H, BPP, log2, gop = geom
    os.environ[var] = "0"
    dev = v9.Device(0)
    try:
        dev.configure(W, H, BPP, nbufs=len(frames))
        dev.stage_batch(frames, list(range(len(frames))), refs)
        dev.run_batch()
        dev.sync()
        bad = []
        for i, ref in bench.oracle_frames(v9, orc, frames, refs, (W, H, BPP, log2, gop)):
            d = bench.compare_frame(v9, dev.download(i), ref, geom)
            if d:
                bad.append((i, d))
        assert not bad, "%s=0 %s: frames differing from the oracle: %s" % (var, config, bad)
    finally:
        dev.close()
        del os.environ[var]
