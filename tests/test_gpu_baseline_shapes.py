"""GPU parity at the BASELINE.md shapes, through the code path bench.py times.

Each case builds the config's synthetic packets exactly as bench.py does
(`bench.make_frames`: same generator, seeds, GOP references, tile columns), stages them as
one batch, replays the batch's launch sequence twice (the first run captures the HIP
graph, the second replays it, as in the bench's timed steps), and compares every visible
plane of every frame with the CPU oracle (`oracle.decode_frame`, the scalar restatement of
vp9dsp_template.c / vp9recon.c / vp9lpf.c / vp9_mc_template.c), sample-exact.

Frame counts are cut down from the bench's 120 / 60 so the oracle finishes in seconds, but
every schedule the bench's full batch uses is exercised:
  - C3 / C4: 2 frame groups (the default) of >= 8 keyframes each, i.e. wide phases (k_resid
    launches, fused k_plf intra + LF diagonals, 4 tile columns) on 2 concurrent HIP streams;
    C3 also with VP9HIP_STREAMS=3 (3 groups, the round-1 default);
  - C2: GOP chains of key + P frames, i.e. narrow phases (the inter level schedule of k_pred,
    k_mc, the row-pipelined k_lfr over 17 SB rows), 2 chains on 2 streams;
  - C5: 8K 10-bit, 8 tile columns, key + 2 P (k_lfr over 68 SB rows x 120 SB columns).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

SHAPES = [
    # (config, frames, VP9HIP_STREAMS or None, frame groups expected): GOP lengths are the
    # config's (C2 / C5: 32; the cut keeps key + P chains)
    ("C3", 28, None, 2),                 # chains split evenly over the groups (stage: nroots % G)
    ("C3", 27, "3", 3),
    ("C4", 24, None, 2),
    ("C2", 6, None, 2),
    ("C5", 3, None, 1),
]


def _two_chains(frames, refs, geom, n_per_chain):
    """C2: two independent GOP chains of n frames (key + P), taken from the first two GOPs."""
    gop = geom[4]
    keep = list(range(n_per_chain)) + list(range(gop, gop + n_per_chain))
    remap = {old: new for new, old in enumerate(keep)}
    fr = [frames[i] for i in keep]
    rf = [None if refs[i] is None else tuple(remap[r] for r in refs[i]) for i in keep]
    return fr, rf


@pytest.mark.parametrize("config,n,streams,groups", SHAPES)
def test_baseline_shape_parity(v9, orc, monkeypatch, config, n, streams, groups):
    if streams is None:
        monkeypatch.delenv("VP9HIP_STREAMS", raising=False)
    else:
        monkeypatch.setenv("VP9HIP_STREAMS", streams)   # read when the context opens
    if config == "C2":
        frames, refs, geom = bench.make_frames(v9, config, 32 + n // 2)
        frames, refs = _two_chains(frames, refs, geom, n // 2)
    else:
        frames, refs, geom = bench.make_frames(v9, config, n)
    W, H, BPP, log2, gop = geom
    dev = v9.Device(0)
    try:
        dev.configure(W, H, BPP, nbufs=len(frames))
        inter = any(r is not None for r in refs)
        dev.stage_batch(frames, list(range(len(frames))), refs if inter else None)
        dev.set_timing(False)             # the bench's timed configuration: graph capture + replay
        for _ in range(2):
            dev.run_batch()
            dev.sync()
        assert dev.groups() == groups
        # C2: decode order of the two chains is chain-major in `frames`
        bad = []
        for i, ref in bench.oracle_frames(v9, orc, frames, refs, (W, H, BPP, log2, len(frames)
                                                                   if config == "C2" else gop)):
            d = bench.compare_frame(v9, dev.download(i), ref, geom)
            if d:
                bad.append((i, d))
        assert not bad, "%s: frames differing from the oracle (frame, samples): %s" % (config, bad)
    finally:
        dev.close()
