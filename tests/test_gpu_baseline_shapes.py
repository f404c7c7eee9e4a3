"""GPU parity at the BASELINE.md shapes, through the code path bench.py times.

Each case builds the config's synthetic packets exactly as bench.py does
(`bench.make_frames`: same generator, seeds, GOP references, tile columns) and compares
every visible plane of every frame with the CPU oracle (`oracle.decode_frame`, the scalar
restatement of vp9dsp_template.c / vp9recon.c / vp9lpf.c / vp9_mc_template.c),
sample-exact. Frame counts are cut down from the bench's 120 / 60 so the oracle finishes in
seconds.

The timed shape (TIMED): the library defaults (one frame-group stream per batch slot) with
the bench's batches in flight, C3 / C4 at 3 slots (VP9HIP_PIPELINE_SLOTS, as the decoder
and the FFHWAccel adapter run) and C2 at 4: the workload staged into every slot
(`bench.stage_slots`), every frame buffer poisoned, then `bench.run_slots` rotating over
the slots with HIP graph replay and no host wait between batches, exactly the bench's timed
loop; every frame of every slot is checked.

Single-slot schedules (SINGLE), one batch replayed twice (capture, then replay):
  - C3 / C4 at 2 and 3 frame groups (VP9HIP_STREAMS): wide phases (k_resid launches, fused
    k_plf intra + LF diagonals, 4 tile columns) on concurrent HIP streams;
  - C2: GOP chains of key + P frames, i.e. narrow phases (the inter level schedule, k_mcq,
    the row-pipelined k_lfro with intra workers), 2 chains on 2 streams;
  - C5: 8K 10-bit, 8 tile columns, key + 2 P (k_lfro over 68 SB rows x 120 SB columns).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

SINGLE = [
    # (config, frames, VP9HIP_STREAMS, frame groups expected): GOP lengths are the config's
    # (C2 / C5: 32; the cut keeps key + P chains)
    ("C3", 28, "2", 2),                  # chains split evenly over the groups (stage: nroots % G)
    ("C3", 27, "3", 3),
    ("C4", 24, "2", 2),
    ("C2", 6, "2", 2),
    ("C5", 3, None, 1),
]

TIMED = [
    # (config, frames per slot): batches in flight = bench.INFLIGHT[config]
    ("C3", 24),
    ("C4", 16),
    ("C2", 8),                           # two GOP chains of key + 3 P per slot
]


def _two_chains(frames, refs, geom, n_per_chain):
    """C2: two independent GOP chains of n frames (key + P), taken from the first two GOPs."""
    gop = geom[4]
    keep = list(range(n_per_chain)) + list(range(gop, gop + n_per_chain))
    remap = {old: new for new, old in enumerate(keep)}
    fr = [frames[i] for i in keep]
    rf = [None if refs[i] is None else tuple(remap[r] for r in refs[i]) for i in keep]
    return fr, rf


def _workload(v9, config, n):
    if config == "C2":
        frames, refs, geom = bench.make_frames(v9, config, 32 + n // 2)
        frames, refs = _two_chains(frames, refs, geom, n // 2)
        geom = geom[:4] + (len(frames),)         # decode order is chain-major in `frames`
    else:
        frames, refs, geom = bench.make_frames(v9, config, n)
    return frames, refs, geom


def _compare(v9, orc, dev, frames, refs, geom, slots):
    """Every frame of every slot (slot k holds frame i in buffer k * n + i) vs the oracle."""
    n, bad = len(frames), []
    for i, ref in bench.oracle_frames(v9, orc, frames, refs, geom):
        for k in range(slots):
            d = bench.compare_frame(v9, dev.download(k * n + i), ref, geom)
            if d:
                bad.append((k, i, d))
    return bad


@pytest.mark.parametrize("config,n,streams,groups", SINGLE)
def test_baseline_shape_parity(v9, orc, monkeypatch, config, n, streams, groups):
    if streams is None:
        monkeypatch.delenv("VP9HIP_STREAMS", raising=False)
    else:
        monkeypatch.setenv("VP9HIP_STREAMS", streams)   # read when the context opens
    frames, refs, geom = _workload(v9, config, n)
    W, H, BPP = geom[:3]
    dev = v9.Device(0)
    try:
        dev.configure(W, H, BPP, nbufs=len(frames))
        inter = any(r is not None for r in refs)
        dev.stage_batch(frames, list(range(len(frames))), refs if inter else None)
        dev.set_timing(False)             # graph capture + replay
        for _ in range(2):
            dev.run_batch()
            dev.sync()
        assert dev.groups() == groups
        bad = _compare(v9, orc, dev, frames, refs, geom, 1)
        assert not bad, "%s: frames differing from the oracle (slot, frame, samples): %s" % (config, bad)
    finally:
        dev.close()


@pytest.mark.parametrize("config,n", TIMED)
def test_timed_shape_parity(v9, orc, monkeypatch, config, n):
    monkeypatch.delenv("VP9HIP_STREAMS", raising=False)     # the library default: 1 per slot
    inflight = bench.INFLIGHT[config]
    frames, refs, geom = _workload(v9, config, n)
    W, H, BPP = geom[:3]
    gop = 1 if all(r is None for r in refs) else geom[4]
    dev = v9.Device(0)
    try:
        dev.configure(W, H, BPP, nbufs=n * inflight)
        bench.stage_slots(dev, frames, refs, gop, inflight)
        dev.set_timing(False)
        bench.run_slots(dev, inflight, inflight)                  # warm-up: graph capture per slot
        dev.sync()
        dev.fill(0, n * inflight, bench.POISON)
        dev.sync()
        bench.run_slots(dev, 2 * inflight + 1, inflight)          # replays, no host wait between
        dev.sync()
        for k in range(inflight):
            dev.set_slot(k)
            assert dev.groups() == 1
        dev.set_slot(0)
        bad = _compare(v9, orc, dev, frames, refs, geom, inflight)
        assert not bad, "%s: frames differing from the oracle (slot, frame, samples): %s" % (config, bad)
    finally:
        dev.close()
