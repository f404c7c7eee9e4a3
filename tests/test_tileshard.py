"""Tile-column sharding of one stream: ffmpeg-hybrid_amd/tileshard.py.

CPU (gloo): the exchange logic against a fake device whose frames are numpy planes.
- Each rank "reconstructs" only its tile columns with a known pattern.
- After the all-gather, every rank's pre-LF frame must be complete before its loop
  filter runs.
- Cases: uneven tile splits and ranks without tiles.

GPU: real shards vs the CPU oracle, bit-exact, on an inter stream with intra blocks.
- In one process: one context per shard, the exchange done by hand.
- Across two processes (gloo, both on cuda:0).
"""
import ctypes
import importlib
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ts():
    return importlib.import_module("ffmpeg-hybrid_amd.tileshard")


class FakeDev:
    """Stripe geometry of vp9hip_stripe (tile offsets of vp9.c:1244-1250, 8-aligned
    size, 4:2:0) over numpy frames; RECON writes the rank's own columns only."""
    PART_RECON, PART_LF = 0, 1

    def __init__(self, w, h, log2, phases, lo, hi):
        self.w8, self.h8 = (w + 7) & ~7, (h + 7) & ~7
        self.sb_cols, self.log2 = (w + 63) >> 6, log2
        self.ph = phases                     # list of frame-index lists
        self.lo, self.hi = lo, hi
        self.frames = {i: [np.zeros((self.h8 >> (p > 0), self.w8 >> (p > 0)), np.uint8) for p in range(3)]
                       for fr in phases for i in fr}
        self.checked = []

    def _x(self, t):
        nt = 1 << self.log2
        return min(min(min(t, nt) * self.sb_cols >> self.log2, self.sb_cols) * 64, self.w8)

    def _pattern(self, i, p):
        a = self.frames[i][p]
        y, x = np.mgrid[0:a.shape[0], 0:a.shape[1]]
        return ((i * 7 + x * 3 + y * 5 + p) & 255).astype(np.uint8)

    def phases(self):
        return len(self.ph)

    def phase_frames(self, ph):
        return list(self.ph[ph])

    def sync(self):
        pass

    def run_phase(self, ph, part):
        for i in self.ph[ph]:
            for p in range(3):
                x0, x1 = self._x(self.lo) >> (p > 0), self._x(self.hi) >> (p > 0)
                if part == self.PART_RECON:
                    self.frames[i][p][:, x0:x1] = self._pattern(i, p)[:, x0:x1]
                else:
                    self.checked.append(bool(np.array_equal(self.frames[i][p], self._pattern(i, p))))

    def stripe(self, i, lo, hi, dev_ptr=None, to_frame=False):
        off = 0
        for p in range(3):
            x0, x1 = self._x(lo) >> (p > 0), self._x(hi) >> (p > 0)
            a = self.frames[i][p]
            n = (x1 - x0) * a.shape[0]
            if dev_ptr and n:
                if to_frame:
                    buf = ctypes.string_at(dev_ptr + off, n)
                    a[:, x0:x1] = np.frombuffer(buf, np.uint8).reshape(a.shape[0], x1 - x0)
                else:
                    src = np.ascontiguousarray(a[:, x0:x1])       # kept alive across the copy
                    ctypes.memmove(dev_ptr + off, src.ctypes.data, n)
            off += n
        return off


def _cpu_worker(rank, world, port, w, h, log2, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ts = _ts()
        lo, hi = ts.tile_ranges(1 << log2, world)[rank]
        dev = FakeDev(w, h, log2, [[0, 1], [2], [3, 4]], lo, hi)
        sh = ts.TileShard(dev, 1 << log2, rank, world)
        sh.run()
        q.put((rank, dev.checked, sh.bytes_per_phase()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,log2", [(2, 1000, 200, 2), (3, 600, 70, 1)])
def test_exchange_completes_every_frame(world, w, h, log2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + world
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, w, h, log2, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, checked, bpp in res:
        assert len(checked) == 5 * 3 and all(checked), (rank, checked)
        assert all(m > 0 for m, _ in bpp)


def test_nccl_exchange_is_stream_ordered(monkeypatch):
    """The RCCL branch, host logic only (no GPU here): the all-gather is issued under the
    context's stream (vp9hip_frame_device's handle as an ExternalStream) and the host never
    syncs the context inside a pass; the exchanged stripes still complete every frame."""
    import contextlib
    ts = _ts()
    w, h, log2, world, rank = 1000, 200, 2, 2, 0
    phases = [[0, 1], [2], [3, 4]]
    ranges = ts.tile_ranges(1 << log2, world)

    class Dev(FakeDev):
        syncs = 0

        def sync(self):
            Dev.syncs += 1

        def frame_device(self, buf):
            return None, None, (w, h), 0xC0FFEE

    dev = Dev(w, h, log2, phases, *ranges[rank])
    peer = FakeDev(w, h, log2, phases, *ranges[1 - rank])
    for ph in range(len(phases)):
        peer.run_phase(ph, FakeDev.PART_RECON)
    state = {"stream": None, "ph": None, "issued": []}

    class Ext:
        def __init__(self, handle, device=None):
            self.handle = handle

    @contextlib.contextmanager
    def under(s):
        state["stream"] = s
        try:
            yield
        finally:
            state["stream"] = None

    def gather(out, inp, group=None):
        s = state["stream"]
        state["issued"].append(s.handle if s is not None else None)
        m = inp.numel()
        out[rank * m:(rank + 1) * m].copy_(inp)
        off = (1 - rank) * m
        for i in phases[state["ph"]]:
            off += peer.stripe(i, *ranges[1 - rank], out.data_ptr() + off)

    monkeypatch.setattr(ts.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(ts.dist, "all_gather_into_tensor", gather)
    monkeypatch.setattr(ts.torch.cuda, "ExternalStream", Ext)
    monkeypatch.setattr(ts.torch.cuda, "stream", under)
    sh = ts.TileShard(dev, 1 << log2, rank, world)
    for ph in range(len(phases)):
        state["ph"] = ph
        sh.run_phase(ph)
    assert Dev.syncs == 0
    assert state["issued"] == [0xC0FFEE] * len(phases)
    assert len(dev.checked) == 5 * 3 and all(dev.checked), dev.checked


def test_tile_ranges():
    ts = _ts()
    assert ts.tile_ranges(8, 2) == [(0, 4), (4, 8)]
    assert ts.tile_ranges(4, 3) == [(0, 1), (1, 2), (2, 4)]
    assert ts.tile_ranges(2, 4) == [(0, 0), (0, 1), (1, 1), (1, 2)]   # ranks without tiles still filter


# ---------------------------------------------------------------- GPU

def _stream(v9, w, h, log2, bpp=8):
    """key + 3 P frames: LAST = previous, GOLDEN = key, compound / bilinear variants,
    intra blocks inside the P frames (synth default)."""
    frames, refs = [v9.SynthFrame(v9.synth_params(w, h, bpp, seed=900, log2_tile_cols=log2))], [None]
    for k in range(1, 4):
        kw = {"compound": 1} if k == 2 else {"bilinear": 1} if k == 3 else {}
        frames.append(v9.SynthFrame(v9.synth_params(w, h, bpp, seed=900 + k, inter=1, log2_tile_cols=log2, **kw)))
        refs.append((k - 1, 0, k - 1))
    return frames, refs


def _oracle(v9, orc, frames, refs, w, h, bpp):
    dec = []
    for f, r in zip(frames, refs):
        out = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, out, None if r is None else [dec[r[0]], dec[r[1]], dec[r[2]]])
        dec.append(out)
    return dec


def _cmp(v9, got, ref, w, h, what):
    for p, (a, b) in enumerate(zip(v9.visible(got, w, h), v9.visible(ref, w, h))):
        if not np.array_equal(a, b):
            ys, xs = np.nonzero(a != b)
            raise AssertionError("%s plane %d: %d px differ, first at (x=%d, y=%d)" % (what, p, len(ys), xs[0], ys[0]))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,log2,bpp,nshards", [(1024, 136, 2, 8, 2), (520, 72, 1, 10, 3), (256, 64, 0, 8, 1)])
def test_shards_in_one_process_match_oracle(v9, orc, w, h, log2, bpp, nshards):
    """One context per shard on the same GPU; the all-gather done by hand through
    device buffers: every shard must end each phase with the oracle's frames."""
    frames, refs = _stream(v9, w, h, log2, bpp)
    ranges = _ts().tile_ranges(1 << log2, nshards)
    devs = []
    for lo, hi in ranges:
        d = v9.Device(0)
        d.configure(w, h, bpp, nbufs=len(frames))
        d.stage_batch(frames, list(range(len(frames))), refs, tiles=(lo, hi))
        devs.append(d)
    assert all(d.phases() == len(frames) for d in devs)
    for ph in range(devs[0].phases()):
        (i,) = devs[0].phase_frames(ph)
        for d in devs:
            d.run_phase(ph, d.PART_RECON)
        bufs = []
        for d, (lo, hi) in zip(devs, ranges):
            n = d.stripe(i, lo, hi)
            t = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda:0")
            if n:
                d.stripe(i, lo, hi, t.data_ptr())
            d.sync()
            bufs.append((t, n))
        for d in devs:
            for q, (lo, hi) in enumerate(ranges):
                if bufs[q][1]:
                    d.stripe(i, lo, hi, bufs[q][0].data_ptr(), to_frame=True)
            d.run_phase(ph, d.PART_LF)
            d.sync()
    ref = _oracle(v9, orc, frames, refs, w, h, bpp)
    for k, d in enumerate(devs):
        for i in range(len(frames)):
            _cmp(v9, d.download(i), ref[i], w, h, "shard %d frame %d" % (k, i))
    for d in devs:
        d.close()


def _gpu_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v9 = importlib.import_module("ffmpeg-hybrid_amd")
        ts = _ts()
        w, h, log2 = 1032, 72, 2
        frames, refs = _stream(v9, w, h, log2)
        lo, hi = ts.tile_ranges(1 << log2, world)[rank]
        dev = v9.Device(0)
        dev.configure(w, h, 8, nbufs=len(frames))
        dev.stage_batch(frames, list(range(len(frames))), refs, tiles=(lo, hi))
        ts.TileShard(dev, 1 << log2, rank, world, device="cuda:0").run()
        outs = [dev.download(i) for i in range(len(frames))]
        dev.close()
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_tileshard_matches_oracle(v9, orc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w, h = 1032, 72
    frames, refs = _stream(v9, w, h, 2)
    ref = _oracle(v9, orc, frames, refs, w, h, 8)
    for rank, outs in res:
        for i, o in enumerate(outs):
            _cmp(v9, o, ref[i], w, h, "rank %d frame %d" % (rank, i))
