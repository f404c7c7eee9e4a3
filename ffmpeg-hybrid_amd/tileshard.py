"""Tile-column sharding of ONE VP9 stream over ranks (inter streams with tiles).

VP9 tile columns decode independently: entropy, residuals, MC and intra are all local
to a tile column. Intra `have_left` stops at the tile start (vp9recon.c:46), above-right
never reaches past the block, and MC reads only reference frames. The loop filter and
the next frame's MC are frame-global. The reference's slice-threaded decode follows the
same split: tile-column jobs (decode_tiles_mt, vp9.c:1442-1520), then the loop filter
(loopfilter_proc, vp9.c:1522-1551).

One process per GPU. Each rank:
- stages the whole stream but reconstructs only its tile columns;
- per phase (the frames of one chain position), exchanges the pre-LF stripes of those
  frames with one all-gather, then runs the loop filter over whole frames.
Every rank ends a phase holding the full post-LF frames that later phases reference.
The collective is RCCL (`nccl` backend) on device buffers, stream-ordered: the packs,
the all-gather and the unpacks all follow the context's HIP stream (the one
vp9hip_frame_device returns), so a phase never waits on the host. The `gloo` backend
(the CPU tests, several ranks sharing one GPU) stages the same bytes through host
tensors, which needs a host sync per phase.

Per phase, rank r ships the stripes of its tile columns: about P/N bytes (P = frame
bytes, N = ranks). It receives P(N-1)/N, padded to the largest stripe.
"""
import torch
import torch.distributed as dist


def tile_ranges(n_tiles, world):
    """Contiguous tile-column ranges [lo, hi) per rank (empty for ranks beyond n_tiles)."""
    return [(r * n_tiles // world, (r + 1) * n_tiles // world) for r in range(world)]


def stream_tiles(frames):
    """Tile columns of a stream; sharding needs one tiling for all its frames."""
    logs = {int((f.pkt if hasattr(f, "pkt") else f).log2_tile_cols) for f in frames}
    if len(logs) != 1:
        raise ValueError("tile sharding needs one log2_tile_cols for the whole batch, got %s" % sorted(logs))
    return 1 << logs.pop()


class TileShard:
    """Drive a staged, tile-sharded batch on `dev` (a Device, or any object with the same
    phases / phase_frames / run_phase / stripe / sync methods)."""

    def __init__(self, dev, n_tiles, rank, world, group=None, device=None):
        self.dev, self.rank, self.world, self.group = dev, rank, world, group
        self.ranges = tile_ranges(n_tiles, world)
        self.lo, self.hi = self.ranges[rank]
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.host_staged = world > 1 and dist.get_backend(group) != "nccl"
        # exchange layout per phase: for each rank, its frames' stripes back to back
        self.plan = []
        for ph in range(dev.phases()):
            fr = dev.phase_frames(ph)
            sizes = [[dev.stripe(i, lo, hi) for i in fr] for lo, hi in self.ranges]
            self.plan.append((fr, sizes, max(sum(s) for s in sizes)))
        m = max((p[2] for p in self.plan), default=0) if world > 1 else 0
        self.send = torch.empty(max(m, 1), dtype=torch.uint8, device=self.device)
        self.recv = torch.empty(max(m, 1) * world, dtype=torch.uint8, device=self.device)
        self._ext = None

    def _stream(self):
        """The context's HIP stream as a torch stream: every launch of run_phase and every
        vp9hip_stripe copy is enqueued on it."""
        if self._ext is None:
            st = self.dev.frame_device(0)[3]
            self._ext = torch.cuda.ExternalStream(st, device=self.device)
        return self._ext

    def bytes_per_phase(self):
        """(bytes sent, bytes received) by this rank per phase, padded as exchanged."""
        if self.world == 1:
            return [(0, 0) for _ in self.plan]
        return [(m, m * (self.world - 1)) for _, _, m in self.plan]

    def _all_gather(self, m):
        if self.world == 1:
            return
        if not self.host_staged:
            # RCCL's stream waits for the context stream (the packs), and the context
            # stream waits for RCCL's (the unpacks that follow): no host round trip
            with torch.cuda.stream(self._stream()):
                dist.all_gather_into_tensor(self.recv[:m * self.world], self.send[:m], group=self.group)
            return
        self.dev.sync()                         # packed stripes complete before the host copy
        parts = [torch.empty(m, dtype=torch.uint8) for _ in range(self.world)]
        dist.all_gather(parts, self.send[:m].cpu(), group=self.group)
        self.recv[:m * self.world].copy_(torch.cat(parts))
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def run_phase(self, ph):
        dev = self.dev
        fr, sizes, m = self.plan[ph]
        dev.run_phase(ph, dev.PART_RECON)
        if self.world > 1 and m:
            off = 0
            for i, n in zip(fr, sizes[self.rank]):
                if n:
                    dev.stripe(i, self.lo, self.hi, self.send.data_ptr() + off, to_frame=False)
                off += n
            self._all_gather(m)
            base = self.recv.data_ptr()
            for q, (lo, hi) in enumerate(self.ranges):
                if q == self.rank:
                    continue
                off = q * m
                for i, n in zip(fr, sizes[q]):
                    if n:
                        dev.stripe(i, lo, hi, base + off, to_frame=True)
                    off += n
        dev.run_phase(ph, dev.PART_LF)

    def run(self):
        """One pass over the staged stream (every phase, in chain order)."""
        for ph in range(len(self.plan)):
            self.run_phase(ph)
        self.dev.sync()
