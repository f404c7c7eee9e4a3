"""CPU (gloo, world_size 2): the N>1 path of bench.py — distinct frames per rank (frame
sharding, no data-path collective), max-over-ranks timing, whole-job aggregate."""
import importlib.util
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench()
        import importlib
        v9 = importlib.import_module("ffmpeg-hybrid_amd")
        # each rank plans its own frames (host planner, no GPU needed)
        f = v9.SynthFrame(v9.synth_params(512, 256, 8, seed=b.frame_seed(rank, 0), log2_tile_cols=1))
        st = v9.plan_stats(f)
        elapsed = 1.0 + rank                   # rank 1 is the slow one
        dist.barrier()
        emax = b.reduce_elapsed(elapsed, dist)
        fps, ms = b.aggregate(frames_per_rank=120, steps=5, world=world, elapsed_max=emax)
        q.put((rank, b.frame_seed(rank, 0), st["pjobs"], emax, fps, ms))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_max_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, j0, e0, f0, m0), (r1, s1, j1, e1, f1, m1) = res
    assert s0 != s1                            # disjoint frame streams per rank
    assert j0 != j1                            # ... so different work
    assert e0 == e1 == 2.0                     # both ranks report the max
    assert f0 == pytest.approx(120 * 5 * 2 / 2.0) and f0 == f1
    assert m0 == pytest.approx(400.0)


def test_single_rank_aggregate_is_identity():
    b = _bench()
    assert b.reduce_elapsed(3.0, None) == 3.0
    fps, ms = b.aggregate(120, 4, 1, 2.0)
    assert fps == pytest.approx(240.0) and ms == pytest.approx(500.0)


@pytest.mark.gpu
def test_two_rank_bench_verifies_every_rank():
    """bench.py at world 2 as the driver launches it (torch.distributed.run, one process per
    rank; both ranks share the box's one GPU here): every rank decodes its own frames after a
    poison fill and compares a sample of them with the oracle; rank 0 reports each rank's
    result and device."""
    import json
    import subprocess
    import sys
    port = 29700 + os.getpid() % 200
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--frames", "8", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2
    v = d["verify"]
    assert v["mismatched"] == []
    assert [p["rank"] for p in v["per_rank"]] == [0, 1]
    assert all(p["frames"] == 2 * 2 for p in v["per_rank"])          # 2 frames x 2 batch slots per rank
    assert d["verified_frames"] == 8
    assert [x["rank"] for x in d["config"]["ranks"]] == [0, 1]
    assert all(x["pci_bus_id"] for x in d["config"]["ranks"])
