#!/usr/bin/env python3
"""Benchmark: decoded frames/s of the VP9 pixel path on MI355X (BASELINE.json metric).

Workload (config C3 of BASELINE.md, the default): 3840x2160 VP9 Profile-0 8-bit, 4 tile
columns, all keyframes, 120 frames per stream, synthetic pass-1 packets with the
SURVEY.md §8(d) stream statistics (seed 0x56503900 + config index + rank).
--config C2 / C4 / C5 measure the other BASELINE.md shapes (1080p GOPs of key + 31 P,
4K 10-bit keyframes, 8K 10-bit GOPs); P frames chain on the previous frame (LAST,
GOLDEN) and the GOP's keyframe (ALTREF), GOPs are independent chains.

One step = reconstruct + loop-filter the whole 120-frame stream on the GPU with all
inputs (pass-1 packets -> device work lists + coefficients) already resident in HBM.
Multi-GPU: one process per GPU; frames are independent (keyframes reset all state,
vp9.c:565,882-892), so every rank decodes its own stream with no data-path
collective (weak scaling); the barrier and the max-over-ranks timing reduction use
torch.distributed (gloo, control plane only).

Prints one JSON line (rank 0) with the driver's fields plus "roofline" (dominant
kernel, algorithmic bytes / HIP-event kernel time vs the 8 TB/s HBM peak) and
"cpu_baseline" (the scalar C oracle on a bounded sample of the same frames).
"""
import argparse
import importlib
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# (index, w, h, bpp, log2 tile cols, GOP length (1 = all keyframes), frames)
CONFIGS = {
    "C2": (1, 1920, 1080, 8, 0, 32, 120),
    "C3": (2, 3840, 2160, 8, 2, 1, 120),
    "C4": (3, 3840, 2160, 10, 2, 1, 120),
    "C5": (4, 7680, 4320, 10, 3, 32, 60),
}
# Batches in flight of the default lines, each slot on ONE frame-group stream (the library
# default, VP9HIP_STREAMS = 1) so the slots' streams fit the 4 hardware queues
# (profiles/r05z): C3 / C4 / C5 at 3 = VP9HIP_PIPELINE_SLOTS, the depth the decoder and the
# FFHWAccel adapter run; C2 (GOP-chain latency) at 4 = VP9HIP_MAX_SLOTS
INFLIGHT = {"C2": 4, "C3": 3, "C4": 3, "C5": 3}

W, H, BPP, LOG2_TILE_COLS = 3840, 2160, 8, 2
CONFIG_INDEX = 2               # C3
CHROMA = {"420": (1, 1), "422": (1, 0), "440": (0, 1), "444": (0, 0)}   # (ss_h, ss_v)
SEED0 = 0x56503900 + CONFIG_INDEX
# rocprofv3 passes of the default C3 bench's serialised timing steps (tools/profile.sh with
# --serial-only): the kernel trace the roofline's launch duration is checked against, and
# the PMC passes its traffic / issue fields come from
TRAFFIC_PROFILE = "r06t/C3"
POISON = 0xA5                  # fill byte of the frame buffers before the timed steps


def frame_seed(rank, i, config_index=CONFIG_INDEX):
    """Seed of frame i of rank `rank`: every rank decodes its own, distinct frames."""
    return 0x56503900 + config_index + rank * 100003 + i


def gop_refs(n, gop):
    """Reference buffers per frame: keyframes (i % gop == 0) none; P frames LAST = GOLDEN =
    previous frame, ALTREF = the GOP's keyframe. Frame i writes buffer i."""
    return [None if i % gop == 0 else (i - 1, i - 1, i - i % gop) for i in range(n)]


def make_frames(v, config, nframes=None, rank=0, chroma="420", **kw):
    """The synthetic pass-1 packets of a BASELINE config exactly as the bench stages them:
    (frames, refs, (W, H, BPP, log2 tile cols, gop)). refs[i] = (LAST, GOLDEN, ALTREF)
    buffer ids or None (keyframes); frame i writes buffer i. Extra synth params in kw."""
    import concurrent.futures    # the C generator releases the GIL: frames in parallel
    cidx, W, H, BPP, log2, gop, nf = CONFIGS[config]
    n = nf if nframes is None else nframes
    refs = gop_refs(n, gop)
    ssh, ssv = CHROMA[chroma]
    with concurrent.futures.ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        frames = list(ex.map(lambda i: v.SynthFrame(v.synth_params(
            W, H, BPP, seed=frame_seed(rank, i, cidx), log2_tile_cols=log2,
            inter=int(refs[i] is not None), ss_h=ssh, ss_v=ssv, **kw)), range(n)))
    return frames, refs, (W, H, BPP, log2, gop)


def oracle_frames(v, oracle, frames, refs, geom, chroma="420", count=None, keep=None):
    """Decode frames 0..count-1 with the CPU oracle (test infrastructure) in decode order,
    yielding (i, planes). Only frames later ones reference are kept in memory."""
    W, H, BPP, _, gop = geom
    ssh, ssv = CHROMA[chroma]
    outs = {}
    n = len(frames) if count is None else min(count, len(frames))
    for i in range(n):
        out = v.alloc_planes(W, H, BPP, ssh, ssv)
        r = refs[i]
        oracle.decode_frame(frames[i].pkt, out, None if r is None else [outs[r[0]], outs[r[1]], outs[r[2]]])
        outs[i] = out
        for k in [k for k in outs if k < i - gop]:     # keep only what later frames reference
            del outs[k]
        yield i, out


def compare_frame(v, got, ref, geom, chroma="420"):
    """Number of visible samples that differ between two frames' planes (0 = bit-exact)."""
    import numpy as np
    W, H = geom[0], geom[1]
    ssh, ssv = CHROMA[chroma]
    return sum(int(np.count_nonzero(a != b))
               for a, b in zip(v.visible(got, W, H, ssh, ssv), v.visible(ref, W, H, ssh, ssv)))


def stage_slots(dev, frames, refs, gop, inflight):
    """The bench's staging: the same workload into `inflight` batch slots, slot k writing
    buffers k * n .. k * n + n - 1 (its references shifted alike); slot 0 selected after."""
    n = len(frames)
    for k in range(inflight):
        dev.set_slot(k)
        dev.stage_batch(frames, [k * n + i for i in range(n)],
                        None if gop == 1 else [None if r is None else tuple(k * n + x for x in r) for r in refs])
    dev.set_slot(0)


def run_slots(dev, steps, inflight, start=0):
    """The timed loop: steps run_batch calls rotating over the slots (each replays its HIP
    graph: device planning, then the pixel kernels), with no host wait between them."""
    for k in range(start, start + steps):
        dev.set_slot(k % inflight)
        dev.run_batch()
        if inflight == 1:
            dev.sync()


def reduce_elapsed(elapsed, dist):
    """Max over ranks of the timed region (the slowest rank defines the job time)."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate(frames_per_rank, steps, world, elapsed_max):
    """Whole-job throughput: all frames of all ranks over the max-over-ranks time."""
    total = frames_per_rank * steps * world
    return total / elapsed_max, elapsed_max * 1000.0 / steps


def dominant_kernel(names, ksum):
    """The roofline's kernel class: the largest serialised time among the pixel kernels
    (the planner's span "k_plan" is excluded, see main)."""
    pix = [k for k in names if k != "k_plan"]
    return max(pix, key=lambda k: ksum.get(k, [0.0, 0])[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=None, help="frames per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify-all", action="store_true",
                    help="compare every timed frame with the oracle (the default at 1 GPU; kept for old scripts)")
    ap.add_argument("--verify-frames", type=int, default=None,
                    help="at 1 GPU: compare only the first N frames (decode order) of each slot with the oracle")
    ap.add_argument("--verify-frames-per-rank", type=int, default=2,
                    help="at N > 1 GPUs: the frames per slot every rank compares with the oracle")
    ap.add_argument("--serial-only", action="store_true",
                    help="profiling runs (tools/profile.sh): only the serialised timing steps the roofline's "
                         "launch durations come from (every launch of the batch on one stream), then a summary line")
    ap.add_argument("--timed-events", action="store_true",
                    help="per-launch HIP events inside the timed steps (no graph replay)")
    ap.add_argument("--chroma", choices=sorted(CHROMA), default="420",
                    help="chroma format (profiles 1/3: 422, 440, 444); the BASELINE configs are 4:2:0")
    ap.add_argument("--inflight", type=int, default=None, choices=[1, 2, 3, 4],
                    help="batches in flight: that many of the context's batch slots (VP9HIP_MAX_SLOTS) hold the same workload and "
                         "alternate steps; each slot runs on HIP streams of its own, so the batches run "
                         "concurrently (as the decoder loop and the FFHWAccel adapter run them). Measured "
                         "with per-slot streams (profiles/r03g): C2 7,778 vs 4,485 fps at 1, C5 761 vs 593. "
                         "Default: 4 for C2, 3 for C3 / C4 / C5, each slot on one stream (the slots on the 4 "
                         "hardware queues; profiles/r05z: C2 17,598-17,786 vs 13,752-13,815 fps at 2, C3 "
                         "11,205 vs 10,821, C4 8,554 vs 8,380, C5 1,316-1,329 vs 1,286-1,304)")
    ap.add_argument("--shard", choices=["frames", "tiles"], default="frames",
                    help="frames: every rank decodes its own stream (weak scaling, default); tiles: all ranks "
                         "decode ONE stream, each its tile columns, pre-LF stripes all-gathered (strong scaling)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    if args.inflight is None:
        args.inflight = INFLIGHT.get(args.config, 2)
    v = importlib.import_module("ffmpeg-hybrid_amd")
    if args.shard == "tiles":
        return bench_tiles(args, v, dist, world, rank, local_rank)
    cidx, W, H, BPP, LOG2_TILE_COLS, gop, nf = CONFIGS[args.config]
    if args.frames is None:
        args.frames = nf
    t0 = time.time()
    ssh, ssv = CHROMA[args.chroma]
    frames, refs, geom = make_frames(v, args.config, args.frames, rank, args.chroma)
    t_gen = time.time() - t0

    # the library's defaults: one frame-group stream per batch slot (VP9HIP_STREAMS unset)
    dev = v.Device(_device_of(local_rank))
    dev.configure(W, H, BPP, nbufs=args.frames * args.inflight, ss_h=ssh, ss_v=ssv)
    t0 = time.time()
    stage_slots(dev, frames, refs, gop, args.inflight)
    t_stage = (time.time() - t0) / args.inflight

    def barrier():
        if dist is not None:
            dist.barrier()

    # per-launch HIP-event kernel timing (roofline): its own steps, launches enqueued one by one
    dev.set_timing(True)
    for _ in range(args.warmup):
        dev.run_batch()
    dev.sync()
    ksum = {}
    for _ in range(args.steps):
        dev.run_batch()
        dev.sync()          # collects the per-launch HIP-event times of this step
        for k, (ms, n) in dev.timing().items():
            a = ksum.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += n

    if args.serial_only:
        kl = {k: int(ksum[k][1] / args.steps) for k in ksum}
        print(json.dumps({"metric": "serial timing steps only (profiling run)", "serial_only": True,
                          "config": {"workload": args.config, "frames_per_gpu": args.frames,
                                     "streams_per_gpu": dev.groups(), "batches_in_flight": 1},
                          "roofline": {"kernel_ms": {k: round(ksum[k][0] / args.steps, 3) for k in ksum},
                                       "kernel_launches": kl}}), flush=True)
        dev.close()
        return

    # timed steps: the batch's launch sequence replayed as one HIP graph
    dev.set_timing(args.timed_events)
    run_slots(dev, args.warmup * args.inflight, args.inflight)
    dev.sync()
    # poison every frame buffer of both slots: the frames verified below can only have been
    # written by the timed steps (a replay that did nothing would leave the poison byte)
    dev.fill(0, args.frames * args.inflight, POISON)
    dev.sync()
    barrier()
    t0 = time.perf_counter()
    run_slots(dev, args.steps, args.inflight)
    dev.sync()                     # every slot's work; checks every slot
    barrier()
    elapsed = time.perf_counter() - t0
    dev.set_slot(0)
    slots_run = min(args.inflight, args.steps)   # slots the timed steps wrote

    elapsed = reduce_elapsed(elapsed, dist)

    alg = dev.alg_bytes()           # per step, per kernel class
    names = list(alg.keys())
    fps, ms_per_step = aggregate(args.frames, args.steps, world, elapsed)
    streams = dev.groups()          # frame groups = concurrent HIP streams of the batch

    # dominant kernel (largest device time; the timing steps run every launch on one stream,
    # so these are serialised launch durations, as under a rocprofv3 kernel trace). The
    # planner's class ("k_plan") is one span over its ~10 kernels (k_pblk, the scans, k_psb,
    # k_pjplan, k_pllf, ...; the largest of them, k_pjplan, is 3.4 ms of its 4.2 per C3 step),
    # not a kernel, and its bytes are not part of BASELINE.md's B: the roofline is taken for
    # the largest pixel kernel
    dom = dominant_kernel(names, ksum)
    kms, kn = ksum[dom]
    launches_per_step = kn / args.steps
    bytes_per_launch = alg[dom] / launches_per_step if launches_per_step else 0.0
    avg_launch_s = (kms / 1000.0) / kn if kn else float("nan")
    achieved = bytes_per_launch / avg_launch_s / 1e9 if kn else 0.0
    # BASELINE.md's algorithmic bytes (coefficients, prediction, reconstruction, LF): the
    # pixel kernels'; the planner's own (the packet it reads) are not part of B
    frame_bytes = sum(b for k, b in alg.items() if k != "k_plan") / args.frames
    kernel_ms_step = sum(ksum[k][0] for k in ksum) / args.steps
    # HBM traffic per launch of the same kernel on the same workload, from the committed
    # rocprofv3 PMC pass (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; tools/traffic.py)
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", TRAFFIC_PROFILE, "traffic.json")
    shape_ok, shape_note = False, None
    if os.path.exists(tf) and args.config == "C3" and args.chroma == "420":
        tj = json.load(open(tf))
        # the profile must have been taken at this run's launch shape: same frames per launch
        # (frame groups / streams, frames per batch) and the same launches of the kernel per step
        run_shape = {"launches_per_step": int(round(launches_per_step)), "streams_per_gpu": streams,
                     "frames_per_gpu": args.frames}
        prof_shape = tj.get("shape", {}).get(dom)
        shape_ok = prof_shape == run_shape
        if not shape_ok:
            shape_note = "refused: profiles/%s launch shape %s != this run's %s" % (TRAFFIC_PROFILE, prof_shape, run_shape)
        per = tj["per_launch"].get(dom)
        if per and shape_ok:
            traffic, traffic_src = round(per["traffic_bytes"]), "profiles/%s/traffic.json" % TRAFFIC_PROFILE
        elif shape_note:
            traffic_src = shape_note
    # the same launches' durations under the committed rocprofv3 kernel trace of those
    # serialised steps (profiles/<P>/kernel_stats.csv): the profile figure `frac` must agree with
    trace = None
    kf = os.path.join(ROOT, "profiles", TRAFFIC_PROFILE, "kernel_stats.csv")
    if os.path.exists(kf) and shape_ok:
        import csv
        for r in csv.DictReader(open(kf)):
            m = re.search(r"\b(k_\w+?)\s*[<(]", r["Name"])
            if m and m.group(1) == dom:
                t_us = float(r["AverageNs"]) / 1000.0
                t_frac = bytes_per_launch / (t_us * 1e-6) / 1e9 / HBM_PEAK_GBS
                trace = {"avg_launch_us": round(t_us, 2), "calls": int(r["Calls"]), "frac": round(t_frac, 5),
                         "frac_ratio": round(achieved / HBM_PEAK_GBS / t_frac, 4) if t_frac else None,
                         "source": "profiles/%s/kernel_stats.csv" % TRAFFIC_PROFILE}
                break
    # instruction issue of the same kernel from the committed SQ pass (profiles/<P>/pmc_summary.txt):
    # VALU wave-instructions per launch / its mean duration there, vs the VALU issue peak:
    # 256 CUs x 4 SIMD-32s, each issuing one wave64 VALU instruction per 2 cycles at 2.4 GHz
    # (MI355X_MICROARCH.md, Wave scheduling; = the 157.3 TF FP32 vector peak / 128 FLOP)
    issue = None
    pf = os.path.join(ROOT, "profiles", TRAFFIC_PROFILE, "pmc_summary.txt")
    if os.path.exists(pf) and shape_ok:
        cur, vals = None, {}
        for line in open(pf):
            if not line.startswith(" "):
                cur = line.strip()
            elif cur in (dom, dom + "d"):          # k_lfr: the k_lfrd kernel
                f = line.split()
                vals[f[0]] = float(f[2].split("=")[1])
        if "SQ_INSTS_VALU" in vals and vals.get("duration_us"):
            peak = 256 * 4 * 2.4e9 / 2
            rate = vals["SQ_INSTS_VALU"] / (vals["duration_us"] * 1e-6)
            issue = {"valu_instr_per_launch": vals["SQ_INSTS_VALU"], "salu_instr_per_launch": vals.get("SQ_INSTS_SALU"),
                     "duration_us": vals["duration_us"], "valu_frac": round(rate / peak, 4),
                     "wait_frac": round(vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"], 4) if vals.get("SQ_WAVE_CYCLES") else None,
                     "source": "profiles/%s/pmc_summary.txt" % TRAFFIC_PROFILE}
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": traffic_src,
        "kernel": dom, "launches_per_step": int(launches_per_step),
        "alg_bytes_per_launch": round(bytes_per_launch),
        "avg_launch_us": round(avg_launch_s * 1e6, 2),
        # whole device: algorithmic bytes of a step / step wall time (all kernels, all chains)
        "gpu_wall_frac": round(frame_bytes * args.frames / (ms_per_step / 1000.0) / 1e9 / HBM_PEAK_GBS, 5),
        # algorithmic bytes of a step / the sum of its serialised kernel durations (planner included)
        "all_kernels_frac": round(frame_bytes * args.frames / (kernel_ms_step / 1000.0) / 1e9 / HBM_PEAK_GBS, 5)
        if kernel_ms_step > 0 else None,
        "launch_time_note": "avg_launch_us: HIP-event durations of the kernel's launches in separate steps of "
                            "slot 0's batch with every launch on one stream, enqueued one by one (each launch "
                            "alone on the GPU); trace: the same serialised steps under rocprofv3 --kernel-trace "
                            "(bench.py --serial-only, tools/profile.sh). The timed steps replay HIP graphs of "
                            "%d batch slots concurrently (%d frame-group stream(s) each), where launches of "
                            "different slots overlap and a trace's durations include the overlap"
                            % (args.inflight, streams),
        "trace": trace,
        "kernel_ms": {k: round(ksum[k][0] / args.steps, 3) for k in ksum},
        "kernel_launches": {k: int(ksum[k][1] / args.steps) for k in ksum},
        "issue": issue,
    }

    # bit-exactness of the timed frames: the oracle's frames are compared with the device's,
    # in every batch slot the timed steps wrote (the buffers were poisoned before them)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker + CPU baseline leg only: the scalar C restatement
    cpu, verify = None, None
    sample = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the first frames as a VP9 stream: the CPU baseline's whole-stream legs and the host
        # entropy / decoder / adapter legs below
        sample = encode_sample(v, frames, gop, min(len(frames), max(gop, 16)))
    if world == 1:
        cpu, verify = cpu_baseline(v, oracle, dev, frames, refs, geom, args, slots_run, sample)
    else:
        # every rank checks a sample of its own frames (the first frames of each slot in
        # decode order); rank 0 reports all ranks' results
        verify = verify_frames(v, oracle, dev, frames, refs, geom, args, slots_run,
                               range(min(args.verify_frames_per_rank, len(frames))), threads=1)
        verify["rank"] = rank
    rank_info = {"rank": rank, "local_rank": local_rank, "device": _device_of(local_rank),
                 "host": os.uname().nodename}
    rank_info.update(_device_ids(v, rank_info["device"]))
    ranks = [rank_info]
    if dist is not None:
        got = [None] * world
        dist.all_gather_object(got, (rank_info, verify))
        ranks = [g[0] for g in got]
        per = [g[1] for g in got]
        verify = {"frames": sum(p["frames"] for p in per), "of": len(frames) * slots_run * world,
                  "mismatched": [[p["rank"]] + m for p in per for m in p["mismatched"]],
                  "what": "per rank: visible Y/U/V of its first %d frames (decode order) in each of its %d batch "
                          "slot(s), written by the timed steps after a poison fill, vs the CPU oracle"
                          % (min(args.verify_frames_per_rank, len(frames)), slots_run),
                  "per_rank": [{"rank": p["rank"], "frames": p["frames"], "mismatched": len(p["mismatched"])}
                               for p in per]}

    host = e2e = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = host_entropy_rate(v, sample, gop, args)
        dev.close()                                     # free the batch's HBM before the decoder runs
        dev = None
        e2e = e2e_rate(v, sample, args, local_rank)
        # the same shapes at a realistic coefficient density (~0.1 MB per 4K frame instead of
        # 1.6 MB: 90 % of tx blocks without coefficients, 70 % skip blocks)
        nlow = min(len(frames), max(gop, 16))
        low = [v.SynthFrame(v.synth_params(W, H, BPP, seed=frame_seed(rank, i, cidx), log2_tile_cols=LOG2_TILE_COLS,
                                           inter=int(refs[i] is not None), ss_h=ssh, ss_v=ssv,
                                           p_zero_eob=0.9, p_skip=0.7)) for i in range(nlow)]
        lsample = encode_sample(v, low, gop, nlow)
        e2e["low_rate"] = e2e_rate(v, lsample, args, local_rank)
        e2e["low_rate"]["bytes_per_frame"] = int(sum(len(d) for g in lsample for d in g) / nlow)
        e2e["low_rate"]["host_parse"] = host_entropy_rate(v, lsample, gop, args)["fps_threads"]
        # the FFHWAccel surface avcodec_receive_frame() reaches (tests/c/hwaccel_harness plays
        # vp9.c around it) on the same realistic-density stream, and on a C2 one
        hw = {args.config: hwaccel_rate(v, lsample, W, H, BPP, args)}
        if args.config != "C2" and args.chroma == "420":
            c2f, c2refs, c2geom = make_frames(v, "C2", 32, rank, p_zero_eob=0.9, p_skip=0.7)
            hw["C2"] = hwaccel_rate(v, encode_sample(v, c2f, 32, 32), 1920, 1080, 8, args)
        e2e["hwaccel_path"] = hw

    out = {
        "metric": "decoded frames/sec (bit-exact) 4K VP9 Profile-0 @ 1/2/4/8 MI355X; % HBM roofline",
        "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8" if BPP == 8 else "u16", "data": "synthetic",
        "config": {"workload": "%s: %dx%d VP9 Profile-%d %d-bit%s, %d tile columns, %s, %d frames per GPU per step, "
                               "pass-1 packets resident in HBM"
                               % (args.config, W, H, (0 if BPP == 8 else 2) | (args.chroma != "420"), BPP,
                                  "" if args.chroma == "420" else " 4:%s:%s" % (args.chroma[1], args.chroma[2]),
                                  1 << LOG2_TILE_COLS,
                                  "all keyframes" if gop == 1 else "GOPs of key + %d P" % (gop - 1), args.frames),
                   "global_batch": args.frames * world, "frames_per_gpu": args.frames,
                   "parallelism": "frame-sharded x%d (independent %s, no collective)"
                                  % (world, "keyframes" if gop == 1 else "GOPs"),
                   "streams_per_gpu": streams, "batches_in_flight": args.inflight,
                   "ranks": ranks,
                   "host_gen_s": round(t_gen, 2), "host_stage_s": round(t_stage, 2)},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "verify": verify,
        "verified_frames": verify["frames"] if verify else 0,
        "host_entropy": host,
        "e2e_decoder": e2e,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dev is not None:
        dev.close()
    if dist is not None:
        dist.destroy_process_group()
    if verify and verify["mismatched"]:
        sys.exit("bench: %d timed frames differ from the oracle: %s" % (len(verify["mismatched"]), verify["mismatched"]))


def _compare_slots(v, dev, i, out, geom, args, slots_run, lock=None):
    """Compare frame i's oracle planes with the device frame in every slot the timed steps
    wrote (slot k holds frame i in buffer k * frames + i); returns the mismatches."""
    bad = []
    for k in range(slots_run):
        b = k * args.frames + i
        if lock is not None:
            with lock:
                got = dev.download(b)
        else:
            got = dev.download(b)
        d = compare_frame(v, got, out, geom, args.chroma)
        if d:
            bad.append([i, k, d])
    return bad


def verify_frames(v, oracle, dev, frames, refs, geom, args, slots_run, idx, threads=None):
    """Verify frames `idx` (decode-order indices) of every written slot against the oracle,
    on a thread pool: keyframes independently, inter frames by GOP chain from its keyframe
    (ctypes releases the GIL in the oracle; device downloads are serialised)."""
    import concurrent.futures
    import threading
    idx = sorted(set(idx))
    gop = geom[4]
    if not idx:
        return {"frames": 0, "mismatched": []}
    lock = threading.Lock()
    W, H, BPP = geom[0], geom[1], geom[2]
    ssh, ssv = CHROMA[args.chroma]

    def unit(chain):
        outs, bad, n = {}, [], 0
        for i in range(chain[0], chain[-1] + 1):
            out = v.alloc_planes(W, H, BPP, ssh, ssv)
            r = refs[i]
            oracle.decode_frame(frames[i].pkt, out, None if r is None else [outs[r[0]], outs[r[1]], outs[r[2]]])
            outs[i] = out
            for k in [k for k in outs if k < i - 1 and k != chain[0] - chain[0] % gop]:
                del outs[k]
            if i in want:
                bad += _compare_slots(v, dev, i, out, geom, args, slots_run, lock)
                n += slots_run
        return n, bad

    want = set(idx)
    if gop == 1:
        chains = [[i] for i in idx]
    else:
        chains = {}
        for i in idx:
            g0 = i - i % gop
            chains.setdefault(g0, [g0, i])[1] = i
        chains = list(chains.values())
    nthr = threads or min(16, os.cpu_count() or 1)
    with concurrent.futures.ThreadPoolExecutor(nthr) as ex:
        res = list(ex.map(unit, chains))
    return {"frames": sum(r[0] for r in res), "mismatched": [m for r in res for m in r[1]]}


def _device_ids(v, ordinal):
    """PCI identity of a rank's GPU (so a multi-GPU line shows each rank on its own card)."""
    try:
        bus, name = v.device_info(ordinal)
        return {"pci_bus_id": bus, "gpu_name": name}
    except Exception as e:                      # no GPU (CPU rehearsal)
        return {"pci_bus_id": None, "error": str(e)}


def _cpu_quota():
    """CPUs the cgroup grants this process (cpu.max quota / period), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_info():
    """The host the CPU legs ran on: nproc, the CPU share used, the lscpu model name."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"nproc": os.cpu_count(), "threads_used": min(16, os.cpu_count() or 1), "model": model,
            "affinity": affinity, "cpu_quota": _cpu_quota()}


def stream_cpu(v, oracle, datas, geom, chroma):
    """The whole CPU decode of one stream (entropy + reconstruction + loop
    filter): the host parse (vp9h_stream, the restatement of vp9.c / vp9block.c) into pass-1
    packets, the oracle's reconstruction and loop filter, reference slots by refresh mask
    (vp9.c:1686-1691). Returns the frames decoded."""
    W, H, BPP = geom[:3]
    ssh, ssv = CHROMA[chroma]
    st, slots, n = v.Stream(), [None] * 8, 0
    for d in datas:
        p, info = st.decode(d)
        if p is None:
            continue
        pk = p.pkt
        out = v.alloc_planes(W, H, BPP, ssh, ssv)
        intra = pk.keyframe or pk.intraonly
        oracle.decode_frame(pk, out, None if intra else [slots[s] for s in info.ref_slot])
        for s in range(8):
            if info.refresh_mask & (1 << s):
                slots[s] = out
        n += 1
    return n


def cpu_baseline(v, oracle, dev, frames, refs, geom, args, slots_run, sample=None):
    """CPU baseline legs on this box's host cores, and the bit-exactness
    check of the timed frames. `value`: the whole stream (host entropy decode + oracle
    reconstruction + loop filter, stream_cpu) over the encoded sample, independent
    keyframes (C3 / C4) or GOP chains (C2 / C5) on the box's 16-thread share; the same on 1
    thread beside it. Reconstruction-only legs from the pass-1 packets: leg 1 the scalar C
    oracle on 1 thread over a bounded sample
    in decode order; every frame it decodes is compared with the device's frame in each
    batch slot the timed steps wrote (downloads and compares are outside the CPU timer).
    The frames leg 1 did not reach are then verified with the oracle on a thread pool.
    Leg 2: tile-column threads per frame (the reference's slice threading). Leg 3:
    frame-parallel over the box's CPU share (16 threads): independent keyframes (C3/C4) or
    independent GOP chains (C2/C5), one oracle decode per thread (ctypes releases the GIL).
    Leg 4: the same over every host thread nproc reports. Returns (cpu_baseline, verify)."""
    import concurrent.futures
    W, H, BPP, log2, gop = geom
    nf = len(frames)
    bounded = not args.no_cpu_baseline
    budget = args.cpu_seconds if bounded else 0.0
    want = nf if args.verify_frames is None else min(nf, args.verify_frames)
    t_or, n, bad = 0.0, 0, []
    gen = oracle_frames(v, oracle, frames, refs, geom, args.chroma)
    while n < nf:
        t0 = time.perf_counter()
        item = next(gen, None)
        t_or += time.perf_counter() - t0
        if item is None:
            break
        i, out = item
        n += 1
        if i < want:
            bad += _compare_slots(v, dev, i, out, geom, args, slots_run)
        if n >= 2 and t_or >= budget:
            break
    gen = None
    rest = verify_frames(v, oracle, dev, frames, refs, geom, args, slots_run, range(n, want))
    bad += rest["mismatched"]
    checked = min(n, want) * slots_run + rest["frames"]
    verify = {"frames": checked, "of": nf * slots_run, "mismatched": bad, "slots": slots_run,
              "poisoned": True,
              "what": "visible Y/U/V of frames 0..%d (decode order) of each of the %d batch slot(s) the timed "
                      "steps wrote (every frame buffer filled with 0x%02X before them) vs the CPU oracle, "
                      "sample-exact" % (want - 1, slots_run, POISON)}
    if not bounded:
        return None, verify
    one = n / t_or
    info = cpu_info()
    thr = info["threads_used"]
    # leg 2: the reference's slice threads: the tile columns of each SB row on their own
    # threads, the loop filter of the previous row overlapped (vp9.c:1442-1551), frames one
    # after another in decode order (vp9o_decode_frame_tiles, same output as leg 1)
    tthr = min(1 << log2, thr)
    t_tile, n_tile = 0.0, 0
    outs = {}
    ssh_, ssv_ = CHROMA[args.chroma]
    for i in range(len(frames)):
        out = v.alloc_planes(W, H, BPP, ssh_, ssv_)
        r = refs[i]
        t0 = time.perf_counter()
        oracle.decode_frame(frames[i].pkt, out, None if r is None else [outs[r[0]], outs[r[1]], outs[r[2]]],
                            tile_threads=tthr)
        t_tile += time.perf_counter() - t0
        n_tile += 1
        outs[i] = out
        for k in [k for k in outs if k < i - gop]:
            del outs[k]
        if n_tile >= 2 and t_tile >= budget / 3:
            break
    outs = None
    tiles = n_tile / t_tile
    # leg 3: frame-parallel (keyframes) / GOP-parallel (inter streams) over thr threads
    if gop == 1:
        units = [[i] for i in range(len(frames))]
    else:
        units = [list(range(g, min(len(frames), g + gop))) for g in range(0, len(frames), gop)]
    per_unit = len(units[0]) / one
    reps = max(1, int(budget / 2 * thr / max(per_unit * len(units), 1e-9)) + 1)
    work = (units * reps)[:max(thr, int(budget / 2 * thr / per_unit) + 1)]
    ssh, ssv = CHROMA[args.chroma]

    def run_unit(idx):
        outs = {}
        for i in idx:
            out = v.alloc_planes(W, H, BPP, ssh, ssv)
            r = refs[i]
            oracle.decode_frame(frames[i].pkt, out, None if r is None else [outs[r[0]], outs[r[1]], outs[r[2]]])
            outs[i] = out
            for k in [k for k in outs if k < i - 1 and k != idx[0]]:
                del outs[k]
        return len(idx)

    with concurrent.futures.ThreadPoolExecutor(thr) as ex:
        t0 = time.perf_counter()
        done = sum(ex.map(run_unit, work))
        par = done / (time.perf_counter() - t0)
    # leg 4: the same pool over every host thread the box reports (nproc); the cgroup's CPU
    # quota, when there is one, bounds what these threads get
    nall = os.cpu_count() or 1
    eff = min(x for x in (nall, info["cpu_quota"], info["affinity"]) if x)   # CPUs the threads can get
    par_all, all_note = None, None
    work_all = (units * max(1, -(-nall // len(units))))[:nall]       # one unit per thread
    est = len(work_all) * per_unit / eff
    if nall > thr and est > 2 * budget:
        all_note = "skipped: %d %s on %d threads would take ~%.0f s on %.4g CPUs" % (
            len(work_all), "keyframes" if gop == 1 else "GOP chains", nall, est, eff)
    elif nall > thr:
        with concurrent.futures.ThreadPoolExecutor(nall) as ex:
            t0 = time.perf_counter()
            done = sum(ex.map(run_unit, work_all))
            par_all = done / (time.perf_counter() - t0)
    legs = [
        {"leg": "1 thread", "value": round(one, 3), "cores": 1,
         "sample": "%d frames in decode order" % n},
        {"leg": "tile-column threads", "value": round(tiles, 3), "cores": tthr + 1,
         "sample": "%d frames in decode order, %d tile-column threads + the loop filter on the calling thread"
                   % (n_tile, tthr)},
        {"leg": "%s-parallel" % ("frame" if gop == 1 else "GOP"), "value": round(par, 3), "cores": thr,
         "sample": "%d %s on %d threads" % (len(work), "keyframes" if gop == 1 else "GOP chains", thr)},
    ]
    if par_all is not None or all_note:
        legs.append({"leg": "%s-parallel, all host threads" % ("frame" if gop == 1 else "GOP"),
                     "value": None if par_all is None else round(par_all, 3), "cores": nall,
                     "sample": all_note or "%d %s on %d threads (nproc); cgroup CPU quota %s, affinity %s CPUs"
                               % (len(work_all), "keyframes" if gop == 1 else "GOP chains", nall, info["cpu_quota"],
                                  info["affinity"])})
    for lg in legs:
        lg["leg"] = "reconstruction + LF, " + lg["leg"]
    cpu = {"value": round(par, 3), "unit": "frames/s", "cores": thr, "kind": "port",
           "sample": "%s %s frames, scalar C oracle (the build's restatement, without the reference's SIMD; "
                     "reconstruction + loop filter from the same pass-1 packets, host entropy decode excluded), "
                     "%s-parallel over %d of the %s host threads"
                     % (len(work) if gop == 1 else sum(len(u) for u in work), args.config,
                        "frame" if gop == 1 else "GOP", thr, info["nproc"]),
           "legs": legs, "host": info}
    if sample:
        # the whole stream as BASELINE.md §3 states it: the encoded sample parsed and
        # reconstructed, 1 thread, then units (keyframes / GOPs) over the 16-thread share
        t0, n1, k = time.perf_counter(), 0, 0
        while k < len(sample) or time.perf_counter() - t0 < budget / 4:
            n1 += stream_cpu(v, oracle, sample[k % len(sample)], geom, args.chroma)
            k += 1
        one_ws = n1 / (time.perf_counter() - t0)
        per = sum(len(g) for g in sample) / len(sample) / one_ws          # seconds per unit, 1 thread
        nunits = max(thr, int(budget / 3 * thr / per) + 1)
        with concurrent.futures.ThreadPoolExecutor(thr) as ex:
            t0 = time.perf_counter()
            done = sum(ex.map(lambda g: stream_cpu(v, oracle, g, geom, args.chroma),
                              [sample[i % len(sample)] for i in range(nunits)]))
            par_ws = done / (time.perf_counter() - t0)
        unit = "keyframes" if gop == 1 else "GOP chains"
        legs.insert(0, {"leg": "whole stream (entropy + reconstruction + LF), 1 thread", "value": round(one_ws, 3),
                        "cores": 1, "sample": "%d frames of the %d-frame sample stream" % (n1, sum(map(len, sample)))})
        legs.insert(1, {"leg": "whole stream, %s-parallel" % ("frame" if gop == 1 else "GOP"), "value": round(par_ws, 3),
                        "cores": thr, "sample": "%d %s of the sample stream on %d threads" % (nunits, unit, thr)})
        cpu.update({"value": round(par_ws, 3),
                    "sample": "%d %s frames as VP9 bitstreams (%s of the timed workload, encoded by vp9h_stream): host "
                              "entropy decode (vp9h_stream) + scalar C oracle reconstruction + loop filter (the build's "
                              "restatement, without the reference's SIMD), %s-parallel over %d of the %s host threads"
                              % (done, args.config, unit, "frame" if gop == 1 else "GOP", thr, info["nproc"])})
    return cpu, verify


def encode_sample(v, frames, gop, n):
    """The first n frames as VP9 streams (vp9h_stream_encode), one per GOP (keyframe to
    keyframe; LAST = ALTREF = the previous frame, GOLDEN = the keyframe), GOPs encoded in
    parallel (ctypes drops the GIL)."""
    import concurrent.futures

    def enc_gop(g0):
        enc, datas = v.Stream(), []
        for i in range(g0, min(n, g0 + gop)):
            kw = {}
            if i > g0:
                prev = (i - 1 - g0) % 8
                kw = {"ref_slot": (prev, 0, prev), "refresh_mask": 1 << ((i - g0) % 8)}
            datas.append(enc.encode(frames[i], base_q_idx=frames[i].params.q_idx, **kw)[0])
        return datas

    with concurrent.futures.ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        return list(ex.map(enc_gop, range(0, n, gop)))


def host_entropy_rate(v, gops, gop, args):
    """The host side of the hybrid split: the sample stream parsed back
    into pass-1 packets by vp9h_stream_decode, timed on this box's cores: 1 thread, then a
    pool decoding independent GOPs (keyframe to keyframe) in parallel. Not `value` (the GPU
    path is timed with packets resident); the rate at which the host front end could feed it."""
    import concurrent.futures
    n = sum(len(g) for g in gops)

    def decode_gop(datas, tile_threads=1):
        dec = v.Stream(threads=tile_threads)
        for d in datas:
            dec.decode(d)
        return len(datas)

    t0 = time.perf_counter()
    done = k = 0
    while time.perf_counter() - t0 < args.cpu_seconds / 2 or k < len(gops):
        done += decode_gop(gops[k % len(gops)])
        k += 1
    one = done / (time.perf_counter() - t0)
    threads = min(16, os.cpu_count() or 1)             # the box's CPU share
    reps = max(1, int(one * args.cpu_seconds / 2 * threads / n / 4) + 1)
    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        many = sum(ex.map(decode_gop, gops * reps)) / (time.perf_counter() - t0)
    # one stream at a time, its frames' tile columns on threads (decode_tiles_mt,
    # vp9.c:1441-1520): the rate of a single GOP chain, which GOP-parallel parsing cannot raise
    ntc = 1 << CONFIGS[args.config][4]
    tiles = None
    if ntc > 1:
        tt = min(threads, ntc)
        t0 = time.perf_counter()
        done = k = 0
        while time.perf_counter() - t0 < args.cpu_seconds / 4 or k < len(gops):
            done += decode_gop(gops[k % len(gops)], tt)
            k += 1
        tiles = {"fps": round(done / (time.perf_counter() - t0), 2), "tile_threads": tt}
    return {"fps_1_thread": round(one, 2), "fps_threads": round(many, 2), "threads": threads,
            "tile_threaded": tiles,
            "bytes_per_frame": int(sum(len(d) for g in gops for d in g) / n),
            "sample": "%d synthetic %s frames as a VP9 stream (%s), parsed to pass-1 packets"
                      % (n, args.config, "keyframes" if gop == 1 else "GOPs of %d" % gop)}


def hwaccel_rate(v, gops, W, H, BPP, args):
    """Frames/s through the FFHWAccel adapter (include/vp9hip_hwaccel.h) driven in vp9.c's
    call order by tests/c/hwaccel_harness: the sample stream repeated `reps` times as one
    IVF stream (every repeat starts at a keyframe), frames read 16 behind the decoder
    (FFmpeg's frame-threading delay) by a device consumer (vp9hip_hwframe_sync) and by a
    download consumer (transfer_data_from: a D2H copy per frame into pageable host memory).
    Host parse on the adapter's pool; async depth 16 (frames per launch)."""
    import subprocess
    import tempfile
    harness = os.path.join(ROOT, "tests", "c", "hwaccel_harness")
    if not os.access(harness, os.X_OK):
        return {"error": "tests/c/hwaccel_harness not built"}
    pkts = [d for g in gops for d in g]
    ssh, ssv = CHROMA[args.chroma]
    nbytes = sum(map(len, pkts))
    # lag 16 (a 16-thread frame delay); async depth = frame_params' default for it (the power
    # of two <= extra / 2 with extra = 2 + lag: 8)
    out = {"sample_frames": len(pkts), "bytes_per_frame": int(nbytes / len(pkts)), "lag": 16, "async_depth": 8}
    with tempfile.TemporaryDirectory() as td:
        ivf = os.path.join(td, "s.ivf")
        for mode in ("device", "download"):
            reps = 2
            while True:
                with open(ivf, "wb") as f:
                    f.write(v.ivf_write(pkts * reps, W, H))
                r = subprocess.run([harness, ivf, "-", str(BPP), str(ssh), str(ssv), "1", "16", mode, "0"],
                                   capture_output=True, text=True, timeout=300)
                f = r.stdout.split()
                if r.returncode or len(f) < 4:
                    out[mode] = {"error": r.stderr.strip()[-300:]}
                    break
                n, sec = int(f[1]), float(f[3])
                cap = max(1, int(400e6 / nbytes))          # stream files up to ~400 MB
                if sec >= args.cpu_seconds / 4 or reps >= cap:
                    out[mode] = {"fps": round(n / sec, 2), "frames": n, "seconds": round(sec, 3)}
                    break
                reps = min(cap, max(reps * 2, int(reps * args.cpu_seconds / 4 / max(sec, 1e-3)) + 1))
    return out


def e2e_rate(v, gops, args, device):
    """Whole decoder, bitstream in -> frames in HBM out: vp9hip_decoder (host parse on a
    thread pool, batched planning + H2D staging, GPU reconstruction), the sample stream sent
    `reps` times, frames received as device buffers and released. Not `value`: this one
    includes the host parse and the PCIe copy of every frame's packet."""
    pkts = [d for g in gops for d in g]
    threads = min(16, os.cpu_count() or 1)
    dec = v.Decoder(device, max_batch=16, parse_threads=threads)

    def run(reps):
        n = 0
        for _, info in dec.decode(pkts * reps, download=False):
            dec.release(info.buf)
            n += 1
        dec.flush()
        return n

    t0 = time.perf_counter()
    run(1)                                              # configure + warm-up
    dt = time.perf_counter() - t0
    reps = max(1, int(args.cpu_seconds / 2 / max(dt, 1e-3)))
    t0 = time.perf_counter()
    n = run(reps)
    dt = time.perf_counter() - t0
    dec.close()
    return {"fps": round(n / dt, 2), "frames": n, "parse_threads": threads, "max_batch": 16,
            "sample": "the %d-frame %s sample stream sent %d times through vp9hip_decoder "
                      "(send_packet / receive_frame, device frames)" % (len(pkts), args.config, reps)}


def _device_of(local_rank):
    """One rank per GPU; ranks beyond the visible GPUs share them round-robin (a multi-rank
    rehearsal on a 1-GPU box). Counting devices does not initialise the GPU."""
    import torch
    n = torch.cuda.device_count()
    return local_rank % n if n > 0 else local_rank


def bench_tiles(args, v, dist, world, rank, local_rank):
    """--shard tiles: one stream over all ranks (tileshard.py). Every
    rank stages the same frames and reconstructs its tile columns. Per chain position
    the pre-LF stripes go through one RCCL all-gather (an nccl group beside the gloo
    control group), then every rank loop-filters the whole frame."""
    import torch
    ts = importlib.import_module("ffmpeg-hybrid_amd.tileshard")
    cidx, W, H, BPP, log2, gop, nf = CONFIGS[args.config]
    if args.frames is None:
        args.frames = nf
    refs = gop_refs(args.frames, gop)
    frames = [v.SynthFrame(v.synth_params(W, H, BPP, seed=frame_seed(0, i, cidx), log2_tile_cols=log2,
                                          inter=int(refs[i] is not None))) for i in range(args.frames)]
    torch.cuda.set_device(local_rank)
    group = dist.new_group(backend="nccl") if dist is not None else None
    lo, hi = ts.tile_ranges(1 << log2, world)[rank]
    dev = v.Device(local_rank)
    dev.configure(W, H, BPP, nbufs=args.frames)
    dev.stage_batch(frames, list(range(args.frames)), refs, tiles=(lo, hi))
    dev.set_timing(False)
    sh = ts.TileShard(dev, 1 << log2, rank, world, group=group, device="cuda:%d" % local_rank)
    for _ in range(args.warmup):
        sh.run()
    if dist is not None:
        dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sh.run()
    dev.sync()
    if dist is not None:
        dist.barrier()
    elapsed = reduce_elapsed(time.perf_counter() - t0, dist)
    fps, ms_per_step = aggregate(args.frames, args.steps, 1, elapsed)     # one stream: strong scaling
    step_bytes = sum(dev.alg_bytes().values())
    sent, recvd = zip(*sh.bytes_per_phase())
    achieved = step_bytes / (ms_per_step / 1000.0) / 1e9
    out = {
        "metric": "decoded frames/sec (bit-exact) 4K VP9 Profile-0 @ 1/2/4/8 MI355X; % HBM roofline",
        "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8" if BPP == 8 else "u16", "data": "synthetic",
        "config": {"workload": "%s: %dx%d %d-bit, %d tile columns, %s, ONE %d-frame stream over all GPUs"
                               % (args.config, W, H, BPP, 1 << log2,
                                  "all keyframes" if gop == 1 else "GOPs of key + %d P" % (gop - 1), args.frames),
                   "parallelism": "tile-sharded x%d: tile columns %d..%d on rank %d, RCCL all-gather of pre-LF "
                                  "stripes per chain position, redundant full-frame LF" % (world, lo, hi - 1, rank),
                   "exchange_bytes_per_phase": {"sent": max(sent), "received": max(recvd)}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "whole step on rank 0 (algorithmic bytes of its share / step wall time)"},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
