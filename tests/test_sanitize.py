"""The host side under the sanitizers, and the FFHWAccel adapter without a GPU (CPU suite).

`make -C ffmpeg-hybrid_amd/csrc sanitize` builds, from the library's own host sources and
without HIP:
- tests/c/host_san.cpp: streams encoded and parsed back serially, on 2 / 3 / 8 tile-column
  threads, frame-pipelined (headers in order, each frame's tiles on a thread of its own,
  waiting per SB row for the previous frame's MVs; probability adaptation off and on,
  use_last_frame_mvs set) and through the parse pool (every packet equal byte for byte), corrupted and
  truncated streams, IVF / WebM files demuxed, parsed and mutated;
- the call-order harness (tests/c/hwaccel_harness.c) over csrc/vp9hip_hwaccel.cpp with
  tests/c/fake_device.cpp in place of the device (the oracle reconstructs on a worker thread,
  asynchronously, like a device queue).
Each as a plain, an ASan + UBSan and a TSan binary. A sanitizer report fails the test (the
binaries abort on UBSan findings; ASan / TSan reports are read from stderr). The harness's
output must equal the oracle's decode loop, including with the consumer on a thread of its
own (MODE "thread": FFmpeg's user thread transferring and unreferencing frames while the
decoder keeps calling the hwaccel). tools/sanitize.sh runs larger inputs and keeps the logs
under profiles/.
"""
import fcntl
import os
import subprocess

import numpy as np
import pytest

from test_ivf_decoder import _oracle_outputs, _stream
from test_hwaccel_harness import _read_frames

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "c", "build")
VARIANTS = ("plain", "asan", "tsan")


@pytest.fixture(scope="module")
def sanbins():
    # one make at a time: pytest-xdist workers each set this fixture up, and a worker linking
    # while another rewrites a host object links a truncated object
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "ffmpeg-hybrid_amd", "csrc"), "sanitize"],
                           capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return BUILD


def _clean(r):
    err = r.stderr
    return r.returncode == 0 and "ERROR: AddressSanitizer" not in err and "WARNING: ThreadSanitizer" not in err \
        and "runtime error" not in err


@pytest.fixture(scope="module")
def containers(v9, tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    pk = _stream(v9, 200, 130)
    files = []
    for name, data in (("s.ivf", v9.ivf_write(pk, 200, 130)),
                       ("s.webm", v9.webm_write(pk, 200, 130)),
                       ("x.webm", v9.webm_write(pk, 200, 130, lacing="xiph", block_groups=False, voids=True)),
                       ("e.webm", v9.webm_write(pk, 200, 130, lacing="ebml", unknown_sizes=True, other_track=True))):
        p = d / name
        p.write_bytes(data)
        files.append(str(p))
    return files


@pytest.mark.parametrize("variant", VARIANTS)
def test_host_side_clean(sanbins, containers, variant):
    r = subprocess.run([os.path.join(sanbins, "host_san_" + variant), "24"] + containers, capture_output=True,
                       text=True, timeout=600)
    assert _clean(r) and "host_san: ok" in r.stdout, (r.stdout[-500:], r.stderr[-3000:])


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("lag,mode,depth", [(0, "download", 16), (8, "device", 4), (20, "download", 0),
                                            (0, "thread", 16), (3, "thread", 1), (8, "thread", 4)])
def test_hwaccel_adapter_on_cpu(v9, orc, sanbins, tmp_path, variant, lag, mode, depth):
    pk = _stream(v9, 200, 130) * 2
    ivf = tmp_path / "s.ivf"
    ivf.write_bytes(v9.ivf_write(pk, 200, 130))
    out = tmp_path / "o.yuv"
    r = subprocess.run([os.path.join(sanbins, "hwaccel_cpu_" + variant), str(ivf), str(out), "8", "1", "1", "2",
                        str(lag), mode, str(depth)], capture_output=True, text=True, timeout=600)
    assert _clean(r), r.stderr[-3000:]
    ref = _oracle_outputs(v9, orc, pk)
    assert int(r.stdout.split()[1]) == 2 * len(ref)
    if mode != "device":
        got = _read_frames(str(out), 200, 130, 8, 1, 1)
        assert len(got) == 2 * len(ref)
        for i, (g, o) in enumerate(zip(got, ref + ref)):
            for p in range(3):
                assert np.array_equal(g[p], o[p]), "%s frame %d plane %d" % (variant, i, p)


@pytest.mark.parametrize("variant", ("plain", "asan"))
def test_hwaccel_adapter_default_extra_on_cpu(v9, orc, sanbins, tmp_path, variant):
    """FFmpeg's default extra_hw_frames (-1) handed to frame_params unclamped."""
    pk = _stream(v9, 200, 130)
    ivf = tmp_path / "s.ivf"
    ivf.write_bytes(v9.ivf_write(pk, 200, 130))
    r = subprocess.run([os.path.join(sanbins, "hwaccel_cpu_" + variant), str(ivf), str(tmp_path / "o.yuv"), "8", "1",
                        "1", "1", "0", "download", "0", "-1"], capture_output=True, text=True, timeout=300)
    assert _clean(r), r.stderr[-3000:]
    got = _read_frames(str(tmp_path / "o.yuv"), 200, 130, 8, 1, 1)
    ref = _oracle_outputs(v9, orc, pk)
    assert len(got) == len(ref) and all(np.array_equal(g[p], o[p]) for g, o in zip(got, ref) for p in range(3))
