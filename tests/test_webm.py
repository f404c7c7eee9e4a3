"""WebM / Matroska demux of a VP9 track (libavformat/matroskadec.c).

The reference's VP9 conformance vectors are .webm files (tests/fate/vpx.mak:98-104); they are
not in this container, so the demuxer is checked against streams written by the package's
small muxer (v9.webm_write, matroskaenc.c's element layout) in every form matroskadec.c
handles for a video track: known- and unknown-size Segment / Clusters, SimpleBlocks and
BlockGroups, Xiph / fixed / EBML lacing, interleaved blocks of another track, Void and Cues
elements; plus matroska_probe's scores and the header errors matroska_read_header reports.
Parse parity with matroskadec.c itself is unpinned (no reference binary, no vectors).

GPU: a VP9 stream demuxed from WebM decodes bit-exact against the oracle.
"""
import struct

import numpy as np
import pytest

from test_ivf_decoder import _decode_all, _oracle_outputs, _same, _stream

FRAMES = [(i * 33, bytes([(7 * i) & 255]) * (5 + 97 * i % 700)) for i in range(23)]


@pytest.mark.parametrize("kw", [{}, dict(unknown_sizes=True), dict(block_groups=True), dict(other_track=True),
                                dict(voids=True, cluster_frames=3), dict(lacing="fixed"),
                                dict(unknown_sizes=True, other_track=True, voids=True)])
def test_webm_round_trip(v9, kw):
    data = v9.webm_write(FRAMES, 352, 288, **kw)
    assert v9.webm_probe(data) == 100
    info, got = v9.webm_read(data)
    assert (info.doctype, info.codec_id, info.track, info.width, info.height, info.timecode_scale) == \
        (b"webm", b"V_VP9", 1, 352, 288, 1000000)
    assert [(p, d) for p, d, _ in got] == FRAMES
    assert got[0][2] == (-1 if kw.get("block_groups") else 1)          # SimpleBlock keyframe flag


@pytest.mark.parametrize("lacing", ["xiph", "ebml", "fixed"])
@pytest.mark.parametrize("groups", [False, True])
def test_webm_lacing(v9, lacing, groups):
    frames = FRAMES if lacing != "fixed" else [(p, bytes([i]) * 300) for i, (p, _) in enumerate(FRAMES)]
    # a 255-byte multiple and a zero-length lace exercise the Xiph run encoding
    if lacing == "xiph":
        frames = frames[:4] + [(frames[4][0], b"\x09" * 510), (frames[5][0], b"")] + frames[6:]
    data = v9.webm_write(frames, 64, 64, lacing=lacing, block_groups=groups)
    _, got = v9.webm_read(data)
    assert [d for _, d, _ in got] == [d for _, d in frames]
    # laces after the first: pts from the BlockGroup's BlockDuration, else none
    pts = [p for p, _, _ in got]
    for i, (p, _) in enumerate(frames):
        if i % 2 == 0 or groups:
            assert pts[i] == p
        else:
            assert pts[i] == v9.NOPTS


def test_webm_timecode_scale_and_negative_relative(v9):
    frames = [(100, b"a"), (90, b"b"), (130, b"c")]       # B-frame-like order: a negative relative timecode
    data = v9.webm_write(frames, 16, 16, timecode_scale=100000, cluster_frames=8)
    info, got = v9.webm_read(data)
    assert info.timecode_scale == 100000
    assert [(p, d) for p, d, _ in got] == frames


def test_webm_probe_scores(v9):
    data = v9.webm_write(FRAMES[:2], 16, 16)
    assert v9.webm_probe(data) == 100
    mk = data.replace(b"webm", b"matroska"[:4])                      # "matr": not a known doctype
    assert v9.webm_probe(mk) == 50
    assert v9.webm_probe(b"DKIF" + data[4:]) == 0
    assert v9.webm_probe(data[:6]) == 0                               # the header must be inside the probe data


def test_webm_errors(v9):
    good = v9.webm_write(FRAMES[:4], 16, 16)
    with pytest.raises(v9.Vp9HipError) as e:                          # no VP9 track
        v9.webm_read(good.replace(b"V_VP9", b"V_VP8"))
    assert e.value.code == v9.EINVALIDDATA
    bad = bytearray(good)
    i = bad.index(b"\x42\xf7\x81\x01")                                # EBMLReadVersion 1 -> 2
    bad[i + 3] = 2
    with pytest.raises(v9.Vp9HipError):
        v9.webm_read(bytes(bad))
    with pytest.raises(v9.Vp9HipError):                               # 0x00 as an EBML number's first byte
        v9.webm_read(b"\x1a\x45\xdf\xa3\x00" + good[5:])
    # a truncated file: the frames before the cut, then an error for the cut block
    cut = good[:len(good) - 40]
    with pytest.raises(v9.Vp9HipError) as e:
        v9.webm_read(cut)
    assert e.value.code == v9.EINVALIDDATA


def test_webm_vp9_stream_parses(v9):
    pkts = _stream(v9)
    _, got = v9.webm_read(v9.webm_write(pkts, 200, 130))
    assert [d for _, d, _ in got] == pkts
    st = v9.Stream()
    shown = 0
    for _, d, _ in got:
        for fr in v9.superframe_split(d):
            _, info = st.decode(fr)
            shown += info.show_frame or info.show_existing_frame
    assert shown == 6


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(unknown_sizes=True, lacing="xiph", other_track=True)])
def test_decoder_webm_stream_matches_oracle(v9, orc, kw):
    pkts = _stream(v9, 176, 144)
    _, got = v9.webm_read(v9.webm_write(pkts, 176, 144, **kw))
    data = [d for _, d, _ in got]
    _same(_decode_all(v9, data, max_batch=3), _oracle_outputs(v9, orc, pkts), "webm %s" % kw)
