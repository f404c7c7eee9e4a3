"""IVF container and the bitstream decode loop.

CPU: IVF read / write against the layout of libavformat/ivfdec.c and ivfenc.c (probe,
header fields, frame headers, pts, a zero time base, a short last frame), and an IVF
round trip of an encoded VP9 stream through the host parser.

GPU: vp9hip_decoder (avcodec_send_packet / avcodec_receive_frame for VP9) decodes IVF
streams with superframes, hidden frames, show_existing_frame, compound prediction and
profile 1 / 2 formats, bit-exact against the oracle driven by the same reference-slot
rules (vp9.c:1636-1653, 1686-1691, 1845-1849), at several batch sizes (decoder delay).
Parity of the parse itself is unpinned (no conformance bitstreams offline).
"""
import struct

import numpy as np
import pytest

from test_stream import _frames


def _stream(v9, w=200, h=130, bpp=8, ssh=1, ssv=1, n=6):
    """An IVF-ready packet list: key, P, [hidden ALTREF + P] superframe, P, show_existing of
    the hidden frame, compound P on (LAST, GOLDEN, ALTREF = hidden)."""
    fr = _frames(v9, w, h, n, bpp=bpp, compound=1, ss_h=ssh, ss_v=ssv)
    enc = v9.Stream()
    d0, _ = enc.encode(fr[0])
    d1, _ = enc.encode(fr[1], ref_slot=(0, 0, 0), refresh_mask=1 << 1)
    dh, _ = enc.encode(fr[2], show_frame=0, ref_slot=(1, 0, 0), refresh_mask=1 << 2)      # hidden
    d3, _ = enc.encode(fr[3], ref_slot=(1, 0, 2), refresh_mask=1 << 3, refresh_ctx=1, parallel=0)
    d4, _ = enc.encode(fr[4], ref_slot=(3, 0, 2), refresh_mask=1 << 4)
    dx, _ = enc.encode(None, show_existing_frame=1, show_slot=2)
    d5, _ = enc.encode(fr[5], ref_slot=(4, 0, 2), refresh_mask=1 << 5)
    return [d0, d1, v9.superframe_join([dh, d3]), d4, dx, d5]


def _oracle_outputs(v9, orc, packets):
    """The reference decode loop on the CPU: host parse + oracle reconstruction, slots by
    refresh mask, outputs = shown frames and show_existing_frame."""
    st = v9.Stream()
    slots = [None] * 8
    outs = []
    for data in packets:
        for fr in v9.superframe_split(data):
            p, info = st.decode(fr)
            if info.show_existing_frame:
                outs.append(slots[info.show_slot])
                continue
            pk = p.pkt
            planes = v9.alloc_planes(pk.width, pk.height, pk.bpp, pk.ss_h, pk.ss_v)
            intra = pk.keyframe or pk.intraonly
            refs = None if intra else [slots[s][0] for s in info.ref_slot]
            sizes = None if intra else [slots[s][1] for s in info.ref_slot]
            orc.decode_frame(pk, planes, refs, sizes)
            entry = (planes, (pk.width, pk.height), (pk.ss_h, pk.ss_v))
            for s in range(8):
                if info.refresh_mask & (1 << s):
                    slots[s] = entry
            if info.show_frame:
                outs.append(entry)
    return [v9.visible(pl, w, h, ss[0], ss[1]) for pl, (w, h), ss in outs]


# ------------------------------------------------------------------ CPU: IVF
def test_ivf_layout_and_round_trip(v9):
    frames = [(0, b"\x82\x49\x83"), (1, b""), (7, bytes(range(200))), (1 << 40, b"\xff" * 3)]
    data = v9.ivf_write(frames, 352, 288, time_base=(1, 30))
    # ivfenc.c write_header: DKIF, version 0, header 32, VP90, w, h, den, num, frames, 0
    assert data[:32] == b"DKIF" + struct.pack("<HH4sHHIII", 0, 32, b"VP90", 352, 288, 30, 1, 4) + b"\0" * 4
    assert data[32:44] == struct.pack("<IQ", 3, 0)
    assert v9.ivf_probe(data) == 98 and v9.ivf_probe(b"RIFF" + data[4:]) == 0
    h, got = v9.ivf_read(data)
    assert (h.fourcc, h.width, h.height, h.time_base_num, h.time_base_den, h.nb_frames) == (b"VP90", 352, 288, 1, 30, 4)
    assert got == frames               # an empty frame is an empty packet (av_get_packet of 0 bytes)


def test_ivf_errors(v9):
    data = v9.ivf_write([(0, b"abcdef"), (1, b"ghijkl")], 64, 64)
    with pytest.raises(v9.Vp9HipError) as e:
        v9.ivf_read(data[:20])
    assert e.value.code == v9.EINVALIDDATA
    bad = data[:16] + b"\0" * 8 + data[24:]                    # time base 0/0: "Invalid frame rate"
    with pytest.raises(v9.Vp9HipError) as e:
        v9.ivf_read(bad)
    assert e.value.code == v9.EINVALIDDATA
    _, got = v9.ivf_read(data[:-2])                            # short last frame: what is there
    assert got == [(0, b"abcdef"), (1, b"ghij")]
    _, got = v9.ivf_read(data[:-6 - 5])                        # partial frame header: end of stream
    assert got == [(0, b"abcdef")]


def test_ivf_vp9_stream_parses(v9):
    pkts = _stream(v9)
    data = v9.ivf_write(pkts, 200, 130)
    _, got = v9.ivf_read(data)
    assert [d for _, d in got] == pkts
    st = v9.Stream()
    shown = 0
    for _, d in got:
        for fr in v9.superframe_split(d):
            p, info = st.decode(fr)
            shown += info.show_frame or info.show_existing_frame
    assert shown == 6


# ------------------------------------------------------------------ GPU: decoder
def _decode_all(v9, packets, **kw):
    dec = v9.Decoder(0, **kw)
    out = [planes for planes, info in dec.decode([(d, i) for i, d in enumerate(packets)])]
    assert dec.eof
    dec.close()
    return out


def _same(a, b, what):
    assert len(a) == len(b), "%s: %d frames vs %d" % (what, len(a), len(b))
    for i, (x, y) in enumerate(zip(a, b)):
        for p, (u, v) in enumerate(zip(x, y)):
            assert u.shape == v.shape and np.array_equal(u, v), "%s: frame %d plane %d" % (what, i, p)


@pytest.mark.gpu
@pytest.mark.parametrize("max_batch,threads", [(1, 0), (3, 4), (16, 16), (4, 1)])
def test_decoder_ivf_stream_matches_oracle(v9, orc, max_batch, threads):
    pkts = _stream(v9)
    _, frames = v9.ivf_read(v9.ivf_write(pkts, 200, 130))
    ref = _oracle_outputs(v9, orc, [d for _, d in frames])
    got = _decode_all(v9, [d for _, d in frames], max_batch=max_batch, parse_threads=threads)
    _same(got, ref, "batch %d threads %d" % (max_batch, threads))


@pytest.mark.gpu
def test_decoder_parallel_gops_and_keyframes(v9, orc):
    """Keyframes start new parse chains (vp9h_frame_type == 0): three GOPs and a run of
    keyframes parse concurrently on the pool, outputs stay in order and bit-exact."""
    pkts = []
    for g in range(3):
        fr = _frames(v9, 136, 72, 4, seed=800 + 10 * g, compound=1)
        enc = v9.Stream()
        pkts += [enc.encode(f, **({} if i == 0 else dict(ref_slot=(0, 0, 0), refresh_mask=2 if i % 2 else 4)))[0]
                 for i, f in enumerate(fr)]
    for k in range(6):
        pkts.append(v9.encode_frame(v9.SynthFrame(v9.synth_params(136, 72, 8, seed=900 + k)), 60))
    assert [v9.vp9h_type(d) for d in pkts] == ([0, 1, 1, 1] * 3 + [0] * 6)
    ref = _oracle_outputs(v9, orc, pkts)
    for threads, batch in ((8, 5), (2, 16)):
        _same(_decode_all(v9, pkts, max_batch=batch, parse_threads=threads), ref, "threads %d" % threads)


@pytest.mark.gpu
@pytest.mark.parametrize("bpp,ssh,ssv", [(10, 1, 1), (8, 0, 0), (12, 1, 0)])
def test_decoder_formats(v9, orc, bpp, ssh, ssv):
    pkts = _stream(v9, 176, 144, bpp, ssh, ssv)
    _same(_decode_all(v9, pkts, max_batch=4), _oracle_outputs(v9, orc, pkts), "fmt %d %d%d" % (bpp, ssh, ssv))


@pytest.mark.gpu
def test_decoder_eagain_flush_and_restart(v9, orc):
    """send_packet's EAGAIN when no buffer is free (frames held by the caller), receive's
    EAGAIN inside the decoder delay, flush (seek) then a new keyframe."""
    fr = _frames(v9, 136, 72, 60)          # more than the parse lookahead + the buffer pool
    enc = v9.Stream()
    long_gop = [enc.encode(fr[0])[0]] + [enc.encode(f, ref_slot=(1 if i else 0, 0, 0), refresh_mask=2)[0]
                                         for i, f in enumerate(fr[1:])]
    pkts = _stream(v9)
    ref = _oracle_outputs(v9, orc, pkts)
    dec = v9.Decoder(0, max_batch=4, extra_bufs=1, parse_threads=1)   # 17 buffers, <= 5 frames in parse
    held = []
    sent = 0
    with pytest.raises(v9.Vp9HipError) as e:
        for d in long_gop:
            dec.send_packet(d)
            sent += 1
            while True:
                got = dec.receive_frame(download=False)
                if got is None:
                    break
                held.append(got[1].buf)                     # hold every frame: the pool runs dry
    assert e.value.code == v9.EAGAIN and 0 < sent < len(long_gop)
    for b in held:
        dec.release(b)
    dec.flush()
    assert dec.receive_frame() is None and not dec.eof
    got = [pl for pl, _ in dec.decode(pkts)]
    _same(got, ref, "after flush")
    dec.close()


@pytest.mark.gpu
def test_decoder_rejects_inter_without_keyframe(v9):
    """The parse runs ahead on the pool, so the error surfaces on the call that consumes
    the frame (send_packet or receive_frame), as with libavcodec's frame threads."""
    pkts = _stream(v9)
    for threads in (0, 4):
        dec = v9.Decoder(0, parse_threads=threads)
        with pytest.raises(v9.Vp9HipError) as e:
            dec.send_packet(pkts[1])
            dec.send_packet(None)
            dec.receive_frame()
        assert e.value.code == v9.EINVALIDDATA
        dec.close()
