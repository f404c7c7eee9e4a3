"""MI355X VP9 hybrid decoder — Python host bindings.

The product is the C-ABI shared library ``libvp9hip.so`` (include/vp9hip.h): host
runtime + gfx950 HIP kernels for the VP9 pixel path (inverse transforms, intra
prediction, motion compensation, loop filter). This module only binds it with
ctypes and mirrors the reference's decode API for this path
(``avcodec_send_packet`` / ``avcodec_receive_frame``, libavcodec/avcodec.c:707-717;
the VP9 decoder's frame loop vp9.c:1606-1863) at the pass-1 packet level.

There is no CPU fallback: if the HIP library cannot be loaded, every entry point
raises :class:`Vp9HipUnavailable`.
"""
import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvp9hip.so")

# AVERROR codes (include/vp9hip.h)
EINVAL = -22
ENOMEM = -12
ENOSYS = -38
EAGAIN = -11
EOF = -541478725
EINVALIDDATA = -1094995529
EEXTERNAL = -542398533
EBUG = -558323010

BS_64x64, BS_64x32, BS_32x64, BS_32x32, BS_32x16, BS_16x32, BS_16x16, BS_16x8, BS_8x16, \
    BS_8x8, BS_8x4, BS_4x8, BS_4x4 = range(13)


class Vp9HipUnavailable(RuntimeError):
    pass


class Vp9HipError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with AVERROR %d" % (fn, code))
        self.code = code


class Block(ctypes.Structure):
    """vp9h_block (include/vp9hip.h) == VP9Block (vp9dec.h:89-97)."""
    _fields_ = [("row", ctypes.c_uint16), ("col", ctypes.c_uint16), ("bs", ctypes.c_uint8),
                ("tx", ctypes.c_uint8), ("uvtx", ctypes.c_uint8), ("skip", ctypes.c_uint8),
                ("intra", ctypes.c_uint8), ("comp", ctypes.c_uint8), ("seg_id", ctypes.c_uint8),
                ("filter", ctypes.c_uint8), ("mode", ctypes.c_uint8 * 4), ("uvmode", ctypes.c_uint8),
                ("ref", ctypes.c_uint8 * 2), ("pad0", ctypes.c_uint8),
                ("mv", ctypes.c_int16 * 16)]


class FramePacket(ctypes.Structure):
    """vp9h_frame: one pass-1 frame packet."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("bpp", ctypes.c_uint8),
                ("ss_h", ctypes.c_uint8), ("ss_v", ctypes.c_uint8), ("keyframe", ctypes.c_uint8),
                ("intraonly", ctypes.c_uint8), ("lossless", ctypes.c_uint8),
                ("filter_level", ctypes.c_uint8), ("sharpness", ctypes.c_uint8),
                ("log2_tile_cols", ctypes.c_uint8), ("log2_tile_rows", ctypes.c_uint8),
                ("pad0", ctypes.c_uint8 * 2), ("lflvl", ctypes.c_uint8 * 64),
                ("ref_w", ctypes.c_int32 * 3), ("ref_h", ctypes.c_int32 * 3),
                ("nblocks", ctypes.c_uint32), ("neobs", ctypes.c_uint32), ("ncoefs", ctypes.c_uint64),
                ("blocks", ctypes.POINTER(Block)), ("eobs", ctypes.POINTER(ctypes.c_uint16)),
                ("coefs", ctypes.c_void_p)]


class SegParams(ctypes.Structure):
    """vp9h_seg_params: segmentation and LF deltas in effect for a frame."""
    _fields_ = [("enabled", ctypes.c_int32), ("update_map", ctypes.c_int32), ("temporal", ctypes.c_int32),
                ("update_data", ctypes.c_int32), ("abs_delta", ctypes.c_int32), ("q_en", ctypes.c_int32),
                ("lf_en", ctypes.c_int32), ("q", ctypes.c_int32 * 8), ("lf", ctypes.c_int32 * 8),
                ("nseg", ctypes.c_int32), ("lf_delta_update", ctypes.c_int32), ("lf_ref", ctypes.c_int32 * 4),
                ("lf_mode", ctypes.c_int32 * 2)]


def seg_params(**kw):
    """A SegParams from keyword fields (lists for q / lf / lf_ref / lf_mode)."""
    p = SegParams()
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        if k in ("q", "lf", "lf_ref", "lf_mode"):
            v = (ctypes.c_int32 * {"q": 8, "lf": 8, "lf_ref": 4, "lf_mode": 2}[k])(*v)
        setattr(p, k, v)
    return p


class SynthParams(ctypes.Structure):
    """vp9h_synth_params."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("bpp", ctypes.c_int32),
                ("ss_h", ctypes.c_int32), ("ss_v", ctypes.c_int32), ("log2_tile_cols", ctypes.c_int32),
                ("inter", ctypes.c_int32), ("compound", ctypes.c_int32), ("q_idx", ctypes.c_int32),
                ("lossless", ctypes.c_int32), ("filter_level", ctypes.c_int32),
                ("sharpness", ctypes.c_int32), ("bilinear", ctypes.c_int32),
                ("coef_stress", ctypes.c_int32), ("p_zero_eob", ctypes.c_float),
                ("p_skip", ctypes.c_float), ("seed", ctypes.c_uint64), ("seg", SegParams)]


class FrameInfo(ctypes.Structure):
    """vp9h_frame_info: the frame header's reference bookkeeping."""
    _fields_ = [("show_existing_frame", ctypes.c_int32), ("show_slot", ctypes.c_int32),
                ("show_frame", ctypes.c_int32), ("refresh_mask", ctypes.c_int32),
                ("ref_slot", ctypes.c_int32 * 3), ("sign_bias", ctypes.c_int32 * 3),
                ("error_res", ctypes.c_int32), ("refresh_ctx", ctypes.c_int32), ("parallel", ctypes.c_int32),
                ("ctx_id", ctypes.c_int32), ("allow_hp", ctypes.c_int32), ("interp", ctypes.c_int32),
                ("comp_mode", ctypes.c_int32), ("tx_mode", ctypes.c_int32),
                ("header_size", ctypes.c_uint32), ("compressed_header_size", ctypes.c_uint32)]


class EncParams(ctypes.Structure):
    """vp9h_enc_params: the encoder's per-frame choices."""
    _fields_ = [("base_q_idx", ctypes.c_int32), ("show_existing_frame", ctypes.c_int32),
                ("show_slot", ctypes.c_int32), ("show_frame", ctypes.c_int32), ("error_res", ctypes.c_int32),
                ("refresh_mask", ctypes.c_int32), ("ref_slot", ctypes.c_int32 * 3),
                ("sign_bias", ctypes.c_int32 * 3), ("refresh_ctx", ctypes.c_int32), ("parallel", ctypes.c_int32),
                ("ctx_id", ctypes.c_int32), ("reset_ctx", ctypes.c_int32), ("allow_hp", ctypes.c_int32),
                ("interp", ctypes.c_int32), ("comp_mode", ctypes.c_int32), ("tx_mode", ctypes.c_int32),
                ("prob_updates", ctypes.c_int32), ("keep_modes", ctypes.c_int32), ("seg", SegParams)]


_lib_handle = None
# torch's ROCm wheel ships its own libamdhip64 under the same soname as /opt/rocm's, which
# libvp9hip.so links: whichever process loads first serves both. torch's device init fails
# ("No HIP GPUs are available") on the newer /opt/rocm runtime, so torch interop
# (frame_tensors) needs torch imported before this library is loaded.
_torch_first = False

ABI_VERSION = 2                # VP9HIP_ABI_VERSION of include/vp9hip.h these bindings mirror
PIPELINE_SLOTS = 3             # VP9HIP_PIPELINE_SLOTS: batch slots the decoder / adapter rotate
# Exported symbols of include/vp9hip.h (checked by the CPU test suite).
ABI_SYMBOLS = ["vp9hip_open", "vp9hip_close", "vp9hip_configure", "vp9hip_submit_frame",
               "vp9hip_stage_batch", "vp9hip_stage_batch_refs", "vp9hip_run_batch", "vp9hip_sync",
               "vp9hip_download_frame",
               "vp9hip_upload_frame", "vp9hip_flush", "vp9hip_last_timing", "vp9hip_set_timing",
               "vp9hip_alg_bytes", "vp9hip_plan_stats", "vp9hip_plan_sb_costs", "vp9hip_abi_version", "vp9hip_set_graph",
               "vp9hip_stage_batch_tiles", "vp9hip_batch_phases", "vp9hip_phase_frames", "vp9hip_run_phase",
               "vp9hip_stripe", "vp9hip_frame_device", "vp9hip_batch_groups", "vp9hip_set_batch_slot", "vp9hip_sync_slot", "vp9hip_slot_busy",
               "vp9hip_fill_buffers", "vp9hip_device_info", "vp9hip_test_hooks", "vp9hip_batch_frame_status",
               "vp9h_decode_frame", "vp9h_encode_frame", "vp9h_frame_free", "vp9h_buffer_free",
               "vp9h_stream_open", "vp9h_stream_close", "vp9h_stream_set_threads", "vp9h_stream_decode", "vp9h_stream_encode",
               "vp9h_enc_defaults", "vp9h_superframe_split", "vp9h_frame_type", "vp9h_frame_peek",
               "vp9hip_slot_stream_wait",
               "vp9hip_synth_defaults", "vp9hip_synth_frame", "vp9hip_synth_free",
               "vp9h_ivf_probe", "vp9h_ivf_read_header", "vp9h_ivf_read_frame", "vp9h_ivf_write_header",
               "vp9h_ivf_write_frame_header", "vp9h_webm_probe", "vp9h_webm_read_header", "vp9h_webm_read_frame",
               "vp9hip_decoder_defaults", "vp9hip_decoder_open", "vp9hip_decoder_close", "vp9hip_decoder_context",
               "vp9hip_decoder_send_packet", "vp9hip_decoder_receive_frame", "vp9hip_decoder_release",
               "vp9hip_decoder_flush"]


def lib():
    """Load libvp9hip.so (fails loudly: there is no CPU fallback)."""
    global _lib_handle
    if _lib_handle is not None:
        return _lib_handle
    if not os.path.exists(LIB_PATH):
        raise Vp9HipUnavailable("libvp9hip.so not built: run __graft_entry__.build() (%s)" % LIB_PATH)
    global _torch_first
    _torch_first = "torch" in sys.modules
    L = ctypes.CDLL(LIB_PATH)
    # the struct mirrors below are the header's of this ABI version (vp9h_synth_params and
    # vp9h_enc_params grew in version 2): a library built from another header is refused
    if L.vp9hip_abi_version() != ABI_VERSION:
        raise Vp9HipUnavailable("libvp9hip.so ABI version %d, these bindings need %d: rebuild it (%s)"
                                % (L.vp9hip_abi_version(), ABI_VERSION, LIB_PATH))
    vp = ctypes.c_void_p
    L.vp9hip_open.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.vp9hip_close.argtypes = [vp]
    L.vp9hip_close.restype = None
    L.vp9hip_configure.argtypes = [vp] + [ctypes.c_int] * 6
    L.vp9hip_submit_frame.argtypes = [vp, ctypes.POINTER(FramePacket), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.vp9hip_stage_batch.argtypes = [vp, ctypes.POINTER(FramePacket), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.vp9hip_stage_batch_refs.argtypes = [vp, ctypes.POINTER(FramePacket), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int)]
    L.vp9hip_stage_batch_tiles.argtypes = [vp, ctypes.POINTER(FramePacket), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int]
    L.vp9hip_batch_phases.argtypes = [vp]
    L.vp9hip_batch_groups.argtypes = [vp]
    L.vp9hip_set_batch_slot.argtypes = [vp, ctypes.c_int]
    L.vp9hip_sync_slot.argtypes = [vp, ctypes.c_int]
    L.vp9hip_batch_frame_status.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.vp9hip_slot_busy.argtypes = [vp, ctypes.c_int]
    L.vp9hip_phase_frames.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.vp9hip_run_phase.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    L.vp9hip_stripe.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.vp9hip_stripe.restype = ctypes.c_int64
    L.vp9hip_frame_device.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_ssize_t),
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_void_p)]
    L.vp9hip_device_info.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.vp9hip_fill_buffers.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.vp9hip_test_hooks.argtypes = [ctypes.c_int, ctypes.c_uint32]
    L.vp9hip_test_hooks.restype = None
    L.vp9hip_run_batch.argtypes = [vp]
    L.vp9hip_sync.argtypes = [vp]
    L.vp9hip_download_frame.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_ssize_t)]
    L.vp9hip_upload_frame.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_ssize_t)]
    L.vp9hip_flush.argtypes = [vp]
    L.vp9hip_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.vp9hip_alg_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    L.vp9hip_set_timing.argtypes = [vp, ctypes.c_int]
    L.vp9hip_synth_defaults.argtypes = [ctypes.POINTER(SynthParams), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.vp9hip_synth_defaults.restype = None
    L.vp9hip_synth_frame.argtypes = [ctypes.POINTER(FramePacket), ctypes.POINTER(SynthParams)]
    L.vp9hip_synth_free.argtypes = [ctypes.POINTER(FramePacket)]
    L.vp9hip_synth_free.restype = None
    L.vp9h_decode_frame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(FramePacket)]
    L.vp9h_encode_frame.argtypes = [ctypes.POINTER(FramePacket), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                    ctypes.POINTER(ctypes.c_size_t)]
    L.vp9h_frame_free.argtypes = [ctypes.POINTER(FramePacket)]
    L.vp9h_frame_free.restype = None
    L.vp9h_buffer_free.argtypes = [ctypes.c_void_p]
    L.vp9h_buffer_free.restype = None
    L.vp9h_stream_open.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    L.vp9h_stream_set_threads.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.vp9h_stream_close.argtypes = [ctypes.c_void_p]
    L.vp9h_stream_close.restype = None
    L.vp9h_stream_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(FramePacket),
                                     ctypes.POINTER(FrameInfo)]
    L.vp9h_stream_encode.argtypes = [ctypes.c_void_p, ctypes.POINTER(FramePacket), ctypes.POINTER(EncParams),
                                     ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(FramePacket)]
    L.vp9h_enc_defaults.argtypes = [ctypes.POINTER(EncParams)]
    L.vp9h_enc_defaults.restype = None
    L.vp9h_superframe_split.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]
    L.vp9h_frame_type.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.vp9h_frame_peek.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(FrameInfo)]
    L.vp9hip_slot_stream_wait.argtypes = [vp, ctypes.c_int, ctypes.c_void_p]
    L.vp9h_ivf_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.vp9h_ivf_read_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(IvfHeader)]
    L.vp9h_ivf_read_frame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.vp9h_ivf_write_header.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32]
    L.vp9h_ivf_write_frame_header.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64]
    L.vp9h_ivf_write_frame_header.restype = None
    L.vp9h_webm_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.vp9h_webm_read_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(WebmInfo),
                                        ctypes.POINTER(WebmCursor)]
    L.vp9h_webm_read_frame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(WebmCursor),
                                       ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.vp9hip_decoder_defaults.argtypes = [ctypes.POINTER(DecoderParams)]
    L.vp9hip_decoder_defaults.restype = None
    L.vp9hip_decoder_open.argtypes = [ctypes.POINTER(DecoderParams), ctypes.POINTER(vp)]
    L.vp9hip_decoder_close.argtypes = [vp]
    L.vp9hip_decoder_close.restype = None
    L.vp9hip_decoder_context.argtypes = [vp]
    L.vp9hip_decoder_context.restype = vp
    L.vp9hip_decoder_send_packet.argtypes = [vp, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64]
    L.vp9hip_decoder_receive_frame.argtypes = [vp, ctypes.POINTER(DecodedFrameInfo)]
    L.vp9hip_decoder_release.argtypes = [vp, ctypes.c_int]
    L.vp9hip_decoder_flush.argtypes = [vp]
    _lib_handle = L
    return L


class IvfHeader(ctypes.Structure):
    _fields_ = [("fourcc", ctypes.c_char * 5), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("time_base_den", ctypes.c_uint32), ("time_base_num", ctypes.c_uint32),
                ("nb_frames", ctypes.c_uint32), ("header_size", ctypes.c_uint32)]


class WebmInfo(ctypes.Structure):
    _fields_ = [("doctype", ctypes.c_char * 16), ("codec_id", ctypes.c_char * 32), ("track", ctypes.c_uint64),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("timecode_scale", ctypes.c_uint64)]


class WebmCursor(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_uint64), ("seg_end", ctypes.c_uint64), ("cluster_end", ctypes.c_uint64),
                ("track", ctypes.c_uint64), ("cluster_tc", ctypes.c_int64), ("block_pts", ctypes.c_int64),
                ("block_duration", ctypes.c_int64), ("cluster_unknown", ctypes.c_int32), ("keyframe", ctypes.c_int32),
                ("nlaces", ctypes.c_int32), ("lace_idx", ctypes.c_int32), ("lace_pos", ctypes.c_uint64),
                ("lace_size", ctypes.c_uint32 * 256)]


class DecoderParams(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_batch", ctypes.c_int32), ("extra_bufs", ctypes.c_int32),
                ("max_width", ctypes.c_int32), ("max_height", ctypes.c_int32), ("parse_threads", ctypes.c_int32)]


class DecodedFrameInfo(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("bpp", ctypes.c_int32), ("ss_h", ctypes.c_int32), ("ss_v", ctypes.c_int32),
                ("pts", ctypes.c_int64)]


def _check(fn, r):
    if r < 0:
        raise Vp9HipError(fn, r)
    return r


def synth_params(width, height, bpp=8, **kw):
    """§8(d) default stream settings, overridable by keyword."""
    p = SynthParams()
    lib().vp9hip_synth_defaults(ctypes.byref(p), width, height, bpp)
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        if k == "seg" and isinstance(v, dict):
            v = seg_params(**v)
        setattr(p, k, v)
    return p


class SynthFrame:
    """A pass-1 frame packet generated by vp9hip_synth_frame (owns its C arrays)."""

    def __init__(self, params):
        self.params = params
        self.pkt = FramePacket()
        _check("vp9hip_synth_frame", lib().vp9hip_synth_frame(ctypes.byref(self.pkt), ctypes.byref(params)))

    def __del__(self):
        if getattr(self, "pkt", None) is not None and _lib_handle is not None:
            _lib_handle.vp9hip_synth_free(ctypes.byref(self.pkt))
            self.pkt = None

    @property
    def nbytes_coefs(self):
        return self.pkt.ncoefs * (2 if self.pkt.bpp == 8 else 4)

    def blocks(self):
        return [self.pkt.blocks[i] for i in range(self.pkt.nblocks)]


def encode_frame(frame, base_q_idx):
    """Write a pass-1 packet (SynthFrame or FramePacket) as a VP9 frame bitstream
    (vp9h_encode_frame): returns bytes."""
    pkt = frame.pkt if hasattr(frame, "pkt") else frame
    buf, n = ctypes.c_void_p(), ctypes.c_size_t()
    _check("vp9h_encode_frame", lib().vp9h_encode_frame(ctypes.byref(pkt), base_q_idx, ctypes.byref(buf), ctypes.byref(n)))
    try:
        return ctypes.string_at(buf.value, n.value)
    finally:
        lib().vp9h_buffer_free(buf)


class DecodedFrame:
    """The pass-1 packet of one VP9 frame bitstream, parsed on the host by
    vp9h_decode_frame (owns its C arrays); usable wherever a SynthFrame is."""

    def __init__(self, data):
        self._data = bytes(data)
        self.pkt = FramePacket()
        _check("vp9h_decode_frame", lib().vp9h_decode_frame(self._data, len(self._data), ctypes.byref(self.pkt)))

    def __del__(self):
        if getattr(self, "pkt", None) is not None and _lib_handle is not None:
            _lib_handle.vp9h_frame_free(ctypes.byref(self.pkt))
            self.pkt = None


class _OwnedPacket:
    """A pass-1 packet whose arrays the library allocated (vp9h_frame_free)."""

    def __init__(self):
        self.pkt = FramePacket()

    def __del__(self):
        if getattr(self, "pkt", None) is not None and _lib_handle is not None:
            _lib_handle.vp9h_frame_free(ctypes.byref(self.pkt))
            self.pkt = None

    def blocks(self):
        return [self.pkt.blocks[i] for i in range(self.pkt.nblocks)]


def enc_params(**kw):
    """vp9h_enc_defaults, overridable by keyword (ref_slot / sign_bias take 3-sequences)."""
    p = EncParams()
    lib().vp9h_enc_defaults(ctypes.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        if k in ("ref_slot", "sign_bias"):
            v = (ctypes.c_int32 * 3)(*v)
        if k == "seg" and isinstance(v, dict):
            v = seg_params(**v)
        setattr(p, k, v)
    return p


class Stream:
    """A stream's host parse state (vp9h_stream): decode or encode frames in order."""

    def __init__(self, threads=1):
        self._s = ctypes.c_void_p()
        _check("vp9h_stream_open", lib().vp9h_stream_open(ctypes.byref(self._s)))
        if threads != 1:
            self.set_threads(threads)

    def set_threads(self, n):
        """Tile-column threads of decode (vp9h_stream_set_threads)."""
        _check("vp9h_stream_set_threads", lib().vp9h_stream_set_threads(self._s, int(n)))

    def close(self):
        if self._s:
            lib().vp9h_stream_close(self._s)
            self._s = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, data):
        """One frame of compressed data -> (packet or None for show_existing_frame, FrameInfo)."""
        data = bytes(data)
        out, info = _OwnedPacket(), FrameInfo()
        _check("vp9h_stream_decode", lib().vp9h_stream_decode(self._s, data, len(data), ctypes.byref(out.pkt),
                                                               ctypes.byref(info)))
        return (None if info.show_existing_frame else out), info

    def encode(self, frame, params=None, **kw):
        """Write one frame (a packet, or None with show_existing_frame=1): returns
        (bytes, coded packet or None)."""
        p = params if params is not None else enc_params(**kw)
        pkt = None if frame is None else (frame.pkt if hasattr(frame, "pkt") else frame)
        buf, n = ctypes.c_void_p(), ctypes.c_size_t()
        coded = _OwnedPacket()
        _check("vp9h_stream_encode", lib().vp9h_stream_encode(self._s, ctypes.byref(pkt) if pkt is not None else None,
                                                               ctypes.byref(p), ctypes.byref(buf), ctypes.byref(n),
                                                               ctypes.byref(coded.pkt)))
        try:
            data = ctypes.string_at(buf.value, n.value)
        finally:
            lib().vp9h_buffer_free(buf)
        return data, (coded if pkt is not None else None)


def superframe_split(data):
    """The frames of a superframe (vp9h_superframe_split), as bytes objects."""
    data = bytes(data)
    offs, sizes = (ctypes.c_size_t * 8)(), (ctypes.c_size_t * 8)()
    n = _check("vp9h_superframe_split", lib().vp9h_superframe_split(data, len(data), offs, sizes, 8))
    return [data[offs[i]:offs[i] + sizes[i]] for i in range(n)]


def superframe_join(frames):
    """Pack frames into one superframe with the index vp9_superframe_split reads."""
    if len(frames) == 1:
        return bytes(frames[0])
    mx = max(len(f) for f in frames)
    ln = 1 if mx < 1 << 8 else 2 if mx < 1 << 16 else 3 if mx < 1 << 24 else 4
    marker = 0xc0 | (ln - 1) << 3 | (len(frames) - 1)
    idx = bytes([marker]) + b"".join(len(f).to_bytes(ln, "little") for f in frames) + bytes([marker])
    return b"".join(bytes(f) for f in frames) + idx


def alloc_planes(width, height, bpp, ss_h=1, ss_v=1, pad=64):
    """Host planes padded to 64 luma pixels (the layout the oracle expects)."""
    dt = np.uint8 if bpp == 8 else np.uint16
    W = (width + pad - 1) // pad * pad
    H = (height + pad - 1) // pad * pad
    return [np.zeros((H, W), dt), np.zeros((H >> ss_v, W >> ss_h), dt), np.zeros((H >> ss_v, W >> ss_h), dt)]


def visible(planes, width, height, ss_h=1, ss_v=1):
    cw, ch = (width + ss_h) >> ss_h, (height + ss_v) >> ss_v
    return [planes[0][:height, :width], planes[1][:ch, :cw], planes[2][:ch, :cw]]


def decode_frame(data):
    """Host entropy decode of one VP9 frame -> DecodedFrame (pass-1 packet)."""
    return DecodedFrame(data)


def test_hooks(reject_batch=0, lfr_spin=0, reject_frame=0):
    """Test hooks copied by every context opened afterwards (vp9hip_test_hooks): frame
    reject_frame of the reject_batch-th batch a context stages starts with an intra block
    whose mode the planner rejects; lfr_spin bounds the row loop filter's hand-off waits
    (0, 0: off)."""
    lib().vp9hip_test_hooks(int(reject_batch) | int(reject_frame) << 16 if reject_batch else 0, int(lfr_spin))


def device_info(device):
    """(PCI bus id, name) of HIP device `device` (vp9hip_device_info)."""
    bus, name = ctypes.create_string_buffer(64), ctypes.create_string_buffer(256)
    _check("vp9hip_device_info", lib().vp9hip_device_info(device, bus, 64, name, 256))
    return bus.value.decode(), name.value.decode()


class Device:
    """A vp9hip context on one GPU (vp9hip_open / vp9hip_configure)."""

    def __init__(self, device=0):
        self._c = ctypes.c_void_p()
        _check("vp9hip_open", lib().vp9hip_open(device, ctypes.byref(self._c)))
        self.w = self.h = 0
        self.bpp = 8

    def close(self):
        if self._c:
            lib().vp9hip_close(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def configure(self, width, height, bpp=8, nbufs=4, ss_h=1, ss_v=1):
        _check("vp9hip_configure", lib().vp9hip_configure(self._c, width, height, bpp, ss_h, ss_v, nbufs))
        self.w, self.h, self.bpp, self.ss_h, self.ss_v = width, height, bpp, ss_h, ss_v

    def submit(self, frame, out_buf, refs=(0, 0, 0)):
        r = (ctypes.c_int * 3)(*refs)
        pkt = frame.pkt if hasattr(frame, "pkt") else frame
        _check("vp9hip_submit_frame", lib().vp9hip_submit_frame(self._c, ctypes.byref(pkt), out_buf, r))

    def stage_batch(self, frames, out_bufs, ref_bufs=None, tiles=None):
        """Stage a batch; ref_bufs: per frame (LAST, GOLDEN, ALTREF) buffer ids or None
        (keyframes). Dependent frames are chained, independent chains run concurrently.
        tiles=(lo, hi): reconstruct only tile columns [lo, hi) (a shard of a tile-sharded
        stream, run with run_phase; see tileshard.py)."""
        arr = (FramePacket * len(frames))(*[f.pkt if hasattr(f, "pkt") else f for f in frames])
        ob = (ctypes.c_int * len(out_bufs))(*out_bufs)
        self._staged = (arr, frames)   # keep host packets alive
        if ref_bufs is None and tiles is None:
            _check("vp9hip_stage_batch", lib().vp9hip_stage_batch(self._c, arr, len(frames), ob))
            return
        flat = []
        for r in (ref_bufs if ref_bufs is not None else [None] * len(frames)):
            flat += list(r) if r is not None else [0, 0, 0]
        rb = (ctypes.c_int * len(flat))(*flat)
        if tiles is not None:
            _check("vp9hip_stage_batch_tiles",
                   lib().vp9hip_stage_batch_tiles(self._c, arr, len(frames), ob, rb, int(tiles[0]), int(tiles[1])))
            return
        _check("vp9hip_stage_batch_refs", lib().vp9hip_stage_batch_refs(self._c, arr, len(frames), ob, rb))

    PART_RECON, PART_LF = 0, 1
    MAX_SLOTS = 4                  # VP9HIP_MAX_SLOTS (include/vp9hip.h)

    def set_slot(self, slot):
        """Select batch slot 0 .. MAX_SLOTS - 1 (vp9hip_set_batch_slot): staged batches run in
        turn overlap one batch's device planning and pixel chains with the others'."""
        _check("vp9hip_set_batch_slot", lib().vp9hip_set_batch_slot(self._c, int(slot)))

    def phases(self):
        """Number of phases (chain positions) of the staged batch."""
        return _check("vp9hip_batch_phases", lib().vp9hip_batch_phases(self._c))

    def groups(self):
        """Frame groups (concurrent HIP streams) of the staged batch."""
        return _check("vp9hip_batch_groups", lib().vp9hip_batch_groups(self._c))

    def phase_frames(self, phase):
        """Batch indices of the frames in `phase`."""
        n = _check("vp9hip_phase_frames", lib().vp9hip_phase_frames(self._c, phase, None, 0))
        a = (ctypes.c_int * max(n, 1))()
        _check("vp9hip_phase_frames", lib().vp9hip_phase_frames(self._c, phase, a, n))
        return list(a[:n])

    def run_phase(self, phase, part):
        _check("vp9hip_run_phase", lib().vp9hip_run_phase(self._c, phase, part))

    def stripe(self, frame, tile_lo, tile_hi, dev_ptr=None, to_frame=False):
        """Pack / unpack the pre-LF columns of tile columns [lo, hi) of batch frame `frame`
        to / from device memory at dev_ptr (an int address); returns the byte count."""
        return _check("vp9hip_stripe", lib().vp9hip_stripe(self._c, frame, tile_lo, tile_hi,
                                                           ctypes.c_void_p(dev_ptr) if dev_ptr else None,
                                                           int(bool(to_frame))))

    def run_batch(self):
        _check("vp9hip_run_batch", lib().vp9hip_run_batch(self._c))

    def sync(self):
        _check("vp9hip_sync", lib().vp9hip_sync(self._c))

    def sync_slot(self, slot):
        """Wait for batch slot `slot`'s last run and check its loop-filter hand-offs."""
        _check("vp9hip_sync_slot", lib().vp9hip_sync_slot(self._c, int(slot)))

    def frame_status(self, slot):
        """Per-frame outcome of the slot's last stage / run after it reported
        AVERROR_INVALIDDATA (vp9hip_batch_frame_status): 0 reconstructed, EINVALIDDATA
        rejected, EAGAIN valid but not run."""
        n = _check("vp9hip_batch_frame_status", lib().vp9hip_batch_frame_status(self._c, int(slot), None, 0))
        a = (ctypes.c_int * max(n, 1))()
        _check("vp9hip_batch_frame_status", lib().vp9hip_batch_frame_status(self._c, int(slot), a, n))
        return list(a[:n])

    def fill(self, buf0, count, value):
        """Fill device buffers [buf0, buf0 + count) with byte `value` (async, context stream)."""
        _check("vp9hip_fill_buffers", lib().vp9hip_fill_buffers(self._c, int(buf0), int(count), int(value)))

    def set_timing(self, on):
        _check("vp9hip_set_timing", lib().vp9hip_set_timing(self._c, int(bool(on))))

    def timing(self):
        names = (ctypes.c_char_p * 8)()
        ms = (ctypes.c_double * 8)()
        cnt = (ctypes.c_int * 8)()
        n = _check("vp9hip_last_timing", lib().vp9hip_last_timing(self._c, names, ms, cnt, 8))
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(n)}

    def alg_bytes(self):
        """Algorithmic bytes of the staged batch per kernel class, keyed like timing()."""
        b = (ctypes.c_double * 8)()
        n = _check("vp9hip_alg_bytes", lib().vp9hip_alg_bytes(self._c, b, 8))
        names = list(self.timing().keys())
        return {names[i]: b[i] for i in range(n)}

    def _plane_args(self, planes):
        ptrs = (ctypes.c_void_p * 3)(*[p.ctypes.data for p in planes])
        ls = (ctypes.c_ssize_t * 3)(*[p.strides[0] for p in planes])
        return ptrs, ls

    def download(self, buf):
        planes = alloc_planes(self.w, self.h, self.bpp, self.ss_h, self.ss_v)
        ptrs, ls = self._plane_args(planes)
        _check("vp9hip_download_frame", lib().vp9hip_download_frame(self._c, buf, ptrs, ls))
        return planes

    def frame_device(self, buf):
        """Device planes of buffer `buf` without a copy: ([ptr] * 3, [pitch bytes] * 3,
        (width, height), hipStream_t handle) -- vp9hip_frame_device."""
        ptrs = (ctypes.c_void_p * 3)()
        ls = (ctypes.c_ssize_t * 3)()
        w, h, st = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
        _check("vp9hip_frame_device", lib().vp9hip_frame_device(self._c, buf, ptrs, ls, ctypes.byref(w), ctypes.byref(h),
                                                                ctypes.byref(st)))
        return list(ptrs), list(ls), (w.value, h.value), st.value

    def frame_tensors(self, buf, device=None):
        """Zero-copy torch views (uint8 / int16 storage of the u16 samples) of buffer
        `buf`'s visible planes, via __cuda_array_interface__. Call sync() first (or order
        consumers after the context's stream). Needs torch imported before the library was
        loaded (see _torch_first)."""
        if not _torch_first:
            raise Vp9HipUnavailable("frame_tensors: import torch before ffmpeg-hybrid_amd loads libvp9hip.so "
                                    "(both use libamdhip64; torch's device init needs its own runtime loaded first)")
        import torch
        ptrs, ls, (w, h), _ = self.frame_device(buf)
        bpp = 1 if self.bpp == 8 else 2
        out = []
        for p in range(3):
            pw = w if p == 0 else (w + self.ss_h) >> self.ss_h
            ph = h if p == 0 else (h + self.ss_v) >> self.ss_v

            class _View:
                __cuda_array_interface__ = {"shape": (ph, pw), "typestr": "|u1" if bpp == 1 else "<i2",
                                            "data": (ptrs[p], False), "strides": (ls[p], bpp), "version": 2}
            out.append(torch.as_tensor(_View(), device=device or "cuda"))
        return out

    def upload(self, buf, planes):
        planes = [np.ascontiguousarray(p) for p in planes]
        ptrs, ls = self._plane_args(planes)
        _check("vp9hip_upload_frame", lib().vp9hip_upload_frame(self._c, buf, ptrs, ls))

    def flush(self):
        _check("vp9hip_flush", lib().vp9hip_flush(self._c))


class PacketDecoder:
    """send_packet / receive_frame over pass-1 frame packets (no bitstream parse).

    Reference slots are simplified: every decoded frame becomes LAST, GOLDEN and
    ALTREF of the next inter frame. Bitstreams go through Decoder.
    """

    def __init__(self, device=0, nbufs=4):
        self.dev = Device(device)
        self.nbufs = nbufs
        self._configured = None
        self._queue = []
        self._last = None
        self._next = 0

    def send_packet(self, frame):
        pkt = frame.pkt if hasattr(frame, "pkt") else frame
        cfg = (pkt.width, pkt.height, pkt.bpp)
        if self._configured != cfg:
            self.dev.configure(pkt.width, pkt.height, pkt.bpp, self.nbufs, pkt.ss_h, pkt.ss_v)
            self._configured = cfg
            self._last = None
        out = self._next
        self._next = (self._next + 1) % self.nbufs
        ref = self._last if self._last is not None else out
        self.dev.submit(pkt, out, (ref, ref, ref))
        self._last = out
        self._queue.append(out)

    def receive_frame(self):
        """Returns the next decoded frame as visible numpy planes, or None (EAGAIN)."""
        if not self._queue:
            return None
        buf = self._queue.pop(0)
        w, h, bpp = self._configured
        return visible(self.dev.download(buf), w, h)


class Decoder:
    """avcodec_send_packet / avcodec_receive_frame for AV_CODEC_ID_VP9 (vp9hip_decoder):
    compressed VP9 packets in, decoded frames out. The host parses each frame
    (vp9h_stream), the MI355X reconstructs them in batches of up to max_batch frames.

    send_packet(data, pts) -> None; raises Vp9HipError with code EAGAIN when frames must
    be received first. send_packet(None) drains. receive_frame() -> (planes, info) with
    visible numpy planes (download=True) or a device-buffer handle, None when more input
    is needed (EAGAIN) or after the drain (EOF, which also sets .eof).
    """

    def __init__(self, device=0, max_batch=16, extra_bufs=4, max_width=0, max_height=0, parse_threads=None):
        self.params = DecoderParams()
        lib().vp9hip_decoder_defaults(ctypes.byref(self.params))
        self.params.device, self.params.max_batch, self.params.extra_bufs = device, max_batch, extra_bufs
        self.params.max_width, self.params.max_height = max_width, max_height
        if parse_threads is not None:
            self.params.parse_threads = parse_threads
        self._d = ctypes.c_void_p()
        _check("vp9hip_decoder_open", lib().vp9hip_decoder_open(ctypes.byref(self.params), ctypes.byref(self._d)))
        self.eof = False

    def close(self):
        if self._d:
            lib().vp9hip_decoder_close(self._d)
            self._d = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def send_packet(self, data, pts=0):
        if data is None:
            _check("vp9hip_decoder_send_packet", lib().vp9hip_decoder_send_packet(self._d, None, 0, 0))
            return
        data = bytes(data)
        _check("vp9hip_decoder_send_packet", lib().vp9hip_decoder_send_packet(self._d, data, len(data), pts))

    def receive_frame(self, download=True):
        """Next output frame: (visible planes, DecodedFrameInfo) with download=True, else
        (None, info) with info.buf valid until release(info.buf). None: EAGAIN / EOF."""
        info = DecodedFrameInfo()
        r = lib().vp9hip_decoder_receive_frame(self._d, ctypes.byref(info))
        if r == EAGAIN:
            return None
        if r == EOF:
            self.eof = True
            return None
        _check("vp9hip_decoder_receive_frame", r)
        if not download:
            return None, info
        planes = alloc_planes(info.width, info.height, info.bpp, info.ss_h, info.ss_v)
        ptrs = (ctypes.c_void_p * 3)(*[p.ctypes.data for p in planes])
        ls = (ctypes.c_ssize_t * 3)(*[p.strides[0] for p in planes])
        try:
            _check("vp9hip_download_frame", lib().vp9hip_download_frame(self.context(), info.buf, ptrs, ls))
        finally:
            self.release(info.buf)
        return visible(planes, info.width, info.height, info.ss_h, info.ss_v), info

    def release(self, buf):
        _check("vp9hip_decoder_release", lib().vp9hip_decoder_release(self._d, buf))

    def context(self):
        return ctypes.c_void_p(lib().vp9hip_decoder_context(self._d))

    def flush(self):
        _check("vp9hip_decoder_flush", lib().vp9hip_decoder_flush(self._d))
        self.eof = False

    def decode(self, packets, download=True):
        """Decode an iterable of (data, pts) or data: yields receive_frame results in
        output order, draining at the end (the ffmpeg -i ... -f null - loop)."""
        for item in packets:
            data, pts = item if isinstance(item, tuple) else (item, 0)
            while True:
                try:
                    self.send_packet(data, pts)
                    break
                except Vp9HipError as e:
                    if e.code != EAGAIN:
                        raise
                    got = self.receive_frame(download)
                    if got is None:
                        raise
                    yield got
            while True:
                got = self.receive_frame(download)
                if got is None:
                    break
                yield got
        self.send_packet(None)
        while True:
            got = self.receive_frame(download)
            if got is None:
                break
            yield got


def frame_peek(data):
    """(type, FrameInfo) from the start of the uncompressed header (vp9h_frame_peek): type 0
    keyframe, 1 inter, 2 show_existing_frame, 3 intra-only; slot bookkeeping without state."""
    data = bytes(data)
    info = FrameInfo()
    t = _check("vp9h_frame_peek", lib().vp9h_frame_peek(data, len(data), ctypes.byref(info)))
    return t, info


def vp9h_type(data):
    """Frame type from the header's first bits (vp9h_frame_type): 0 key, 1 other, 2
    show_existing_frame, or a negative AVERROR."""
    data = bytes(data)
    return lib().vp9h_frame_type(data, len(data))


# ---- IVF (libavformat/ivfdec.c, ivfenc.c) -------------------------------------------
def ivf_probe(data):
    data = bytes(data[:32])
    return lib().vp9h_ivf_probe(data, len(data))


def ivf_read(data):
    """IVF bytes -> (IvfHeader, [(pts, frame bytes)]). A short last frame is returned
    as far as it goes (av_get_packet)."""
    data = bytes(data)
    h = IvfHeader()
    _check("vp9h_ivf_read_header", lib().vp9h_ivf_read_header(data, len(data), ctypes.byref(h)))
    frames = []
    pos = ctypes.c_size_t(32)
    ptr, n, pts, tr = ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_int64(), ctypes.c_int()
    base = ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p).value
    while True:
        r = lib().vp9h_ivf_read_frame(data, len(data), ctypes.byref(pos), ctypes.byref(ptr), ctypes.byref(n),
                                      ctypes.byref(pts), ctypes.byref(tr))
        if r == EOF:
            break
        _check("vp9h_ivf_read_frame", r)
        off = ptr.value - base
        frames.append((pts.value, data[off:off + n.value]))
    return h, frames


def ivf_write(frames, width, height, time_base=(1, 30)):
    """[(pts, bytes)] or [bytes] -> IVF bytes (fourcc VP90, frame count filled in)."""
    hdr = ctypes.create_string_buffer(32)
    _check("vp9h_ivf_write_header", lib().vp9h_ivf_write_header(hdr, width, height, time_base[1], time_base[0],
                                                                 len(frames)))
    out = [hdr.raw]
    fh = ctypes.create_string_buffer(12)
    for i, f in enumerate(frames):
        pts, data = f if isinstance(f, tuple) else (i, f)
        lib().vp9h_ivf_write_frame_header(fh, len(data), pts)
        out += [fh.raw, bytes(data)]
    return b"".join(out)


NOPTS = -(1 << 63)


def webm_probe(data):
    data = bytes(data)
    return lib().vp9h_webm_probe(data, len(data))


def webm_read(data):
    """WebM / Matroska bytes -> (WebmInfo, [(pts, frame bytes, keyframe)]) of the first VP9
    video track (vp9h_webm_read_header / _read_frame; pts in TimecodeScale units, NOPTS
    for later laces of a block without a duration)."""
    data = bytes(data)
    info, cur = WebmInfo(), WebmCursor()
    _check("vp9h_webm_read_header", lib().vp9h_webm_read_header(data, len(data), ctypes.byref(info), ctypes.byref(cur)))
    frames = []
    ptr, n, pts, key = ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_int64(), ctypes.c_int()
    base = ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p).value
    while True:
        r = lib().vp9h_webm_read_frame(data, len(data), ctypes.byref(cur), ctypes.byref(ptr), ctypes.byref(n),
                                       ctypes.byref(pts), ctypes.byref(key))
        if r == EOF:
            break
        _check("vp9h_webm_read_frame", r)
        off = ptr.value - base
        frames.append((pts.value, data[off:off + n.value], key.value))
    return info, frames


# ---- a small WebM muxer (matroskaenc.c's element layout) for tests and tools: not the product
def _ebml_id(i):
    return i.to_bytes((i.bit_length() + 7) // 8, "big")


def _ebml_size(n, width=None, unknown=False):
    if unknown:
        w = width or 8
        return bytes([0xFF >> (w - 1) | (0x80 >> (w - 1))] + [0xFF] * (w - 1)) if w > 1 else b"\xff"
    w = width or next(k for k in range(1, 9) if n < (1 << (7 * k)) - 1)
    return (n | (1 << (7 * w))).to_bytes(w, "big")


def _el(i, payload, unknown=False, width=None):
    return _ebml_id(i) + _ebml_size(len(payload), width, unknown) + payload


def _uint(i, v):
    return _el(i, v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big"))


def webm_write(frames, width, height, timecode_scale=1000000, cluster_frames=8, lacing=None,
               unknown_sizes=False, block_groups=False, other_track=False, voids=False):
    """[(pts, bytes)] or [bytes] -> WebM bytes with one V_VP9 track (number 1). Options for
    tests: lacing = "xiph" / "fixed" / "ebml" (frames laced in pairs), unknown-size Segment
    and Clusters, BlockGroup + Block instead of SimpleBlock, an interleaved second track's
    blocks, Void elements."""
    fr = [f if isinstance(f, tuple) else (i, f) for i, f in enumerate(frames)]
    hdr = _el(0x1A45DFA3, _uint(0x4286, 1) + _uint(0x42F7, 1) + _uint(0x42F2, 4) + _uint(0x42F3, 8) +
              _el(0x4282, b"webm") + _uint(0x4287, 4) + _uint(0x4285, 2))
    info = _el(0x1549A966, _uint(0x2AD7B1, timecode_scale) + _el(0x4D80, b"vp9hip"))
    video = _el(0xE0, _uint(0xB0, width) + _uint(0xBA, height))
    tracks = [_el(0xAE, _uint(0xD7, 1) + _uint(0x73C5, 1) + _uint(0x83, 1) + _el(0x86, b"V_VP9") + video)]
    if other_track:
        tracks.append(_el(0xAE, _uint(0xD7, 2) + _uint(0x73C5, 2) + _uint(0x83, 2) + _el(0x86, b"A_OPUS")))
    body = [info, _el(0x1654AE6B, b"".join(tracks))]
    if voids:
        body.insert(1, _el(0xEC, b"\0" * 5))

    def block(track, rel, flags, payloads, kind):
        head = bytes([0x80 | track]) + (rel & 0xFFFF).to_bytes(2, "big")
        if kind is None:
            return head + bytes([flags]) + payloads[0]
        n = len(payloads)
        if kind == "xiph":
            lace = bytes([n - 1]) + b"".join(b"\xff" * (len(p) // 255) + bytes([len(p) % 255]) for p in payloads[:-1])
            return head + bytes([flags | 0x02]) + lace + b"".join(payloads)
        if kind == "fixed":
            return head + bytes([flags | 0x04]) + bytes([n - 1]) + b"".join(payloads)
        sizes = _ebml_size(len(payloads[0]))                        # EBML lacing: size, then signed deltas
        for a, b in zip(payloads, payloads[1:-1]):
            d = len(b) - len(a)
            w = next(k for k in range(1, 9) if abs(d) < (1 << (7 * k - 1)) - 1)
            sizes += (d + (1 << (7 * w - 1)) - 1 | (1 << (7 * w))).to_bytes(w, "big")
        return head + bytes([flags | 0x06]) + bytes([n - 1]) + sizes + b"".join(payloads)

    for c0 in range(0, len(fr), cluster_frames):
        grp = fr[c0:c0 + cluster_frames]
        tc = grp[0][0]
        parts = [_uint(0xE7, tc)]
        k = 0
        while k < len(grp):
            n = 2 if lacing and k + 1 < len(grp) and (lacing != "fixed" or len(grp[k][1]) == len(grp[k + 1][1])) else 1
            pays = [d for _, d in grp[k:k + n]]
            rel = grp[k][0] - tc
            if block_groups:
                parts.append(_el(0xA0, _el(0xA1, block(1, rel, 0, pays, lacing if n > 1 else None)) +
                                 (_uint(0x9B, n * (grp[1][0] - grp[0][0] if len(grp) > 1 else 1)) if n > 1 else b"")))
            else:
                parts.append(_el(0xA3, block(1, rel, 0x80 if k == 0 and c0 == 0 else 0, pays, lacing if n > 1 else None)))
            if other_track:
                parts.append(_el(0xA3, block(2, rel, 0x80, [b"\x01\x02\x03"], None)))
            if voids and k == 0:
                parts.append(_el(0xEC, b"\0\0"))
            k += n
        payload = b"".join(parts)
        body.append(_el(0x1F43B675, payload, unknown=unknown_sizes))
    body.append(_el(0x1C53BB6B, _el(0xBB, _uint(0xB3, 0))))        # a Cues element after the clusters
    return hdr + _el(0x18538067, b"".join(body), unknown=unknown_sizes)


PLAN_STAT_NAMES = ("sbs", "passes", "pjobs", "rjobs", "jobs_4x4", "jobs_8x8", "jobs_16x16",
                   "jobs_32x32", "lane_use", "max_passes_sb", "lf_records", "mc_units", "pred_steps",
                   "lf_steps", "levels", "pass_rows", "level_steps", "asap_passes", "firstfit_passes", "firstfit_height_passes",
                   "mc_out_bytes", "mc_alg_bytes", "mc_line_bytes")


def plan_sb_costs(frame):
    """Per SB of one packet (raster order) the pixel rows its intra passes loop over, as staged
    for the device (vp9hip_plan_sb_costs; host only, tools/wave_tail.py)."""
    n = ((frame.pkt.width + 63) >> 6) * ((frame.pkt.height + 63) >> 6)
    out = (ctypes.c_double * n)()
    got = _check("vp9hip_plan_sb_costs", lib().vp9hip_plan_sb_costs(ctypes.byref(frame.pkt), out, n))
    return np.array(out[:got])


def plan_stats(frame):
    """Host-only work-planning statistics of one pass-1 packet (vp9hip_plan_stats)."""
    out = (ctypes.c_double * len(PLAN_STAT_NAMES))()
    _check("vp9hip_plan_stats", lib().vp9hip_plan_stats(ctypes.byref(frame.pkt), out, len(PLAN_STAT_NAMES)))
    return dict(zip(PLAN_STAT_NAMES, list(out)))
