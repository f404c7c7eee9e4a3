"""ORACLE loader — test infrastructure only.

ctypes binding of oracle/liboracle.so, the scalar C restatement of the reference
VP9 pixel path (see vp9_oracle.h for the reference file:line map). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_L = None


class Planes(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * 3), ("stride", ctypes.c_ssize_t * 3),
                ("w", ctypes.c_int), ("h", ctypes.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        _L = ctypes.CDLL(LIB)
        _L.vp9o_decode_frame.argtypes = [ctypes.c_void_p, ctypes.POINTER(Planes), ctypes.POINTER(Planes)]
        _L.vp9o_decode_frame_tiles.argtypes = [ctypes.c_void_p, ctypes.POINTER(Planes), ctypes.POINTER(Planes),
                                               ctypes.c_int]
        _L.vp9o_itxfm_add.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _L.vp9o_itxfm_add.restype = None
        _L.vp9o_intra_pred.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        _L.vp9o_intra_pred.restype = None
        _L.vp9o_loop_filter.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t] + [ctypes.c_int] * 7
        _L.vp9o_loop_filter.restype = None
        _L.vp9o_mc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p,
                               ctypes.c_ssize_t] + [ctypes.c_int] * 6
        _L.vp9o_mc.restype = None
        _L.vp9o_mc_scaled.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p,
                                      ctypes.c_ssize_t] + [ctypes.c_int] * 8
        _L.vp9o_mc_scaled.restype = None
        _L.vp9o_scan.argtypes = [ctypes.c_int, ctypes.c_int]
        _L.vp9o_scan.restype = ctypes.POINTER(ctypes.c_int16)
    return _L


def _planes(arrs, w, h):
    p = Planes()
    for i in range(3):
        p.data[i] = arrs[i].ctypes.data
        p.stride[i] = arrs[i].strides[0] // arrs[i].itemsize
    p.w, p.h = w, h
    return p


def decode_frame(pkt, out_planes, ref_planes=None, ref_sizes=None, tile_threads=0):
    """Reconstruct + loop-filter one pass-1 packet into out_planes (padded numpy planes).

    ref_planes: list of 3 plane-lists (LAST, GOLDEN, ALTREF) for inter frames.
    tile_threads > 0: the slice-threaded form (tile columns of an SB row on that many
    threads, vp9o_decode_frame_tiles); same output."""
    cur = _planes(out_planes, pkt.width, pkt.height)
    refs = None
    if ref_planes is not None:
        refs = (Planes * 3)()
        for i in range(3):
            rw, rh = (ref_sizes[i] if ref_sizes else (pkt.width, pkt.height))
            refs[i] = _planes(ref_planes[i], rw, rh)
    if tile_threads > 0:
        r = lib().vp9o_decode_frame_tiles(ctypes.addressof(pkt), ctypes.byref(cur), refs, int(tile_threads))
    else:
        r = lib().vp9o_decode_frame(ctypes.addressof(pkt), ctypes.byref(cur), refs)
    if r < 0:
        raise RuntimeError("vp9o_decode_frame failed: %d" % r)
    return out_planes


def scan(tx, txtp):
    n = 16 << (2 * (tx & 3))
    p = lib().vp9o_scan(tx, txtp)
    return np.array([p[i] for i in range(n)], dtype=np.int64)


def itxfm_add(bpp, dst, coef, eob, tx, txtp):
    """In-place itxfm_add on a 2-D numpy pixel block (coef is zeroed like the reference)."""
    lib().vp9o_itxfm_add(bpp, dst.ctypes.data, dst.strides[0] // dst.itemsize, coef.ctypes.data, eob, tx, txtp)


def intra_pred(bpp, dst, left, top_with_tl, tx, mode):
    """top_with_tl[0] is the top-left pixel; top row follows."""
    lib().vp9o_intra_pred(bpp, dst.ctypes.data, dst.strides[0] // dst.itemsize, left.ctypes.data,
                          top_with_tl.ctypes.data + top_with_tl.itemsize, tx, mode)


def loop_filter(bpp, buf, off, stride, kind, wd1, wd2, direction, E, I, H):
    lib().vp9o_loop_filter(bpp, buf.ctypes.data + off * buf.itemsize, stride, kind, wd1, wd2, direction, E, I, H)


def mc_scaled(bpp, dst, src, off, sstride, w, h, mx, my, dx, dy, filt, avg):
    lib().vp9o_mc_scaled(bpp, dst.ctypes.data, dst.strides[0] // dst.itemsize, src.ctypes.data + off * src.itemsize,
                         sstride, w, h, mx, my, dx, dy, filt, avg)


def mc(bpp, dst, src, off, sstride, w, h, mx, my, filt, avg):
    lib().vp9o_mc(bpp, dst.ctypes.data, dst.strides[0] // dst.itemsize, src.ctypes.data + off * src.itemsize,
                  sstride, w, h, mx, my, filt, avg)
