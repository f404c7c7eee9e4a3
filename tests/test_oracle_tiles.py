"""CPU: the slice-threaded oracle (vp9o_decode_frame_tiles: the tile columns of each SB row
on worker threads, the previous row's loop filter overlapped, after decode_tiles_mt +
loopfilter_proc, vp9.c:1442-1551) gives the same frames as the serial oracle. It is the
bench's tile-column CPU leg, so its output must not depend on threads."""
import numpy as np
import pytest

from test_stream import _frames


@pytest.mark.parametrize("w,h,bpp,log2,threads", [(1032, 200, 8, 2, 4), (1032, 200, 8, 2, 2), (2048, 136, 10, 3, 8),
                                                   (300, 140, 8, 0, 3), (2048, 136, 8, 3, 3)])
def test_tile_threads_match_serial(v9, orc, w, h, bpp, log2, threads):
    fr = _frames(v9, w, h, 4, bpp=bpp, log2_tile_cols=log2, seed=1200 + w)
    prev_a = prev_b = None
    for i, f in enumerate(fr):
        a, b = v9.alloc_planes(w, h, bpp), v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, a, None if i == 0 else [prev_a] * 3)
        orc.decode_frame(f.pkt, b, None if i == 0 else [prev_b] * 3, tile_threads=threads)
        for p in range(3):
            assert np.array_equal(a[p], b[p]), "frame %d plane %d" % (i, p)
        prev_a, prev_b = a, b
