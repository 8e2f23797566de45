"""Pipelined device encodes (dmmt_ctx_set_lanes): consecutive dmmt_encode_device
calls with stream NULL run on different workspaces and streams at once; every
output must still be byte-identical to the oracle's encode of its frame."""
import numpy as np
import pytest

import dmmt_jpeg
import oracle
from conftest import synthetic

pytestmark = pytest.mark.gpu


def _opts(sub, q):
    luma, chroma = dmmt_jpeg.quality_tables(q)
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma)


@pytest.mark.parametrize("lanes", [2, 3, 8])
def test_pipelined_frames_equal_oracle(encoder, lanes):
    w, h, sub = 328, 200, 2
    opts = _opts(sub, 80)
    frames = [synthetic(w, h, frame=40 + i) for i in range(2 * lanes + 1)]
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_in = [encoder.malloc(f.nbytes) for f in frames]
    d_out = [encoder.malloc(stride) for _ in frames]
    d_len = [encoder.malloc(4) for _ in frames]
    try:
        for d, f in zip(d_in, frames):
            encoder.h2d(d, f)
        encoder.set_lanes(lanes)
        for i in range(len(frames)):  # all enqueued before any completes
            encoder.encode_device(d_in[i], 1, w, h, opts, d_out[i], stride, d_len[i])
        encoder.synchronize()
        for i, f in enumerate(frames):
            n = int(np.frombuffer(encoder.d2h(d_len[i], 4), np.uint32)[0])
            assert encoder.d2h(d_out[i], n) == oracle.encode(f, 255, sub, opts.luma_table, opts.chroma_table), i
        # host calls between pipelined ones (lane 0, the context stream)
        assert encoder.encode(dmmt_jpeg.Image.from_array(frames[0]), opts) == \
            oracle.encode(frames[0], 255, sub, opts.luma_table, opts.chroma_table)
    finally:
        encoder.set_lanes(1)
        for d in d_in + d_out + d_len:
            encoder.free(d)


def test_pipelined_table_change_between_calls(encoder):
    """new quantisation tables wait for the lanes still reading the old ones"""
    w, h, sub = 96, 64, 0
    frames = [synthetic(w, h, frame=70 + i) for i in range(6)]
    qs = [50, 90, 50, 75, 95, 50]
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_in = [encoder.malloc(f.nbytes) for f in frames]
    d_out = [encoder.malloc(stride) for _ in frames]
    d_len = [encoder.malloc(4) for _ in frames]
    try:
        for d, f in zip(d_in, frames):
            encoder.h2d(d, f)
        encoder.set_lanes(3)
        for i in range(len(frames)):
            encoder.encode_device(d_in[i], 1, w, h, _opts(sub, qs[i]), d_out[i], stride, d_len[i])
        encoder.synchronize()
        for i, f in enumerate(frames):
            o = _opts(sub, qs[i])
            n = int(np.frombuffer(encoder.d2h(d_len[i], 4), np.uint32)[0])
            assert encoder.d2h(d_out[i], n) == oracle.encode(f, 255, sub, o.luma_table, o.chroma_table), i
    finally:
        encoder.set_lanes(1)
        for d in d_in + d_out + d_len:
            encoder.free(d)


def test_set_lanes_bounds(encoder):
    for bad in (0, -1, 9):
        with pytest.raises(dmmt_jpeg.Error):
            encoder.set_lanes(bad)
    encoder.set_lanes(8)
    encoder.set_lanes(1)
