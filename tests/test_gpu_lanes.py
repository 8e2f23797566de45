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


@pytest.mark.parametrize("lanes", [1, 2])
def test_async_error_surfaces_at_synchronize(encoder, lanes):
    """an asynchronous encode's error is reported by synchronize, never by (or lost
    to) a host call made in between, whichever lane the bad frame ran on"""
    w, h, sub = 64, 48, 0
    opts = _opts(sub, 75)
    good = synthetic(w, h, frame=3)
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_in = [encoder.malloc(good.nbytes) for _ in range(2)]
    d_out = [encoder.malloc(stride) for _ in range(2)]
    d_len = [encoder.malloc(4) for _ in range(2)]
    try:
        for d in d_in:
            encoder.h2d(d, good)
        encoder.set_lanes(lanes)
        encoder.encode_device(d_in[0], 1, w, h, opts, d_out[0], stride, d_len[0])
        # maxval 100 with samples up to 255: the RangeColorFormat panic (color.rs:63-65),
        # on lane 1 with two lanes, on lane 0 with one
        encoder.encode_device(d_in[1], 1, w, h, opts, d_out[1], stride, d_len[1], maxval=100)
        assert encoder.encode(dmmt_jpeg.Image.from_array(good), opts) == \
            oracle.encode(good, 255, sub, opts.luma_table, opts.chroma_table)
        with pytest.raises(dmmt_jpeg.Error) as ei:
            encoder.synchronize()
        assert ei.value.name == "ValueExceedsMax"
        encoder.synchronize()  # reported once, then clear
        n = int(np.frombuffer(encoder.d2h(d_len[0], 4), np.uint32)[0])
        assert encoder.d2h(d_out[0], n) == oracle.encode(good, 255, sub, opts.luma_table, opts.chroma_table)
    finally:
        encoder.set_lanes(1)
        for d in d_in + d_out + d_len:
            encoder.free(d)


def test_async_error_kept_when_lanes_dropped(encoder):
    w, h, sub = 40, 24, 1
    opts = _opts(sub, 60)
    bad = synthetic(w, h, frame=5)
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_in, d_out, d_len = encoder.malloc(bad.nbytes), encoder.malloc(stride), encoder.malloc(4)
    try:
        encoder.h2d(d_in, bad)
        encoder.set_lanes(3)
        encoder.encode_device(d_in, 1, w, h, opts, d_out, stride, d_len)  # lane 0
        encoder.encode_device(d_in, 1, w, h, opts, d_out, stride, d_len)  # lane 1
        encoder.encode_device(d_in, 1, w, h, opts, d_out, stride, d_len, maxval=7)  # lane 2: error
        encoder.set_lanes(1)  # lane 2 is freed; its error is not
        with pytest.raises(dmmt_jpeg.Error) as ei:
            encoder.synchronize()
        assert ei.value.name == "ValueExceedsMax"
    finally:
        encoder.set_lanes(1)
        for d in (d_in, d_out, d_len):
            encoder.free(d)


def test_caller_stream_mixed_with_lanes(encoder):
    """calls on a caller's stream use lane 0's workspace; interleaved with the
    round-robin calls (lane 0 among them) every output stays exact"""
    import torch
    w, h, sub = 200, 136, 2
    opts = _opts(sub, 85)
    frames = [synthetic(w, h, frame=90 + i) for i in range(8)]
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_in = [encoder.malloc(f.nbytes) for f in frames]
    d_out = [encoder.malloc(stride) for _ in frames]
    d_len = [encoder.malloc(4) for _ in frames]
    s = torch.cuda.Stream(device=0)
    try:
        for d, f in zip(d_in, frames):
            encoder.h2d(d, f)
        encoder.set_lanes(2)
        for i in range(len(frames)):
            stream = s.cuda_stream if i % 2 else None
            encoder.encode_device(d_in[i], 1, w, h, opts, d_out[i], stride, d_len[i], stream=stream)
        encoder.synchronize()
        s.synchronize()
        for i, f in enumerate(frames):
            n = int(np.frombuffer(encoder.d2h(d_len[i], 4), np.uint32)[0])
            assert encoder.d2h(d_out[i], n) == oracle.encode(f, 255, sub, opts.luma_table, opts.chroma_table), i
    finally:
        encoder.set_lanes(1)
        for d in d_in + d_out + d_len:
            encoder.free(d)
