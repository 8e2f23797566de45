"""One image over several GPUs as MCU-row stripes (BASELINE config 4's structure):
dmmt_stripe_analyze -> histogram sum (the one exchange) -> dmmt_stripe_encode.
The stripes concatenated must equal, byte for byte, the single encode of the whole
image with the same restart interval (and so the oracle's)."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import dmmt_jpeg
import oracle
from conftest import synthetic

pytestmark = pytest.mark.gpu

MCU_H = {0: 8, 1: 8, 2: 16}
MCU_W = {0: 8, 1: 16, 2: 16}


def _opts(sub, q, ri):
    luma, chroma = dmmt_jpeg.quality_tables(q)
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma, restart_interval=ri)


def _striped_on_one_gpu(rgb, sub, q, rows_per_interval, n_stripes):
    h, w, _ = rgb.shape
    mcux, mcuy = -(-w // MCU_W[sub]), -(-h // MCU_H[sub])
    opts = _opts(sub, q, mcux * rows_per_interval)
    encs = [dmmt_jpeg.Encoder(0) for _ in range(n_stripes)]
    parts, stripes, bufs = [], [], []
    try:
        hist = np.zeros(dmmt_jpeg.STRIPE_HIST_WORDS, np.uint64)
        for r, enc in enumerate(encs):
            row0, rows = dmmt_jpeg.stripe_rows(mcuy, n_stripes, r, rows_per_interval)
            y0, y1 = row0 * MCU_H[sub], min((row0 + rows) * MCU_H[sub], h)
            px = np.ascontiguousarray(rgb[y0:y1])
            d_in = enc.malloc(px.nbytes)
            enc.h2d(d_in, px)
            st = enc.stripe(d_in, w, h, row0, rows)
            cap = enc.stripe_max_bytes(st, opts)
            d_out = enc.malloc(cap)
            bufs.append((enc, d_in, d_out, cap))
            stripes.append(st)
            hist += enc.stripe_analyze(st, opts)  # in a real run: all-reduce over ranks
        for (enc, d_in, d_out, cap) in bufs:
            n = enc.stripe_encode(hist, d_out, cap)
            parts.append(enc.d2h(d_out, n))
    finally:
        for (enc, d_in, d_out, cap) in bufs:
            enc.free(d_in)
            enc.free(d_out)
        for enc in encs:
            enc.close()
    return b"".join(parts), opts


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("shape,n_stripes,rpi", [((120, 200), 3, 1), ((37, 53), 2, 1), ((256, 96), 4, 2),
                                                  ((64, 64), 1, 1)])
def test_stripes_equal_single_encode(encoder, sub, shape, n_stripes, rpi):
    h, w = shape
    rgb = synthetic(w, h, frame=h)
    data, opts = _striped_on_one_gpu(rgb, sub, 75, rpi, n_stripes)
    whole = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts)
    assert data == whole
    assert data == oracle.encode(rgb, 255, sub, opts.luma_table, opts.chroma_table,
                                 restart_interval=opts.restart_interval)


def test_stripes_4k_8way(encoder):
    rgb = synthetic(3840, 2160, frame=11)
    data, opts = _striped_on_one_gpu(rgb, 0, 90, 1, 8)
    assert data == oracle.encode(rgb, 255, 0, opts.luma_table, opts.chroma_table, threads=8,
                                 restart_interval=opts.restart_interval)


def test_stripe_must_align_to_restart_intervals(encoder):
    opts = _opts(0, 75, 3)  # 3 MCUs per interval on an 8-MCU-wide image: row 1 starts mid-interval
    d = encoder.malloc(64 * 8 * 3)
    try:
        st = encoder.stripe(d, 64, 16, 1, 1)
        with pytest.raises(dmmt_jpeg.Error) as e:
            encoder.stripe_analyze(st, opts)
        assert e.value.code == -102
        with pytest.raises(dmmt_jpeg.Error):  # no restart interval: stripes are not independent
            encoder.stripe_analyze(encoder.stripe(d, 64, 16, 0, 1), _opts(0, 75, 0))
    finally:
        encoder.free(d)


def _rank(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "dmmt-jpeg-encoder_amd"))
    import torch  # noqa: F401
    import torch.distributed as dist
    import dmmt_jpeg as dj
    dist.init_process_group("gloo")
    w, h, sub = 320, 176, 2
    enc = dj.Encoder(0)
    mcux, mcuy = w // 16, h // 16
    row0, rows = dj.stripe_rows(mcuy, world, rank)
    y0, y1 = row0 * 16, min((row0 + rows) * 16, h)
    d_in = enc.malloc(w * (y1 - y0) * 3)
    enc.fill_synthetic_rows(d_in, w, h, y0, y1 - y0, frame=5)
    opts = _opts(sub, 75, mcux)
    st = enc.stripe(d_in, w, h, row0, rows)
    cap = enc.stripe_max_bytes(st, opts)
    d_out = enc.malloc(cap)
    n, off, total = dj.encode_striped(enc, st, opts, d_out, cap)
    with open(os.path.join(out_dir, f"part{rank}.bin"), "wb") as f:
        f.write(enc.d2h(d_out, n))
    with open(os.path.join(out_dir, f"meta{rank}.json"), "w") as f:
        json.dump({"n": n, "off": off, "total": total}, f)
    enc.free(d_in)
    enc.free(d_out)
    enc.close()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_stripes_two_processes_gloo(tmp_path):
    """The multi-rank protocol for real: two processes (one context each, both on
    GPU 0 here), the histogram all-reduce and size all-gather over gloo."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_rank, args=(2, port, str(tmp_path)), nprocs=2, start_method="spawn")
    metas = [json.load(open(tmp_path / f"meta{r}.json")) for r in range(2)]
    data = b"".join(open(tmp_path / f"part{r}.bin", "rb").read() for r in range(2))
    assert metas[1]["off"] == metas[0]["n"] and metas[0]["total"] == len(data)
    rgb = synthetic(320, 176, frame=5)
    opts = _opts(2, 75, 320 // 16)
    assert data == oracle.encode(rgb, 255, 2, opts.luma_table, opts.chroma_table,
                                 restart_interval=opts.restart_interval)
