"""BASELINE.json configs 3, 4 and 5 at their stated sizes, byte for byte.

* config 3: a batch of 256 distinct 1920x1080 frames, 4:2:0, q75, encoded by one
  device launch (as bench.py does) and by the host batch API; every frame is
  compared with the oracle.
* config 4: one 32768x32768 image, 4:2:0, q75 (25.17 M blocks, 2048 MCU rows --
  twice the u16 MCU count of 16384 per side): the whole-image encode and eight
  MCU-row stripes on eight contexts (the multi-GPU protocol, here on one GPU), in
  both stripe modes -- restart intervals of one MCU row (config 4 as written) and
  joined stripes (no restart intervals, the reference's own single scan,
  encoder.rs:125-135, 264-282).  Stripes, whole image and oracle must agree.
* config 5: the 8K q75 point of the quality sweep (q50 and q95 are in
  test_gpu_parity.py).

The frames come from the library's device generator and are copied
to the host for the oracle, which runs in threads while the GPU encodes (ctypes
releases the GIL); its front half is split over threads for the 32768^2 image
(oracle.forward(threads=...), the same blocks as the serial restatement)."""
import concurrent.futures as cf
import os

import numpy as np
import pytest

import dmmt_jpeg
import oracle

pytestmark = pytest.mark.gpu

CPU_THREADS = min(16, len(os.sched_getaffinity(0)))


def _opts(sub, q, ri=0):
    luma, chroma = dmmt_jpeg.quality_tables(q)
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma, restart_interval=ri)


def _device_frames(enc, w, h, n, first=0):
    """n synthetic frames in HBM (pointer) and on the host (uint8 array)"""
    d = enc.malloc(w * h * 3 * n)
    enc.fill_synthetic(d, w, h, n, first_frame=first)
    host = np.frombuffer(enc.d2h(d, w * h * 3 * n), np.uint8).reshape(n, h, w, 3)
    return d, host


def _encode_device(enc, d_rgb, n, w, h, opts):
    stride = (dmmt_jpeg.max_jpeg_bytes(w, h, int(opts.chroma_subsampling_preset)) + 255) // 256 * 256
    d_out = enc.malloc(stride * n)
    d_len = enc.malloc(4 * n)
    try:
        enc.encode_device(d_rgb, n, w, h, opts, d_out, stride, d_len)
        enc.synchronize()
        lens = np.frombuffer(enc.d2h(d_len, 4 * n), np.uint32)
        return [enc.d2h(d_out + i * stride, int(lens[i])) for i in range(n)]
    finally:
        enc.free(d_out)
        enc.free(d_len)


@pytest.mark.timeout(600)
def test_config3_1080p_batch_of_256(encoder):
    w, h, n, sub, q = 1920, 1080, 256, 2, 75
    opts = _opts(sub, q)
    d, frames = _device_frames(encoder, w, h, n, first=1000)
    try:
        with cf.ThreadPoolExecutor(CPU_THREADS) as pool:
            refs = pool.map(lambda f: oracle.encode(f, 255, sub, opts.luma_table, opts.chroma_table), frames)
            gpu = _encode_device(encoder, d, n, w, h, opts)  # one launch of 256 frames (bench.py's step)
            refs = list(refs)
    finally:
        encoder.free(d)
    assert len(set(refs)) == n  # 256 distinct frames
    for i in range(n):
        assert gpu[i] == refs[i], f"frame {i}"
    # the host batch API (one upload, one batched launch, one download)
    host = encoder.encode_batch([dmmt_jpeg.Image.from_array(f) for f in frames], opts)
    assert host == refs


@pytest.mark.timeout(600)
def test_config5_8k_q75(encoder):
    w, h, sub = 7680, 4320, 2
    opts = _opts(sub, 75)
    d, frames = _device_frames(encoder, w, h, 2, first=77)
    try:
        gpu = _encode_device(encoder, d, 2, w, h, opts)
    finally:
        encoder.free(d)
    with cf.ThreadPoolExecutor(2) as pool:
        refs = list(pool.map(lambda f: oracle.encode(f, 255, sub, opts.luma_table, opts.chroma_table,
                                                     threads=CPU_THREADS // 2, parallel=True), frames))
    assert gpu == refs


def _stripes_on_contexts(d_img, w, h, sub, opts, n_stripes):
    """the stripe protocol of SURVEY 8(e) with one context per stripe (as one per GPU),
    the stripes' pixels read in place from the whole image in HBM"""
    mcu_h = 16 if sub == 2 else 8
    mcu_w = 8 if sub == 0 else 16
    mcux, mcuy = -(-w // mcu_w), -(-h // mcu_h)
    ri = opts.restart_interval
    rpi = max(1, ri // mcux) if ri else 1
    encs = [dmmt_jpeg.Encoder(0) for _ in range(n_stripes)]
    bufs = []
    try:
        sts, hists = [], []
        for r, enc in enumerate(encs):
            row0, rows = dmmt_jpeg.stripe_rows(mcuy, n_stripes, r, rpi)
            st = enc.stripe(d_img + row0 * mcu_h * w * 3, w, h, row0, rows)
            cap = enc.stripe_max_bytes(st, opts)
            d_out = enc.malloc(cap)
            bufs.append((enc, d_out, cap))
            sts.append(st)
            hists.append(enc.stripe_analyze(st, opts))
        parts = []
        if ri:
            total = np.sum(hists, axis=0, dtype=np.uint64)
            for enc, d_out, cap in bufs:
                parts.append(enc.d2h(d_out, enc.stripe_encode(total, d_out, cap)))
        else:
            edges = [enc.stripe_dc_edges() for enc in encs]
            prevs = [[0, 0, 0]] + [edges[r - 1][1] for r in range(1, n_stripes)]
            total = np.zeros(dmmt_jpeg.STRIPE_HIST_WORDS, np.uint64)
            for r in range(n_stripes):
                total += dmmt_jpeg.Encoder.stripe_fix_dc_hist(hists[r], edges[r][0], prevs[r]) if r else hists[r]
            heads = [enc.stripe_measure(total, prevs[r], d_out, cap) for r, (enc, d_out, cap) in enumerate(bufs)]
            bits, f16 = [b for b, _ in heads], [f for _, f in heads]
            for r, (enc, d_out, cap) in enumerate(bufs):
                parts.append(enc.d2h(d_out, enc.stripe_write(*dmmt_jpeg.stripe_seam(bits, f16, r))))
        return b"".join(parts)
    finally:
        for enc, d_out, cap in bufs:
            enc.free(d_out)
        for enc in encs:
            enc.close()


@pytest.mark.timeout(900)
def test_config4_32768_square_both_stripe_modes(encoder):
    w = h = 32768
    sub, q = 2, 75
    mcux = w // 16
    o_r, o_j = _opts(sub, q, mcux), _opts(sub, q, 0)
    d, host = _device_frames(encoder, w, h, 1, first=0)
    rgb = host[0]
    try:
        with cf.ThreadPoolExecutor(2) as pool:
            def ref_both():
                coef = oracle.forward(rgb, 255, sub, o_j.luma_table, o_j.chroma_table, threads=CPU_THREADS)
                with cf.ThreadPoolExecutor(2) as p2:
                    fj = p2.submit(oracle.encode_coefficients, coef, w, h, sub, o_j.luma_table, o_j.chroma_table)
                    fr = p2.submit(oracle.encode_coefficients, coef, w, h, sub, o_r.luma_table, o_r.chroma_table,
                                   restart_interval=mcux)
                    return fr.result(), fj.result()
            ref = pool.submit(ref_both)
            whole_r = _encode_device(encoder, d, 1, w, h, o_r)[0]
            whole_j = _encode_device(encoder, d, 1, w, h, o_j)[0]
            striped_r = _stripes_on_contexts(d, w, h, sub, o_r, 8)
            striped_j = _stripes_on_contexts(d, w, h, sub, o_j, 8)
            ref_r, ref_j = ref.result()
    finally:
        encoder.free(d)
    assert striped_r == whole_r
    assert striped_j == whole_j
    assert whole_r == ref_r, "restart mode differs from the oracle"
    assert whole_j == ref_j, "joined (reference) stream differs from the oracle"
    assert ref_j[-2:] == b"\xff\xd9" and len(ref_j) > 1 << 20
