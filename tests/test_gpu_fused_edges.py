"""The edges of the two "last arriver does the rest" fusions, byte for byte against
the oracle.

* k_emit's fused chunk offsets: rounds of kFusedRoundChunks = 1536
  chunks, at most kFusedOffsetsMaxChunks = 6144 chunks per frame (k_offsets
  above).  Frames of exactly 1536 and 1537 chunks (one round, a carry into a
  second), 6144 (four rounds, the largest fused frame) and just above 6144 (the
  k_offsets launch), alone, in multi-frame launches (per-frame arrival counters,
  32-bit carries per frame) and with restart intervals (segmented scans).
  [binary_stream.rs:38-96, segment_marker_injector.rs:13-30: the bytes those
  offsets place]
* k_hist's fused Huffman tables (tables_tail): frames up to tables_fusable's
  bound take them; 1 to 3 frames per launch; the DMMT_FUSE_TABLES=0 build path
  (k_tables) must give the same files.  [length_limited.rs:37-134,
  symbol_counting.rs:55-94, huffman/encoder.rs:45-157, encoder.rs:125-262]"""
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


def _chunks(w, h, sub):
    hr, vr = (1, 1) if sub == 0 else ((2, 1) if sub == 1 else (2, 2))
    mcus = -(-w // (8 * hr)) * -(-h // (8 * vr))
    return -(-mcus * (hr * vr + 2) // 256)


def _encode_device(enc, w, h, n, opts, first=0):
    d = enc.malloc(w * h * 3 * n)
    stride = (dmmt_jpeg.max_jpeg_bytes(w, h, int(opts.chroma_subsampling_preset)) + 255) // 256 * 256
    d_out, d_len = enc.malloc(stride * n), enc.malloc(4 * n)
    try:
        enc.fill_synthetic(d, w, h, n, first_frame=first)
        host = np.frombuffer(enc.d2h(d, w * h * 3 * n), np.uint8).reshape(n, h, w, 3)
        enc.encode_device(d, n, w, h, opts, d_out, stride, d_len)
        enc.synchronize()
        lens = np.frombuffer(enc.d2h(d_len, 4 * n), np.uint32)
        return host, [enc.d2h(d_out + i * stride, int(lens[i])) for i in range(n)]
    finally:
        for p in (d, d_out, d_len):
            enc.free(p)


def _oracle_all(frames, sub, opts):
    luma, chroma = list(opts.luma_table), list(opts.chroma_table)
    ri = opts.restart_interval
    with cf.ThreadPoolExecutor(min(len(frames), 4)) as ex:
        return list(ex.map(lambda f: oracle.encode(f, 255, sub, luma, chroma, restart_interval=ri,
                                                   threads=max(1, CPU_THREADS // len(frames)), parallel=True), frames))


@pytest.mark.parametrize("w,h,sub,nch", [
    (4096, 2048, 0, 1536),   # one round, exactly full
    (2400, 3496, 0, 1537),   # the carry into a second round
    (8192, 8192, 2, 6144),   # four rounds: the largest fused frame
    (8192, 8208, 2, 6156),   # above: k_offsets
])
def test_fused_offsets_round_edges(encoder, w, h, sub, nch):
    assert _chunks(w, h, sub) == nch
    opts = _opts(sub, 90)
    host, gpu = _encode_device(encoder, w, h, 1, opts, first=nch)
    assert gpu == _oracle_all(list(host), sub, opts)


@pytest.mark.parametrize("nf", [2, 3])
def test_fused_offsets_multi_frame_launch(encoder, nf):
    """nf frames of 1537 chunks in one launch: every frame's own counters and carries"""
    opts = _opts(0, 75)
    host, gpu = _encode_device(encoder, 2400, 3496, nf, opts, first=7)
    assert gpu == _oracle_all(list(host), 0, opts)


@pytest.mark.parametrize("ri", [1, 37, 300])
def test_fused_offsets_restart_segments(encoder, ri):
    """restart intervals: the chunk grid restarts per segment and the scans are
    segmented; 1537-chunk-class frame, two per launch"""
    opts = _opts(0, 90, ri)
    host, gpu = _encode_device(encoder, 2400, 3496, 2, opts, first=11)
    assert gpu == _oracle_all(list(host), 0, opts)


@pytest.mark.parametrize("w,h,sub", [(64, 48, 0), (1920, 1080, 2), (3840, 2160, 0), (333, 97, 1)])
def test_fused_tables_match_k_tables(w, h, sub):
    """the tables built in k_hist's last workgroup and by the k_tables launch
    (DMMT_FUSE_TABLES=0 context): the same files, and the oracle's"""
    opts = _opts(sub, 90)
    outs = {}
    for fuse in ("1", "0"):
        os.environ["DMMT_FUSE_TABLES"] = fuse
        try:
            enc = dmmt_jpeg.Encoder(0)
        finally:
            os.environ.pop("DMMT_FUSE_TABLES")
        try:
            host, outs[fuse] = _encode_device(enc, w, h, 3, opts, first=w)
        finally:
            enc.close()
    assert outs["1"] == outs["0"] == _oracle_all(list(host), sub, opts)


def test_fused_tables_skewed_histograms(encoder):
    """flat frames (one symbol dominates, others rare: the length limit of 15 binds)
    and a noise frame (wide histograms, long codes) through the fused tables"""
    rng = np.random.default_rng(3)
    frames = [np.zeros((64, 96, 3), np.uint8), np.full((40, 40, 3), 200, np.uint8),
              rng.integers(0, 256, (96, 128, 3), dtype=np.uint8)]
    frames[0][5, 7] = 255
    for sub in (0, 2):
        for q in (1, 50, 100):
            opts = _opts(sub, q)
            for f in frames:
                got = encoder.encode(dmmt_jpeg.Image.from_array(f), opts)
                assert got == oracle.encode(f, 255, sub, list(opts.luma_table), list(opts.chroma_table))


@pytest.mark.timeout(300)
def test_fused_tables_u64_keys(encoder):
    """A symbol counted 2^24 times or more: the fused tail ranks that table with
    64-bit keys (phase 1's u32 keys need every frequency below 2^24) and the others
    with 32-bit ones -- the back half from crafted blocks: 4:2:0, 267,264 luma
    blocks whose 63 AC coefficients are all 1 (the symbol 0x01 counted 16,837,632
    times), every 97th block noise, still within tables_fusable's bound."""
    w, h, sub = 4096, 4176, 2
    mcus = (w // 16) * (h // 16)
    rng = np.random.default_rng(24)
    coef = np.ones((mcus * 6, 64), np.int16)
    coef[:, 0] = 0
    noisy = np.arange(0, coef.shape[0], 97)
    coef[noisy] = rng.integers(-50, 51, (noisy.size, 64), dtype=np.int16)
    assert (mcus * 4) * 63 >= 1 << 24 and coef.shape[0] * 64 * 16 < 1 << 30
    luma, chroma = dmmt_jpeg.quality_tables(90)
    opts = _opts(sub, 90)
    ref = oracle.encode_coefficients(coef, w, h, sub, luma, chroma)
    assert encoder.encode_coefficients(coef, w, h, opts) == ref


@pytest.mark.parametrize("sub,w,h", [(0, 264, 256), (2, 528, 512)])
def test_fused_offsets_ff_counts_past_a_byte(encoder, sub, w, h):
    """k_emit's fused offsets read each chunk's 0xFF counts packed one byte each
    (global_load_lds into LDS with the first loads) and take the full count from
    chunk_ff where the byte holds 255.  Crafted blocks: every AC coefficient of the
    first blocks 32767 (category 15, fifteen 1-bits of extra bits after a one-bit
    code: about one 0xFF byte per coefficient at every alignment, thousands per
    chunk), the rest sparse noise (counts below 255), an odd number of chunks (the
    last 16-byte piece reads the padding).  [binary_stream.rs:38-96,
    segment_marker_injector.rs:13-30]"""
    nl = 1 if sub == 0 else 4
    mcus = (w // (8 * (1 if sub == 0 else 2))) * (h // (8 * (1 if sub == 0 else 2)))
    nb = mcus * (nl + 2)
    assert _chunks(w, h, sub) % 2 == 1
    rng = np.random.default_rng(255)
    coef = np.where(rng.random((nb, 64)) < 0.05, rng.integers(-20, 21, (nb, 64)), 0).astype(np.int16)
    heavy = nb // 2
    coef[:heavy, 1:] = 32767
    coef[:heavy, 0] = 0
    luma, chroma = dmmt_jpeg.quality_tables(75)
    ref = oracle.encode_coefficients(coef, w, h, sub, luma, chroma)
    assert ref.count(b"\xff\x00") > 4 * 255 * _chunks(w, h, sub) // 2
    assert encoder.encode_coefficients(coef, w, h, _opts(sub, 75)) == ref
