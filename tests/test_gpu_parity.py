"""Parity of the gfx950 HIP path (through the C ABI) with the CPU oracle.
Bar: bit-exact -- quantised coefficients and every JPEG byte."""
import io
import json
import os

import numpy as np
import pytest

import dmmt_jpeg
import oracle
from oracle import jpeg_scan
from conftest import GOLDEN, synthetic

pytestmark = pytest.mark.gpu

SUBS = [0, 1, 2]


def opts(sub, luma, chroma, bits=8):
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), bits, luma_table=luma,
                                              chroma_table=chroma)


def natural(zz):
    q = [0] * 64
    for i, z in enumerate(jpeg_scan.ZIGZAG):
        q[z] = zz[i]
    return q


def test_dct_operator_matches_oracle(encoder):
    rng = np.random.default_rng(1)
    blocks = rng.uniform(-128, 127, (1000, 64)).astype(np.float32)
    gpu = encoder.dct_transform(blocks)
    cpu = np.stack([oracle.dct_block(b) for b in blocks])
    assert np.array_equal(gpu.view(np.uint32), cpu.view(np.uint32))


def test_dct_operator_reference_kat(encoder):  # arai.rs:190-202 vs the naive transform, 1e-4
    from test_oracle_kat import TEST_VALUES, naive_dct
    out = dmmt_jpeg.AraiDiscrete8x8CosineTransformer(encoder).transform(TEST_VALUES)
    assert np.max(np.abs(out - naive_dct(TEST_VALUES))) <= 1e-4


@pytest.mark.parametrize("sub", SUBS)
def test_forward_blocks_fixtures(encoder, fixture_images, presets, sub):
    for name, (rgb, mx) in fixture_images.items():
        for p in presets:
            img = dmmt_jpeg.Image.from_array(rgb, mx)
            gpu = encoder.forward_blocks(img, opts(sub, p["luma"], p["chroma"]))
            cpu = oracle.forward(rgb, mx, sub, p["luma"], p["chroma"])
            assert np.array_equal(gpu, cpu), (name, sub, p["name"])


def test_whole_file_committed_goldens(encoder, fixture_images, presets):
    manifest = json.load(open(os.path.join(GOLDEN, "oracle_manifest.json")))
    for fn, m in sorted(manifest.items()):
        rgb, mx = fixture_images[m["image"]]
        p = presets[m["preset"]]
        gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb, mx), opts(m["subsampling"], p["luma"], p["chroma"]))
        assert gpu == open(os.path.join(GOLDEN, fn), "rb").read(), fn


def test_G1_back_half_on_gpu():
    """The reference encoder's own file (output_image_2.jpg) reproduced by the
    GPU back half from its decoded coefficients."""
    enc = dmmt_jpeg.Encoder(0)
    data = open(os.path.join(GOLDEN, "ref_output_image_2.jpg"), "rb").read()
    jf, blocks, _ = jpeg_scan.decode_coefficients(data)
    out = enc.encode_coefficients(blocks, jf.width, jf.height, opts(0, natural(jf.dqt[0]), natural(jf.dqt[1])))
    assert out == data


@pytest.mark.parametrize("sub", SUBS)
@pytest.mark.parametrize("shape", [(1, 1), (2, 3), (8, 8), (17, 7), (16, 16), (33, 65), (200, 120), (257, 513)])
def test_synthetic_shapes(encoder, spec_tables, sub, shape):
    h, w = shape
    rgb = synthetic(w, h, frame=h)
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(sub, *spec_tables))
    assert gpu == oracle.encode(rgb, 255, sub, *spec_tables)


@pytest.mark.parametrize("sub", SUBS)
@pytest.mark.parametrize("shape", [(9, 65520), (65520, 9), (1, 65519), (65519, 2)])
def test_extreme_aspect_at_u16_limit(encoder, spec_tables, sub, shape):
    """Widths and heights at the u16 limit of Image / PaddedImage (image.rs:7-11,
    padder.rs:3-9): one MCU row of 4096 MCUs, one MCU column, ragged both ways."""
    h, w = shape
    rgb = synthetic(w, h, frame=3)
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(sub, *spec_tables))
    assert gpu == oracle.encode(rgb, 255, sub, *spec_tables)


@pytest.mark.parametrize("sub,shape", [(0, (1, 65535)), (2, (65530, 1)), (1, (3, 65535))])
def test_padded_size_above_u16_is_an_error(encoder, spec_tables, sub, shape):
    """padder.rs:12-14 computes the padded size in u16; one past 65535 overflows
    there (a panic in the reference): an error code here, as in the oracle."""
    h, w = shape
    rgb = np.zeros((h, w, 3), np.uint8)
    with pytest.raises(oracle.OracleError) as eo:
        oracle.encode(rgb, 255, sub, *spec_tables)
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(sub, *spec_tables))
    assert e.value.code == eo.value.code == -102


@pytest.mark.parametrize("sub", SUBS)
def test_full_range_noise_all_tables(encoder, presets, sub):
    """uniform noise: large coefficients, long runs of categories, every table."""
    rng = np.random.default_rng(100 + sub)
    rgb = rng.integers(0, 256, (72, 136, 3), dtype=np.uint8)
    for p in presets:
        gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(sub, p["luma"], p["chroma"]))
        assert gpu == oracle.encode(rgb, 255, sub, p["luma"], p["chroma"]), p["name"]


def test_q1_extreme_and_flat(encoder):
    rng = np.random.default_rng(5)
    ones = [1] * 64
    for rgb in (rng.integers(0, 256, (64, 64, 3), dtype=np.uint8), np.zeros((64, 64, 3), np.uint8),
                np.full((40, 24, 3), 255, np.uint8)):
        for sub in SUBS:
            gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(sub, ones, ones))
            assert gpu == oracle.encode(rgb, 255, sub, ones, ones)


@pytest.mark.parametrize("maxval", [1, 15, 1000, 65535])
def test_16bit_and_odd_maxval(encoder, spec_tables, maxval):
    rng = np.random.default_rng(maxval)
    rgb = rng.integers(0, maxval + 1, (30, 50, 3)).astype(np.uint16)
    img = dmmt_jpeg.Image(50, 30, maxval, rgb if maxval > 255 else rgb.astype(np.uint8))
    for sub in SUBS:
        assert encoder.encode(img, opts(sub, *spec_tables)) == oracle.encode(rgb, maxval, sub, *spec_tables)


@pytest.mark.parametrize("sub", SUBS)
@pytest.mark.parametrize("shape", [(1, 1), (9, 13), (16, 16), (61, 203), (270, 480)])
def test_image_f32_input(encoder, spec_tables, sub, shape):
    """sample_bytes 4: the reference's Image<f32> dots (`v as f32 / max as f32`,
    color.rs:45-53, computed here in float32) -- the JpegImageWriter seam."""
    h, w = shape
    rgb = synthetic(w, h, frame=w)
    for maxval in (255, 1000):
        raw = rgb.astype(np.uint16) * (maxval // 255)
        f32 = raw.astype(np.float32) / np.float32(maxval)
        gpu = encoder.encode(dmmt_jpeg.Image.from_array(f32, maxval), opts(sub, *spec_tables))
        assert gpu == oracle.encode(raw, maxval, sub, *spec_tables)


def test_value_above_maxval_is_an_error(encoder, spec_tables):
    rgb = np.full((8, 8, 3), 200, np.uint8)
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode(dmmt_jpeg.Image(8, 8, 100, rgb), opts(0, *spec_tables))
    assert e.value.code == -100
    # the context stays usable afterwards
    ok = synthetic(16, 16)
    assert encoder.encode(dmmt_jpeg.Image.from_array(ok), opts(2, *spec_tables)) == oracle.encode(ok, 255, 2, *spec_tables)


@pytest.mark.parametrize("where", ["ac", "dc", "dc_diff"])
def test_category_out_of_range_is_an_error(encoder, spec_tables, where):
    """categorize.rs:25-30 panics on -32768 (category 16): an AC coefficient, a
    first-block DC (difference from predictor 0) or a DC difference that wraps
    to -32768 in i16 -- the oracle's CategoryOutOfRange, as an error code here."""
    blocks = np.zeros((3 * 4, 64), np.int16)  # 32x8 pixels, 4:4:4: 4 MCUs
    if where == "ac":
        blocks[4, 5] = -32768
    elif where == "dc":
        blocks[0, 0] = -32768
    else:
        blocks[0, 0], blocks[3, 0] = 16384, -16384  # luma DCs of MCUs 0, 1: -16384 - 16384 wraps
    with pytest.raises(oracle.OracleError) as eo:
        oracle.encode_coefficients(blocks, 32, 8, 0, *spec_tables)
    assert eo.value.code == -101
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode_coefficients(blocks, 32, 8, opts(0, *spec_tables))
    assert e.value.code == -101
    # the context stays usable afterwards
    ok = synthetic(16, 16)
    assert encoder.encode(dmmt_jpeg.Image.from_array(ok), opts(0, *spec_tables)) == oracle.encode(ok, 255, 0, *spec_tables)


def test_category_out_of_range_from_f32_dots(encoder, spec_tables):
    """Image<f32> dots far outside [0, 1] saturate `as i16` (quantizer.rs:60) to
    -32768, whose category the reference cannot encode (categorize.rs:25-30)."""
    dots = np.full((8, 8, 3), -1000.0, np.float32)
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode(dmmt_jpeg.Image.from_array(dots, 255), opts(0, *spec_tables))
    assert e.value.code == -101
    dots[:, 4:, :] = 1000.0  # a saturated AC coefficient beside a finite DC
    dots[:, :4, :] = -1000.0
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode(dmmt_jpeg.Image.from_array(dots, 255), opts(0, *spec_tables))
    assert e.value.code == -101


def test_bits_per_channel_written_to_sof(encoder, spec_tables):
    rgb = synthetic(24, 16)
    for bits in (8, 16, 32):
        gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(2, *spec_tables, bits=bits))
        assert gpu == oracle.encode(rgb, 255, 2, *spec_tables, bits_per_channel=bits)


def test_batch_api_mixed_geometry(encoder, spec_tables):
    imgs = [synthetic(64, 48, frame=f) for f in range(5)] + [synthetic(31, 17, frame=9), synthetic(64, 48, frame=11)]
    outs = encoder.encode_batch([dmmt_jpeg.Image.from_array(a) for a in imgs], opts(2, *spec_tables))
    for a, o in zip(imgs, outs):
        assert o == oracle.encode(a, 255, 2, *spec_tables)


def test_batch_error_mid_batch(encoder, spec_tables):
    """A sample above maxval in frame 2 of 4: the whole call fails (color.rs:63-65),
    no output is returned, and the context stays usable."""
    frames = [np.full((16, 24, 3), 90, np.uint8) for _ in range(4)]
    frames[2][3, 5, 1] = 200
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode_batch([dmmt_jpeg.Image(24, 16, 100, f) for f in frames], opts(2, *spec_tables))
    assert e.value.code == -100
    ok = [synthetic(24, 16, frame=f) for f in range(3)]
    outs = encoder.encode_batch([dmmt_jpeg.Image.from_array(a) for a in ok], opts(2, *spec_tables))
    assert outs == [oracle.encode(a, 255, 2, *spec_tables) for a in ok]


def test_device_resident_api_and_generator(encoder, spec_tables):
    w, h, n = 320, 240, 6
    d_in = encoder.malloc(w * h * 3 * n)
    stride = dmmt_jpeg.max_jpeg_bytes(w, h, 2)
    d_out = encoder.malloc(stride * n)
    d_len = encoder.malloc(4 * n)
    try:
        encoder.fill_synthetic(d_in, w, h, n, first_frame=2)
        host = np.frombuffer(encoder.d2h(d_in, w * h * 3 * n), np.uint8).reshape(n, h, w, 3)
        for f in range(n):
            assert np.array_equal(host[f], synthetic(w, h, frame=2 + f))
        encoder.encode_device(d_in, n, w, h, opts(2, *spec_tables), d_out, stride, d_len)
        encoder.synchronize()
        lens = np.frombuffer(encoder.d2h(d_len, 4 * n), np.uint32)
        for f in range(n):
            data = encoder.d2h(d_out + f * stride, int(lens[f]))
            assert data == oracle.encode(host[f], 255, 2, *spec_tables), f
    finally:
        for p in (d_in, d_out, d_len):
            encoder.free(p)


@pytest.mark.parametrize("sub", SUBS)
@pytest.mark.parametrize("sample_bytes", [1, 2])
def test_device_frames_misaligned_interior_tiles(encoder, spec_tables, sub, sample_bytes):
    """Frames packed at odd byte offsets, widths a multiple of the 256-pixel tile:
    k_front's interior-tile loads (aligned 16-byte chunks, no masking) start a
    chunk up to 15 bytes before a row and read the next tile's bytes; the first
    and last tiles of each frame take the guarded path."""
    w, h, n = 512, 24, 3
    rng = np.random.default_rng(17 + sub)
    maxval = 255 if sample_bytes == 1 else 1023
    dt = np.uint8 if sample_bytes == 1 else np.uint16
    frames = rng.integers(0, maxval + 1, (n, h, w, 3)).astype(dt)
    fbytes = w * h * 3 * sample_bytes
    stride = fbytes + 6 * sample_bytes  # every frame starts at a different residue mod 16
    buf = np.zeros(stride * n + 16, np.uint8)
    for f in range(n):
        buf[3 * sample_bytes + f * stride:3 * sample_bytes + f * stride + fbytes] = frames[f].reshape(-1).view(np.uint8)
    d_in = encoder.malloc(buf.nbytes)
    ostride = dmmt_jpeg.max_jpeg_bytes(w, h, sub)
    d_out = encoder.malloc(ostride * n)
    d_len = encoder.malloc(4 * n)
    try:
        encoder.h2d(d_in, buf)
        encoder.encode_device(d_in + 3 * sample_bytes, n, w, h, opts(sub, *spec_tables), d_out, ostride, d_len,
                              frame_stride=stride, maxval=maxval, sample_bytes=sample_bytes)
        encoder.synchronize()
        lens = np.frombuffer(encoder.d2h(d_len, 4 * n), np.uint32)
        for f in range(n):
            assert encoder.d2h(d_out + f * ostride, int(lens[f])) == oracle.encode(frames[f], maxval, sub, *spec_tables), f
    finally:
        for p in (d_in, d_out, d_len):
            encoder.free(p)


def test_4k_quality90_444(encoder):
    """BASELINE config 2 workload at full size."""
    luma, chroma = dmmt_jpeg.quality_tables(90)
    rgb = synthetic(3840, 2160, frame=0)
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(0, luma, chroma))
    assert gpu == oracle.encode(rgb, 255, 0, luma, chroma)


@pytest.mark.parametrize("quality", [50, 95])
def test_8k_quality_sweep_420(encoder, quality):
    """BASELINE config 5 frame (7680x4320, 4:2:0) at the ends of the quality sweep;
    q50 is the reference's Specification preset."""
    luma, chroma = dmmt_jpeg.quality_tables(quality)
    rgb = synthetic(7680, 4320, frame=quality)
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(2, luma, chroma))
    assert gpu == oracle.encode(rgb, 255, 2, luma, chroma, threads=8)


def test_1080p_batch_quality75_420(encoder):
    """BASELINE config 3 shape (a few of the 256 frames; each byte-exact)."""
    luma, chroma = dmmt_jpeg.quality_tables(75)
    frames = [synthetic(1920, 1080, frame=f) for f in range(4)]
    outs = encoder.encode_batch([dmmt_jpeg.Image.from_array(a) for a in frames], opts(2, luma, chroma))
    for a, o in zip(frames, outs):
        assert o == oracle.encode(a, 255, 2, luma, chroma)


def test_pillow_roundtrip(encoder, spec_tables):
    PIL = pytest.importorskip("PIL.Image")
    rgb = synthetic(200, 150)
    data = encoder.encode(dmmt_jpeg.Image.from_array(rgb), opts(2, *spec_tables))
    im = np.asarray(PIL.open(io.BytesIO(data)).convert("RGB"))
    assert im.shape == rgb.shape


def test_cli_and_convert_ppm(tmp_path, spec_tables):
    import subprocess
    src = os.path.join(GOLDEN, "7x17.ppm")
    out = tmp_path / "o.jpg"
    r = subprocess.run([dmmt_jpeg.CLI_PATH, src, str(out), "-p", "P422", "-q", "Flat"], capture_output=True)
    assert r.returncode == 0, r.stderr
    from oracle import ppm
    rgb, mx = ppm.read_p3(open(src, "rb").read())
    flat = [16] * 64
    assert out.read_bytes() == oracle.encode(rgb, mx, 1, flat, flat)
    out2 = tmp_path / "o2.jpg"
    dmmt_jpeg.convert_ppm_to_jpeg(dmmt_jpeg.Arguments(src, str(out2)))
    assert out2.read_bytes() == oracle.encode(rgb, mx, 2, *spec_tables)
    r = subprocess.run([dmmt_jpeg.CLI_PATH, str(tmp_path / "missing.ppm"), str(out)], capture_output=True)
    assert r.returncode == 1 and b"Conversion failed because of" in r.stderr


def test_seeded_random_sweep(encoder):
    """200 seeded random cases across the option space, each byte-compared with the
    oracle: shape (1..300 x 1..300), subsampling, IJG quality 1..100, 8/16-bit
    samples with any maxval, sample content (noise, smooth, flat, sparse), restart
    interval (0 or 1..40 MCUs)."""
    rng = np.random.default_rng(20261016)
    for case in range(200):
        h, w = int(rng.integers(1, 301)), int(rng.integers(1, 301))
        sub = int(rng.integers(0, 3))
        q = int(rng.integers(1, 101))
        maxval = int(rng.choice([255, int(rng.integers(1, 256)), int(rng.integers(256, 65536))]))
        kind = int(rng.integers(0, 4))
        if kind == 0:
            px = rng.integers(0, maxval + 1, (h, w, 3))
        elif kind == 1:
            yy, xx = np.mgrid[0:h, 0:w]
            px = ((np.stack([xx, yy, xx + yy], -1) * maxval) // max(w + h, 1)) % (maxval + 1)
        elif kind == 2:
            px = np.full((h, w, 3), int(rng.integers(0, maxval + 1)))
        else:
            px = np.where(rng.random((h, w, 3)) < 0.02, rng.integers(0, maxval + 1, (h, w, 3)), 0)
        rgb = px.astype(np.uint8 if maxval < 256 else np.uint16)
        ri = 0 if rng.random() < 0.5 else int(rng.integers(1, 41))
        luma, chroma = dmmt_jpeg.quality_tables(q)
        o = opts(sub, luma, chroma)
        o.restart_interval = ri
        gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb, maxval), o)
        ref = oracle.encode(rgb, maxval, sub, luma, chroma, restart_interval=ri)
        assert gpu == ref, dict(case=case, h=h, w=w, sub=sub, q=q, maxval=maxval, kind=kind, ri=ri)
