"""Pin the CPU oracle to the reference's own outputs and cross-check the two
independent restatements (C cpu_ref vs numpy np_ref)."""
import json
import os

import numpy as np
import pytest

import oracle
from oracle import jpeg_scan, np_ref
from conftest import GOLDEN, synthetic


def natural(zz):
    q = [0] * 64
    for i, z in enumerate(jpeg_scan.ZIGZAG):
        q[z] = zz[i]
    return q


def test_G1_back_half_reproduces_reference_file():
    """tests/output_image_2.jpg was written by the reference encoder:
    decode its coefficients, re-encode with the oracle's back half -> identical file."""
    data = open(os.path.join(GOLDEN, "ref_output_image_2.jpg"), "rb").read()
    jf, blocks, pad_ok = jpeg_scan.decode_coefficients(data)
    assert pad_ok and blocks.shape == (19260, 64)
    out = oracle.encode_coefficients(blocks, jf.width, jf.height, oracle.P444, natural(jf.dqt[0]), natural(jf.dqt[1]),
                                     jf.precision)
    assert out == data


def test_G1_numpy_back_half_too():
    data = open(os.path.join(GOLDEN, "ref_output_image_2.jpg"), "rb").read()
    jf, blocks, _ = jpeg_scan.decode_coefficients(data)
    out = np_ref.encode_coefficients(blocks, jf.width, jf.height, 0, natural(jf.dqt[0]), natural(jf.dqt[1]))
    assert out == data


def test_G2_front_half_flat_red_block():
    """tests/output_image.jpg (older reference revision, 8x8 red, P444, q_DC = 16):
    its scan decodes to DC Y -26, Cb -22, Cr 64 with all AC zero."""
    data = open(os.path.join(GOLDEN, "ref_output_image.jpg"), "rb").read()
    _, blocks, _ = jpeg_scan.decode_coefficients(data)
    rgb = np.zeros((8, 8, 3), np.uint16)
    rgb[..., 0] = 255
    mine = oracle.forward(rgb, 255, oracle.P444, [16] * 64, [16] * 64)
    assert np.array_equal(mine, blocks)
    assert list(blocks[:, 0]) == [-26, -22, 64]


@pytest.mark.parametrize("sub", [0, 1, 2])
def test_crosscheck_fixtures_front_half(fixture_images, presets, sub):
    for name, (rgb, mx) in fixture_images.items():
        for p in presets:
            a = oracle.forward(rgb, mx, sub, p["luma"], p["chroma"])
            b = np_ref.forward(rgb, mx, sub, p["luma"], p["chroma"])
            assert np.array_equal(a, b), (name, sub, p["name"])


@pytest.mark.parametrize("sub", [0, 1, 2])
def test_crosscheck_synthetic_noise(presets, sub):
    rng = np.random.default_rng(7 + sub)
    imgs = [synthetic(67, 45, frame=3), rng.integers(0, 256, (40, 56, 3), dtype=np.uint8),
            rng.integers(0, 4096, (23, 31, 3), dtype=np.uint16)]
    for k, rgb in enumerate(imgs):
        mx = 4095 if rgb.dtype == np.uint16 else 255
        for p in presets[:3]:
            a = oracle.forward(rgb, mx, sub, p["luma"], p["chroma"])
            b = np_ref.forward(rgb, mx, sub, p["luma"], p["chroma"])
            assert np.array_equal(a, b), (k, p["name"])
            ja = oracle.encode_coefficients(a, rgb.shape[1], rgb.shape[0], sub, p["luma"], p["chroma"])
            jb = np_ref.encode_coefficients(b, rgb.shape[1], rgb.shape[0], sub, p["luma"], p["chroma"])
            assert ja == jb
            jf, dec, pad_ok = jpeg_scan.decode_coefficients(ja)
            assert pad_ok and np.array_equal(dec, a)


def test_committed_oracle_goldens(fixture_images, presets):
    manifest = json.load(open(os.path.join(GOLDEN, "oracle_manifest.json")))
    assert len(manifest) == 105
    for fn, m in manifest.items():
        rgb, mx = fixture_images[m["image"]]
        p = presets[m["preset"]]
        assert oracle.encode(rgb, mx, m["subsampling"], p["luma"], p["chroma"]) == open(os.path.join(GOLDEN, fn), "rb").read(), fn


def test_pillow_decodes_oracle_output(fixture_images, spec_tables):
    PIL = pytest.importorskip("PIL.Image")
    import io
    rgb = synthetic(96, 64)
    for sub in (0, 1, 2):
        data = oracle.encode(rgb, 255, sub, *spec_tables)
        im = np.asarray(PIL.open(io.BytesIO(data)).convert("RGB")).astype(float)
        psnr = 10 * np.log10(255 ** 2 / ((im - rgb) ** 2).mean())
        assert psnr > 20, (sub, psnr)  # sharp wrap-around edges + noise at q50


def test_oracle_multithreaded_dct_identical(spec_tables):
    rgb = synthetic(320, 200, frame=1)
    assert oracle.encode(rgb, 255, 2, *spec_tables, threads=4) == oracle.encode(rgb, 255, 2, *spec_tables)


def test_oracle_errors(spec_tables):
    with pytest.raises(oracle.OracleError) as e:
        oracle.encode(np.full((4, 4, 3), 300, np.uint16), 255, 0, *spec_tables)
    assert e.value.code == -100
    with pytest.raises(oracle.OracleError) as e:
        oracle.encode(np.zeros((0, 4, 3), np.uint16), 255, 0, *spec_tables)
    assert e.value.code == -102
