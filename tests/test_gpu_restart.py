"""Restart intervals on the GPU path (extension: DRI + RSTn every N MCUs, DC
predictors reset per interval), byte-exact against the oracle's restart encoding
(tests/test_oracle_restart.py pins that one by decode equivalence)."""
import numpy as np
import pytest

import dmmt_jpeg
import oracle
from oracle import jpeg_scan
from conftest import synthetic

pytestmark = pytest.mark.gpu

MCU = {0: (8, 8), 1: (16, 8), 2: (16, 16)}


def ropts(sub, luma, chroma, ri):
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma, restart_interval=ri)


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("shape", [(37, 53), (120, 200), (8, 8)])
@pytest.mark.parametrize("ri_kind", ["one", "two", "five", "row", "huge"])
def test_restart_matches_oracle(encoder, spec_tables, sub, shape, ri_kind):
    h, w = shape
    rgb = synthetic(w, h, frame=w + h)
    mw, mh = MCU[sub]
    mcux = -(-w // mw)
    ri = {"one": 1, "two": 2, "five": 5, "row": mcux, "huge": 65535}[ri_kind]
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), ropts(sub, *spec_tables, ri))
    assert gpu == oracle.encode(rgb, 255, sub, *spec_tables, restart_interval=ri)


def test_restart_noise_all_tables(encoder, presets):
    rng = np.random.default_rng(17)
    rgb = rng.integers(0, 256, (48, 80, 3), dtype=np.uint8)
    for p in presets:
        for sub, ri in ((0, 3), (2, 1), (1, 7)):
            gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), ropts(sub, p["luma"], p["chroma"], ri))
            assert gpu == oracle.encode(rgb, 255, sub, p["luma"], p["chroma"], restart_interval=ri), p["name"]


@pytest.mark.parametrize("ri_kind", ["row", "one"])
def test_restart_4k(encoder, ri_kind):
    """BASELINE config 4's stripe structure on a 4K frame: one restart per MCU row,
    and the extreme of one per MCU (129,600 segments)."""
    luma, chroma = dmmt_jpeg.quality_tables(90)
    rgb = synthetic(3840, 2160, frame=4)
    ri = 3840 // 8 if ri_kind == "row" else 1
    gpu = encoder.encode(dmmt_jpeg.Image.from_array(rgb), ropts(0, luma, chroma, ri))
    ref = oracle.encode(rgb, 255, 0, luma, chroma, threads=8, restart_interval=ri)
    assert gpu == ref
    jf, blocks, pad_ok = jpeg_scan.decode_coefficients(gpu) if ri_kind == "row" else (None, None, True)
    assert pad_ok


def test_restart_interval_out_of_range(encoder, spec_tables):
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.encode(dmmt_jpeg.Image.from_array(synthetic(16, 16)), ropts(0, *spec_tables, 70000))
    assert e.value.code == -102
