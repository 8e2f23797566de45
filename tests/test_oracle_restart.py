"""Restart intervals (DRI/RSTn): an extension the reference does not have
(BASELINE config 4's row stripes).  With no reference
output to pin it, the oracle's restart encoding is checked by equivalence: the
scan decodes (RST markers in sequence, 1-padded segments, DC predictors reset)
to exactly the quantised blocks of the reference-exact encode, and a
third-party decoder (Pillow) reconstructs the same pixels."""
import io

import numpy as np
import pytest

import oracle
from oracle import jpeg_scan
from conftest import synthetic

MCU = {0: (8, 8), 1: (16, 8), 2: (16, 16)}


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("ri_kind", ["one", "three", "row", "all"])
def test_restart_decodes_to_the_same_blocks(spec_tables, sub, ri_kind):
    h, w = 37, 53
    rgb = synthetic(w, h, frame=7)
    mw, mh = MCU[sub]
    mcux, mcuy = -(-w // mw), -(-h // mh)
    ri = {"one": 1, "three": 3, "row": mcux, "all": mcux * mcuy + 5}[ri_kind]
    plain = oracle.encode(rgb, 255, sub, *spec_tables)
    rst = oracle.encode(rgb, 255, sub, *spec_tables, restart_interval=ri)
    jf, blocks, pad_ok = jpeg_scan.decode_coefficients(rst)
    assert jf.restart_interval == ri and pad_ok
    assert np.array_equal(blocks, oracle.forward(rgb, 255, sub, *spec_tables))
    nmcu = mcux * mcuy
    assert rst.count(b"\xff\xdd\x00\x04") == 1
    nmarkers = sum(rst.count(bytes([0xFF, 0xD0 + m])) for m in range(8))
    assert nmarkers == (nmcu - 1) // ri
    if ri >= nmcu:  # no marker: the scan equals the reference-exact one
        assert rst.replace(b"\xff\xdd\x00\x04" + bytes([ri >> 8, ri & 255]), b"") == plain


def test_restart_pixels_match_pillow(spec_tables):
    Image = pytest.importorskip("PIL.Image")
    rgb = synthetic(96, 64, frame=3)
    for sub in (0, 2):
        a = np.asarray(Image.open(io.BytesIO(oracle.encode(rgb, 255, sub, *spec_tables))).convert("RGB"))
        b = np.asarray(Image.open(io.BytesIO(oracle.encode(rgb, 255, sub, *spec_tables, restart_interval=2)))
                       .convert("RGB"))
        assert np.array_equal(a, b)


def test_restart_marker_sequence_is_checked(spec_tables):
    rgb = synthetic(64, 8, frame=1)
    rst = bytearray(oracle.encode(rgb, 255, 0, *spec_tables, restart_interval=1))
    i = rst.index(b"\xff\xd1")
    rst[i + 1] = 0xD3
    with pytest.raises(ValueError):
        jpeg_scan.decode_coefficients(bytes(rst))
