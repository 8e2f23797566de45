"""PPM ingest on the GPU (dmmt_decode_ppm_device): the P3 body
decoded in HBM must give exactly the samples of the reference tokenizer/parser
(ppm.rs:41-77, 224-252; restated by oracle/ppm.py and the host mirror
dmmt_parse_ppm) and the same error variant, whatever the whitespace, comments
(a '#' comment runs to its '\\n' and does not end a token), '+' signs, leading
zeros, chunk boundaries (4096-byte chunks) and buffer alignment."""
import os
import re

import numpy as np
import pytest

import dmmt_jpeg
import oracle
from conftest import GOLDEN, synthetic
from oracle import ppm

pytestmark = pytest.mark.gpu

WS = [b" ", b"\n", b"\t", b"\r", b"\x0c"]


def p3_text(rgb, maxval, rng, ws_max=3, comments=0.0, plus=0.0, zeros=0.0, header=b"P3\n"):
    """a P3 file of rgb with random separators, comments, '+' signs, leading zeros"""
    h, w, _ = rgb.shape
    parts = [header, b"%d %d\n%d\n" % (w, h, maxval)]
    for v in rgb.reshape(-1).tolist():
        tok = b"%d" % v
        if zeros and rng.random() < zeros:
            tok = b"0" * int(rng.integers(1, 6)) + tok
        if plus and rng.random() < plus:
            tok = b"+" + tok
        if comments and rng.random() < comments:  # a comment inside the token: does not split it
            k = int(rng.integers(0, len(tok) + 1))
            tok = tok[:k] + b"#c # x\n" + tok[k:]
        parts.append(tok)
        sep = b"".join(WS[int(i)] for i in rng.integers(0, len(WS), int(rng.integers(1, ws_max + 1))))
        if comments and rng.random() < comments:
            sep += b"# comment between tokens\n" + WS[int(rng.integers(0, len(WS)))]
        parts.append(sep)
    return b"".join(parts)


def decode_gpu(encoder, data, align=0):
    """the whole file at a device address with the given misalignment"""
    h = dmmt_jpeg.parse_ppm_header(data)
    n = h.width * h.height * 3
    sb = 1 if h.maxval <= 255 else 2
    d_text = encoder.malloc(len(data) + 64)
    d_rgb = encoder.malloc(max(n * sb, 1))
    try:
        if data:
            encoder.h2d(d_text + align, np.frombuffer(data, np.uint8))
        encoder.decode_ppm_device(d_text + align, len(data), h, d_rgb)
        return np.frombuffer(encoder.d2h(d_rgb, n * sb), np.uint8 if sb == 1 else np.uint16).reshape(
            h.height, h.width, 3), h.maxval
    finally:
        encoder.free(d_text)
        encoder.free(d_rgb)


def host_code(data):
    try:
        dmmt_jpeg.PPMImageReader(data).read_image()
        return 0
    except dmmt_jpeg.Error as e:
        return e.code


def check_equal(encoder, data, align=0):
    rgb, mx = ppm.read_p3(data)
    got, gmx = decode_gpu(encoder, data, align)
    assert gmx == mx
    assert np.array_equal(got.astype(np.uint16), rgb)


@pytest.mark.parametrize("name", ["16x16", "8x8", "7x17", "small"])
def test_reference_fixtures(encoder, name):
    check_equal(encoder, open(os.path.join(GOLDEN, name + ".ppm"), "rb").read())


@pytest.mark.parametrize("w,h,ws_max,seed", [(37, 23, 1, 0), (160, 90, 3, 1), (300, 200, 8, 2), (1, 1, 1, 3)])
def test_random_separators(encoder, w, h, ws_max, seed):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    for align in (0, 5):
        check_equal(encoder, p3_text(rgb, 255, rng, ws_max=ws_max), align)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_comments_signs_leading_zeros(encoder, seed):
    rng = np.random.default_rng(10 + seed)
    rgb = rng.integers(0, 256, (61, 97, 3), dtype=np.uint8)
    data = p3_text(rgb, 255, rng, comments=0.05, plus=0.05, zeros=0.05,
                   header=b"P3 # a header comment\n# another\n")
    for align in (0, 3, 15):
        check_equal(encoder, data, align)


def test_sixteen_bit_samples(encoder):
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 1001, (50, 70, 3), dtype=np.uint16)
    check_equal(encoder, p3_text(rgb, 1000, rng, ws_max=2, comments=0.01))
    rgb = rng.integers(0, 65536, (20, 30, 3), dtype=np.uint16)
    check_equal(encoder, p3_text(rgb, 65535, rng))


def test_long_runs_across_chunks(encoder):
    """whitespace runs, comments and tokens longer than a chunk (4096 B) and its staged tail"""
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    parts = [b"P3\n11 9\n255\n"]
    for i, v in enumerate(rgb.reshape(-1).tolist()):
        if i % 37 == 0:
            parts.append(b"0" * 5000 + b"%d" % v)           # a 5000-byte token
        elif i % 41 == 0:
            parts.append(b"%d#" % v + b"x" * 9000 + b"\n")  # a 9 KB comment before the separator
        else:
            parts.append(b"%d" % v)
        parts.append(b" " * (6000 if i % 29 == 0 else 1))
    data = b"".join(parts)
    check_equal(encoder, data)
    check_equal(encoder, data, 7)


def test_synthetic_4k_frame(encoder):
    """a whole 3840x2160 frame as P3 (~35 MB of text), as bench.py's ingest line"""
    import bench
    rgb = synthetic(3840, 2160)
    data = bench.p3_bytes(rgb)
    got, mx = decode_gpu(encoder, data)
    assert mx == 255 and np.array_equal(got, rgb)


@pytest.mark.parametrize("text", [
    b"P3 1 1 255 0 0", b"P3 2 1 255 0 0 0", b"P3 1 1 255 0 0 0 1 1 1", b"P3 1 1 255 0 256 0",
    b"P3 1 1 15 0 16 0", b"P3 1 1 255 0 0 -1", b"P3 1 1 255 0 + 1", b"P3 1 1 255 0 1a 1",
    b"P3 1 1 255 0 65536 1", b"P3 1 1 255 0 0 1#x", b"P3 1 1 255 0 0 1 #x\n", b"P3 1 1 255 1 2 ++3",
    b"P3 1 1 255 1 2 3 4 5", b"P3 2 1 255 1 2 3 4 5 x", b"P3 0 0 255", b"P3 0 0 255 ", b"P3 1 1 255",
    b"P3 1 1 255\n1 2\xff 3", b"P3 2 2 255 " + b"1 " * 12 + b"# trailing comment"])
def test_errors_match_host_reader(encoder, text):
    code = host_code(text)
    h = dmmt_jpeg.parse_ppm_header(text)
    n = max(h.width * h.height * 3, 1)
    d_text = encoder.malloc(len(text))
    d_rgb = encoder.malloc(2 * n)
    try:
        encoder.h2d(d_text, np.frombuffer(text, np.uint8))
        try:
            encoder.decode_ppm_device(d_text, len(text), h, d_rgb)
            got = 0
        except dmmt_jpeg.Error as e:
            got = e.code
    finally:
        encoder.free(d_text)
        encoder.free(d_rgb)
    assert got == code


@pytest.mark.parametrize("text", [
    b"P3 65535 65535 255 1 2 3", b"P3 65535 65535 255 1 2", b"P3 65535 65535 255 1 x 3",
    b"P3 40000 3 65535 " + b"7 " * 300, b"P6 65535 65535 255\n\x01\x02\x03", b"P6 30000 2 65535\n" + b"\x00" * 10])
def test_short_body_claiming_a_large_image(encoder, tmp_path, text):
    """A few bytes of text under a header that claims up to 65535 x 65535: the
    frame buffer is sized by what the text can fill (a sample per token, a token
    and a separator per two bytes), never by the header; the error is the host
    reader's, through the mirror's decode and through convert_ppm_to_jpeg."""
    code = host_code(text)
    assert code != 0
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.read_ppm_device(text)
    assert e.value.code == code
    src = tmp_path / "short.ppm"
    src.write_bytes(text)
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.convert_ppm_to_jpeg(dmmt_jpeg.Arguments(str(src), str(tmp_path / "o.jpg")))
    assert e.value.code == code
    rgb = np.arange(3 * 9 * 5, dtype=np.uint8).reshape(5, 9, 3)  # the context still decodes
    got, _ = decode_gpu(encoder, b"P6 9 5 255\n" + rgb.tobytes())
    assert np.array_equal(got, rgb)


def test_p6_samples(encoder):
    rgb = np.arange(3 * 5 * 7, dtype=np.uint8).reshape(5, 7, 3)
    got, _ = decode_gpu(encoder, b"P6\n7 5\n255\n" + rgb.tobytes())
    assert np.array_equal(got, rgb)
    rgb16 = (np.arange(3 * 4 * 3, dtype=np.uint16) * 997).reshape(4, 3, 3)
    got, _ = decode_gpu(encoder, b"P6 3 4 65535\n" + rgb16.astype(">u2").tobytes())
    assert np.array_equal(got, rgb16)


def test_convert_decodes_on_the_gpu(tmp_path, spec_tables):
    """convert_ppm_to_jpeg: file bytes -> GPU decode -> GPU encode, byte-identical"""
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (45, 67, 3), dtype=np.uint8)
    src = tmp_path / "in.ppm"
    src.write_bytes(p3_text(rgb, 255, rng, comments=0.02))
    out = tmp_path / "o.jpg"
    dmmt_jpeg.convert_ppm_to_jpeg(dmmt_jpeg.Arguments(str(src), str(out)))
    assert out.read_bytes() == oracle.encode(rgb, 255, 2, *spec_tables)
    bad = tmp_path / "bad.ppm"
    bad.write_bytes(b"P3 2 2 255 1 2 3 4 5 6 7 8 9 10 11 x")
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.convert_ppm_to_jpeg(dmmt_jpeg.Arguments(str(bad), str(out)))
    assert e.value.code == -2


from test_abi import PPM_KATS  # noqa: E402  (ppm.rs:266-306 as data)


@pytest.mark.parametrize("name,text,err", PPM_KATS, ids=[k[0] for k in PPM_KATS])
def test_reference_ppm_unit_tests_on_gpu(encoder, name, text, err):
    """the reference's five PPM unit tests (ppm.rs:266-306) with the body decoded on
    the GPU (dmmt_decode_ppm_device); IncompletePixelParsed carries n == 2"""
    data = text.encode()
    if err is None:
        img = encoder.read_ppm_device(data)
        host = dmmt_jpeg.PPMImageReader(data).read_image()
        assert img.height == 2 and np.array_equal(img.samples, host.samples)
        return
    with pytest.raises(dmmt_jpeg.Error) as e:
        encoder.read_ppm_device(data)
    assert e.value.code == err[0]
    if err[1] is not None:
        assert e.value.n == err[1]


def test_convert_device_batch(encoder, spec_tables):
    """dmmt_convert_ppm_device_batch: a stream of files in HBM decoded and encoded back
    to back over three lanes, each file speculatively on the comment-free path; every
    JPEG byte-identical to the oracle's and every code the one the file gets on its
    own (host reader, then the encoder's range check): clean P3 files of several
    sizes, comments (redone on the general path), 16-bit samples, P6, a token that
    does not parse, an incomplete pixel, a body too short for the fast path, a sample
    above maxval, a header too large for the output buffer, a short body whose
    header claims 65535 x 65535 (no buffer is sized by the header)."""
    rng = np.random.default_rng(21)
    cases = []  # (file bytes, samples or None, maxval)
    for w, h in [(67, 45), (128, 96), (300, 211), (640, 360)]:
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        cases.append((p3_text(rgb, 255, rng), rgb, 255))
    rgb = rng.integers(0, 256, (40, 52, 3), dtype=np.uint8)
    cases.append((p3_text(rgb, 255, rng, comments=0.02, plus=0.02), rgb, 255))
    rgb16 = rng.integers(0, 1001, (33, 41, 3), dtype=np.uint16)
    cases.append((p3_text(rgb16, 1000, rng), rgb16, 1000))
    rgb6 = rng.integers(0, 256, (7, 19, 3), dtype=np.uint8)
    cases.append((b"P6 19 7 255\n" + rgb6.tobytes(), rgb6, 255))
    cases.append((b"P3 2 2 255 " + b" ".join(b"%d" % v for v in range(11)) + b" x" + b" " * 100, None, 255))
    cases.append((b"P3 2 4 255\n" + b"9 " * 23 + b" " * 100, None, 255))
    small = np.array([[[1, 2, 3]]], np.uint8)
    cases.append((b"P3 1 1 255 1 2 3", small, 255))
    over = rng.integers(0, 201, (30, 40, 3), dtype=np.uint16)
    over[5, 7, 1] = 250
    cases.append((p3_text(over, 200, rng), over, 200))
    cases.append((b"P3 65535 65535 255 " + b"7 " * 300, None, 255))  # a short body claiming a huge image
    cases = cases + cases[::-1]  # 24 files: every lane sees every kind
    L = dmmt_jpeg.lib()
    allocs, files, expect = [], [], []
    try:
        for k, (data, rgb, mx) in enumerate(cases):
            hdr = dmmt_jpeg.parse_ppm_header(data)
            cap = L.dmmt_max_jpeg_bytes(max(hdr.width, 1), max(hdr.height, 1), 2)
            if hdr.width * hdr.height > 1 << 24:
                cap = 4096  # the huge header: its decode fails before the capacity check
            if k == 3:
                cap -= 1  # too small: DMMT_E_CAPACITY after a successful decode
            d_text, d_out, d_len = encoder.malloc(len(data)), encoder.malloc(cap), encoder.malloc(4)
            allocs += [d_text, d_out, d_len]
            encoder.h2d(d_text, np.frombuffer(data, np.uint8))
            encoder.h2d(d_len, np.array([0xFFFFFFFF], np.uint32))
            files.append((d_text, len(data), hdr, d_out, cap, d_len))
            code = host_code(data)
            if code == 0 and rgb is not None and int(rgb.max()) > mx:
                code = -100  # DMMT_E_VALUE_EXCEEDS_MAX (color.rs:63-65)
            if code == 0 and k == 3:
                code = -203
            expect.append((code, None if code else oracle.encode(rgb, mx, 2, *spec_tables)))
        encoder.set_lanes(3)
        codes = encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions(), check=False)
        assert codes == [e[0] for e in expect]
        for (d_text, n, hdr, d_out, cap, d_len), (code, jpeg) in zip(files, expect):
            size = int(np.frombuffer(encoder.d2h(d_len, 4), np.uint32)[0])
            if code:
                assert size == 0
            else:
                assert encoder.d2h(d_out, size) == jpeg
    finally:
        encoder.set_lanes(1)
        for p in allocs:
            encoder.free(p)


def _device_files(encoder, datas, allocs):
    L = dmmt_jpeg.lib()
    files = []
    for data in datas:
        hdr = dmmt_jpeg.parse_ppm_header(data)
        cap = L.dmmt_max_jpeg_bytes(max(hdr.width, 1), max(hdr.height, 1), 2)
        d_text, d_out, d_len = encoder.malloc(len(data)), encoder.malloc(cap), encoder.malloc(4)
        allocs += [d_text, d_out, d_len]
        encoder.h2d(d_text, np.frombuffer(data, np.uint8))
        files.append((d_text, len(data), hdr, d_out, cap, d_len))
    return files


def test_convert_device_batch_error_payload_is_the_first_failures(encoder):
    """dmmt_convert_ppm_device_batch returns the first failing file's code, and the
    payload dmmt_last_error_detail keeps is that file's (IncompletePixelParsed(1)),
    not the one of a file redone after it (a commented file that succeeds, then
    IncompletePixelParsed(2)) [ppm.rs:239-245, error.rs:3-22]"""
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (12, 20, 3), dtype=np.uint8)
    body = b" ".join(b"%d" % v for v in rgb.reshape(-1))
    datas = [b"P3 2 2 255\n" + b"9 " * 10 + b" " * 100,              # 10 samples: n = 1
             b"P3 20 12 255\n# a comment\n" + body + b"\n",          # redone, succeeds
             b"P3 2 2 255\n" + b"9 " * 11 + b" " * 100]              # 11 samples: n = 2
    allocs = []
    try:
        files = _device_files(encoder, datas, allocs)
        for lanes in (1, 3):
            encoder.set_lanes(lanes)
            with pytest.raises(dmmt_jpeg.Error) as e:
                encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions())
            assert e.value.code == -3 and e.value.n == 1, str(e.value)
            assert "got 1." in str(e.value)
            codes = encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions(), check=False)
            assert codes == [-3, 0, -3]
            assert dmmt_jpeg.lib().dmmt_last_error_detail() == 1
    finally:
        encoder.set_lanes(1)
        for p in allocs:
            encoder.free(p)


def test_convert_device_batch_redoes_only_the_failing_file(encoder, spec_tables):
    """A commented file in a batch is redone on its own; the clean files on its lane
    are not (each speculative encode reports into its own status words), and every
    JPEG is the oracle's"""
    rng = np.random.default_rng(6)
    cases = []
    for k in range(12):
        rgb = rng.integers(0, 256, (24 + k, 40, 3), dtype=np.uint8)
        cases.append((p3_text(rgb, 255, rng, comments=0.05 if k == 4 else 0.0), rgb))
    allocs = []
    try:
        files = _device_files(encoder, [d for d, _ in cases], allocs)
        for lanes in (1, 2):
            encoder.set_lanes(lanes)
            codes = encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions())
            assert codes == [0] * len(cases)
            assert encoder.batch_redone() == 1
            for (d_text, n, hdr, d_out, cap, d_len), (data, rgb) in zip(files, cases):
                size = int(np.frombuffer(encoder.d2h(d_len, 4), np.uint32)[0])
                assert encoder.d2h(d_out, size) == oracle.encode(rgb, 255, 2, *spec_tables)
    finally:
        encoder.set_lanes(1)
        for p in allocs:
            encoder.free(p)


def test_convert_device_batch_leading_zeros_8bit(encoder, spec_tables):
    """An 8-bit body with leading zeros ("007", tokens of four or more bytes): the
    comment-free pass for 8-bit samples does not parse such tokens, flags them and the
    file is redone on its own on the general path -- its samples and JPEG exactly the
    oracle's; the clean files of the batch are not redone [ppm.rs:41-77, 247-251:
    str::parse::<u16> accepts leading zeros]"""
    rng = np.random.default_rng(77)
    cases = []
    for k in range(6):
        rgb = rng.integers(0, 256, (20 + k, 36, 3), dtype=np.uint8)
        cases.append((p3_text(rgb, 255, rng, zeros=0.05 if k == 2 else 0.0), rgb))
    assert re.search(rb"\s0[0-9]", cases[2][0])  # (a token with a leading zero)
    allocs = []
    try:
        files = _device_files(encoder, [d for d, _ in cases], allocs)
        codes = encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions())
        assert codes == [0] * len(cases)
        assert encoder.batch_redone() == 1
        for (d_text, n, hdr, d_out, cap, d_len), (data, rgb) in zip(files, cases):
            size = int(np.frombuffer(encoder.d2h(d_len, 4), np.uint32)[0])
            assert encoder.d2h(d_out, size) == oracle.encode(rgb, 255, 2, *spec_tables)
        got, mx = decode_gpu(encoder, cases[2][0])
        assert mx == 255 and np.array_equal(got, cases[2][1])
    finally:
        for p in allocs:
            encoder.free(p)


def _random_file(rng):
    """a random small PPM file: P3 (separators, sometimes comments, signs, leading
    zeros, a broken token, a missing or extra sample, a sample above maxval) or P6"""
    w, h = int(rng.integers(1, 90)), int(rng.integers(1, 70))
    mx = int(rng.choice([255, 255, 255, 100, 1000, 65535]))
    rgb = rng.integers(0, mx + 1, (h, w, 3)).astype(np.uint16)
    if mx < 65535 and rng.random() < 0.1:
        rgb.reshape(-1)[int(rng.integers(0, rgb.size))] = mx + 1 + int(rng.integers(0, 5))
    if rng.random() < 0.15 and mx == 255 and int(rgb.max()) <= 255:
        return b"P6 %d %d 255\n" % (w, h) + rgb.astype(np.uint8).tobytes(), rgb, mx
    r = rng.random()
    data = p3_text(rgb, mx, rng, ws_max=int(rng.integers(1, 4)),
                   comments=0.02 if r < 0.15 else 0.0, plus=0.02 if r < 0.25 else 0.0,
                   zeros=0.03 if r < 0.35 else 0.0)
    k = rng.random()
    if k < 0.06:  # a token that does not parse
        data = data[:-3] + b" 1x "
    elif k < 0.12:  # one sample missing
        data = data.rstrip()
        data = data[:data.rfind(b" ") if b" " in data[-8:] else len(data)]
    elif k < 0.16:  # one sample too many
        data += b" 7 "
    return data, rgb, mx


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_convert_device_batch_fuzz(encoder, spec_tables, seed):
    """dmmt_convert_ppm_device_batch on 40 random files per seed, 1-4 lanes: every
    code the host reader's (then the encoder's range check), every JPEG the
    oracle's"""
    rng = np.random.default_rng(100 + seed)
    cases = [_random_file(rng) for _ in range(40)]
    L = dmmt_jpeg.lib()
    allocs, files, expect = [], [], []
    try:
        for data, rgb, mx in cases:
            hdr = dmmt_jpeg.parse_ppm_header(data)
            cap = L.dmmt_max_jpeg_bytes(max(hdr.width, 1), max(hdr.height, 1), 2)
            d_text, d_out, d_len = encoder.malloc(len(data)), encoder.malloc(cap), encoder.malloc(4)
            allocs += [d_text, d_out, d_len]
            encoder.h2d(d_text, np.frombuffer(data, np.uint8))
            files.append((d_text, len(data), hdr, d_out, cap, d_len))
            code = host_code(data)
            if code == 0 and int(rgb.max()) > mx:
                code = -100
            expect.append((code, None if code else oracle.encode(rgb, mx, 2, *spec_tables)))
        encoder.set_lanes(int(rng.integers(1, 5)))
        codes = encoder.convert_ppm_device_batch(files, dmmt_jpeg.JpegTransformationOptions(), check=False)
        assert codes == [e[0] for e in expect]
        for (d_text, n, hdr, d_out, cap, d_len), (code, jpeg) in zip(files, expect):
            size = int(np.frombuffer(encoder.d2h(d_len, 4), np.uint32)[0])
            assert size == 0 if code else encoder.d2h(d_out, size) == jpeg
    finally:
        encoder.set_lanes(1)
        for p in allocs:
            encoder.free(p)
