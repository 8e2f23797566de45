"""The reference's own known-answer tests, ported as data, run
against the CPU oracle.  Each test cites the reference test it restates."""
import numpy as np
import pytest

import oracle
from oracle import jpeg_scan


def f32(x):
    return np.float32(x)


# ---- color.rs:106-209
def test_rgb_to_ycbcr_ranges():  # color.rs:106-129
    y, cb, cr = oracle.rgb_to_ycbcr(0.25, 0.75, 0.333)
    assert 12.95 <= y < 13.05 and -31.68 <= cb < -31.58 and -55.13 <= cr < -55.03


def test_rgb_white_and_black():  # color.rs:131-167
    y, cb, cr = oracle.rgb_to_ycbcr(1.0, 1.0, 1.0)
    assert 126.99999 <= y <= 127.00001 and -0.5 <= cb <= 0.5 and -0.5 <= cr <= 0.5
    assert oracle.rgb_to_ycbcr(0.0, 0.0, 0.0) == (-128.0, 0.0, 0.0)


def test_normalize():  # color.rs:169-209
    assert 7.209e-3 <= oracle.normalize(128, 17734) <= 7.219e-3
    assert oracle.normalize(0xFFFF, 0xFFFF) == 1.0
    assert 0.133333 <= oracle.normalize(2, 15) <= 0.133334
    assert oracle.normalize(15, 15) == 1.0


def test_k128_constant_bits():  # 128/255 as f32 is 0x3f008081
    assert np.float32(128.0) / np.float32(255.0) == np.frombuffer(np.uint32(0x3F008081).tobytes(), np.float32)[0]


# ---- subsampling.rs:332-550
CH1 = np.arange(1, 17, dtype=np.float32).reshape(4, 4)
CH2 = np.arange(1, 65, dtype=np.float32).reshape(8, 8)


def test_block_iter_with_single_fit_image():  # subsampling.rs:441-462
    out = oracle.subsample_resort(CH1, 1, 1, False, square=4)
    assert np.array_equal(out, CH1.reshape(-1))


def test_square_resorter_with_1x1_subsampling():  # subsampling.rs:464-491
    out = oracle.subsample_resort(CH2, 1, 1, False, square=4)
    expect = [1, 2, 3, 4, 9, 10, 11, 12, 17, 18, 19, 20, 25, 26, 27, 28, 5, 6, 7, 8, 13, 14, 15, 16, 21, 22, 23, 24,
              29, 30, 31, 32, 33, 34, 35, 36, 41, 42, 43, 44, 49, 50, 51, 52, 57, 58, 59, 60, 37, 38, 39, 40, 45, 46,
              47, 48, 53, 54, 55, 56, 61, 62, 63, 64]
    assert list(out) == expect


def test_square_resorter_with_2x2_subsampling():  # subsampling.rs:493-518 (Skip)
    out = oracle.subsample_resort(CH2, 2, 2, False, square=4)
    assert list(out) == [1, 3, 5, 7, 17, 19, 21, 23, 33, 35, 37, 39, 49, 51, 53, 55]


def test_square_resorter_with_1x2_subsampling():  # subsampling.rs:520-550 (Skip, vertical 2)
    out = oracle.subsample_resort(CH2, 1, 2, False, square=4)
    assert list(out) == [1, 2, 3, 4, 17, 18, 19, 20, 33, 34, 35, 36, 49, 50, 51, 52, 5, 6, 7, 8, 21, 22, 23, 24, 37,
                         38, 39, 40, 53, 54, 55, 56]


def test_average_subsampling():  # average_subsampling_test, subsampling.rs:372-393: rate 1x2 -> (6+10)/2... at (1,1)
    out = oracle.subsample_resort(CH1, 1, 2, True, square=2)
    # row view 1 = rows 2..3, column 1: (10 + 14) / 2 = 12; resorted index of (sy 1, sx 1) with square 2 is 3
    assert out.reshape(-1)[3] == 12.0


def test_resort_8x8_squares_16x16():
    p = np.arange(256, dtype=np.float32).reshape(16, 16)
    out = oracle.subsample_resort(p, 1, 1, False).reshape(4, 8, 8)
    assert np.array_equal(out[1], p[0:8, 8:16]) and np.array_equal(out[2], p[8:16, 0:8])


def test_average_2x2_sum_order():  # Subsampler::rect order x outer, y inner (subsampling.rs:108-122)
    p = np.zeros((16, 16), np.float32)
    p[0, 0], p[1, 0], p[0, 1], p[1, 1] = 1e8, 1.0, -1e8, 1.0
    out = oracle.subsample_resort(p, 2, 2, True)
    expect = (((f32(1e8) + f32(1.0)) + f32(-1e8)) + f32(1.0)) / f32(4)
    assert out[0] == expect and expect == f32(0.25)


# ---- arai.rs:186-219
TEST_VALUES = np.array([
    1, 2, 1, 2, 3, 2, 3, 2, 3, 2, 1, 2, 3, 4, 3, 2, 3, 4, 3, 2, 3, 4, 5, 6, 7, 6, 5, 4, 3, 2, 3, 2,
    3, 4, 5, 5, 6, 5, 2, 3, 4, 3, 2, 3, 4, 5, 4, 3, 2, 3, 4, 5, 6, 5, 4, 3, 2, 3, 4, 5, 3, 4, 3, 4], np.float32)
A1, A2, A4, A5 = f32(0.70710678118654752440), f32(0.5411961), f32(1.3065629), f32(0.3826834)
A3 = A1
S = [f32(v) for v in (0.3535533, 0.2548978, 0.27059805, 0.30067244, 0.35355338, 0.4499881, 0.6532815, 1.2814577)]


def closed_form(i):
    """arai.rs:117-166 y0..y7, evaluated left to right in f32"""
    i = [f32(v) for v in i]
    s = f32(0)
    for v in i:
        s = s + v
    y0 = s * S[0]
    y4 = (i[0] + i[7] + i[3] + i[4] - i[1] - i[6] - i[2] - i[5]) * S[4]
    y2 = ((i[0] + i[1] - i[2] - i[3] - i[4] - i[5] + i[6] + i[7]) * A1 + i[0] + i[7] - i[3] - i[4]) * S[2]
    y6 = ((i[0] + i[1] - i[2] - i[3] - i[4] - i[5] + i[6] + i[7]) * -A1 + i[0] + i[7] - i[3] - i[4]) * S[6]
    y5 = (A2 * (i[3] - i[4] + i[2] - i[5]) + A5 * (i[3] - i[4] + i[2] - i[5] - i[1] + i[6] - i[0] + i[7]) + i[0] - i[7]
          - A3 * (i[2] - i[5] + i[1] - i[6])) * S[5]
    t = i[1] - i[6] + i[0] - i[7]
    y1 = (i[0] - i[7] + A3 * (i[2] - i[5] + i[1] - i[6]) + A4 * t - A5 * (t - i[3] + i[4] - i[0] + i[7])) * S[1]
    y7 = (i[0] - i[7] + A3 * (i[2] - i[5] + i[1] - i[6]) - A4 * t + A5 * (t - i[3] + i[4] - i[0] + i[7])) * S[7]
    t = i[3] - i[4] + i[2] - i[5]
    y3 = (-A2 * t - A5 * (t - i[1] + i[6] - i[0] + i[7]) + i[0] - i[7] - A3 * (i[2] - i[5] + i[1] - i[6])) * S[3]
    return [y0, y1, y2, y3, y4, y5, y6, y7]


def test_fast_arai_exact_closed_form():  # compare_fast_own, arai.rs:204-219 (assert_eq!)
    out = oracle.fast_arai(TEST_VALUES[:8].copy(), 1)
    assert [float(v) for v in out] == [float(v) for v in closed_form(TEST_VALUES[:8])]


def naive_dct(block):  # simple.rs:45-59 (the O(n^4) transform the reference compares against)
    b = block.reshape(8, 8).astype(np.float64)
    out = np.zeros((8, 8))
    for v in range(8):
        for u in range(8):
            cu = 1 / np.sqrt(2) if u == 0 else 1.0
            cv = 1 / np.sqrt(2) if v == 0 else 1.0
            s = 0.0
            for y in range(8):
                for x in range(8):
                    s += b[y, x] * np.cos((2 * x + 1) * u * np.pi / 16) * np.cos((2 * y + 1) * v * np.pi / 16)
            out[v, u] = 0.25 * cu * cv * s
    return out.reshape(64)


def test_arai_vs_naive():  # test_fast_simple, arai.rs:190-202, tolerance 1e-4
    out = oracle.dct_block(TEST_VALUES)
    assert np.max(np.abs(out - naive_dct(TEST_VALUES))) <= 1e-4


# ---- frequency_block.rs:63-100
def test_zigzag_order():
    data = [0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31,
            40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61,
            35, 36, 48, 49, 57, 58, 62, 63]
    assert [data[z] for z in jpeg_scan.ZIGZAG] == list(range(64))


# ---- categorize.rs:175-289
@pytest.mark.parametrize("v,length,pattern", [
    (57, 6, 0b11100100_00000000), (45, 6, 0b10110100_00000000), (1, 1, 0b10000000_00000000),
    (-30, 5, 0b00001000_00000000), (32767, 15, 0b11111111_11111110), (-32767, 15, 0), (0, 0, 0)])
def test_categorize(v, length, pattern):
    c = oracle.category(v)
    assert c == length and oracle.category_pattern(v, c) == pattern


def test_categorize_min_panics():  # test_categorize_integer_lower_than_min_value
    assert oracle.category(-32768) == -1


def test_sum_zeros_before_values():  # categorize.rs:254-289 via the numpy restatement's tokenizer
    from oracle import np_ref
    seq = [57, 45, 0, 0, 0, 0, 23, 0, -30, -16] + [0] * 19 + [1, 0]
    blk = [99] + seq + [0] * (63 - len(seq))
    toks = np_ref.tokens(np.array(blk))
    expect = [(0, 57), (0, 45), (4, 23), (1, -30), (0, -16), (15, 0), (3, 1), (0, 0)]
    got = [(s >> 4, v) for s, v in toks]
    assert got == expect
    assert [s & 15 for s, _ in toks] == [6, 6, 5, 5, 5, 0, 1, 0]


# ---- length_limited.rs:209-255
@pytest.mark.parametrize("freqs,limit,expect", [
    ([1, 2, 5, 8, 10, 11, 14, 14, 15, 18, 20], 4, [4, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3]),
    ([1, 1, 1, 2, 2, 2, 3, 6, 17, 20], 5, [5, 5, 4, 4, 4, 4, 4, 3, 2, 2]),
    ([1, 1, 1, 2, 2, 2, 3, 6, 17, 20], 4, [4, 4, 4, 4, 4, 4, 4, 4, 2, 2])])
def test_package_merge(freqs, limit, expect):
    assert oracle.package_merge(freqs, limit) == expect
    from oracle import np_ref
    assert np_ref.package_merge(freqs, limit) == expect


def test_package_merge_too_many_symbols():  # test_generate_too_long_input_array (panics)
    with pytest.raises(oracle.OracleError):
        oracle.package_merge([1, 1, 1, 2, 2, 2, 3, 6, 17, 20], 3)


# ---- huffman/encoder.rs:213-269: 32 symbols, limit 6, +1, exact 22 output bytes
SYMFREQ = [(1, 14), (2, 30), (3, 4), (4, 7), (5, 9), (6, 4), (7, 42), (8, 1), (9, 14), (10, 5), (11, 14), (12, 30),
           (13, 4), (14, 7), (15, 9), (16, 4), (17, 42), (18, 1), (19, 14), (20, 5), (21, 14), (22, 30), (23, 4),
           (24, 7), (25, 9), (26, 4), (27, 42), (28, 1), (29, 14), (30, 12), (31, 32), (32, 1)]
SEQ = [27, 17, 7, 31, 22, 12, 2, 29, 21, 19, 11, 9, 1, 30, 25, 15, 5, 24, 14, 4, 20, 10, 26, 23, 16, 13, 6, 3, 32, 28,
       18, 8]
BYTES = [0b00000100, 0b01101000, 0b10101100, 0b11110000, 0b10001100, 0b10100111, 0b01001010, 0b11011010, 0b11101011,
         0b11110000, 0b11000111, 0b00101100, 0b11110100, 0b11010111, 0b01101101, 0b11111000, 0b11100111, 0b10101110,
         0b11111100, 0b11110111, 0b11101111, 0b11000000]


def test_coder_encode_kat():
    syms = sorted(SYMFREQ, key=lambda t: t[1])  # stable sort by frequency
    lens = oracle.package_merge([f for _, f in syms], 6)
    lens[0] += 1
    codes = oracle.assign_codes([s for s, _ in syms], lens)
    acc, n, out = 0, 0, []
    for s in SEQ:
        c, ln = codes[s]
        acc = (acc << ln) | c
        n += ln
    pad = (-n) % 8  # BitWriter::new(.., false): zero padding in this test
    acc <<= pad
    n += pad
    out = list(acc.to_bytes(n // 8, "big"))
    assert out == BYTES


@pytest.mark.parametrize("prev,plen,expect", [(0b1100 << 12, 4, 0b1101 << 12), (0b11010 << 11, 5, 0b11011 << 11),
                                              (0b11110 << 11, 5, 0b11111 << 11)])
def test_calculate_bit_pattern(prev, plen, expect):  # huffman/encoder.rs:271-302
    assert (prev + (1 << (16 - plen))) & 0xFFFF == expect


# ---- symbol_counting.rs:108-198 (via the oracle's histogram inside code_lengths)
def test_code_lengths_stable_order():
    hist = [0] * 256
    for s, f in [(0b00001001, 1), (0b11110000, 4), (0b01000011, 1), (0, 4), (0b00001010, 2), (0b01000100, 1),
                 (0b00000111, 1), (0b00100011, 1), (0b00000001, 1)]:
        hist[s] = f
    syms, lens = oracle.code_lengths(hist)
    # ascending by frequency, equal frequencies in symbol order (stable sort of the filtered list)
    assert syms == [0b00000001, 0b00000111, 0b00001001, 0b00100011, 0b01000011, 0b01000100, 0b00001010, 0, 0b11110000]
    assert lens[0] == max(lens)


# ---- encoder.rs:449-550 segment bytes, checked inside a whole oracle file
def test_segments_in_oracle_file(spec_tables):
    rgb = np.zeros((2, 3, 3), np.uint16)
    data = oracle.encode(rgb, 255, oracle.P444, *spec_tables)
    assert data[:2] == b"\xff\xd8"
    assert data[2:20] == bytes([0xFF, 0xE0, 0x00, 0x10, 74, 70, 73, 70, 0, 1, 2, 0, 0, 0x48, 0, 0x48, 0, 0])
    dqt = bytes([0xFF, 0xDB, 0x00, 0x43, 0x00, 16, 11, 12, 14, 12, 10, 16, 14, 13, 14, 18, 17, 16, 19, 24, 40, 26, 24,
                 22, 22, 24, 49, 35, 37, 29, 40, 58, 51, 61, 60, 57, 51, 56, 55, 64, 72, 92, 78, 64, 68, 87, 69, 55,
                 56, 80, 109, 81, 87, 95, 98, 103, 104, 103, 62, 77, 113, 121, 112, 100, 120, 92, 101, 103, 99])
    assert data[20:89] == dqt  # encoder.rs:519-537 (there with id 2)
    assert data[158:177] == bytes([0xFF, 0xC0, 0, 0x11, 8, 0, 2, 0, 3, 3, 1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1])
    sos = bytes([0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x01, 0x02, 0x23, 0x03, 0x23, 0x00, 0x3F, 0x00])
    assert sos in data and data[-2:] == b"\xff\xd9"


def test_sof_ratio_bytes(spec_tables):  # encoder.rs:855-880
    rgb = np.zeros((8, 8, 3), np.uint16)
    for sub, ratio in ((0, 0x11), (1, 0x21), (2, 0x22)):
        data = oracle.encode(rgb, 255, sub, *spec_tables)
        assert data[158 + 11] == ratio


def test_one_padding_and_stuffing():  # binary_stream.rs:298-306, segment_marker_injector.rs:37-59
    # an all-black 8x8 image: every scan byte pattern ends in 1-padding
    from oracle import np_ref
    blocks = np.zeros((3, 64), np.int16)
    data = np_ref.encode_coefficients(blocks, 8, 8, 0, [1] * 64, [1] * 64)
    assert data == oracle.encode_coefficients(blocks, 8, 8, 0, [1] * 64, [1] * 64)
    jf, dec, pad_ok = jpeg_scan.decode_coefficients(data)
    assert pad_ok and np.array_equal(dec, blocks)
