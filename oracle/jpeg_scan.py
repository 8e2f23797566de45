"""Baseline JPEG parser / Huffman decoder to quantised coefficients (TEST INFRASTRUCTURE).

Used to pin the back half of the oracle (and of the HIP path) against the file
the reference encoder itself wrote, /root/reference/tests/output_image_2.jpg
(committed as tests/golden/ref_output_image_2.jpg): decode its scan to the
quantised zigzag coefficients, re-encode them, and demand the identical file.
It is also used to sanity-check every encoder output (marker structure, table
ids, scan decodes to exactly the coefficients that were encoded).

Handles what the reference writes: SOF0, 1x1/2x1/2x2 luma sampling with 1x1
chroma, one interleaved scan, no restart markers -- plus DRI/RSTn for the
restart-interval extension of this build.
"""
from __future__ import annotations

import struct

import numpy as np

ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
          13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59,
          52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


class JpegFile:
    def __init__(self):
        self.segments = []  # (marker, payload bytes)
        self.dqt = {}
        self.dht = {}  # (class, id) -> (bits[16], huffval list)
        self.width = self.height = 0
        self.precision = 0
        self.components = []  # (id, h, v, tq)
        self.scan_components = []  # (id, td, ta)
        self.restart_interval = 0
        self.scan = b""  # entropy-coded data incl. RST markers, stuffing intact
        self.trailer = b""


def parse(data: bytes) -> JpegFile:
    if data[:2] != b"\xff\xd8":
        raise ValueError("missing SOI")
    jf = JpegFile()
    pos = 2
    while pos < len(data):
        if data[pos] != 0xFF:
            raise ValueError(f"expected marker at {pos}")
        marker = data[pos + 1]
        if marker == 0xD9:
            jf.trailer = data[pos:]
            break
        (length,) = struct.unpack(">H", data[pos + 2:pos + 4])
        payload = data[pos + 4:pos + 2 + length]
        jf.segments.append((marker, payload))
        pos += 2 + length
        if marker == 0xDB:
            p = 0
            while p < len(payload):
                pq, tq = payload[p] >> 4, payload[p] & 15
                if pq != 0:
                    raise ValueError("16-bit DQT unsupported")
                jf.dqt[tq] = list(payload[p + 1:p + 65])
                p += 65
        elif marker == 0xC4:
            p = 0
            while p < len(payload):
                tc, th = payload[p] >> 4, payload[p] & 15
                bits = list(payload[p + 1:p + 17])
                n = sum(bits)
                vals = list(payload[p + 17:p + 17 + n])
                jf.dht[(tc, th)] = (bits, vals)
                p += 17 + n
        elif marker in (0xC0, 0xC1):
            jf.precision = payload[0]
            jf.height, jf.width = struct.unpack(">HH", payload[1:5])
            nc = payload[5]
            for i in range(nc):
                cid, hv, tq = payload[6 + 3 * i:9 + 3 * i]
                jf.components.append((cid, hv >> 4, hv & 15, tq))
        elif marker == 0xDD:
            (jf.restart_interval,) = struct.unpack(">H", payload[:2])
        elif marker == 0xDA:
            ns = payload[0]
            for i in range(ns):
                cid, t = payload[1 + 2 * i:3 + 2 * i]
                jf.scan_components.append((cid, t >> 4, t & 15))
            # entropy-coded segment runs to the next non-RST, non-stuffed marker
            end = pos
            while True:
                j = data.index(b"\xff", end)
                nxt = data[j + 1]
                if nxt == 0x00 or 0xD0 <= nxt <= 0xD7:
                    end = j + 2
                    continue
                break
            jf.scan = data[pos:j]
            pos = j
    return jf


def _huff_lookup(bits, vals):
    """canonical decode table: (length, code) -> symbol"""
    table = {}
    code = 0
    k = 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            table[(length, code)] = vals[k]
            k += 1
            code += 1
        code <<= 1
    return table


class _BitReader:
    def __init__(self, scan: bytes):
        # remove stuffing; split at RST markers
        self.segments = []
        cur = bytearray()
        i = 0
        while i < len(scan):
            b = scan[i]
            if b == 0xFF:
                nb = scan[i + 1]
                if nb == 0x00:
                    cur.append(0xFF)
                    i += 2
                    continue
                if 0xD0 <= nb <= 0xD7:
                    if nb - 0xD0 != len(self.segments) % 8:  # RSTm cycles 0..7 (T.81 F.1.2.3)
                        raise ValueError("restart marker out of sequence")
                    self.segments.append(bytes(cur))
                    cur = bytearray()
                    i += 2
                    continue
                raise ValueError("unexpected marker in scan")
            cur.append(b)
            i += 1
        self.segments.append(bytes(cur))
        self.seg = 0
        self._load()

    def _load(self):
        self.data = self.segments[self.seg]
        self.nbits = len(self.data) * 8
        self.pos = 0

    def next_segment(self):
        self.seg += 1
        self._load()

    def bit(self):
        if self.pos >= self.nbits:
            raise ValueError("scan exhausted")
        p = self.pos
        self.pos = p + 1
        return (self.data[p >> 3] >> (7 - (p & 7))) & 1

    def bits(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

    def remaining_padding_ok(self):
        """all bits after pos must be ones (1-padding), and < 8 of them"""
        rest = self.nbits - self.pos
        if rest >= 8:
            return False
        return rest == 0 or (self.data[-1] & ((1 << rest) - 1)) == (1 << rest) - 1


def _decode_symbol(br, table):
    code = 0
    for length in range(1, 17):
        code = (code << 1) | br.bit()
        s = table.get((length, code))
        if s is not None:
            return s
    raise ValueError("bad huffman code")


def _extend(v, t):
    return v if t == 0 or v >= (1 << (t - 1)) else v - (1 << t) + 1


def decode_coefficients(data: bytes):
    """Decode a baseline JPEG to quantised zigzag coefficient blocks in MCU
    emission order.  Returns (JpegFile, ndarray[nblocks, 64] int16, padding_ok)."""
    jf = parse(data)
    comps = {c[0]: c for c in jf.components}
    hmax = max(c[1] for c in jf.components)
    vmax = max(c[2] for c in jf.components)
    mcux = -(-jf.width // (8 * hmax))
    mcuy = -(-jf.height // (8 * vmax))
    tables = {k: _huff_lookup(*v) for k, v in jf.dht.items()}
    br = _BitReader(jf.scan)
    pred = {c[0]: 0 for c in jf.scan_components}
    blocks = []
    nmcu = mcux * mcuy
    ri = jf.restart_interval
    padding_ok = True
    for m in range(nmcu):
        if ri and m and m % ri == 0:
            padding_ok &= br.remaining_padding_ok()
            br.next_segment()
            pred = {c[0]: 0 for c in jf.scan_components}
        for cid, td, ta in jf.scan_components:
            _, h, v, _ = comps[cid]
            for _ in range(h * v):
                blk = np.zeros(64, dtype=np.int16)
                t = _decode_symbol(br, tables[(0, td)])
                diff = _extend(br.bits(t), t)
                pred[cid] += diff
                blk[0] = pred[cid]
                k = 1
                while k < 64:
                    rs = _decode_symbol(br, tables[(1, ta)])
                    r, s = rs >> 4, rs & 15
                    if s == 0:
                        if r == 15:
                            k += 16
                            continue
                        break
                    k += r
                    blk[k] = _extend(br.bits(s), s)
                    k += 1
                blocks.append(blk)
    padding_ok &= br.remaining_padding_ok()
    return jf, np.stack(blocks) if blocks else np.zeros((0, 64), np.int16), padding_ok
