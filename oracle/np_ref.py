"""Second, independent restatement of the reference encode path (TEST INFRASTRUCTURE).

numpy float32 for the front half (every ufunc rounds once, no contraction),
pure Python integers for the back half.  Written separately from cpu_ref.c so
the two restatements cross-check each other (tests/test_oracle_crosscheck.py);
only tests import it.  Citations are reference file:line.
"""
from __future__ import annotations

import heapq

import numpy as np

from .jpeg_scan import ZIGZAG

f32 = np.float32

A1 = f32(0.70710678118654752440)  # arai.rs:7 FRAC_1_SQRT_2
A2 = f32(0.5411961)
A3 = A1
A4 = f32(1.3065629)
A5 = f32(0.3826834)
S = [f32(0.3535533), f32(0.2548978), f32(0.27059805), f32(0.30067244), f32(0.35355338), f32(0.4499881),
     f32(0.6532815), f32(1.2814577)]


def rgb_to_ycbcr(r, g, b):
    """color.rs:75-100 on float32 arrays"""
    k = f32(128.0) / f32(255.0)
    y = (((r * f32(0.299) + g * f32(0.587)) + b * f32(0.114)) - k) * f32(255.0)
    cb = ((r * f32(-0.1687) + g * f32(-0.3312)) + b * f32(0.5)) * f32(255.0)
    cr = ((r * f32(0.5) + g * f32(-0.4186)) + b * f32(-0.0813)) * f32(255.0)
    return y, cb, cr


def arai(v):
    """arai.rs:29-92 along the last axis (length 8) of a float32 array."""
    v0, v1, v2, v3, v4, v5, v6, v7 = (v[..., i] for i in range(8))
    v10, v11, v12, v13 = v0 + v7, v1 + v6, v2 + v5, v3 + v4
    v14, v15, v16, v17 = v3 - v4, v2 - v5, v1 - v6, v0 - v7
    v20, v21, v22, v23 = v10 + v13, v11 + v12, v11 - v12, v10 - v13
    v24, v25, v26 = (-v14) - v15, v15 + v16, v16 + v17
    v30, v31, v32 = v20 + v21, v20 - v21, v22 + v23
    v42 = v32 * A1
    v44 = ((-v24) * A2) - ((v24 + v26) * A5)
    v45 = v25 * A3
    v46 = (v26 * A4) - ((v26 + v24) * A5)
    v52, v53, v55, v57 = v42 + v23, v23 - v42, v45 + v17, v17 - v45
    v64, v65, v66, v67 = v44 + v57, v55 + v46, v55 - v46, v57 - v44
    out = np.empty_like(v)
    out[..., 0] = v30 * S[0]
    out[..., 4] = v31 * S[4]
    out[..., 2] = v52 * S[2]
    out[..., 6] = v53 * S[6]
    out[..., 5] = v64 * S[5]
    out[..., 1] = v65 * S[1]
    out[..., 7] = v66 * S[7]
    out[..., 3] = v67 * S[3]
    return out


def dct_blocks(blocks):
    """arai.rs:95-104: rows then columns; blocks shape (n, 8, 8) float32"""
    rows = arai(blocks)
    cols = arai(np.swapaxes(rows, 1, 2))
    return np.swapaxes(cols, 1, 2)


def round_half_away(x):
    t = np.trunc(x)
    frac = x - t  # exact
    return t + np.where(np.abs(frac) >= f32(0.5), np.sign(x), f32(0.0)).astype(np.float32)


def quantize(coef, table):
    """quantizer.rs:60 incl. Rust's saturating `as i16` (NaN -> 0)"""
    x = round_half_away(coef / np.asarray(table, dtype=np.float32).reshape(8, 8))
    x = np.where(np.isnan(x), f32(0), x)
    return np.clip(x, -32768, 32767).astype(np.int16)


def to_blocks(plane):
    """ChannelSquareResorter: (H, W) -> (H/8 * W/8, 8, 8) in block raster order"""
    h, w = plane.shape
    return plane.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8)


def forward(rgb, maxval, preset, luma_q, chroma_q):
    """Front half -> (nblocks, 64) int16 zigzag blocks in MCU emission order."""
    rgb = np.asarray(rgb)
    h, w, _ = rgb.shape
    hr = 1 if preset == 0 else 2
    vr = 2 if preset == 2 else 1
    wp = -(-w // (8 * hr)) * 8 * hr
    hp = -(-h // (8 * vr)) * 8 * vr
    norm = rgb.astype(np.float32) / f32(maxval)
    padded = np.zeros((hp, wp, 3), np.float32)
    padded[:h, :w] = norm
    y, cb, cr = rgb_to_ycbcr(padded[..., 0], padded[..., 1], padded[..., 2])

    def sub(p):
        if preset == 0:
            return p
        if preset == 1:  # rect 2x1: x then x+1
            return (p[:, 0::2] + p[:, 1::2]) / f32(2.0)
        # rect 2x2, x outer / y inner: (x,y) (x,y+1) (x+1,y) (x+1,y+1)
        return (((p[0::2, 0::2] + p[1::2, 0::2]) + p[0::2, 1::2]) + p[1::2, 1::2]) / f32(4.0)

    yb = quantize(dct_blocks(to_blocks(y)), luma_q).reshape(-1, 64)
    cbb = quantize(dct_blocks(to_blocks(sub(cb))), chroma_q).reshape(-1, 64)
    crb = quantize(dct_blocks(to_blocks(sub(cr))), chroma_q).reshape(-1, 64)
    line = wp // 8
    cbx = wp // hr // 8
    out = []
    for m in range(cbb.shape[0]):
        mx, my = m % cbx, m // cbx
        if preset == 0:
            ys = [m]
        elif preset == 1:
            ys = [my * line + 2 * mx, my * line + 2 * mx + 1]
        else:
            r0 = 2 * my * line
            ys = [r0 + 2 * mx, r0 + 2 * mx + 1, r0 + line + 2 * mx, r0 + line + 2 * mx + 1]
        out.extend(yb[i] for i in ys)
        out.append(cbb[m])
        out.append(crb[m])
    blocks = np.stack(out)
    return blocks[:, ZIGZAG]


# ------------------------------------------------------------------ back half

def category(v):
    return abs(int(v)).bit_length()


def tokens(blk):
    """categorize.rs:132-151 -> list of (symbol, value) for the AC part"""
    out = []
    zeros = 0
    for v in blk[1:]:
        v = int(v)
        if v == 0:
            zeros += 1
            continue
        while zeros > 15:
            out.append((0xF0, 0))
            zeros -= 16
        out.append(((zeros << 4) | category(v), v))
        zeros = 0
    if zeros:
        out.append((0x00, 0))
    return out


def package_merge(freqs, limit):
    """length_limited.rs:37-134, written with heapq instead of BinaryHeap"""
    n = len(freqs)
    leaves = [(f, 0) for f in freqs]
    levels = [list(leaves)]
    for _ in range(1, limit):
        prev = levels[-1]
        pk = [(prev[2 * i][0] + prev[2 * i + 1][0], 1) for i in range(len(prev) // 2)]
        levels.append(list(heapq.merge(pk, leaves)))
    lengths = [0] * n
    packages = n - 1
    for lvl in reversed(levels):
        take = lvl[:2 * packages]
        leafs = sum(1 for _, k in take if k == 0)
        packages = len(take) - leafs
        for i in range(leafs):
            lengths[i] += 1
    return lengths


def huffman_table(hist):
    """symbol_counting.rs:55-94 + huffman/encoder.rs:45-119.
    Returns (symbols ascending by frequency, lengths, {symbol: (code, len)})."""
    syms = [s for s in range(len(hist)) if hist[s] > 0]
    syms.sort(key=lambda s: hist[s])  # stable
    lens = package_merge([hist[s] for s in syms], 15)
    lens[0] += 1
    codes = {}
    pat, plen = 0, 0
    for i in range(len(syms) - 1, -1, -1):
        pat = 0 if i == len(syms) - 1 else (pat + (1 << (16 - plen))) & 0xFFFF
        plen = lens[i]
        codes[syms[i]] = (pat >> (16 - plen), plen)
    return syms, lens, codes


def encode_coefficients(blocks, width, height, preset, luma_q, chroma_q, bits=8):
    n_luma = {0: 1, 1: 2, 2: 4}[preset]
    bpm = n_luma + 2
    hist = [[0] * 256 for _ in range(4)]
    last = [0, 0, 0]
    items = []
    for e, blk in enumerate(blocks):
        k = e % bpm
        comp = 0 if k < n_luma else (1 if k == n_luma else 2)
        t = 0 if comp == 0 else 2
        d = int(np.int16(int(blk[0]) - last[comp]))
        last[comp] = int(blk[0])
        c = category(d)
        hist[t][c] += 1
        toks = tokens(blk)
        for s, _ in toks:
            hist[t + 1][s] += 1
        items.append((t, d, toks))
    tabs = [huffman_table(h) for h in hist]
    out = bytearray(b"\xff\xd8")

    def seg(m, content):
        out.extend(bytes([0xFF, m]) + (len(content) + 2).to_bytes(2, "big") + bytes(content))

    seg(0xE0, b"JFIF\x00\x01\x02\x00\x00\x48\x00\x48\x00\x00")
    seg(0xDB, bytes([0] + [luma_q[z] for z in ZIGZAG]))
    seg(0xDB, bytes([1] + [chroma_q[z] for z in ZIGZAG]))
    hr = 1 if preset == 0 else 2
    vr = 2 if preset == 2 else 1
    seg(0xC0, bytes([bits]) + height.to_bytes(2, "big") + width.to_bytes(2, "big")
        + bytes([3, 1, (hr << 4) | vr, 0, 2, 0x11, 1, 3, 0x11, 1]))
    for kind, t in ((0x11, 1), (0x00, 0), (0x13, 3), (0x02, 2)):
        syms, lens, _ = tabs[t]
        bitsc = [0] * 16
        for ln in lens:
            bitsc[ln - 1] += 1
        seg(0xC4, bytes([kind] + bitsc + syms[::-1]))
    seg(0xDA, bytes([3, 1, 1, 2, 0x23, 3, 0x23, 0, 0x3F, 0]))
    acc, nacc = 0, 0
    scan = bytearray()

    def put(v, n):
        nonlocal acc, nacc
        acc = (acc << n) | (v & ((1 << n) - 1))
        nacc += n
        while nacc >= 8:
            b = (acc >> (nacc - 8)) & 0xFF
            scan.append(b)
            if b == 0xFF:
                scan.append(0)
            nacc -= 8
        acc &= (1 << nacc) - 1

    def extra(v, c):
        return v if v > 0 else (1 << c) - 1 + v

    for t, d, toks in items:
        c = category(d)
        code, ln = tabs[t][2][c]
        put(code, ln)
        put(extra(d, c), c)
        for s, v in toks:
            code, ln = tabs[t + 1][2][s]
            put(code, ln)
            c = s & 15
            put(extra(v, c), c)
    if nacc:
        put((1 << (8 - nacc)) - 1, 8 - nacc)
    out.extend(scan)
    out.extend(b"\xff\xd9")
    return bytes(out)
