"""P3 reader restating ppm.rs:41-237 (TEST INFRASTRUCTURE; tests parse fixtures with it).

Tokenizer: '#' starts a comment to end of line, ASCII whitespace separates
tokens (ppm.rs:41-77).  Parser: "P3", width, height, max value (u16 each),
then RGB triples; an incomplete last pixel or a pixel count different from
width*height is an error (ppm.rs:145-252).
"""
from __future__ import annotations

import numpy as np


class PPMError(ValueError):
    pass


def tokens(data: bytes):
    buf = bytearray()
    in_comment = False
    for byte in data:
        if in_comment:
            if byte == 0x0A:
                in_comment = False
            continue
        if byte == 0x23:
            in_comment = True
            continue
        if byte in b" \t\n\x0c\r":
            if buf:
                yield buf.decode()
                buf = bytearray()
        else:
            buf.append(byte)
    if buf:
        yield buf.decode()


def _u16(tok, name):
    # Rust `str::parse::<u16>` (core::num from_str_radix): one optional leading '+',
    # then at least one ASCII digit; no '-' for unsigned types; value <= 65535
    digits = tok[1:] if tok.startswith("+") else tok
    if not digits or any(c not in "0123456789" for c in digits):
        raise PPMError(f"ParsingOfTokenFailed({name})")
    sig = digits.lstrip("0") or "0"  # leading zeros are accepted, however many
    if len(sig) > 5 or int(sig) > 65535:
        raise PPMError(f"ParsingOfTokenFailed({name})")
    return int(sig)


def read_p3(data: bytes):
    """-> (rgb uint16 HxWx3, maxval)"""
    it = tokens(data)
    header = next(it, None)
    if header is None or header != "P3":
        raise PPMError("PPMFileDoesNotContainRequiredToken(P3 Header)")
    w = next(it, None)
    if w is None:
        raise PPMError("PPMFileDoesNotContainRequiredToken(Width Header)")
    w = _u16(w, "Width Header")
    h = next(it, None)
    if h is None:
        raise PPMError("PPMFileDoesNotContainRequiredToken(Height Header)")
    h = _u16(h, "Height Header")
    mx = next(it, None)
    if mx is None:
        raise PPMError("PPMFileDoesNotContainRequiredToken(Max Value Header)")
    mx = _u16(mx, "Max Value Header")
    vals = [_u16(t, "Color Component Value") for t in it]
    if len(vals) % 3:
        raise PPMError(f"IncompletePixelParsed({len(vals) % 3})")
    if len(vals) != 3 * w * h:
        raise PPMError("MismatchOfSizeBetweenHeaderAndValues")
    arr = np.array(vals, dtype=np.uint16).reshape(h, w, 3)
    if (arr > mx).any():
        raise PPMError("value exceeds max (color.rs:63-65 panics)")
    return arr, mx
