"""numpy twin of the device synthetic-frame generator (kernels.hip k_synthetic).

SURVEY.md 8(d): base = (x + 8y) % 256 (the reference's own pattern,
src/bin/dct_timing.rs:150-160); R = base, G = (base + 85 f + (y >> 3)) % 256,
B = (255 - base + (x >> 4)) % 256; plus per-channel 4-bit noise from
xorshift32(seed ^ (f*W*H + y*W + x)) (bits 0-3 / 4-7 / 8-11), clamped to 255.
Test/bench infrastructure: used to check the device generator and to feed the
CPU baseline the same frames the GPU encodes.
"""
import numpy as np


def synthetic(w, h, frame=0, seed=0x9E3779B9, noise_bits=4):
    y, x = np.mgrid[0:h, 0:w].astype(np.uint64)
    base = (x + 8 * y) % 256
    idx = (np.uint64(frame) * np.uint64(w * h) + y * np.uint64(w) + x) & np.uint64(0xFFFFFFFF)
    s = (np.uint64(seed) ^ idx) & np.uint64(0xFFFFFFFF)
    s = (s ^ (s << np.uint64(13))) & np.uint64(0xFFFFFFFF)
    s = s ^ (s >> np.uint64(17))
    s = (s ^ (s << np.uint64(5))) & np.uint64(0xFFFFFFFF)
    m = np.uint64((1 << noise_bits) - 1)
    r = base + (s & m)
    g = ((base + np.uint64(85 * frame) + (y >> np.uint64(3))) % 256) + ((s >> np.uint64(4)) & m)
    b = ((np.uint64(255) - base + (x >> np.uint64(4))) % 256) + ((s >> np.uint64(8)) & m)
    return np.minimum(np.stack([r, g, b], -1), 255).astype(np.uint8)
