"""First differing scan bit between a GPU encode and the oracle, mapped to the block
(emission order) the oracle's stream is in at that bit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402
from oracle import jpeg_scan as js  # noqa: E402
from oracle.synth import synthetic  # noqa: E402

w, h, sub, q = [int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (1920, 1080, 0, 95))]
luma, chroma = dmmt_jpeg.quality_tables(q)
opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                           chroma_table=chroma)
rgb = synthetic(w, h, frame=q)
ob = oracle.encode(rgb, 255, sub, luma, chroma, threads=8)
enc = dmmt_jpeg.Encoder(0)
g = enc.encode(dmmt_jpeg.Image.from_array(rgb), opts)
print("equal", g == ob, len(g), len(ob))
jo, jg = js.parse(ob), js.parse(g)
print("same tables", jo.dht == jg.dht)
bo, bg = js._BitReader(jo.scan).data, js._BitReader(jg.scan).data
i = next((k for k in range(min(len(bo), len(bg))) if bo[k] != bg[k]), None)
print("first differing unstuffed byte", i, "of", len(bo), len(bg))
x = bo[i] ^ bg[i]
bit = 8 * i + (7 - x.bit_length() + 1)
print("first differing bit", bit)
# oracle block starts
tables = {k: js._huff_lookup(*v) for k, v in jo.dht.items()}
br = js._BitReader(jo.scan)
comps = {c[0]: c for c in jo.components}
hmax = max(c[1] for c in jo.components)
vmax = max(c[2] for c in jo.components)
nmcu = -(-jo.width // (8 * hmax)) * -(-jo.height // (8 * vmax))
starts = []
oc = oracle.forward(rgb, 255, sub, luma, chroma)
done = False
for m in range(nmcu):
    for cid, td, ta in jo.scan_components:
        for _ in range(comps[cid][1] * comps[cid][2]):
            starts.append(br.pos)
            if br.pos > bit + 2000:
                done = True
                break
            t = js._decode_symbol(br, tables[(0, td)])
            br.bits(t)
            k = 1
            while k < 64:
                rs = js._decode_symbol(br, tables[(1, ta)])
                r, s = rs >> 4, rs & 15
                if s == 0:
                    if r == 15:
                        k += 16
                        continue
                    break
                k += r + 1
                br.bits(s)
        if done:
            break
    if done:
        break
starts = np.array(starts)
b = int(np.searchsorted(starts, bit, side="right") - 1)
print("block", b, "chunk", b // 256, "pos", b % 256, "block bits", starts[b], "..", starts[b + 1], "len", starts[b + 1] - starts[b])
nz = np.nonzero(oc[b])[0]
print("coef", oc[b].tolist(), "last nz", int(nz.max()) if len(nz) else 0)
def bitstr(data, a, n):
    return "".join(str((data[p >> 3] >> (7 - (p & 7))) & 1) for p in range(a, a + n))
print("oracle", bitstr(bo, starts[b], starts[b + 1] - starts[b]))
print("gpu   ", bitstr(bg, starts[b], starts[b + 1] - starts[b]))
# the chunk's blocks: lengths
c0 = (b // 256) * 256
print("chunk-relative start bit", int(starts[b] - starts[c0]), "byte", int(starts[b] - starts[c0]) / 8.0,
      "diff bit rel block", bit - int(starts[b]), "bits differing in block",
      sum(((bo[p >> 3] ^ bg[p >> 3]) >> (7 - (p & 7))) & 1 for p in range(int(starts[b]), int(starts[b + 1]))))
lens = [int(starts[j + 1] - starts[j]) for j in range(c0, min(c0 + 256, len(starts) - 1))]
print("chunk block bits max", max(lens), "over 384:", sum(1 for L in lens if L > 384), "total", sum(lens))
# decode the first symbols of block b from both streams
for name, data in (("oracle", jo.scan), ("gpu", jg.scan)):
    r = js._BitReader(data)
    r.pos = int(starts[b])
    comp_of = []
    for cid, td, ta in jo.scan_components:
        comp_of += [(td, ta)] * (comps[cid][1] * comps[cid][2])
    td, ta = comp_of[b % len(comp_of)]
    p0 = r.pos
    t = js._decode_symbol(r, tables[(0, td)])
    v = js._extend(r.bits(t), t)
    syms = []
    for _ in range(4):
        rs = js._decode_symbol(r, tables[(1, ta)])
        s_ = rs & 15
        syms.append((rs >> 4, s_, js._extend(r.bits(s_), s_)))
    print(name, "DC cat", t, "diff", v, "AC", syms)
prev = oc[:b]
