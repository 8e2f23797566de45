"""Find the first block whose decoded coefficients differ between a GPU encode and
the oracle's, for a few image sizes; print the block, its chunk and its neighbours."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402
from oracle import jpeg_scan  # noqa: E402
from oracle.synth import synthetic  # noqa: E402

enc = dmmt_jpeg.Encoder(0)
done = False
for (w, h, sub, q) in [(640, 480, 2, 95), (1024, 768, 2, 95), (1920, 1080, 2, 95), (1920, 1080, 0, 95), (2048, 2048, 2, 98)]:
    luma, chroma = dmmt_jpeg.quality_tables(q)
    opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                               chroma_table=chroma)
    rgb = synthetic(w, h, frame=q)
    ob = oracle.encode(rgb, 255, sub, luma, chroma, threads=8)
    res = [enc.encode(dmmt_jpeg.Image.from_array(rgb), opts) for _ in range(3)]
    print(w, h, sub, q, [r == ob for r in res], flush=True)
    if done:
        continue
    for g in res:
        if g != ob:
            oc = oracle.forward(rgb, 255, sub, luma, chroma)
            try:
                _, gc, _ = jpeg_scan.decode_coefficients(g)
            except Exception as e:  # noqa: BLE001
                print("decode failed", e)
                break
            n = min(len(gc), len(oc))
            bad = np.nonzero((gc[:n] != oc[:n]).any(axis=1))[0]
            print("differing decoded blocks", len(bad), bad[:8].tolist())
            b = int(bad[0])
            print("chunk", b // 256, "pos in chunk", b % 256)
            print("gpu   ", gc[b].tolist())
            print("oracle", oc[b].tolist())
            nz = np.nonzero(oc[b])[0]
            print("oracle last nz", nz.max() if len(nz) else 0)
            done = True
            break
