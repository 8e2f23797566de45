"""Back half from crafted coefficient blocks: the oracle's blocks with the AC zeroed,
or with the DC zeroed; reports agreement with the oracle over repeats."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402
from oracle.synth import synthetic  # noqa: E402

w, h, sub, q = 1920, 1080, 0, 95
luma, chroma = dmmt_jpeg.quality_tables(q)
opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                           chroma_table=chroma)
rgb = synthetic(w, h, frame=q)
oc = oracle.forward(rgb, 255, sub, luma, chroma)
enc = dmmt_jpeg.Encoder(0)
for name, blocks in (("dc only", np.where(np.arange(64) == 0, oc, 0).astype(np.int16)),
                     ("ac only", np.where(np.arange(64) == 0, 0, oc).astype(np.int16)),
                     ("ac only, dc 5", np.where(np.arange(64) == 0, 5, oc).astype(np.int16)),
                     ("as is", oc)):
    ob = oracle.encode_coefficients(blocks, w, h, sub, luma, chroma)
    print(os.environ.get("DMMT_LIB_PATH", "lib")[-28:], name,
          [enc.encode_coefficients(blocks, w, h, opts) == ob for _ in range(3)], flush=True)
