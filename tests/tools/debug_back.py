"""Back half only (dmmt_encode_coefficients from the oracle's blocks), repeated:
agreement with the oracle's encode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402
from oracle.synth import synthetic  # noqa: E402

w, h, sub, q = [int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (1920, 1080, 0, 95))]
luma, chroma = dmmt_jpeg.quality_tables(q)
opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                           chroma_table=chroma)
rgb = synthetic(w, h, frame=q)
ob = oracle.encode(rgb, 255, sub, luma, chroma, threads=8)
oc = oracle.forward(rgb, 255, sub, luma, chroma)
enc = dmmt_jpeg.Encoder(0)
print(os.environ.get("DMMT_LIB_PATH", "lib")[-28:], [enc.encode_coefficients(oc, w, h, opts) == ob for _ in range(4)])
