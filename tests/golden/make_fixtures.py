"""Regenerate the committed fixtures under tests/golden/ (run in the build container).

1. quantization_presets.json: the 7 presets, parsed as data from the reference's
   src/image/writer/jpeg/quantization_tables.rs (QuantizationTablePreset order,
   quantization_tables.rs:232-243 / 286-327), natural order.
2. 500x500_rgb.npz: the reference's tests/500x500.ppm (P3, 2.2 MB) as uint8 array.
3. The reference's own files are copied verbatim: 16x16.ppm, 8x8.ppm, 7x17.ppm,
   small.ppm (inputs), output_image.jpg / output_image_2.jpg (reference-encoder
   outputs, renamed ref_*.jpg).
4. oracle_*.jpg: JPEGs written by the CPU oracle for every fixture x preset x
   subsampling (regression pins; the oracle itself is pinned by the KATs and
   ref_*.jpg).

Usage: python tests/golden/make_fixtures.py [/root/reference]
"""
import json
import os
import re
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from oracle import ppm  # noqa: E402

ORDER = [
    ("SPECIFICATION", "Specification"), ("FLAT", "Flat"), ("MSSIM_KODAK_TUNED", "MSSIMKodakTuned"),
    ("PSNRHVSNI_KODAK_TUNED", "PSNRHVSNKodakTuned"),
    ("DC_TUNE_PERCEPTUAL_OPTIMIZATION", "DCTunePerceptualOptimization"),
    ("A_VISUAL_DETECTION_MODEL", "AVisualDetectionModel"), ("AN_IMPROVED_DETECTION_MODEL", "AnImprovedDetectionModel"),
]


def parse_presets(path):
    src = open(path).read()
    out = []
    for const, name in ORDER:
        tabs = []
        for kind in ("LUMINANCE", "CHROMINANCE"):
            m = re.search(r"pub const %s_%s_QUANTIZATION_TABLE: \[u8; 64\] =\s*\[(.*?)\];" % (const, kind), src, re.S)
            vals = [int(v) for v in re.findall(r"\d+", m.group(1))]
            assert len(vals) == 64, (const, kind)
            tabs.append(vals)
        out.append({"name": name, "luma": tabs[0], "chroma": tabs[1]})
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    if os.path.isdir(ref):
        presets = parse_presets(os.path.join(ref, "src/image/writer/jpeg/quantization_tables.rs"))
        json.dump(presets, open(os.path.join(HERE, "quantization_presets.json"), "w"), indent=0)
        for f in ("16x16.ppm", "8x8.ppm", "7x17.ppm", "small.ppm"):
            shutil.copyfile(os.path.join(ref, "tests", f), os.path.join(HERE, f))
        shutil.copyfile(os.path.join(ref, "tests/output_image.jpg"), os.path.join(HERE, "ref_output_image.jpg"))
        shutil.copyfile(os.path.join(ref, "tests/output_image_2.jpg"), os.path.join(HERE, "ref_output_image_2.jpg"))
        rgb, mx = ppm.read_p3(open(os.path.join(ref, "tests/500x500.ppm"), "rb").read())
        np.savez_compressed(os.path.join(HERE, "500x500_rgb.npz"), rgb=rgb.astype(np.uint8), maxval=np.array(mx))
    presets = json.load(open(os.path.join(HERE, "quantization_presets.json")))
    images = {f: ppm.read_p3(open(os.path.join(HERE, f + ".ppm"), "rb").read()) for f in ("16x16", "8x8", "7x17", "small")}
    z = np.load(os.path.join(HERE, "500x500_rgb.npz"))
    images["500x500"] = (z["rgb"], int(z["maxval"]))
    manifest = {}
    for name, (rgb, mx) in images.items():
        for sub in (0, 1, 2):
            for pi, p in enumerate(presets):
                data = oracle.encode(rgb, mx, sub, p["luma"], p["chroma"])
                fn = f"oracle_{name}_P{['444', '422', '420'][sub]}_q{pi}.jpg"
                open(os.path.join(HERE, fn), "wb").write(data)
                manifest[fn] = {"image": name, "subsampling": sub, "preset": pi, "bytes": len(data)}
    json.dump(manifest, open(os.path.join(HERE, "oracle_manifest.json"), "w"), indent=0, sort_keys=True)
    print(f"wrote {len(manifest)} oracle goldens")


if __name__ == "__main__":
    main()
