"""Time ppm_ingest (bench.py's PPM leg) with whatever library DMMT_LIB_PATH names.
usage: python scripts/ppm_probe.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dmmt_jpeg  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
enc = dmmt_jpeg.Encoder(0)
print(json.dumps(bench.ppm_ingest(enc, 3840, 2160, steps)))
