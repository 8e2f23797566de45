import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dmmt-jpeg-encoder_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import dmmt_jpeg  # noqa: E402  (imports torch first when present: one HIP runtime per process)
import oracle  # noqa: E402
from oracle import ppm  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); runs the HIP path through the C ABI")


@pytest.fixture(scope="session")
def presets():
    return json.load(open(os.path.join(GOLDEN, "quantization_presets.json")))


@pytest.fixture(scope="session")
def spec_tables(presets):
    return presets[0]["luma"], presets[0]["chroma"]


def load_fixture_images():
    imgs = {}
    for f in ("16x16", "8x8", "7x17", "small"):
        imgs[f] = ppm.read_p3(open(os.path.join(GOLDEN, f + ".ppm"), "rb").read())
    z = np.load(os.path.join(GOLDEN, "500x500_rgb.npz"))
    imgs["500x500"] = (z["rgb"], int(z["maxval"]))
    return imgs


@pytest.fixture(scope="session")
def fixture_images():
    return load_fixture_images()


@pytest.fixture(scope="session")
def encoder():
    """The GPU encoder.  No skip: a gpu test without the library or device fails."""
    if not os.path.exists(dmmt_jpeg.LIB_PATH):
        dmmt_jpeg.build()
    enc = dmmt_jpeg.Encoder(0)
    yield enc
    enc.close()


from oracle.synth import synthetic  # noqa: E402,F401  (numpy twin of the device generator)
