"""A short run of the long seeded parity sweep (tests/tools/fuzz_parity.py): random
images through single, Image<f32>, batch and pipelined device encodes, every JPEG
byte-compared with the oracle.  The 100,000-case run is in DESIGN.md §4."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))

pytestmark = pytest.mark.gpu


def test_seeded_sweep_short():
    import fuzz_parity
    res = fuzz_parity.run(cases=300, seed=11, max_side=400, log=lambda line: None)
    assert "mismatch" not in res, res
    assert res["cases"] == 300
