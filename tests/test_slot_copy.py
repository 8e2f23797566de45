"""CPU unit check of k_emit's clear-free window copy (csrc/slot_copy.hpp, compiled
for the host from the kernel's own source) against a bit-serial model of the
chunk's stream [binary_stream.rs:38-66].

The unmasked replay is the first clear-free build of round 4 (stale slot words
past a block not zeroed): the check must find its fault, and the fault must be
extra 1 bits only -- the symptom of the round-4 `r04_emit1` parity failure
(8K 4:2:0 q95, b'\\x16' -> b'\\x1e'; profiles/STUDIES.md B)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "slot_copy_check.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("slot") / "slot_copy_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unknown-pragmas", "-o", exe, SRC], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_product_copy_matches_bit_serial_stream(checker, seed):
    r = subprocess.run([checker, "1500", str(seed)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok:")


def test_unmasked_copy_is_caught_and_only_adds_bits(checker):
    r = subprocess.run([checker, "1500", "1", "--unmasked"], capture_output=True, text=True)
    assert r.returncode == 1, r.stdout
    assert "FAIL:" in r.stdout and ", 0 of them missing bits" in r.stdout, r.stdout
