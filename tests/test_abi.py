"""CPU-side checks of the C ABI: the library loads, exports every function
include/dmmt_jpeg.h declares, host-only entry points behave like the reference,
and -- without a GPU -- the product refuses to run instead of falling back."""
import ctypes
import os
import re

import numpy as np
import pytest

import dmmt_jpeg
import oracle
from oracle import ppm
from conftest import GOLDEN, ROOT


def declared_functions():
    hdr = open(os.path.join(ROOT, "include", "dmmt_jpeg.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(dmmt_[a-z0-9_]+)\s*\(", hdr)))


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(dmmt_jpeg.LIB_PATH):
        dmmt_jpeg.build()
    return dmmt_jpeg.lib()


def test_exports_every_declared_symbol(L):
    names = declared_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_presets_match_reference_tables(L, presets):
    for i, p in enumerate(presets):
        luma, chroma = dmmt_jpeg.quantization_preset(i)
        assert luma == p["luma"] and chroma == p["chroma"], p["name"]


def test_preset_names_and_aliases():
    Q = dmmt_jpeg.QuantizationTablePreset
    assert Q.from_name("Spec") == Q.Specification == Q.from_name("0") == Q.from_name("Default")
    assert Q.from_name("8") == Q.AnImprovedDetectionModel
    assert Q.from_name("PSNR-HVS-N-Kodak-Tuned") == Q.from_name("4")


def test_quality_tables(L, presets):
    l50, c50 = dmmt_jpeg.quality_tables(50)
    assert l50 == presets[0]["luma"] and c50 == presets[0]["chroma"]
    l90, _ = dmmt_jpeg.quality_tables(90)
    assert l90[0] == 3 and min(l90) >= 1
    l1, _ = dmmt_jpeg.quality_tables(1)
    assert max(l1) == 255
    with pytest.raises(dmmt_jpeg.Error):
        dmmt_jpeg.quality_tables(0)


def test_quality_tables_match_libjpeg(L):
    """dmmt_quality_tables(q) (the IJG quality extension) against an
    independent implementation: libjpeg's jpeg_set_quality(q, force_baseline)
    through Pillow, whose decoded DQT tables come back in natural order, for every
    q = 1..100.  The reference has no quality factor; q50 is its Specification
    preset (quantization_tables.rs:286-327), checked in test_quality_tables."""
    Image = pytest.importorskip("PIL.Image")
    import io
    im = Image.fromarray(np.zeros((8, 8, 3), np.uint8))
    for q in range(1, 101):
        buf = io.BytesIO()
        im.save(buf, "JPEG", quality=q)
        t = Image.open(io.BytesIO(buf.getvalue())).quantization
        luma, chroma = dmmt_jpeg.quality_tables(q)
        assert list(t[0]) == list(luma), q
        assert list(t[1]) == list(chroma), q


def test_default_options(L):
    o = dmmt_jpeg.DmmtOptions()
    L.dmmt_default_options(ctypes.byref(o))
    assert o.subsampling == 2 and o.bits_per_channel == 8 and o.restart_interval == 0
    assert list(o.luma_q)[:4] == [16, 11, 10, 16]


@pytest.mark.parametrize("name", ["16x16", "8x8", "7x17", "small"])
def test_ppm_reader_matches_reference_tokenizer(L, name):
    data = open(os.path.join(GOLDEN, name + ".ppm"), "rb").read()
    img = dmmt_jpeg.PPMImageReader(data).read_image()
    rgb, mx = ppm.read_p3(data)
    assert img.maxval == mx and img.width == rgb.shape[1] and img.height == rgb.shape[0]
    assert np.array_equal(img.samples.astype(np.uint16), rgb)


@pytest.mark.parametrize("text,code", [
    (b"", -1), (b"P5 1 1 255 0 0 0", -1), (b"P3 1", -1), (b"P3 x 1 255", -2), (b"P3 1 1 255 0 0", -3),
    (b"P3 2 1 255 0 0 0", -4), (b"P3 1 1 255 0 0 0 1 1 1", -4), (b"P3 1 1 70000 0 0 0", -2),
    (b"P3 1 1 255 0 256 0", -100), (b"P3 1 1 15 0 16 0", -100), (b"P3 1 1 255 0 0 -1", -2)])
def test_ppm_errors(L, text, code):  # ppm.rs:145-252 error variants
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.PPMImageReader(text).read_image()
    assert e.value.code == code


def test_ppm_tokenizer_quirks(L):
    # '#' comment: its newline is swallowed and does not end the token (ppm.rs:50-55)
    data = b"P3\n# c\n1 1\n255\n1#x\n2 3 4"
    img = dmmt_jpeg.PPMImageReader(data).read_image()
    assert img.samples.reshape(-1).tolist() == [12, 3, 4]
    assert ppm.read_p3(data)[0].reshape(-1).tolist() == [12, 3, 4]
    assert dmmt_jpeg.PPMImageReader(b"P3 1 1 +255 +1 2 3").read_image().maxval == 255


def test_ppm_p6_and_16bit(L):
    rgb = np.arange(12, dtype=np.uint8).reshape(2, 2, 3)
    img = dmmt_jpeg.PPMImageReader(b"P6\n2 2\n255\n" + rgb.tobytes()).read_image()
    assert np.array_equal(img.samples, rgb)
    img = dmmt_jpeg.PPMImageReader(b"P3 1 1 1000 999 0 1000").read_image()
    assert img.samples.dtype == np.uint16 and img.samples.reshape(-1).tolist() == [999, 0, 1000]


def test_error_names(L):
    assert L.dmmt_error_name(-4) == b"MismatchOfSizeBetweenHeaderAndValues"
    assert L.dmmt_error_name(-17) == b"HuffmanSymbolNotPresentInTranslator"
    assert b"no CPU fallback" in L.dmmt_strerror(-202)


def test_max_jpeg_bytes(L):
    assert dmmt_jpeg.max_jpeg_bytes(3840, 2160, 0) > 3840 * 2160 * 3
    assert dmmt_jpeg.max_jpeg_bytes(0, 10, 0) == 0


def test_no_gpu_fails_loudly(L):
    if dmmt_jpeg.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.Encoder(0)
    assert e.value.code == -202  # DMMT_E_NO_DEVICE: no CPU fallback exists


def test_product_does_not_reference_the_oracle():
    pkg = os.path.join(ROOT, "dmmt-jpeg-encoder_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h", "Makefile")):
                src = open(os.path.join(dirpath, f)).read()
                assert "cpu_ref" not in src and "import oracle" not in src and "libcpu_ref" not in src, f


def _category(v):
    return int(abs(int(v))).bit_length()


def test_stripe_fix_dc_hist(L):
    """joined stripes: a stripe's first DC difference per component, counted from
    predictor 0 by the stripe, moves to the category of (first - previous stripe's
    last), as i16 (categorize.rs:153-169)"""
    rng = np.random.default_rng(3)
    for _ in range(50):
        hist = rng.integers(1, 1000, dmmt_jpeg.STRIPE_HIST_WORDS).astype(np.uint64)
        first = [int(x) for x in rng.integers(-1024, 1024, 3)]
        prev = [int(x) for x in rng.integers(-1024, 1024, 3)]
        out = dmmt_jpeg.Encoder.stripe_fix_dc_hist(hist, first, prev)
        want = hist.copy()
        for i, base in enumerate((0, 272, 272)):
            want[base + _category(first[i])] -= 1
            d = ((first[i] - prev[i] + 32768) % 65536) - 32768
            want[base + _category(d)] += 1
        assert np.array_equal(out, want)


def test_stripe_seam_composition():
    """(B_k, next_bits, next16) equal a slice of the concatenated stripe bit strings,
    including stripes shorter than 16 bits and the end of the scan"""
    rng = np.random.default_rng(5)
    for _ in range(200):
        n = int(rng.integers(1, 9))
        lens = [int(x) for x in rng.integers(0, 40, n)]
        strs = ["".join(rng.choice(["0", "1"], size=m)) for m in lens]
        f16 = [int((s[:16] + "0" * 16)[:16], 2) for s in strs]
        whole = "".join(strs)
        for k in range(n):
            b, nb, nx = dmmt_jpeg.stripe_seam(lens, f16, k)
            assert b == sum(lens[:k])
            tail = whole[b + lens[k]:b + lens[k] + 16]
            assert nb == len(tail)
            assert nx == (int((tail + "0" * 16)[:16], 2) if tail else 0)


@pytest.mark.parametrize("text,w,h,mx,binary,off", [
    (b"P3\n2 1\n255\n1 2 3 4 5 6", 2, 1, 255, 0, 11),
    (b"P3 # c\n2 1 # d 9\n255 1", 2, 1, 255, 0, 21),   # comments swallowed with their newline
    (b"P3 2 1 25#x\n5 1", 2, 1, 255, 0, 14),           # a comment inside the max value token
    (b"P6\n3 4\n65535\n", 3, 4, 65535, 1, 13),
    (b"P3 1 1 255", 1, 1, 255, 0, 10)])                # maxval ended by the end of the file
def test_ppm_header(L, text, w, h, mx, binary, off):  # ppm.rs:145-222 on the host
    hd = dmmt_jpeg.parse_ppm_header(text)
    assert (hd.width, hd.height, hd.maxval, hd.binary, hd.body_offset) == (w, h, mx, binary, off)
    if not binary:  # the body from body_offset holds exactly the reference tokenizer's sample tokens
        toks = list(ppm.tokens(text))
        assert list(ppm.tokens(text[off:])) == toks[4:]


def test_ppm_header_errors(L):
    for text, code in [(b"", -1), (b"P5 1 1 1", -1), (b"P3 1 1", -1), (b"P3 1 x 1", -2)]:
        with pytest.raises(dmmt_jpeg.Error) as e:
            dmmt_jpeg.parse_ppm_header(text)
        assert e.value.code == code


def test_multi_gpu_context_without_a_gpu(L):
    """dmmt_ctx_create_multi: bad arguments are refused before any device is
    touched; without a gfx950 GPU it fails like dmmt_ctx_create (no CPU fallback)"""
    out = ctypes.c_void_p()
    ids = (ctypes.c_int * 2)(0, 0)
    assert L.dmmt_ctx_create_multi(ids, 0, ctypes.byref(out)) == -102
    assert L.dmmt_ctx_create_multi(None, 2, ctypes.byref(out)) == -102
    big = (ctypes.c_int * 65)()
    assert L.dmmt_ctx_create_multi(big, 65, ctypes.byref(out)) == -102
    rc = L.dmmt_ctx_create_multi(ids, 2, ctypes.byref(out))
    if rc == 0:  # pragma: no cover - only on a GPU host
        L.dmmt_ctx_destroy(out)
    else:
        assert rc == -202 and not out.value
    assert L.dmmt_ctx_num_devices(None) == 0


# ppm.rs:266-306, the reference's own PPM unit tests, as data
PPM_KATS = [
    ("read_string", "P3\n# Example PPM image string\n3 2\n255\n255 0 0   0 255 0   0 0 255\n255 255 0  255 0 255  0 255 255",
     None),
    ("read_continuous_string", "P3 3 2 255 255 0 0   0 255 0   0 0 255 255 255 0  255 0 255  0 255 255", None),
    ("read_newline_string", "P3\n# Example PPM image newlines\n3\n2\n255\n255\n0\n0\n0\n255\n0\n0\n0\n255\n255\n255\n0\n"
     "255\n0\n255\n0\n255\n255", None),
    ("incomplete_pixel", "P3\n3 2 255 0 0 255 0 0", (-3, 2)),
    ("wrong_size", "P3\n3 2 255 0 0 255", (-4, None)),
]


@pytest.mark.parametrize("name,text,err", PPM_KATS, ids=[k[0] for k in PPM_KATS])
def test_reference_ppm_unit_tests(L, name, text, err):
    """ppm.rs:266-306 through the host reader (PPMImageReader::read_image)"""
    if err is None:
        img = dmmt_jpeg.PPMImageReader(text.encode()).read_image()
        assert img.height == 2 and img.width == 3
        assert img.samples.reshape(-1).tolist()[:6] == [255, 0, 0, 0, 255, 0]
        return
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.PPMImageReader(text.encode()).read_image()
    assert e.value.code == err[0]
    if err[1] is not None:  # IncompletePixelParsed(n), n == 2 (ppm.rs:290-293)
        assert e.value.n == err[1]
        assert "Expected 3 components, but got 2." in str(e.value)


@pytest.mark.parametrize("text,code,token", [(b"", -1, "P3 Header"), (b"P5 1 1 255", -1, "P3 Header"),
                                             (b"P3 1", -1, "Height Header"), (b"P3 x 1 255", -2, "Width Header"),
                                             (b"P3 1 1 99999 0 0 0", -2, "Max Value Header"),
                                             (b"P3 1 1 255 0 0 -1", -2, "Color Component Value")])
def test_ppm_error_payload_token_names(L, text, code, token):
    """error.rs:28-33: the token errors name the token (ppm.rs:80-84)"""
    with pytest.raises(dmmt_jpeg.Error) as e:
        dmmt_jpeg.PPMImageReader(text).read_image()
    assert e.value.code == code and f"'{token}'" in str(e.value)


def test_build_info_reports_no_sdwa_peephole(L):
    """every device object is built without the SDWA peephole (no gain with it:
    profiles/r05_sdwa_ab.txt); the library says so"""
    info = L.dmmt_build_info().decode()
    assert "-amdgpu-sdwa-peephole=false" in info and "gfx950" in info


def test_no_64bit_op_reads_the_last_allocated_vgpr(L):
    """the round-3 k_emit fault pattern (profiles/r03_kemit_fault_study.md, round 5):
    a 64-bit shift whose shift amount is the last VGPR of its kernel's allocation
    computed wrong bits on MI355X; no 64-bit VALU operation of the product library
    reads that register (tools/last_vgpr_check.py, from the built code objects)"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("last_vgpr_check", os.path.join(ROOT, "tools", "last_vgpr_check.py"))
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    hits, kernels = [], 0
    for co in chk.code_objects(dmmt_jpeg.LIB_PATH):
        h, n = chk.check_object(co)
        hits += h
        kernels += n
    assert kernels >= 20 and not hits, hits


@pytest.mark.timeout(300)
def test_last_vgpr_check_flags_the_probe(tmp_path):
    """the checker finds the pattern where it is: tools/last_vgpr_probe.hip (the
    standalone reproduction) built as a library has 64-bit shifts reading v63, the
    last of its kernels' 64 VGPRs, and a control shift reading v62"""
    import importlib.util
    import shutil
    import subprocess
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not installed")
    lib = tmp_path / "libprobe.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-shared", "-fPIC", "-o", str(lib),
                    os.path.join(ROOT, "tools", "last_vgpr_probe.hip")], check=True, capture_output=True)
    spec = importlib.util.spec_from_file_location("last_vgpr_check", os.path.join(ROOT, "tools", "last_vgpr_check.py"))
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    hits = []
    for co in chk.code_objects(str(lib)):
        hits += chk.check_object(co)[0]
    flagged = {ins.split()[0] for _, cnt, last, ins in hits if last == 63 and cnt == 64}
    assert {"v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64"} <= flagged
    assert not any("v62" in ins for _, _, _, ins in hits)
    # the same probe as a compressed offload bundle (--offload-compress): unpacked with
    # clang-offload-bundler, the same hits
    clib = tmp_path / "libprobe_c.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "--offload-compress", "-shared", "-fPIC",
                    "-o", str(clib), os.path.join(ROOT, "tools", "last_vgpr_probe.hip")], check=True,
                   capture_output=True)
    assert chk.elf_section(str(clib), ".hip_fatbin")[:4] == b"CCOB"
    chits = []
    for co in chk.code_objects(str(clib)):
        chits += chk.check_object(co)[0]
    assert sorted(chits) == sorted(hits)
