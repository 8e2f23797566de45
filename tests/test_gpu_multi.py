"""Several GPUs behind one C-ABI context (dmmt_ctx_create_multi).

The reference's fan-out seam is ThreadPool::new(n) (lib.rs:62) handed to
transform_on_threadpool (cosine_transform.rs:55-73); here a context of n member
contexts with one host thread each.  The box has one GPU, so the members are n
contexts on GPU 0: the protocol (stripes, exchanges on the host, seams) is the
same whatever GPU each member drives.  Every output must be byte-identical to the
single-context encode and to the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

import dmmt_jpeg
import oracle
from conftest import GOLDEN, PKG, synthetic

pytestmark = pytest.mark.gpu

MCU_W = {0: 8, 1: 16, 2: 16}
MCU_H = {0: 8, 1: 8, 2: 16}


class _Member(dmmt_jpeg.Encoder):
    """a view of a group's member context (borrowed: the group destroys it)"""

    def __init__(self, handle):
        self._ctx = dmmt_jpeg.ctypes.c_void_p(handle)

    def close(self):
        pass


def _opts(sub, q, ri=0):
    luma, chroma = dmmt_jpeg.quality_tables(q)
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma, restart_interval=ri)


@pytest.fixture(scope="module")
def group4():
    g = dmmt_jpeg.Encoder(devices=[0, 0, 0, 0])
    yield g
    g.close()


def test_group_shape(group4):
    assert group4.num_devices() == 4
    assert all(group4.member(i) for i in range(4)) and group4.member(4) == 0
    e = dmmt_jpeg.Encoder(0)
    try:
        assert e.num_devices() == 1 and e.member(0) == e.handle.value
    finally:
        e.close()


def test_members_on_their_devices(group4):
    """dmmt_ctx_check_device after work on every member: each member's worker thread
    runs on the member's GPU and every pooled buffer (lane workspaces, tables, the
    group's staging) lies there -- the readiness check the group workers also run
    before each member's part of a call (here all members are GPU 0)"""
    rgb = synthetic(300, 260, frame=3)
    img = dmmt_jpeg.Image.from_array(rgb)
    ref = oracle.encode(rgb, 255, 2, *dmmt_jpeg.quality_tables(75))
    assert group4.encode_striped(img, _opts(2, 75)) == ref
    assert group4.encode_batch([img] * 5, _opts(2, 75)) == [ref] * 5
    assert group4.check_device() == 0
    for i in range(4):
        assert _Member(group4.member(i)).check_device() == 0
    e = dmmt_jpeg.Encoder(0)
    try:
        assert e.check_device() == 0  # before any buffer exists
        assert e.encode(img, _opts(2, 75)) == ref
        assert e.check_device() == 0
    finally:
        e.close()


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("shape", [(120, 200), (37, 53), (16, 16), (8, 5), (257, 129), (64, 64)])
@pytest.mark.parametrize("ri_rows", [0, 1, 2])
def test_group_encode_equals_single(encoder, group4, sub, shape, ri_rows):
    """dmmt_jpeg_encode on a 4-member context: stripes (fewer where the image has
    fewer MCU rows), joined mid-byte without restart intervals"""
    h, w = shape
    rgb = synthetic(w, h, frame=h * 7 + w)
    mcux = -(-w // MCU_W[sub])
    opts = _opts(sub, 75, ri_rows * mcux)
    img = dmmt_jpeg.Image.from_array(rgb)
    whole = encoder.encode(img, opts)
    assert group4.encode(img, opts) == whole
    assert whole == oracle.encode(rgb, 255, sub, opts.luma_table, opts.chroma_table,
                                  restart_interval=opts.restart_interval)


@pytest.mark.parametrize("ri", [1, 3, 7, 50])
def test_group_restart_intervals_not_a_row(encoder, group4, ri):
    """restart intervals that are not whole MCU rows: stripes of whole intervals
    (a stripe starts where an interval and an MCU row start together)"""
    rgb = synthetic(100, 90, frame=ri)
    opts = _opts(0, 80, ri)
    img = dmmt_jpeg.Image.from_array(rgb)
    assert group4.encode(img, opts) == encoder.encode(img, opts)


@pytest.mark.parametrize("n_stripes", [1, 2, 3, 4])
def test_encode_striped_counts(encoder, group4, n_stripes):
    rgb = synthetic(320, 240, frame=n_stripes)
    opts = _opts(2, 90)
    img = dmmt_jpeg.Image.from_array(rgb)
    assert group4.encode_striped(img, opts, n_stripes) == encoder.encode(img, opts)
    with pytest.raises(dmmt_jpeg.Error):  # one context: no stripes of its own
        encoder.encode_striped(img, opts, 2)
    assert encoder.encode_striped(img, opts, 1) == encoder.encode(img, opts)


def test_group_4k_8_members(encoder):
    """BASELINE config 2's frame over eight members, both stripe modes"""
    rgb = synthetic(3840, 2160, frame=21)
    g = dmmt_jpeg.Encoder(devices=[0] * 8)
    try:
        for ri in (0, 480):
            opts = _opts(0, 90, ri)
            img = dmmt_jpeg.Image.from_array(rgb)
            data = g.encode(img, opts)
            assert data == encoder.encode(img, opts)
            assert data == oracle.encode(rgb, 255, 0, opts.luma_table, opts.chroma_table, threads=8, parallel=True,
                                         restart_interval=ri)
    finally:
        g.close()


def test_group_batch_round_robin(encoder, group4):
    frames = [synthetic(96 + 16 * (i % 3), 64, frame=i) for i in range(11)]  # mixed geometry
    opts = _opts(1, 60)
    imgs = [dmmt_jpeg.Image.from_array(f) for f in frames]
    assert group4.encode_batch(imgs, opts) == encoder.encode_batch(imgs, opts)


def test_group_errors(group4):
    opts = _opts(0, 75)
    bad = np.full((16, 16, 3), 9, np.uint16)
    with pytest.raises(dmmt_jpeg.Error) as e:  # a sample above maxval, found by a member
        group4.encode(dmmt_jpeg.Image(16, 16, 8, bad), opts)
    assert e.value.code == -100
    with pytest.raises(dmmt_jpeg.Error) as e:
        group4.encode_batch([dmmt_jpeg.Image.from_array(synthetic(16, 16)), dmmt_jpeg.Image(16, 16, 8, bad)], opts)
    assert e.value.code == -100
    # the group still works afterwards
    rgb = synthetic(48, 48, frame=3)
    assert group4.encode(dmmt_jpeg.Image.from_array(rgb), opts) == oracle.encode(rgb, 255, 0, opts.luma_table,
                                                                                 opts.chroma_table)
    for ids in ([], [0] * 65, [99]):
        with pytest.raises(dmmt_jpeg.Error):
            dmmt_jpeg.Encoder(devices=ids)


def test_group_device_resident(encoder, group4):
    """dmmt_encode_device_multi (frames in each member's HBM) and
    dmmt_encode_striped_device (stripes in the members' HBM)"""
    w, h = 256, 160
    opts = _opts(2, 85)
    mall, frames = [], []
    stride = (dmmt_jpeg.max_jpeg_bytes(w, h, 2) + 255) // 256 * 256
    try:
        for i in range(4):
            m = _Member(group4.member(i))
            d_in, d_out, d_len = m.malloc(w * h * 3 * 2), m.malloc(stride * 2), m.malloc(8)
            m.fill_synthetic(d_in, w, h, 2, first_frame=2 * i)
            mall.append((m, d_in, d_out, d_len))
            f = dmmt_jpeg.DmmtDeviceFrames()
            f.d_rgb, f.frame_stride, f.n_frames = d_in, w * h * 3, 2
            f.width, f.height, f.maxval, f.sample_bytes = w, h, 255, 1
            f.d_out, f.out_stride, f.d_out_len = d_out, stride, d_len
            frames.append(f)
        group4.encode_device_multi(frames, opts)
        group4.synchronize()
        for i, (m, d_in, d_out, d_len) in enumerate(mall):
            lens = np.frombuffer(m.d2h(d_len, 8), np.uint32)
            for j in range(2):
                got = m.d2h(d_out + j * stride, int(lens[j]))
                rgb = synthetic(w, h, frame=2 * i + j)
                assert got == oracle.encode(rgb, 255, 2, opts.luma_table, opts.chroma_table)
        # stripes: member k holds MCU rows of one image (10 MCU rows over 4 members)
        rgb = synthetic(w, h, frame=40)
        for ri in (0, w // 16):
            o = _opts(2, 85, ri)
            sts, outs, caps = [], [], []
            for k, (m, d_in, d_out, d_len) in enumerate(mall):
                row0, rows = dmmt_jpeg.stripe_rows(h // 16, 4, k)
                px = np.ascontiguousarray(rgb[row0 * 16:(row0 + rows) * 16])
                m.h2d(d_in, px)
                st = dmmt_jpeg.Encoder.stripe(d_in, w, h, row0, rows)
                sts.append(st)
                outs.append(d_out)
                caps.append(stride * 2)
            lens = group4.encode_striped_device(sts, o, outs, caps)
            data = b"".join(mall[k][0].d2h(outs[k], lens[k]) for k in range(4))
            assert data == oracle.encode(rgb, 255, 2, o.luma_table, o.chroma_table, restart_interval=ri)
    finally:
        for m, d_in, d_out, d_len in mall:
            m.free(d_in)
            m.free(d_out)
            m.free(d_len)


def test_group_convert_ppm_and_cli(tmp_path):
    src = os.path.join(GOLDEN, "7x17.ppm")
    rgb_img = dmmt_jpeg.PPMImageReader(open(src, "rb").read()).read_image()
    g = dmmt_jpeg.Encoder(devices=[0, 0, 0])
    try:
        out = tmp_path / "g.jpg"
        dmmt_jpeg.convert_ppm_to_jpeg(dmmt_jpeg.Arguments(src, str(out)), encoder=g)
        spec = dmmt_jpeg.quantization_preset(0)
        ref = oracle.encode(rgb_img.samples, rgb_img.maxval, 2, spec[0], spec[1])
        assert out.read_bytes() == ref
    finally:
        g.close()
    # the CLI over three contexts on GPU 0, both stripe modes
    cli = os.path.join(PKG, "bin", "dmmt-jpeg-encoder")
    big = tmp_path / "big.ppm"
    rgb = synthetic(200, 120, frame=9)
    big.write_bytes(b"P3\n200 120\n255\n" + " ".join(str(int(v)) for v in rgb.reshape(-1)).encode() + b"\n")
    for extra, ri in ((["--devices", "0,0,0"], 0), (["--devices", "0,0,0", "--restart-interval", "13"], 13)):
        o = tmp_path / f"cli{ri}.jpg"
        subprocess.run([cli, str(big), str(o), "-p", "P444", "--quality", "70"] + extra, check=True, timeout=60)
        opts = _opts(0, 70, ri)
        assert o.read_bytes() == oracle.encode(rgb, 255, 0, opts.luma_table, opts.chroma_table, restart_interval=ri)


@pytest.mark.timeout(300)
def test_multi_gpu_c_driver():
    """tools/multi_gpu.cpp: the same checks through the C ABI alone (no Python)"""
    exe = os.path.join(PKG, "bin", "multi_gpu")
    for args in (["3840", "2160", "0", "90", "8", "0,0,0,0,0,0,0,0", "8"], ["1920", "1080", "2", "75", "3", "0,0,0", "5"]):
        r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["match"] and line["members"] == int(args[4]) and line["batch"]["mismatched"] == 0


def test_bench_inproc_leg_on_the_gpu():
    """bench.py --inproc through the real C-ABI group (two members on GPU 0): the
    contract's one JSON line, every member's pixels counted, JPEGs of the
    workload's size (the stand-in group of tests/test_bench_dist.py checks the
    arithmetic; this runs the real dmmt_encode_device_multi pipeline)"""
    import bench
    lines = []
    bench.main(["--inproc", "--devices", "0,0", "--steps", "4", "--warmup", "1", "--cpu-seconds", "0",
                "--ppm-steps", "0"], emit=lines.append)
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["metric"] == "Mpixel/s encoded (4K PPM, q=90)" and d["n_gpus"] == 1 and d["steps"] == 4
    assert d["config"]["members"] == 2 and d["config"]["device_ids"] == [0, 0]
    assert d["value"] > 0 and d["scaling"] == "weak"
    assert 4e6 < d["config"]["mean_jpeg_bytes"] < 7e6  # a 4K q90 synthetic frame: ~5.3 MB
