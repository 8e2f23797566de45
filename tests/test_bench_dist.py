"""The N>1 bench path on CPU: two ranks over gloo, a stand-in encoder.

bench.py's multi-GPU contract: every rank encodes its own
frames (independent images, weak scaling, no data-path collective); the timed
region is bracketed by barriers; the elapsed time is the MAX over ranks; rank 0
prints one JSON line whose `value` is the whole-job pixel rate.  The stand-in
encoder records which synthetic frames each rank generated and sleeps a
rank-dependent time per step so the MAX reduction is observable.
"""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))

STEP_SLEEP = {0: 0.001, 1: 0.004}  # rank 1 is the slow one


class StandInEncoder:
    def __init__(self, local_rank, rank, log):
        self.rank, self.log = rank, log
        self.mem = {}
        self.mask = 0

    def malloc(self, n):
        h = len(self.mem) + 1
        self.mem[h] = n
        return h

    def free(self, h):
        self.mem.pop(h, None)

    def fill_synthetic(self, d, w, h, n_frames, first_frame=0, seed=0x9E3779B9):
        self.log.append(("frames", self.rank, first_frame, n_frames))

    def encode_device(self, d_in, n, w, h, opts, d_out, out_stride, d_len, frame_stride=0, opt_c=None):
        time.sleep(STEP_SLEEP[self.rank])

    def synchronize(self):
        pass

    def check_device(self):
        return self.rank

    def set_lanes(self, n):
        self.log.append(("lanes", self.rank, n))

    def set_profiling(self, mask):
        self.mask = mask

    def profile(self):
        # summed ms and launches per stage (dmmt_ctx_profile): k_emit the longest
        return {"front": (0.05 * 3, 3), "hist": (0.02 * 3, 3), "tables": (0.01 * 3, 3), "emit": (0.06 * 3, 3),
                "offsets": (0.005 * 3, 3), "stuffwrite": (0.007 * 3, 3)}

    def d2h(self, d, n):
        return np.full(n // 4, 1000, np.uint32).tobytes()

    def close(self):
        pass

    # the stripe calls of BASELINE config 4 (extra_configs)
    def fill_synthetic_rows(self, d, w, h, row0, rows, frame=0):
        self.log.append(("rows", self.rank, row0, rows))

    stripe = staticmethod(lambda *a, **k: __import__("dmmt_jpeg").Encoder.stripe(*a, **k))
    stripe_max_bytes = staticmethod(lambda st, opts: 1 << 20)

    def stripe_analyze(self, st, opts):
        self.log.append(("analyze", self.rank, st.mcu_row0, st.mcu_rows))
        h = np.zeros(544, np.uint64)
        h[0] = h[16] = h[272] = h[288] = 7  # a DC and an AC symbol per table
        return h

    def stripe_encode(self, hist, d_out, cap):
        self.log.append(("stripe_encode", self.rank, int(np.asarray(hist)[0])))
        time.sleep(STEP_SLEEP[self.rank])
        return 1000 + self.rank

    def stripe_dc_edges(self):
        return [1, 2, 3], [4, 5, 6]

    def stripe_measure(self, hist, prev, d_out, cap):
        self.log.append(("measure", self.rank, list(prev)))
        return 8000 + 3 * self.rank, 0xABCD

    def stripe_write(self, bit_offset, next_bits, next16):
        time.sleep(STEP_SLEEP[self.rank])
        return 1001


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import bench
    log, lines = [], []
    bench.main(["--gpus", str(world), "--steps", "20", "--warmup", "2", "--cpu-seconds", "0", "--ppm-steps", "0",
                "--config", "1080p420q75x256", "--no-extras"],
               make_encoder=lambda lr: StandInEncoder(lr, rank, log), emit=lines.append)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"log": log, "lines": lines}, f)


def _worker_same_device(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import bench
    log, lines = [], []

    def make(lr):
        log.append(("local_rank", rank, lr))
        return StandInEncoder(lr, rank, log)

    bench.main(["--gpus", str(world), "--steps", "5", "--warmup", "1", "--cpu-seconds", "0", "--ppm-steps", "0",
                "--config", "1080p420q75x256", "--same-device", "--no-extras"], make_encoder=make, emit=lines.append)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"log": log, "lines": lines}, f)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    r0 = json.load(open(tmp_path / "rank0.json"))
    r1 = json.load(open(tmp_path / "rank1.json"))
    assert len(r0["lines"]) == 1 and r1["lines"] == []  # one JSON line, rank 0 only
    line = json.loads(r0["lines"][0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["steps"] == 20
    # distinct synthetic frames per rank (no two ranks encode the same frames)
    f0 = {tuple(x[2:]) for x in r0["log"] if x[0] == "frames"}
    f1 = {tuple(x[2:]) for x in r1["log"] if x[0] == "frames"}
    # untimed settle steps, then the timed steps, pipelined over the default lanes, then one at a
    # time with events (roofline), then one at a time without them (the plain one-lane latency)
    assert [x[2] for x in r0["log"] if x[0] == "lanes"] == [4, 4, 1, 1]
    assert line["config"]["settle"]["frames"] >= 32 * 256 and line["config"]["settle"]["ms"] >= 60
    assert line["config"]["lanes"] == 4 and line["config"]["single_lane_ms_per_step"] > 0
    assert f0 and f1 and not (f0 & f1)
    # elapsed is the MAX over ranks: at least the slow rank's sleeps
    assert line["ms_per_step"] >= STEP_SLEEP[1] * 1e3 * 0.9
    # value = whole-job pixels / elapsed
    w, h, fps = 1920, 1080, 256
    expect = w * h * fps * 20 * world / (line["ms_per_step"] * 20 / 1e3) / 1e6
    assert line["value"] == pytest.approx(expect, rel=2e-3)
    assert line["config"]["parallelism"] == "independent frames x2"
    # the line validates itself: each rank's own time and rate, its device, the world
    ranks = line["config"]["ranks"]
    assert ranks["world_size"] == 2 and ranks["backend"] == "gloo" and ranks["devices"] == [0, 1]
    assert ranks["one_device_per_rank"] and max(ranks["seconds"]) == pytest.approx(line["ms_per_step"] * 20 / 1e3,
                                                                                   rel=1e-3)
    # (barrier-bracketed: the slow rank bounds both, up to the ranks' barrier-exit skew,
    # a few ms on a loaded CPU)
    assert ranks["seconds"][1] > ranks["seconds"][0] * 0.9
    for sec, rate in zip(ranks["seconds"], ranks["mpixel_s"]):
        assert rate == pytest.approx(w * h * fps * 20 / sec / 1e6, rel=1e-3)


@pytest.mark.timeout(300)
def test_bench_same_device_rehearsal(tmp_path):
    """--same-device (the N>1 path rehearsed on a one-GPU box): every rank's
    encoder is created on device 0 and the collectives go over gloo"""
    world = 2
    mp.start_processes(_worker_same_device, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    r0 = json.load(open(tmp_path / "rank0.json"))
    r1 = json.load(open(tmp_path / "rank1.json"))
    assert [x[2] for x in r0["log"] + r1["log"] if x[0] == "local_rank"] == [0, 0]
    line = json.loads(r0["lines"][0])
    assert line["n_gpus"] == 2 and line["config"]["ranks"]["backend"] == "gloo"


def test_bench_line_fields_single_rank(monkeypatch):
    """N = 1, the BASELINE config (4K 4:4:4 q90): the roofline block names the
    longest kernel of the events pass, prices every kernel's launch against the
    SURVEY 8(d) bytes of the frame, and carries the committed PMC counters."""
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    import bench
    log, lines = [], []
    bench.main(["--steps", "5", "--warmup", "1", "--cpu-seconds", "0", "--ppm-steps", "0", "--no-extras"],
               make_encoder=lambda lr: StandInEncoder(lr, 0, log), emit=lines.append)
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["metric"] == "Mpixel/s encoded (4K PPM, q=90)"
    cfg = line["config"]
    assert cfg["input_slots"] == 12 and cfg["input_slots"] * 3840 * 2160 * 3 > 256 * 2**20  # past the MALL
    assert cfg["single_lane_ms_per_step"] > 0 and cfg["single_lane_plain_ms_per_step"] > 0
    rf = line["roofline"]
    assert rf["kernel"] == "k_emit" and rf["bound"] == "hbm" and rf["peak"] == 8000.0 and rf["unit"] == "GB/s"
    algo = 3840 * 2160 * 3 + 1000  # RGB in + the stand-in's JPEG bytes
    assert rf["algorithmic_bytes_per_launch"] == algo
    assert rf["avg_launch_us"] == pytest.approx(60.0)
    assert rf["frac"] == pytest.approx(algo / 60e-6 / 1e9 / 8000.0, rel=1e-3)
    assert set(rf["kernels"]) == {"k_front", "k_hist", "k_tables", "k_emit", "k_offsets", "k_stuffwrite"}
    for name, k in rf["kernels"].items():
        assert k["frac"] == pytest.approx(algo / (k["avg_launch_us"] * 1e-6) / 1e9 / 8000.0, rel=1e-2)
    pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_4k444q90.json")))
    assert rf["traffic"] == round(pmc["kernels"]["k_emit"]["hbm_bytes"])
    assert rf["kernels"]["k_front"]["valu_wave_insts"] == round(pmc["kernels"]["k_front"]["SQ_INSTS_VALU"])
    assert line["cpu_baseline"] is None and line["ppm_ingest"] is None


def make_standin(local_rank):
    """picklable encoder factory for the spawned ranks"""
    return StandInEncoder(local_rank, local_rank, [])


@pytest.mark.timeout(300)
def test_bench_gpus_flag_spawns_ranks(monkeypatch):
    """`bench.py --gpus 2` without a launcher (no WORLD_SIZE) starts the two rank
    processes itself and reports n_gpus 2."""
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    import bench
    lines = []
    bench.main(["--gpus", "2", "--steps", "10", "--warmup", "1", "--cpu-seconds", "0", "--ppm-steps", "0",
                "--config", "1080p420q75x256", "--no-extras"], make_encoder=make_standin, emit=lines.append)
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "independent frames x2"
    assert line["ms_per_step"] >= STEP_SLEEP[1] * 1e3 * 0.9  # the MAX over ranks


def test_bench_refuses_world_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    import bench
    with pytest.raises(SystemExit):
        bench.main(["--gpus", "4", "--steps", "1", "--warmup", "0", "--cpu-seconds", "0", "--ppm-steps", "0"],
                   make_encoder=lambda lr: StandInEncoder(lr, 0, []), emit=lambda l: None)


class StandInGroup:
    """a multi-device context stand-in: members record their frames, the group
    records each enqueue (one batch of frames per member per call)"""

    def __init__(self, ids, log):
        self.ids, self.log = list(ids), log
        self.members = [StandInEncoder(0, i, log) for i in range(len(ids))]

    def num_devices(self):
        return len(self.ids)

    def member_encoder(self, i):
        return self.members[i]

    def set_lanes(self, n):
        self.log.append(("group_lanes", n))

    def encode_device_multi(self, frames, opts):
        assert len(frames) == len(self.ids)
        self.log.append(("multi", tuple(int(f.d_rgb) for f in frames), tuple(int(f.n_frames) for f in frames)))
        time.sleep(0.001)

    def synchronize(self):
        self.log.append(("sync",))

    def close(self):
        self.log.append(("close",))


def test_bench_inproc_group(monkeypatch):
    """`bench.py --gpus 4 --inproc`: one process, the C ABI's multi-GPU context
    (dmmt_ctx_create_multi); each step is one dmmt_encode_device_multi call with
    one batch per member, every member encoding its own distinct frames; value =
    all members' pixels / elapsed, weak scaling.  Repeated ids (--devices 0,0)
    rehearse it on one GPU."""
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    import bench
    for argv, ids in ((["--gpus", "4"], [0, 1, 2, 3]), (["--gpus", "1", "--devices", "0,0"], [0, 0])):
        log, lines, made = [], [], []

        def make_group(i, log=log, made=made):
            made.append(list(i))
            return StandInGroup(i, log)
        bench.main(argv + ["--inproc", "--steps", "6", "--warmup", "2", "--cpu-seconds", "0", "--ppm-steps", "0"],
                   make_group=make_group, emit=lines.append)
        assert made == [ids] and len(lines) == 1
        line = json.loads(lines[0])
        n = len(ids)
        assert line["n_gpus"] == len(set(ids)) and line["scaling"] == "weak" and line["config"]["members"] == n
        assert line["config"]["device_ids"] == ids
        calls = [x for x in log if x[0] == "multi"]
        assert len(calls) == 8  # warmup + steps, one call per step
        # distinct synthetic frames for every member
        firsts = [x[2] for x in log if x[0] == "frames"]
        assert len(firsts) == len(set(firsts)) == n * line["config"]["input_slots_per_member"]
        expect = n * 3840 * 2160 * 6 / (line["ms_per_step"] * 6 / 1e3) / 1e6
        assert line["value"] == pytest.approx(expect, rel=2e-3)
        assert log[-1] == ("close",)


def test_path_roofline_over_the_launched_kernels():
    """roofline.path's issue ceiling sums the PMC of the kernels the step launched:
    with the chunk offsets fused into k_emit there is no k_offsets launch, and the
    ceiling is still reported; a launched kernel without PMC leaves it null"""
    import bench

    pmc = {"kernels": {n: {"SQ_INSTS_VALU": 1e6, "SQ_INSTS_SALU": 5e5}
                       for n in ("k_front", "k_hist", "k_tables", "k_emit", "k_stuffwrite", "k_ppm_fast")}}
    fused = {"k_front", "k_hist", "k_tables", "k_emit", "k_stuffwrite"}
    p = bench.path_roofline(30e6, 500.0, 50e-6, pmc, fused)
    assert p["valu_wave_insts"] == 5_000_000 and p["salu_wave_insts"] == 2_500_000
    assert p["valu_frac"] == round(5e6 / 50e-6 / bench.VALU_PEAK_PER_S, 4)
    assert bench.path_roofline(30e6, 500.0, 50e-6, pmc, fused | {"k_offsets"})["valu_frac"] is None
    assert bench.path_roofline(30e6, 500.0, 50e-6, None, fused)["valu_frac"] is None


def _worker_extras(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import bench
    log, lines = [], []
    bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--ppm-steps", "0",
                "--extra-steps", "2"], make_encoder=lambda lr: StandInEncoder(lr, rank, log), emit=lines.append)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"log": log, "lines": lines}, f)


@pytest.mark.timeout(300)
def test_bench_extra_configs_two_ranks(tmp_path):
    """`bench.py --gpus 2` (the driver's SCALE command) prints configs 2, 4 and 5 in
    its one line: after the 4K headline, extra_configs holds BASELINE config 4 (the
    32768^2 image as one MCU-row stripe per rank, with restart intervals and
    joined) and config 5 (8K 4:2:0 streams at q50/75/95), each with its own ranks
    block; the stripes' histograms are summed over the ranks on the host (gloo)"""
    world = 2
    mp.start_processes(_worker_extras, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    r0 = json.load(open(tmp_path / "rank0.json"))
    r1 = json.load(open(tmp_path / "rank1.json"))
    assert len(r0["lines"]) == 1 and r1["lines"] == []
    line = json.loads(r0["lines"][0])
    assert line["metric"] == "Mpixel/s encoded (4K PPM, q=90)" and line["n_gpus"] == 2
    ex = line["extra_configs"]
    assert list(ex) == ["32k420r", "32k420", "8k420q50", "8k420q75", "8k420q95"]
    for name in ("32k420r", "32k420"):
        e = ex[name]
        assert "error" not in e, e
        assert e["scaling"] == "strong" and e["n_gpus"] == 2 and e["steps"] == 2
        assert e["config"]["ranks"]["world_size"] == 2 and e["config"]["ranks"]["devices"] == [0, 1]
        assert e["value"] == pytest.approx(32768 * 32768 * 2 / (e["ms_per_step"] * 2 / 1e3) / 1e6, rel=2e-3)
        assert e["config"]["parallelism"] == "MCU-row stripes x2"
    # every rank analysed its own half of the 2048 MCU rows, in each stripe mode
    a0 = {tuple(x[2:]) for x in r0["log"] if x[0] == "analyze"}
    a1 = {tuple(x[2:]) for x in r1["log"] if x[0] == "analyze"}
    assert a0 == {(0, 1024)} and a1 == {(1024, 1024)}
    # the restart-interval stripes encode with the SUM of both ranks' histograms
    assert {x[2] for x in r0["log"] + r1["log"] if x[0] == "stripe_encode"} == {14}
    # joined stripes: rank 1's DC predictors continue rank 0's last DCs
    assert {tuple(x[2]) for x in r1["log"] if x[0] == "measure"} == {(4, 5, 6)}
    for q in (50, 75, 95):
        e = ex[f"8k420q{q}"]
        assert "error" not in e, e
        assert e["scaling"] == "weak" and e["steps"] == 8 and e["config"]["quality"] == q
        assert e["config"]["ranks"]["world_size"] == 2
        assert e["value"] == pytest.approx(7680 * 4320 * 8 * 2 / (e["ms_per_step"] * 8 / 1e3) / 1e6, rel=2e-3)


def test_bench_no_extras_by_flag(monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    import bench
    lines = []
    bench.main(["--steps", "2", "--warmup", "0", "--cpu-seconds", "0", "--ppm-steps", "0", "--no-extras"],
               make_encoder=lambda lr: StandInEncoder(lr, 0, []), emit=lines.append)
    assert "extra_configs" not in json.loads(lines[0])
