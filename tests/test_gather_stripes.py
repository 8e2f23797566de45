"""dmmt_jpeg.gather_striped on CPU: the stripes of the ranks land in rank order in
root's file buffer, over gloo with three processes -- a root that
is not rank 0, an empty stripe, parts with slack after their bytes -- and a tiling
that does not add up is refused on every rank."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SIZES = [5, 0, 7]


def _part(rank):
    return bytes((rank * 40 + i) & 0xFF for i in range(SIZES[rank]))


def _rank(rank, world, port, out_dir, root, bad):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
    import torch
    import torch.distributed as dist
    import dmmt_jpeg as dj
    dist.init_process_group("gloo")
    n = SIZES[rank]
    off, total = sum(SIZES[:rank]), sum(SIZES)
    part = torch.full((n + 9,), 0xEE, dtype=torch.uint8)  # slack past the stripe's bytes
    part[:n] = torch.tensor(list(_part(rank)), dtype=torch.uint8)
    try:
        out = dj.gather_striped(part, n, off + (1 if bad and rank == 2 else 0), total, root=root)
    except ValueError as e:
        out = f"refused: {e}"
    with open(os.path.join(out_dir, f"out{rank}.txt"), "w") as f:
        f.write("None" if out is None else (out if isinstance(out, str) else bytes(out.tolist()).hex()))
    dist.destroy_process_group()


def _run(tmp_path, root, bad):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_rank, args=(3, port, str(tmp_path), root, bad), nprocs=3, start_method="spawn")
    return [open(tmp_path / f"out{r}.txt").read() for r in range(3)]


@pytest.mark.timeout(180)
def test_gather_in_rank_order(tmp_path):
    outs = _run(tmp_path, root=1, bad=False)
    assert outs[0] == "None" and outs[2] == "None"
    assert bytes.fromhex(outs[1]) == b"".join(_part(r) for r in range(3))


@pytest.mark.timeout(180)
def test_gather_refuses_a_bad_tiling(tmp_path):
    outs = _run(tmp_path, root=0, bad=True)
    assert all(o.startswith("refused") for o in outs), outs
