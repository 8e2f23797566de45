"""Host threads (SURVEY.md 8(b) "Threading": re-entrant per dmmt_ctx, the output
bit-identical for any thread count).  The Python mirror's ctypes calls release
the GIL, so the threads below are in the library at the same time:
  * one context per thread, each encoding its own images;
  * one context shared by several threads (its mutex serialises the calls);
every JPEG byte-identical to the oracle's."""
import threading

import pytest

import dmmt_jpeg
import oracle
from conftest import synthetic

pytestmark = pytest.mark.gpu


def _opts(sub, q):
    luma, chroma = dmmt_jpeg.quality_tables(q)
    return dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                              chroma_table=chroma)


def _jobs(n):
    # (image, subsampling, quality): sizes, presets and tables differ per job
    out = []
    for i in range(n):
        w, h = 64 + 24 * i, 40 + 16 * (i % 3)
        out.append((synthetic(w, h, frame=200 + i), i % 3, [50, 75, 90, 95][i % 4]))
    return out


def _run_threads(target, n):
    errs = []

    def wrap(k):
        try:
            target(k)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(k,)) for k in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs


def test_one_context_per_thread():
    jobs = _jobs(8)
    want = [oracle.encode(img, 255, sub, _opts(sub, q).luma_table, _opts(sub, q).chroma_table)
            for img, sub, q in jobs]
    got = [[None] * len(jobs) for _ in range(4)]

    def work(k):
        enc = dmmt_jpeg.Encoder(0)
        try:
            for rep in range(3):
                for j, (img, sub, q) in enumerate(jobs):
                    if (j + k + rep) % 2 == 0:
                        got[k][j] = enc.encode(dmmt_jpeg.Image.from_array(img), _opts(sub, q))
        finally:
            enc.close()

    _run_threads(work, 4)
    for k in range(4):
        for j in range(len(jobs)):
            if got[k][j] is not None:
                assert got[k][j] == want[j], (k, j)


def test_shared_context_across_threads(encoder):
    jobs = _jobs(6)
    want = [oracle.encode(img, 255, sub, _opts(sub, q).luma_table, _opts(sub, q).chroma_table)
            for img, sub, q in jobs]
    got = [[None] * len(jobs) for _ in range(3)]

    def work(k):
        for rep in range(2):
            for j, (img, sub, q) in enumerate(jobs):
                got[k][j] = encoder.encode(dmmt_jpeg.Image.from_array(img), _opts(sub, q))

    _run_threads(work, 3)
    for k in range(3):
        for j in range(len(jobs)):
            assert got[k][j] == want[j], (k, j)
