"""File-based launcher bootstrap (csrc/dist/bootstrap.cpp) with 3 real processes: repeated
all-gathers return every rank's blob in rank order, files of a stale earlier job are
ignored, the finish barrier cleans up, and a missing rank times out instead of hanging."""
import ctypes
import multiprocessing as mp
import os
import time

from hpnn_amd._lib import lib_path


def _worker(rank, world, d, q, rounds):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), HPNN_BOOT_DIR=d, HPNN_BOOT_TIMEOUT_S="5")
    L = ctypes.CDLL(lib_path())
    L.hpnn_boot_allgather.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    out = []
    for i in range(rounds):
        mine = (ctypes.c_int * 4)(rank, i, rank * 10 + i, 7)
        allv = (ctypes.c_int * (4 * world))()
        rc = L.hpnn_boot_allgather(mine, 16, allv)
        out.append((rc, list(allv)))
    L.hpnn_boot_finish()
    q.put((rank, out))


def test_allgather_three_processes(tmp_path):
    d = str(tmp_path / "boot")
    os.makedirs(d)
    # a stale file of an earlier job with the same directory: ignored (older than 2 min)
    with open(os.path.join(d, "0.2"), "wb") as f:
        f.write(b"\xff" * 16)
    old = time.time() - 3600
    os.utime(os.path.join(d, "0.2"), (old, old))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 3, d, q, 4)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    for r in range(3):
        for i, (rc, v) in enumerate(res[r]):
            assert rc == 0
            assert v == [x for q_ in range(3) for x in (q_, i, q_ * 10 + i, 7)]
    # finish removed every exchange file but the last barrier's
    assert len(os.listdir(d)) <= 3


def test_missing_rank_times_out(tmp_path):
    d = str(tmp_path / "boot")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 2, d, q, 1))
    t0 = time.time()
    p.start()
    rank, out = q.get(timeout=60)
    p.join(timeout=30)
    assert out[0][0] < 0 and time.time() - t0 < 40
