"""The node's shared-memory size exchange (yrwi_coll.cpp) across
separate processes, as the ranks of `bench.py --gpus N` use it: no GPU needed.
Every rank runs the same batch parts and exchanges; the sums must be exact, with
more parts than mailbox slots (slots are reused) and ranks started at
different times."""
import multiprocessing as mp
import os

import pytest


def _segment(uid, world):
    """The mailbox's shared-memory name for group id `uid` (hostx_open, yrwi_coll.cpp)."""
    h = 1469598103934665603
    for b in uid:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"yrwi-hx-{h:016x}-{world}"


def _rank(uid, world, rank, nparts, ncalls, n, delay, q):
    import time
    time.sleep(delay)
    from yacy_search_server_amd import _lib
    q.put((rank, _lib.lib().yrwi_hostx_selftest(uid, world, rank, nparts, ncalls, n)))


@pytest.mark.parametrize("world,nparts,ncalls,n", [(2, 40, 3, 1000), (4, 20, 8, 4096), (8, 12, 2, 17)])
def test_hostx_processes(world, nparts, ncalls, n):
    uid = b"YRWI-HOSTX-TEST" + os.urandom(113)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(uid, world, r, nparts, ncalls, n, 0.05 * ((r * 7) % world), q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {r: 0 for r in range(world)}, res
    assert not os.path.exists(os.path.join("/dev/shm", _segment(uid, world)))  # rank 0 unlinked the mailbox


@pytest.mark.parametrize("nparts", [4, 20])  # 20: later parts reuse the aborted part's slots
def test_hostx_failed_part_fails_peers_fast(nparts):
    """A rank whose batch part fails aborts that part in the mailbox (run_batch_part):
    its peers' exchanges of the part fail at once instead of spinning for the whole
    timeout (300 s), and every later part then runs normally on every rank (the
    abort is scoped to the failed part: the selftest returns part 0's status only
    when parts 1..3 all succeed, 1000 + the part otherwise)."""
    import time
    uid = b"YRWI-HOSTX-TEST" + os.urandom(113)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t0 = time.time()
    ps = [ctx.Process(target=_rank, args=(uid, 3, r, nparts, 2, -100, 0.3 if r == 2 else 0.0, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: -6, 1: -6, 2: -6}, res  # YRWI_E_RCCL everywhere
    assert time.time() - t0 < 30


def test_hostx_oversized_vector_not_handled():
    """Vectors longer than the mailbox's slots fall back to the device all-gather."""
    from yacy_search_server_amd import _lib
    uid = b"YRWI-HOSTX-TEST" + os.urandom(113)
    assert _lib.lib().yrwi_hostx_selftest(uid, 1, 0, 1, 1, 10) == 1  # world 1: no mailbox
