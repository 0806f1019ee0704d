"""bench.py's multi-process path on CPU (world size 2, host sockets).

dfl001 does not shard: N ranks run independent replicas,
the timed region is bracketed by barriers and the reported time is the
maximum over ranks; the value is the sum of all ranks' iterations divided
by that time.  This exercises bench.Dist / bench.timed_replicas exactly as
bench.py uses them, with a CPU stand-in for the per-rank solve.
"""
import os
import socket
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import bench
    d = bench.Dist()
    # uneven per-rank work: rank r "iterates" (r + 1) * 3 times, 20 ms each
    iters = (rank + 1) * 3

    def block():
        for _ in range(iters):
            time.sleep(0.02)
        return iters

    res, elapsed = bench.timed_replicas(d, block, lambda: None)
    total = d.sum(res)
    # the convergence gate: every rank must report its solves converged
    gate = d.min(1.0 if rank == 0 else 0.0)
    q.put((rank, res, elapsed, total, gate))
    d.close()


@pytest.mark.timeout(120)
def test_replicas_max_time_and_sum_over_two_gloo_ranks():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (r0, it0, t0, tot0, g0), (r1, it1, t1, tot1, g1) = out
    assert g0 == g1 == 0.0                        # one unconverged rank voids the value everywhere
    assert (it0, it1) == (3, 6)
    assert tot0 == tot1 == 9                      # value numerator: all ranks' iterations
    assert t0 == t1                               # max over ranks, identical on every rank
    assert t0 >= 6 * 0.02                         # at least the slowest rank's work
