"""Block-angular sharding on the CPU: gloo, world size 2.

The sharded KKT factor/solve (kkt_device.hip with an Exchange, exchange.h)
orders each shard's linking rows L last -- the forced dense tail -- and
meets the other shards only there: shard k's tail holds -E_L (shard 0
only) minus its Schur contribution K_LF K_FF^-1 K_FL, the allreduced tail
is the global Schur complement, the tail right-hand side is summed the same
way, every shard solves the tail itself and back-substitutes its own
blocks.  This restates exactly that exchange with dense numpy on each
rank's local problem (ipo_amd.shard_block_angular) and requires the global
KKT solution.  The reductions go over one of two transports:
  * gloo (torch.distributed), the harness's CPU stand-in for RCCL;
  * the library's host transport: exchange.h's HostAllreduceFn as the
    package builds it (ipo_amd.host_allreduce_callback), called through its
    C function pointer exactly as make_host_exchange calls it after staging
    the device buffer, over ipo_amd.hostcomm's sockets.  exchange.cpp's
    staging copies need a device; tests/test_gpu_shard.py runs the same
    transport through them (two processes sharing the GPU).
"""
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIMS = (4, 30, 100, 4, 16, 6, 40)     # blocks, mb, nb, per_col, band, nlink, link_nz


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def dense(p):
    A = np.zeros((p.m, p.n))
    A[p.iA, np.repeat(np.arange(p.n), np.diff(p.kA))] = p.A
    return A


def scaling(p, seed=7):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.5, 2.0, p.m), rng.uniform(0.5, 2.0, p.n), rng.uniform(-1, 1, p.m), rng.uniform(-1, 1, p.n)


def local_index(p, loc):
    """Global row / column index of every local row / column of a shard."""
    b = loc.blocks
    nl = b["nlink"]
    rows = np.r_[np.arange(b["row0"], b["row0"] + loc.m - nl), np.arange(p.m - nl, p.m)]
    return rows, np.arange(b["col0"], b["col0"] + loc.n)


def _allreducer(transport, rank, world):
    """(allreduce-sum-in-place of a float64 array, close)"""
    if transport == "gloo":
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return (lambda a: dist.all_reduce(torch.from_numpy(a))), dist.destroy_process_group
    import ctypes as C

    import ipo_amd
    from ipo_amd.hostcomm import HostComm
    comm = HostComm(rank, world)
    ops = {0: "sum", 1: "max", 2: "min"}
    cb = ipo_amd.host_allreduce_callback(lambda buf, op: comm.allreduce(buf, ops[op]))
    fn = ipo_amd.ALLREDUCE_FN(C.cast(cb, C.c_void_p).value)     # the pointer the C side holds

    def allreduce(a, keep=cb):      # cb owns the thunk behind fn
        assert a.dtype == np.float64 and a.flags.c_contiguous
        assert fn(None, a.ctypes.data_as(C.POINTER(C.c_double)), a.size, 0) == 0
    return allreduce, comm.close


def _rank_main(rank, world, port, q, transport="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [os.path.join(REPO, "linear-programming-vanderbei_amd"), os.path.join(REPO, "tests")]
    import ipo_amd
    allreduce, close = _allreducer(transport, rank, world)
    try:
        p = ipo_amd.synth_block_angular(*DIMS)
        E, D, fy, fx = scaling(p)
        loc = ipo_amd.shard_block_angular(p, world, rank)
        rows, cols = local_index(p, loc)
        nl = loc.blocks["nlink"]
        mf = loc.m - nl
        Al = dense(loc)
        assert np.array_equal(Al, dense(p)[np.ix_(rows, cols)])      # the local LP is the global slice
        El, Dl = E[rows], D[cols]
        KFF = np.block([[-np.diag(El[:mf]), Al[:mf]], [Al[:mf].T, np.diag(Dl)]])
        KLF = np.hstack([np.zeros((nl, mf)), Al[mf:]])
        KLL = -np.diag(El[mf:]) if rank == 0 else np.zeros((nl, nl))
        rF = np.r_[fy[rows[:mf]], fx[cols]]
        rL = fy[rows[mf:]] if rank == 0 else np.zeros(nl)
        X = np.linalg.solve(KFF, np.column_stack([KLF.T, rF]))
        S = KLL - KLF @ X[:, :nl]
        t = rL - KLF @ X[:, nl]
        S = np.ascontiguousarray(S)
        allreduce(S)                # in place: S and t become the global tail
        allreduce(t)
        xL = np.linalg.solve(S, t)
        xF = np.linalg.solve(KFF, rF - KLF.T @ xL)
        q.put((rank, xL, xF[:mf], xF[mf:], None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))
    finally:
        close()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("transport", ["gloo", "host"])
def test_tail_exchange_reproduces_global_kkt_solution(transport):
    import multiprocessing as mp

    import ipo_amd
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, transport)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = sorted((q.get(timeout=150) for _ in procs), key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=30)
        assert pr.exitcode == 0
    for r in out:
        assert r[4] is None, r[4]
    p = ipo_amd.synth_block_angular(*DIMS)
    E, D, fy, fx = scaling(p)
    A = dense(p)
    sol = np.linalg.solve(np.block([[-np.diag(E), A], [A.T, np.diag(D)]]), np.r_[fy, fx])
    dy, dx = sol[:p.m], sol[p.m:]
    for rank, xL, yF, xC, _ in out:
        loc = ipo_amd.shard_block_angular(p, world, rank)
        rows, cols = local_index(p, loc)
        mf = loc.m - loc.blocks["nlink"]
        np.testing.assert_allclose(xL, dy[rows[mf:]], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(yF, dy[rows[:mf]], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(xC, dx[cols], rtol=1e-9, atol=1e-11)
    assert np.array_equal(out[0][1], out[1][1])      # the replicated tail solution is bitwise shared


def test_assemble_block_angular_roundtrip():
    import ipo_amd
    p = ipo_amd.synth_block_angular(*DIMS)
    for world in (1, 2, 4):
        parts = []
        for k in range(world):
            loc = ipo_amd.shard_block_angular(p, world, k)
            parts.append((loc.blocks, (loc.xs, loc.ys, loc.ws, loc.zs)))
        for a, b in zip(ipo_amd.assemble_block_angular(parts), (p.xs, p.ys, p.ws, p.zs)):
            assert np.array_equal(a, b)
