"""Sharded block-angular solve on the GPU (BASELINE configs[4]).

The GPU box has one device and RCCL refuses two ranks on one GPU, so the
two ranks here share it and exchange through the host-callback transport
(exchange.h make_host_exchange) over host sockets (ipo_amd.hostcomm; no
torch in a GPU process, whose bundled HIP runtime would sit beside the
library's); RCCL is the same Exchange
interface and carries bench.py's multi-GPU runs.  Checked, for hsd and
intpt:
  * both ranks report the same status and iteration count;
  * the replicated linking-row y, w come out bitwise identical on both
    ranks (the replication claim of exchange.h);
  * rank 0 prints the trace of the whole LP (global m, n, nz);
  * against the unsharded GPU solve and the CPU oracle on the whole LP:
    same status, iterations within +-1, final objectives within 1e-6
    relative (the tolerances of test_synth.py; the oracle restates the
    reference's algorithm on the same data -- the reference has no
    synthetic problems, so this parity is pinned through the oracle);
  * the assembled HSD solution passes test_synth.py's optimality
    certificate.
nranks = 1 (one process, linking rows forced into the dense tail) is
checked against the oracle the same way.
"""
import os
import socket
import sys

import numpy as np
import pytest

import ipo_amd
import oracle_lib
from test_synth import certificate

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIMS = (4, 300, 1200, 4, 64, 16, 200)     # blocks, mb, nb, per_col, band, nlink, link_nz
METHODS = ("hsd", "intpt")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q, dims=DIMS, methods=METHODS):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [os.path.join(REPO, "linear-programming-vanderbei_amd"), os.path.join(REPO, "tests")]
    import ipo_amd
    from ipo_amd.hostcomm import HostComm
    comm = HostComm(rank, world)
    ops = {0: "sum", 1: "max", 2: "min"}

    def allreduce(buf, op):
        comm.allreduce(buf, ops[op])
    try:
        p = ipo_amd.synth_block_angular(*dims)
        loc = ipo_amd.shard_block_angular(p, world, rank)
        del p
        ctx = ipo_amd.ShardContext(loc, world, rank, host_allreduce=allreduce)
        res = {}
        for method in methods:
            st, stats, text = ctx.run(method, trace=(rank == 0))
            res[method] = (st, stats["iters"], stats["final_pobj"], stats["final_dobj"], ctx.solution(), text)
        ctx.close()
        q.put((rank, loc.blocks, res, None))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
    finally:
        comm.close()


def _check(st, iters, pobj, dobj, ref):
    rst, riters, rpobj, rdobj = ref
    assert st == rst == 0, (st, rst)
    assert abs(iters - riters) <= 1, (iters, riters)
    for a, b in ((pobj, rpobj), (dobj, rdobj)):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(b)), (a, b)


def _references(p, method):
    g = ipo_amd.solver(p, method)
    o = oracle_lib.solve_arrays(p, method)
    return ((g["status"], g["stats"]["iters"], g["stats"]["final_pobj"], g["stats"]["final_dobj"]),
            (o["status"], o["iters"], o["final_pobj"], o["final_dobj"]))


def _run_shards(world, dims=DIMS, methods=METHODS, timeout=240):
    """world host-transport shards of the LP `dims` on the one GPU, one
    spawned process each; their (rank, blocks, results, error) tuples."""
    import multiprocessing as mp
    ipo_amd.require_gpu()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, dims, methods)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        out = sorted((q.get(timeout=timeout) for _ in procs), key=lambda t: t[0])
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.is_alive():
                pr.kill()
    for r in out:
        assert r[3] is None, r[3]
    for pr in procs:
        assert pr.exitcode == 0
    return out


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_shards_on_one_gpu_match_unsharded_and_oracle():
    world = 2
    out = _run_shards(world)
    p = ipo_amd.synth_block_angular(*DIMS)
    nl = DIMS[5]
    for method in METHODS:
        r0, r1 = out[0][2][method], out[1][2][method]
        assert r0[:2] == r1[:2], (method, r0[:2], r1[:2])
        (_, y0, w0, _), (_, y1, w1, _) = r0[4], r1[4]
        assert np.array_equal(y0[-nl:], y1[-nl:]) and np.array_equal(w0[-nl:], w1[-nl:])
        assert f"m = {p.m},n = {p.n},nz = {p.nz}" in r0[5]
        for ref in _references(p, method):
            _check(*r0[:4], ref)
        if method == "hsd":
            x, y, w, z = ipo_amd.assemble_block_angular([(out[k][1], out[k][2][method][4]) for k in range(world)])
            pr_, du, gap = certificate(p, x, y, w, z)
            assert pr_ < 1e-6 and du < 1e-6 and gap < 1e-6, (pr_, du, gap)


@pytest.mark.gpu
def test_forced_tail_single_process_matches_oracle():
    p = ipo_amd.synth_block_angular(*DIMS)
    loc = ipo_amd.shard_block_angular(p, 1, 0)
    ctx = ipo_amd.ShardContext(loc)
    try:
        for method in METHODS:
            st, stats, _ = ctx.run(method)
            o = oracle_lib.solve_arrays(p, method)
            _check(st, stats["iters"], stats["final_pobj"], stats["final_dobj"],
                   (o["status"], o["iters"], o["final_pobj"], o["final_dobj"]))
            if method == "hsd":
                pr_, du, gap = certificate(p, *ctx.solution())
                assert pr_ < 1e-6 and du < 1e-6 and gap < 1e-6, (pr_, du, gap)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_rccl_exchange_one_rank_matches_host_exchange(monkeypatch):
    """The RCCL transport (exchange.cpp) on a one-rank communicator against
    the host-callback transport on one rank: both take every sharded code
    path (summed linking-row products, allreduced tail and scalars) and a
    one-rank allreduce is the identity, so the two solves must agree
    bitwise -- this runs the RCCL calls of bench.py's multi-GPU leg on the
    single-GPU box."""
    p = ipo_amd.synth_block_angular(*DIMS)
    loc = ipo_amd.shard_block_angular(p, 1, 0)
    runs = []
    for transport in ("host", "rccl"):
        if transport == "rccl":
            monkeypatch.setenv("IPO_HIP_SHARD_RCCL", "1")
            ctx = ipo_amd.ShardContext(loc)
        else:
            ctx = ipo_amd.ShardContext(loc, 1, 0, host_allreduce=lambda buf, op: None)
        try:
            st, stats, text = ctx.run("hsd", trace=True)
            runs.append((st, stats["iters"], text, ctx.solution()))
        finally:
            ctx.close()
    (s0, i0, t0, sol0), (s1, i1, t1, sol1) = runs
    assert s0 == s1 == 0 and i0 == i1 and t0 == t1
    for a, b in zip(sol0, sol1):
        assert np.array_equal(a, b)
    o = oracle_lib.solve_arrays(p, "hsd")
    assert abs(i0 - o["iters"]) <= 1


# BASELINE configs[4] at its stated shape: 8 diagonal blocks of
# 25,000 x 100,000 (banded, width 256, 4 nnz per column) + 512 linking rows
# of 2,000 nonzeros each.  No oracle at this size (hours of CPU): the
# one-process solve is held to HSD's own stop and the optimality
# certificate, the 8-way split to the one-process solve.
CONFIG4 = (8, 25000, 100000, 4, 256, 512, 2000)


@pytest.fixture(scope="module")
def config4_one_process():
    p = ipo_amd.synth_block_angular(*CONFIG4)
    loc = ipo_amd.shard_block_angular(p, 1, 0)
    ctx = ipo_amd.ShardContext(loc)
    try:
        st, stats, _ = ctx.run("hsd")
        sol = ctx.solution()
    finally:
        ctx.close()
    return p, st, stats, sol


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_config4_full_size_one_process(config4_one_process):
    """(a) the whole LP in one process, linking rows forced into the dense tail."""
    p, st, stats, sol = config4_one_process
    assert st == 0, st            # HSD's stop (mu < 1e-12 in its homogeneous variables, hsd.c:155) with phi > psi
    pr_, du, gap = certificate(p, *sol)
    assert pr_ < 1e-6 and du < 1e-6 and gap < 1e-6, (pr_, du, gap)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_config4_eight_shards_on_one_gpu_match_one_process(config4_one_process):
    """(b) the 8-way split (one block per shard, the code path of bench.py's
    8-GPU run) as 8 host-transport shards sharing the test box's GPU:
    every rank the same status and iteration count, the replicated
    linking-row y and w bitwise identical on all ranks, and against the
    one-process solve the same status, iterations within +-1, objectives
    within 1e-6 relative; the assembled solution passes the certificate."""
    p, st1, stats1, _ = config4_one_process
    world, nl = 8, CONFIG4[5]
    out = _run_shards(world, CONFIG4, ("hsd",), timeout=540)
    r = [out[k][2]["hsd"] for k in range(world)]
    for k in range(1, world):
        assert r[k][:2] == r[0][:2], (k, r[k][:2], r[0][:2])
        (_, y0, w0, _), (_, yk, wk, _) = r[0][4], r[k][4]
        assert np.array_equal(y0[-nl:], yk[-nl:]) and np.array_equal(w0[-nl:], wk[-nl:]), k
    assert f"m = {p.m},n = {p.n},nz = {p.nz}" in r[0][5]
    _check(*r[0][:4], (st1, stats1["iters"], stats1["final_pobj"], stats1["final_dobj"]))
    x, y, w, z = ipo_amd.assemble_block_angular([(out[k][1], out[k][2]["hsd"][4]) for k in range(world)])
    pr_, du, gap = certificate(p, x, y, w, z)
    assert pr_ < 1e-6 and du < 1e-6 and gap < 1e-6, (pr_, du, gap)
