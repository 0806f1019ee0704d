"""The persistent dense tail's work-item schedules (kkt_dense.hip
tail_run_schedule / tail_chain_schedule, through ipo_hip_tail_schedule; host
code, no GPU): every item of the look-ahead factorisation exactly once, and
every item waiting only on items with smaller tickets -- the property that
lets k_tail_run / k_tail_chain_run drain on any share of the CUs (DESIGN.md
section 6.2).  The waits restated from k_tail_run:
  panel (t, j):  pdone[t - 1] (every panel of step t - 1; with the window
                 hand-off also their published windows), and the visits of
                 its diagonal tile (t, t) and its tile (t + j + 1, t);
  visit (launch t, tile (bi, c), chunk q): pdone[t - 1] and chunks 0 .. q - 1
                 of the same tile.
A chunk applies blocks [b0, b1) of its tile, which must be final before its
launch (b1 - 1 <= t - 1) and the chunk done before the tile's panel (t < c)."""
import ctypes as C
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402

PC = 64


def schedule(kind, nt, K=6, L=2, cap=256):
    lib = ipo_amd.lib()
    f = lib.ipo_hip_tail_schedule
    f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint), C.c_int, C.POINTER(C.c_int)]
    f.restype = C.c_int
    n = f(kind, nt, K, L, cap, None, 0, None)
    assert n > 0, ipo_amd.lib().ipo_hip_last_error
    ntb = (nt + PC - 1) // PC
    items = (C.c_uint * (2 * n))()
    ptr = (C.c_int * (ntb + 1))()
    assert f(kind, nt, K, L, cap, items, n, ptr) == n
    return [(items[2 * i], items[2 * i + 1]) for i in range(n)], list(ptr), ntb


def tail_gp(nt, t):
    return max(1, (nt - t * PC + 63) // 64 - 1)


def check_visits(vis, panel_idx, ntb, nt):
    """vis: list of (index, launch t, bi, c, b0, b1, q)."""
    by_tile = {}
    for it in vis:
        by_tile.setdefault((it[2], it[3]), []).append(it)
    for c in range(ntb):
        for bi in range(c, ntb):
            ch = sorted(by_tile.get((bi, c), []), key=lambda v: v[6])
            want = c - 1       # blocks 0 .. c - 2 by visits, c - 1 by the panel's pre-update
            if want <= 0:
                assert not ch, (bi, c)
                continue
            assert [v[6] for v in ch] == list(range(len(ch))), (bi, c, ch)
            b = 0
            for i, t, _, _, b0, b1, q in ch:
                assert b0 == b and b1 > b0, (bi, c, ch)     # blocks in order, contiguous
                b = b1
                assert b1 - 1 <= t - 1 and t < c, (bi, c, t, b0, b1)
                if q > 0:
                    assert ch[q - 1][0] < i, ("chunk after its predecessor", bi, c, q)
                if t > 0:
                    assert max(panel_idx[(t - 1, jj)] for jj in range(tail_gp(nt, t - 1))) < i, \
                        ("visit after the panels of step t - 1", bi, c, t)
            assert b == want, (bi, c, b, want)
    return by_tile


@pytest.mark.parametrize("nt,K,L,cap", [(4441, 6, 2, 256), (4441, 6, 6, 256), (4441, 6, 2, 80),
                                        (2000, 6, 2, 256), (732, 6, 2, 256), (155, 6, 2, 256), (640, 4, 1, 32)])
def test_run_schedule(nt, K, L, cap):
    items, ptr, ntb = schedule(0, nt, K, L, cap)
    panel_idx, vis = {}, []
    for i, (x, y) in enumerate(items):
        t = y & 0xff
        if y >> 31:
            assert (t, x) not in panel_idx
            panel_idx[(t, x)] = i
        else:
            vis.append((i, t, x & 255, (x >> 8) & 255, (x >> 16) & 255, x >> 24, (y >> 8) & 0xff))
    # every panel workgroup of every step, once
    assert sorted(panel_idx) == sorted((t, j) for t in range(ntb) for j in range(tail_gp(nt, t)))
    by_tile = check_visits(vis, panel_idx, ntb, nt)
    for (t, j), i in panel_idx.items():
        if t > 0:
            assert max(panel_idx[(t - 1, jj)] for jj in range(tail_gp(nt, t - 1))) < i, (t, j)
        for tile in ((t, t), (t + j + 1, t)):
            for v in by_tile.get(tile, []):
                assert v[0] < i, ("panel after its tiles' visits", t, j, tile)
        # the chunk count the panel waits for (y >> 8) is its column's
        nch = (items[i][1] >> 8) & 0xff
        assert nch == len(by_tile.get((t, t), [])), (t, nch)
    # ptr: launch t's items start at ptr[t]; a run resumed at t0 takes items[ptr[t0]:]
    assert ptr[0] == 0 and ptr[ntb] == len(items)
    for i, (x, y) in enumerate(items):
        t = y & 0xff
        assert ptr[t] <= i < ptr[t + 1], (i, t)


@pytest.mark.parametrize("nt", [4441, 2000, 500])
def test_chain_schedule(nt):
    items, ptr, ntb = schedule(1, nt)
    assert items[0] == (0, 1 << 30)              # the chain item, ticket 0
    tiles, vis, panel_idx = {}, [], {}
    for i, (x, y) in enumerate(items[1:], 1):
        t = y & 0xff
        if y >> 31:
            assert (t, x) not in tiles and x >= t + 2
            tiles[(t, x)] = i
        else:
            assert not (y >> 30)
            vis.append((i, t, x & 255, (x >> 8) & 255, (x >> 16) & 255, x >> 24, (y >> 8) & 0xff))
    assert sorted(tiles) == sorted((t, R) for t in range(ntb) for R in range(t + 2, ntb))
    for (t, R), i in tiles.items():
        if t > 0:
            assert tiles[(t - 1, R)] < i
    # the chain factors every panel: its "panels" precede everything
    for t in range(ntb):
        for j in range(tail_gp(nt, t)):
            panel_idx[(t, j)] = 0
    check_visits(vis, panel_idx, ntb, nt)
