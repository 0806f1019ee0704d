#!/usr/bin/env python3
"""Read a k_tail_run item trace (tools/ubench_tail with UB_RUN=1
UB_TRACE=file) and print where the persistent dense tail's time goes:
per step the panels' first ready / last done (the chain), the gap from step
t - 1's last panel to step t's panels being ready, and the visits' durations.
Times in microseconds from the first item drawn (s_memrealtime, 100 MHz).
usage: python tools/tail_run_trace.py file [--steps]"""
import struct
import sys

import numpy as np


def main():
    path = sys.argv[1]
    raw = open(path, "rb").read()
    ntb, ni = struct.unpack_from("ii", raw, 0)
    if ni < 0:
        return chain(raw, ntb, -ni)
    items = np.frombuffer(raw, np.uint32, 2 * ni, 8).reshape(ni, 2)
    tr = np.frombuffer(raw, np.uint64, 4 * ni, 8 + 8 * ni).reshape(ni, 4).astype(np.float64)
    t0 = tr[:, 0].min()
    drawn, ready, done = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0
    panel = (items[:, 1] >> 31) == 1
    step = items[:, 1] & 0xff
    print(f"{ni} items, {panel.sum()} panel workgroups, {(~panel).sum()} visits; run {done.max():.1f} us")
    vis = ~panel
    vdur = done[vis] - ready[vis]
    vwait = ready[vis] - drawn[vis]
    nblk = ((items[vis, 0] >> 24) - ((items[vis, 0] >> 16) & 255)).astype(int)
    print(f"visits: duration mean {vdur.mean():.2f} us (per block {np.mean(vdur / nblk):.2f}), "
          f"wait mean {vwait.mean():.2f} max {vwait.max():.1f}; busy {vdur.sum():.0f} us over {len(vdur)} items")
    for k in sorted(set(nblk)):
        sel = nblk == k
        print(f"  {k} blocks: {sel.sum()} visits, {vdur[sel].mean():.2f} us")
    pdur = done[panel] - ready[panel]
    print(f"panels: ready->done mean {pdur.mean():.2f} us; drawn->ready mean {(ready[panel] - drawn[panel]).mean():.2f}")
    prev_end = 0.0
    rows = []
    for t in range(ntb):
        sel = panel & (step == t)
        r0, r1, d1 = ready[sel].min(), ready[sel].max(), done[sel].max()
        rows.append((t, r0 - prev_end, r0, r1, d1, d1 - r0))
        prev_end = d1
    gaps = np.array([r[1] for r in rows[1:]])
    spans = np.array([r[5] for r in rows])
    print(f"chain: step span (first ready -> last done) mean {spans.mean():.2f} us, "
          f"gap (last done of t - 1 -> first ready of t) mean {gaps.mean():.2f} us")
    if "--steps" in sys.argv:
        for t, gap, r0, r1, d1, span in rows:
            print(f"  step {t:3d}: gap {gap:6.2f} ready {r0:8.1f}..{r1:8.1f} done {d1:8.1f} span {span:6.2f}")


def chain(raw, ntb, ni):
    """k_tail_chain_run's trace: items, then one record per step of the chain
    {step start, passes done, results stored}."""
    items = np.frombuffer(raw, np.uint32, 2 * ni, 8).reshape(ni, 2)
    tr = np.frombuffer(raw, np.uint64, 4 * (ni + ntb), 8 + 8 * ni).reshape(ni + ntb, 4).astype(np.float64)
    t0 = tr[:ni, 0].min()
    drawn, ready, done = (tr[:ni, 0] - t0) / 100.0, (tr[:ni, 1] - t0) / 100.0, (tr[:ni, 2] - t0) / 100.0
    steps = (tr[ni:, :3] - t0) / 100.0
    tile = (items[:, 1] >> 31) == 1
    vis = ((items[:, 1] >> 30) == 0)
    print(f"chain run: {ni} items ({tile.sum()} tile items, {vis.sum()} visits); chain ends {steps[-1, 2]:.1f} us, "
          f"last item done {done.max():.1f} us")
    span = np.diff(steps[:, 0])
    print(f"chain steps: mean {span.mean():.2f} us (start->passes {np.mean(steps[:, 1] - steps[:, 0]):.2f}, "
          f"passes->results {np.mean(steps[:, 2] - steps[:, 1]):.2f}, results->next start "
          f"{np.mean(steps[1:, 0] - steps[:-1, 2]):.2f})")
    vdur = done[vis] - ready[vis]
    print(f"visits: duration mean {vdur.mean():.2f} us, wait mean {(ready[vis] - drawn[vis]).mean():.2f}")
    tdur = done[tile] - drawn[tile]
    print(f"tile items: drawn->done mean {tdur.mean():.2f} us")
    ws = np.frombuffer(raw, np.uint64, ntb * 32, 8 + 8 * ni + 8 * 4 * (ni + ntb)).reshape(ntb, 8, 4).astype(np.float64)
    if "--steps" in sys.argv:
        for t in range(ntb):
            print(f"  step {t:3d}: start {steps[t, 0]:8.1f} passes {steps[t, 1] - steps[t, 0]:6.2f} "
                  f"results {steps[t, 2] - steps[t, 1]:6.2f}")
            if t < 6 or t == ntb // 2:
                for wv in range(8):
                    e = (ws[t, wv] - t0) / 100.0 - steps[t, 0]
                    print(f"      wave {wv}: own window {e[0]:7.2f} .. {e[1]:7.2f}, work done {e[2]:7.2f}, barriers {e[3]:7.2f}")


if __name__ == "__main__":
    main()
