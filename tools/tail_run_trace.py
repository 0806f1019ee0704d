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


if __name__ == "__main__":
    main()
