#!/usr/bin/env python3
"""Per-phase timeline of a conv chain launch (RTENHIP_CHAIN_STAMPS=<path>:
<path> holds {grid, n_phases}, then per block and phase barrier {arrived,
released} s_memrealtime stamps = 100 MHz, u64 [grid][n_phases][2]; the last phase has
no barrier and no stamps).  Tuning aid: per phase, the work time of the
blocks (from their previous release to their arrival: median / max) and the
barrier's own latency (last arrival -> median release).

usage: chain_stamps.py <path>"""
import sys

import numpy as np


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64)
    G, nph = int(raw[0]), int(raw[1])
    a = raw[2:2 + G * nph * 2].reshape(G, nph, 2)
    it = raw[2 + G * nph * 2:].reshape(G, nph, 4) if raw.size >= 2 + G * nph * 6 else None
    arr, rel = a[:, :, 0], a[:, :, 1]
    ok = (arr[:, : nph - 1] > 0).all()
    base = arr[:, 0].min()
    print(f"{G} blocks, {nph} phases{'' if ok else ' (missing stamps)'}")
    print("ph  work_med  work_max  last_arrive->rel_med  rel_spread | first item (blocks with one): "
          "loads  chain  fold+store  (median, max; us)")
    prev = None
    tot_w = tot_b = 0.0
    for p in range(nph - 1):
        start = rel[:, p - 1] if p > 0 else np.full(G, arr[:, 0].min())
        work = (arr[:, p] - start) / 100.0
        last = arr[:, p].max()
        bar = (np.median(rel[:, p]) - last) / 100.0
        spread = (rel[:, p].max() - rel[:, p].min()) / 100.0
        tot_w += np.median(work)
        tot_b += bar
        extra = ""
        if it is not None:
            m = it[:, p, 0] > 0
            if m.any():
                seg = np.diff(it[m, p, :], axis=1) / 100.0
                extra = " | " + "  ".join(f"{np.median(seg[:, j]):5.2f}/{seg[:, j].max():5.2f}" for j in range(3))
        print(f"{p:2d} {np.median(work):9.2f} {work.max():9.2f} {bar:14.2f} {spread:16.2f}{extra}")
    print(f"sum of median work {tot_w:.1f} us, of barrier latency {tot_b:.1f} us; "
          f"span to last release {(rel[:, nph - 2].max() - base) / 100.0:.1f} us")


if __name__ == "__main__":
    main()
