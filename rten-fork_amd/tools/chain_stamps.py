#!/usr/bin/env python3
"""Per-layer timeline of a conv chain launch from its unit timestamps
(RTENHIP_CHAIN_STAMPS=<path>: <path>.<chain> holds {layer | xcc << 8 |
block << 16, start, waited, end} per unit, s_memrealtime = 100 MHz).
Tuning aid: where a chain's time goes (dependency waits vs unit execution).
usage: chain_stamps.py <path>.<chain>"""
import sys

import numpy as np


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
    layer = (a[:, 0] & 0xFF).astype(int)
    t0 = a[:, 1].astype(np.int64)
    t1 = a[:, 2].astype(np.int64)
    t2 = a[:, 3].astype(np.int64)
    base = t0.min()
    us = lambda t: (t - base) / 100.0  # 100 MHz ticks -> us
    print(f"{len(a)} units, span {us(t2.max()):.2f} us")
    print(" L   units  first_start  first_go  last_go  last_end  mean_wait  mean_exec  max_exec")
    prev_end = 0.0
    for L in range(layer.max() + 1):
        m = layer == L
        if not m.any():
            continue
        w = (t1[m] - t0[m]) / 100.0
        e = (t2[m] - t1[m]) / 100.0
        le = us(t2[m].max())
        print(f"{L:2d} {m.sum():7d} {us(t0[m].min()):12.2f} {us(t1[m].min()):9.2f} {us(t1[m].max()):8.2f}"
              f" {le:9.2f} {w.mean():10.2f} {e.mean():10.2f} {e.max():9.2f}   (+{le - prev_end:.2f})")
        prev_end = le


if __name__ == "__main__":
    main()
