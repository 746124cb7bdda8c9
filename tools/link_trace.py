#!/usr/bin/env python3
"""Summarise an MM_LINK_TRACE file (mm_wide_link_kernel: per ticket the wall clock at
start, after the wait and at the end, and the XCD): per pass the span, the mean work and
wait per segment, and the overlap with the previous pass. usage: link_trace.py FILE [MHz]"""
import sys

import numpy as np

f = sys.argv[1]
mhz = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
raw = np.fromfile(f, dtype=np.uint64)
items = int(raw[0])
rec = raw[1:].reshape(-1, 4).astype(np.int64)
rec = rec[rec[:, 2] > 0]
npass = len(rec) // items
t0 = rec[:, 0].min()
us = lambda x: x / mhz  # noqa: E731
print(f"items/pass {items}, passes {npass}, span {us(rec[:, 2].max() - t0):.1f} us")
prev_end = None
for p in range(npass):
    r = rec[p * items:(p + 1) * items]
    s, w, e = r[:, 0] - t0, r[:, 1] - t0, r[:, 2] - t0
    line = (f"pass {p:3d}: start {us(s.min()):9.1f}..{us(s.max()):9.1f} end {us(e.min()):9.1f}.."
            f"{us(e.max()):9.1f}  work {us((e - w).mean()):6.1f} (max {us((e - w).max()):6.1f})"
            f"  wait {us((w - s).mean()):6.1f} (max {us((w - s).max()):6.1f})")
    if prev_end is not None:
        line += f"  first start - prev last end {us(s.min() - prev_end):7.1f}"
    prev_end = e.max()
    if p < 4 or p >= npass - 2 or p % 16 == 0:
        print(line)
xcd = rec[:, 3] & 15
print("XCD counts", np.bincount(xcd, minlength=8))
