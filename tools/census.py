#!/usr/bin/env python3
"""Summarise a DFS_SHA_CENSUS dump: per work item {hw_id, xcc_id << 28 |
shader clocks (s_memtime) of the item, t0, t1} (t0/t1: s_memrealtime, 100 MHz).  Items [0, n_long) are fileId (long) items.

usage: census.py FILE N_LONG  -> JSON summary on stdout"""
import json
import sys

import numpy as np

path, n_long = sys.argv[1], int(sys.argv[2])
a = np.fromfile(path, dtype=np.uint32).reshape(-1, 4).astype(np.int64)
a = a[a[:, 3] != 0]
t0 = a[:, 2] - a[:, 2].min()
t1 = a[:, 3] - a[:, 2].min()
dur = (t1 - t0) / 1e5  # ms
start = t0 / 1e5
idx = np.arange(len(a))
lng = idx < n_long
def q(x):
    return [round(float(v), 3) for v in np.percentile(x, [0, 10, 50, 90, 100])] if len(x) else []
cyc = (a[:, 1] & 0x0FFFFFFF).astype(np.float64)
real_s = (t1 - t0).astype(np.float64) / 1e8
ok = real_s > 0
out = {
    "items": int(len(a)),
    "shader_clock_ghz_weighted": round(float(cyc[ok].sum() / real_s[ok].sum() / 1e9), 4),
    "shader_clock_ghz_long_items": round(float(cyc[ok & lng].sum() / max(real_s[ok & lng].sum(), 1e-12) / 1e9), 4),
    "kernel_ms": round(float(t1.max() / 1e5), 3),
    "long_dur_ms_p0_10_50_90_100": q(dur[lng]),
    "long_start_ms": q(start[lng]),
    "long_end_ms": q((t1[lng]) / 1e5),
    "short_dur_ms": q(dur[~lng]),
    "short_start_ms": q(start[~lng]),
    "short_end_ms": q(t1[~lng] / 1e5),
}
print(json.dumps(out))
