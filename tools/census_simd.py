#!/usr/bin/env python3
"""Per-SIMD view of a DFS_SHA_CENSUS dump: active waves per SIMD over time
and one sample SIMD's items.  usage: census_simd.py FILE N_LONG"""
import collections
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint32).reshape(-1, 4).astype(np.int64)
n_long = int(sys.argv[2])
t0 = (a[:, 2] - a[:, 2].min()) / 1e5
t1 = (a[:, 3] - a[:, 2].min()) / 1e5
hw, xcc = a[:, 0], a[:, 1] >> 28
key = ((xcc & 7) << 10) | (((hw >> 13) & 7) << 7) | (((hw >> 12) & 1) << 6) | (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)
d = collections.defaultdict(list)
for i in range(len(a)):
    d[key[i]].append((t0[i], t1[i], i < n_long))
print("simds", len(d), "items/simd", sorted(collections.Counter(len(v) for v in d.values()).items()))
ts = np.linspace(0, t1.max(), 21)
act = [np.mean([sum(1 for (s, e, l) in v if s <= t < e) for v in d.values()]) for t in ts]
print("active waves/simd:", " ".join(f"{t:.0f}:{x:.2f}" for t, x in zip(ts, act)))
for k in list(d.keys())[5:7]:
    print("sample", sorted((round(s, 1), round(e, 1), l) for s, e, l in d[k]))
