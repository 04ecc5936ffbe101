#!/usr/bin/env python3
"""Is the SHA-256 kernel memory-limited?  Runs the config-2 SHA work
(65,536 x 1 MiB, N=5: fileId + fragment lanes) with the files aliased onto A
distinct 1 MiB files (A = 1 keeps everything L2-resident; A = 65,536 is the
real, HBM-streaming layout) and prints the SHA kernel time for each A.
Same descriptor geometry, same op count: only the memory footprint changes."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))
import dfs_amd  # noqa: E402

F, S, N = 65536, 1 << 20, 5
eng = dfs_amd.FragmentEngine(0)
dev = torch.device("cuda:0")
files = torch.empty(F * S, dtype=torch.uint8, device=dev)
allsp = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(S), np.full(F, S, dtype=np.uint64)], axis=1)
dfs_amd.synth_fill(eng, files.data_ptr(), allsp, 0, 0x5EED5EED)
torch.cuda.synchronize()
fd = torch.empty(F * 32, dtype=torch.uint8, device=dev)
frd = torch.empty(F * N * 32, dtype=torch.uint8, device=dev)
out = {}
conc = "--concurrent" in sys.argv  # SHA || Base64 (the bench's default mode) instead of SHA alone
b64 = None
for A in [int(a) for a in ([x for x in sys.argv[1:] if not x.startswith("--")] or ["1", "64", "1024", "65536"])]:
    sp = np.stack([(np.arange(F, dtype=np.uint64) % np.uint64(A)) * np.uint64(S),
                   np.full(F, S, dtype=np.uint64)], axis=1)
    plan = dfs_amd.UploadPlan(eng, sp, N, align128=True)
    if conc and b64 is None:
        b64 = torch.empty(plan.b64_total, dtype=torch.uint8, device=dev)
    ms, tot = [], []
    for i in range(4):
        eng.set_profiling(True)
        if conc:
            plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
        else:
            plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), 0, dfs_amd.DFS_NO_B64 | dfs_amd.DFS_SERIAL)
        t = eng.timings()
        eng.set_profiling(False)
        if i:
            ms.append(t["sha"])
            tot.append(t["total"])
    torch.cuda.synchronize()
    plan.close()
    out[A] = round(float(np.mean(ms)), 3)
    print(json.dumps({"aliased_files": A, "concurrent": conc, "sha_ms": out[A],
                      "total_ms": round(float(np.mean(tot)), 3)}), flush=True)
eng.close()
