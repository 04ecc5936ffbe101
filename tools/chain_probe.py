"""Latency-bound SHA launches: time dfs_sha256_batch over n equal messages
(device memory) for a sweep of n.  The library picks the pair-lane latency
kernel up to half of dfs::kChainMaxLanes messages (DFS_SHA_CHAIN=1: the
one-lane kernel there too), the one-lane kernel up to kChainMaxLanes and the
persistent kernel above; profiles/r02_chain_vs_persistent.txt was measured
with a temporary build whose threshold came from a DFS_CHAIN_MAX variable
(not in the library)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-file-storage_amd"))
import dfs_amd  # noqa: E402
from dfs_amd.engine import sha256_device  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
counts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16384, 32768, 49152, 65536, 81920]
eng = dfs_amd.FragmentEngine(0)
nmax = max(counts)
buf = torch.empty(nmax * S + 64, dtype=torch.uint8, device="cuda:0")
spans = np.stack([np.arange(nmax, dtype=np.uint64) * np.uint64(S), np.full(nmax, S, dtype=np.uint64)], axis=1)
dfs_amd.synth_fill(eng, buf.data_ptr(), spans, 0, 0x5EED5EED)
torch.cuda.synchronize()
res = {}
for n in counts:
    sha256_device(eng, buf.data_ptr(), spans[:n])
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        sha256_device(eng, buf.data_ptr(), spans[:n])
        ts.append(time.perf_counter() - t0)
    res[n] = round(min(ts) * 1e3, 2)
    print(f"one_lane={os.environ.get('DFS_SHA_CHAIN', '0')} n={n} S={S}: {res[n]} ms", flush=True)
eng.close()
