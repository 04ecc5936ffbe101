"""On the GPU box: the holders' check alone (dfs_replica_check) on the shape of
the N > 1 step's chunk: 65,536 files x 256 KiB, N = 8, one rank; three calls."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))
import dfs_amd
from dfs_amd import placement as P

F, S, N = int(os.environ.get("CHK_FILES", 65536)), int(os.environ.get("CHK_SIZE", 262144)), int(os.environ.get("CHK_N", 8))
with dfs_amd.FragmentEngine(0) as eng:
    spans = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(S), np.full(F, S, dtype=np.uint64)], axis=1)
    files = torch.empty(F * S + 64, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(eng, files.data_ptr(), spans, 0, 0x5EED5EED)
    plan = dfs_amd.UploadPlan(eng, spans, N, frag_major=True, align128=True)
    fd = torch.empty(F * 32, dtype=torch.uint8, device="cuda")
    frd = torch.empty(F * N * 32, dtype=torch.uint8, device="cuda")
    b64 = torch.empty(plan.b64_total, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
    torch.cuda.synchronize()
    comm = P.Comm(eng, P.unique_id(), 1, 0)
    rp = P.ReplicaPlan(comm, N, [S] * F, True)
    held = torch.empty(rp.held_bytes, dtype=torch.uint8, device="cuda")
    raw = torch.empty(rp.raw_bytes + 16, dtype=torch.uint8, device="cuda")
    verdict = torch.empty(rp.nheld, dtype=torch.int32, device="cuda")
    failed = torch.empty(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    comm.place("star", rp.table, b64.data_ptr(), held.data_ptr())
    rp.exchange(frd.data_ptr())
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rep in range(3):
        t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        import time
        a = time.perf_counter()
        rp.check(eng, held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
        torch.cuda.synchronize()
        print(f"one_pass={rp.one_pass} check {1e3 * (time.perf_counter() - a):.2f} ms failed={int(failed[0])}", flush=True)
    rp.close(); comm.close(); plan.close()
