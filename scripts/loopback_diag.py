"""On the GPU box: where does a one-rank placement through RCCL self send /
receive pairs (DFS_COMM_LOOPBACK=1) differ from the plain-copy placement?
Prints, per file count, whether the held buffer equals the expected bytes and
if not the extent of the differences per group."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))
import dfs_amd
from dfs_amd import placement as P

os.environ["DFS_COMM_LOOPBACK"] = "1"
S, N = 262144, 8
with dfs_amd.FragmentEngine(0) as eng:
    for F in [int(x) for x in sys.argv[1:]] or [256, 8192, 32768, 131072]:
        spans = np.array([(f * S, S) for f in range(F)], dtype=np.uint64)
        files = torch.empty(F * S + 64, dtype=torch.uint8, device="cuda")
        dfs_amd.synth_fill(eng, files.data_ptr(), spans, 0, 0x5EED5EED)
        plan = dfs_amd.UploadPlan(eng, spans, N, frag_major=True, align128=True)
        fd = torch.zeros(F * 32, dtype=torch.uint8, device="cuda")
        frd = torch.zeros(F * N * 32, dtype=torch.uint8, device="cuda")
        b64 = torch.zeros(plan.b64_total, dtype=torch.uint8, device="cuda")
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
        torch.cuda.synchronize()
        offs = plan.b64_offsets()
        grp = [int(offs[f]) for f in range(N)] + [int(offs[-1])]
        comm = P.Comm(eng, P.unique_id(), 1, 0)
        table = comm.sizes([grp[f + 1] - grp[f] for f in range(N)])
        lay = P.held_layout(1, 0, N, table)
        for mode in ("star", "ring"):
            held = torch.zeros(int(lay[N]), dtype=torch.uint8, device="cuda")
            comm.place(mode, table, b64.data_ptr(), held.data_ptr())
            torch.cuda.synchronize()
            same = torch.equal(held, b64[:int(lay[N])])
            print(f"F={F} {mode}: group bytes {grp[1] - grp[0]} held {int(lay[N])} equal {same} {comm.counters()}", flush=True)
            if not same:
                for f in range(N):
                    a, b = int(lay[f]), int(lay[f + 1])
                    d = torch.nonzero(held[a:b] != b64[a:b]).flatten()
                    if d.numel():
                        z = int((held[a:b][d] == 0).sum())
                        print(f"   group {f} [{a},{b}): {d.numel()} bytes differ, first {int(d[0])} last {int(d[-1])}, {z} of them zero in held", flush=True)
            del held
        comm.close()
        plan.close()
        del files, b64
