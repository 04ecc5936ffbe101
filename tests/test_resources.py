"""Device and pinned memory come back: contexts, upload / download / replica
plans, a communicator and a batcher are created, used and destroyed twenty
times over; the device's free memory afterwards is what it was after the
first round (hipMemGetInfo through torch), so nothing leaks per cycle."""
import numpy as np
import pytest

import dfs_amd
import oracle as O
from dfs_amd import placement as P
from dfs_amd.batcher import Batcher

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _cycle(torch, dev, i):
    nfiles, S, N = 512, 40000 + i, 5
    spans = np.stack([np.arange(nfiles, dtype=np.uint64) * np.uint64(S), np.full(nfiles, S, np.uint64)], axis=1)
    with dfs_amd.FragmentEngine(0) as eng:
        files = torch.empty(nfiles * S + 64, dtype=torch.uint8, device=dev)
        dfs_amd.synth_fill(eng, files.data_ptr(), spans, 0, O.SYNTH_SEED)
        plan = dfs_amd.UploadPlan(eng, spans, N, frag_major=True, align128=True)
        fd = torch.empty(nfiles * 32, dtype=torch.uint8, device=dev)
        frd = torch.empty(nfiles * N * 32, dtype=torch.uint8, device=dev)
        b64 = torch.empty(max(plan.b64_total, 1), dtype=torch.uint8, device=dev)
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
        dplan = dfs_amd.DownloadPlan(eng, plan.b64_spans([S] * nfiles), nfiles, N, np.full(nfiles, S, np.uint64),
                                     np.arange(nfiles, dtype=np.uint64) * np.uint64(S))
        out = torch.empty(nfiles * S, dtype=torch.uint8, device=dev)
        st = dplan.run(b64.data_ptr(), frd.data_ptr(), fd.data_ptr(), out.data_ptr())
        assert (st == 0).all()
        comm = P.Comm(eng, P.unique_id(), 1, 0)
        rp = P.ReplicaPlan(comm, N, [S] * nfiles, True)
        held = torch.empty(max(rp.held_bytes, 1), dtype=torch.uint8, device=dev)
        comm.place("star", rp.table, b64.data_ptr(), held.data_ptr())
        raw = torch.empty(rp.raw_bytes + 16, dtype=torch.uint8, device=dev)
        verdict = torch.empty(rp.nheld, dtype=torch.int32, device=dev)
        failed = torch.empty(1, dtype=torch.int32, device=dev)
        rp.verify(frd.data_ptr(), held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
        torch.cuda.synchronize(dev)
        assert int(failed[0]) == 0
        rp.close()
        comm.close()
        dplan.close()
        plan.close()
    with Batcher(0, N, max_wait_us=100) as b:
        data = O.c_synth(5, i, 100000)
        fdig, _, texts = b.upload(data)
        stt, back = b.download(texts, len(data), None, fdig)
        assert stt == 0 and back == data
        fdig2, _, texts2 = b.upload_view(np.frombuffer(data, np.uint8))
        assert fdig2 == fdig and texts2 == texts
    del files, fd, frd, b64, out, held, raw, verdict, failed
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()


def test_no_device_memory_leak_over_create_destroy_cycles():
    import torch
    dev = torch.device("cuda", 0)
    _cycle(torch, dev, 0)  # first use: lazily created library state stays
    _cycle(torch, dev, 1)
    torch.cuda.synchronize(dev)
    free0, _ = torch.cuda.mem_get_info(dev)
    for i in range(2, 22):
        _cycle(torch, dev, i)
    torch.cuda.synchronize(dev)
    free1, _ = torch.cuda.mem_get_info(dev)
    print(f"free device memory: {free0} -> {free1} after 20 cycles", flush=True)
    assert free0 - free1 < (64 << 20), f"{(free0 - free1) >> 20} MiB of device memory gone after 20 cycles"
