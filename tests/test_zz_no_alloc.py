"""dfs_sha256_batch_static (the entry point that allocates nothing: its lane
descriptors and queue words live in the library's static device array) against
dfs_sha256_batch on the same device buffers, through the C ABI: two calls in a
row, the second with a smaller input, so the array is reused with stale
contents behind the live part.  Collected last (file name)."""
import numpy as np
import pytest

import dfs_amd
from dfs_amd import _lib as L
from dfs_amd.engine import sha256_device, sha256_static_device

pytestmark = pytest.mark.gpu


def _case(eng, torch, dev, rng, n, max_len):
    lens = rng.integers(0, max_len, n).astype(np.uint64)
    lens[:: max(1, n // 7)] = 0                      # empty messages
    lens[1:: max(1, n // 5)] = [55, 56, 63, 64, 65, 119, 120][: len(lens[1:: max(1, n // 5)])] if n >= 40 else 3
    gaps = rng.integers(0, 5, n).astype(np.uint64)   # ragged, unaligned starts
    offs = np.cumsum(lens + gaps) - (lens + gaps) + gaps
    total = int(offs[-1] + lens[-1]) + 64
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev,
                         generator=torch.Generator(device=dev).manual_seed(int(rng.integers(1 << 30))))
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    spans = np.stack([offs, lens], axis=1).astype(np.uint64)
    want = sha256_device(eng, data.data_ptr(), spans)                     # dfs_sha256_batch, DFS_DEVICE_PTRS
    d_spans = torch.from_numpy(spans.view(np.int64).copy()).to(dev)
    d_dig = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    d_st = torch.full((n,), 7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    rc = sha256_static_device(eng, data.data_ptr(), d_spans.data_ptr(), n, d_dig.data_ptr(), d_st.data_ptr())
    assert rc == L.DFS_OK
    torch.cuda.synchronize(dev)
    got = d_dig.view(n, 32).cpu().numpy()
    assert (d_st.cpu().numpy() == 0).all()
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"n={n}: {bad.size} digests differ, first at message {bad[:5]}"
    return data, spans, want


def test_static_entry_matches_batch_entry_two_calls():
    import hashlib
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(20261113)
    with dfs_amd.FragmentEngine(0) as eng:
        print("static entry: call 1, n=40000 (persistent kernel)", flush=True)
        _case(eng, torch, dev, rng, 40000, 2000)
        print("static entry: call 2, n=1500 (smaller: latency kernel, stale descriptors behind it)", flush=True)
        data, spans, want = _case(eng, torch, dev, rng, 1500, 6000)
        host = data.cpu().numpy()
        for i in (0, 1, 777, 1499):  # and against hashlib, independently of the library
            o, n = int(spans[i, 0]), int(spans[i, 1])
            assert hashlib.sha256(host[o:o + n].tobytes()).digest() == want[i].tobytes()
        print("static entry: call 3, n=33000 again larger", flush=True)
        _case(eng, torch, dev, rng, 33000, 300)
        # beyond the static array: rejected before any launch, with its own message
        rc = sha256_static_device(eng, data.data_ptr(), 8, L.DFS_STATIC_MAX_MSGS + 1, 8)
        assert rc == L.DFS_E_TOOBIG
        assert b"at most 65,536" in dfs_amd.lib().dfs_strerror(rc)
        assert sha256_static_device(eng, 0, 0, 0, 0) == L.DFS_OK


def test_static_entry_in_a_captured_graph():
    """The allocation-free entry under stream capture: one call recorded into a
    HIP graph (torch.cuda.graph on the engine's stream), then replayed four
    times over new input bytes, with eager work (the input refill, the
    reference digests through dfs_sha256_batch on another ctx) and device
    synchronisations between the replays.  Every replay's digests are checked
    against the eager result: the kernels' queue words and descriptors are
    re-initialised by the entry's own prep kernel inside the graph."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    n = 30000  # the persistent kernel
    lens = rng.integers(0, 1500, n).astype(np.uint64)
    offs = np.cumsum(lens + 3) - (lens + 3)
    spans = np.stack([offs, lens], axis=1).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 64
    gen = torch.Generator(device=dev).manual_seed(99)
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    d_spans = torch.from_numpy(spans.view(np.int64).copy()).to(dev)
    d_dig = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    d_st = torch.full((n,), 7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    with dfs_amd.FragmentEngine(0) as eng, dfs_amd.FragmentEngine(0) as ref:
        s = torch.cuda.Stream(dev)
        eng.set_stream(s.cuda_stream)
        args = (data.data_ptr(), d_spans.data_ptr(), n, d_dig.data_ptr(), d_st.data_ptr())
        assert sha256_static_device(eng, *args) == L.DFS_OK  # eager once: everything lazy is loaded
        torch.cuda.synchronize(dev)
        print("static entry: capturing one call into a graph", flush=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            rc = sha256_static_device(eng, *args)
        assert rc == L.DFS_OK
        for rep in range(4):
            data.copy_(torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen))  # eager work
            d_dig.zero_()
            d_st.fill_(7)
            torch.cuda.synchronize(dev)
            want = sha256_device(ref, data.data_ptr(), spans)  # eager, another ctx; synchronises
            print(f"static entry: graph replay {rep + 1}", flush=True)
            g.replay()
            torch.cuda.synchronize(dev)
            got = d_dig.view(n, 32).cpu().numpy()
            assert (d_st.cpu().numpy() == 0).all(), rep
            bad = np.nonzero((got != want).any(axis=1))[0]
            assert bad.size == 0, f"replay {rep + 1}: {bad.size} digests differ, first at message {bad[:5]}"
        eng.set_stream(0)
