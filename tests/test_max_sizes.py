"""One Base64 job of more than 4 GiB on the GPU.

The reference holds a file in one Java byte[] (below 2 GiB); the library takes
messages up to 2^37 bytes, and the bench's batches reach 68 GB, so offsets
inside a batch are exercised far beyond 2^32 there.  What no batch of small
files reaches is a SINGLE job whose own length passes 2^32: here one message
of 4.5 GiB is encoded (StorageNode.java:636) from a source 3 bytes past a
dword boundary, compared byte for byte with Python's base64 of the same bytes,
and decoded back (:281) to a destination 1 byte past a 16-byte boundary.
SHA-256 is left out on purpose: one message is one lane, and a lane hashes
about 36 MB/s (4.5 GiB would take two minutes)."""
import base64
import ctypes

import numpy as np
import pytest

import dfs_amd
import oracle as O
from dfs_amd import _lib as L

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def test_base64_job_over_4_gib():
    import torch
    n = (1 << 32) + (1 << 29) + 4          # message bytes; n % 3 == 1: the encoder pads with "=="
    enc = 4 * ((n + 2) // 3)
    assert n > 1 << 32 and enc > 1 << 32 and n % 3 == 1
    with dfs_amd.FragmentEngine(0) as eng:
        src = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        dfs_amd.synth_fill(eng, src.data_ptr(), np.array([(0, n + 64)], dtype=np.uint64), 3, O.SYNTH_SEED)
        b64 = torch.zeros(enc + 64, dtype=torch.uint8, device="cuda")
        span = np.array([(3, n)], dtype=np.uint64)
        off = np.zeros(2, dtype=np.uint64)
        lib = L.lib()
        torch.cuda.synchronize()  # torch's fills run on its stream, the library on the engine's
        print(f"encode {n} bytes -> {enc} chars", flush=True)
        assert lib.dfs_b64_encode_batch(eng.ctx, ctypes.c_void_p(src.data_ptr()), span.ctypes.data, 1,
                                        ctypes.c_void_p(b64.data_ptr()), enc, off.ctypes.data, L.DFS_DEVICE_PTRS) == 0
        torch.cuda.synchronize()
        assert off.tolist() == [0, enc] and int(b64[enc]) == 0 and bytes(b64[enc - 2:enc].cpu().numpy()) == b"=="
        piece = 192 << 20  # source bytes per comparison step, a multiple of 3
        for a in range(0, n, piece):
            b = min(a + piece, n)
            want = base64.b64encode(src[3 + a:3 + b].cpu().numpy().tobytes())
            got = b64[a // 3 * 4:a // 3 * 4 + len(want)].cpu().numpy().tobytes()
            assert got == want, f"Base64 differs in source bytes [{a}, {b})"
        back = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
        msg = np.array([(0, enc)], dtype=np.uint64)
        out_off = np.array([1], dtype=np.uint64)
        out_len = np.zeros(1, dtype=np.uint64)
        status = np.full(1, 99, dtype=np.int32)
        torch.cuda.synchronize()
        print(f"decode {enc} chars", flush=True)
        assert lib.dfs_b64_decode_batch(eng.ctx, ctypes.c_void_p(b64.data_ptr()), msg.ctypes.data, 1,
                                        ctypes.c_void_p(back.data_ptr()), out_off.ctypes.data, out_len.ctypes.data,
                                        status.ctypes.data, L.DFS_DEVICE_PTRS) == 0
        torch.cuda.synchronize()
        assert int(out_len[0]) == n and int(status[0]) == 0
        assert int(back[0]) == 0 and int(back[1 + n]) == 0
        assert torch.equal(back[1:1 + n], src[3:3 + n])
        # one char outside the alphabet, beyond 2^32: the decoder's IllegalArgumentException (SN:281)
        b64[(1 << 32) + 12345] = ord("!")
        torch.cuda.synchronize()
        assert lib.dfs_b64_decode_batch(eng.ctx, ctypes.c_void_p(b64.data_ptr()), msg.ctypes.data, 1,
                                        ctypes.c_void_p(back.data_ptr()), out_off.ctypes.data, out_len.ctypes.data,
                                        status.ctypes.data, L.DFS_DEVICE_PTRS) == L.DFS_E_DECODE
        assert int(status[0]) == L.DFS_E_DECODE
