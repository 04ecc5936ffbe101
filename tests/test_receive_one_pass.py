"""dfs_receive_fragments_batch in one pass (a lane decodes, stores and hashes
its message; batches of more than 32,768 dword-aligned messages) against the
two-kernel path and the oracle: the replica receiver's decode + hash
(StorageNode.java:281-282) with java.util.Base64's rules for what is accepted
(unpadded 2- and 3-char endings, "xx==", "xxx=") and what throws (a char
outside the alphabet anywhere, a dangling char, padding in the wrong place)."""
import base64
import ctypes
import hashlib
import random

import numpy as np
import pytest

import dfs_amd
import oracle as O
from dfs_amd import _lib as L

pytestmark = pytest.mark.gpu


def _corpus():
    rng = random.Random(23)
    alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/="
    texts = [bytes(rng.choice(alphabet + b"-_ \n\xff") for _ in range(rng.randrange(0, 40))) for _ in range(1500)]
    for n in list(range(0, 260)) + [1000, 4095, 4096, 4097, 20000, 65537]:  # every block / unit phase, padded and not
        d = bytes(rng.getrandbits(8) for _ in range(n))
        t = base64.b64encode(d)
        texts += [t, t.rstrip(b"=")]
    for _ in range(60):  # long texts damaged at one place: first block, last blocks, final unit, padding
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(100, 30000)))
        t = bytearray(base64.b64encode(d))
        where = rng.choice([rng.randrange(len(t)), 1, len(t) - 1, len(t) - 2, len(t) - 3, len(t) - 70])
        t[where] = rng.choice(b"*-_= \nA")
        texts.append(bytes(t))
    return texts


def _receive(eng, texts):
    n = len(texts)
    spans = np.zeros((n, 2), dtype=np.uint64)
    out_off = np.zeros(n, dtype=np.uint64)
    pos = opos = 0
    for i, t in enumerate(texts):
        spans[i] = (pos, len(t))
        out_off[i] = opos
        pos += (len(t) + 3) & ~3      # chars start on dword boundaries
        opos += (3 * ((len(t) + 3) // 4) + 15) & ~15  # decoded bytes at 16-byte aligned places
    buf = np.full(pos + 16, ord("#"), dtype=np.uint8)
    for (o, ln), t in zip(spans, texts):
        buf[int(o):int(o) + int(ln)] = np.frombuffer(t, dtype=np.uint8)
    out = np.full(opos + 16, 0xEE, dtype=np.uint8)
    out_len = np.full(n, 77, dtype=np.uint64)
    dig = np.full((n, 32), 0xDD, dtype=np.uint8)
    status = np.full(n, 99, dtype=np.int32)
    rc = L.lib().dfs_receive_fragments_batch(eng.ctx, buf.ctypes.data, spans.ctypes.data, n, out.ctypes.data,
                                             out_off.ctypes.data, out_len.ctypes.data, dig.ctypes.data, status.ctypes.data, 0)
    assert rc in (L.DFS_OK, L.DFS_E_DECODE)
    return rc, out, out_off, out_len, dig, status


def test_receive_one_pass_vs_two_kernels_and_oracle(monkeypatch):
    corpus = _corpus()
    texts = (corpus * (33000 // len(corpus) + 1))[:33000]
    with dfs_amd.FragmentEngine(0) as eng:
        rc1, out1, off, len1, dig1, st1 = _receive(eng, texts)
        assert eng.stats()["recv_one_pass"] == 1
    monkeypatch.setenv("DFS_RECV_FUSED", "0")
    with dfs_amd.FragmentEngine(0) as eng:
        rc2, out2, _, len2, dig2, st2 = _receive(eng, texts)
        assert eng.stats()["recv_one_pass"] == 0
    assert rc1 == rc2 == L.DFS_E_DECODE
    assert st1.tolist() == st2.tolist() and len1.tolist() == len2.tolist() and (dig1 == dig2).all()
    for i, t in enumerate(texts[:len(corpus)]):
        want = O.c_b64_decode(t)
        if want is None:  # IllegalArgumentException: no bytes, no hash (the 0xDD fill stays)
            assert st1[i] == L.DFS_E_DECODE and len1[i] == 0 and (dig1[i] == 0xDD).all(), t[:40]
        else:
            o = int(off[i])
            assert st1[i] == 0 and int(len1[i]) == len(want), t[:40]
            assert out1[o:o + len(want)].tobytes() == want, t[:40]
            assert dig1[i].tobytes() == hashlib.sha256(want).digest(), t[:40]
