"""Config 4 (files larger than HBM): the chunk schedule of
dfs_amd.streaming, replayed on the CPU with hashlib / base64 (host logic, no
GPU), and the streamed GPU upload against the oracle (gpu)."""
import base64
import hashlib

import numpy as np
import pytest

import oracle as O
from dfs_amd.streaming import GRAIN, ChunkSchedule


def replay(data: bytes, nfrag: int, chunk: int):
    """Feed every message part by part exactly as the GPU path does; return
    (fileId, [fragment digests], [fragment Base64])."""
    sc = ChunkSchedule(len(data), nfrag, chunk)
    h = [hashlib.sha256() for _ in range(nfrag + 1)]
    b64 = [b""] * (nfrag + 1)
    seen_final = [False] * (nfrag + 1)
    for c, lo, hi, items in sc.plan():
        window = data[lo:hi]  # the only bytes the GPU holds for this chunk
        for k, a, n, begin, final in items:
            assert lo <= a and a + n <= hi
            assert final or (n % GRAIN == 0 and n > 0)
            assert begin == (h[k].copy().digest() == hashlib.sha256().digest() and not b64[k] and not seen_final[k])
            part = window[a - lo:a - lo + n]
            h[k].update(part)
            if k:
                b64[k] += base64.b64encode(part)
            seen_final[k] |= final
    assert all(seen_final)
    return h[0].digest(), [x.digest() for x in h[1:]], b64[1:]


@pytest.mark.parametrize("S,N,chunk", [
    (0, 5, 192), (3, 5, 192), (191, 5, 192), (192, 5, 192), (1000, 5, 192), (4096 * 3 + 7, 5, 384),
    (100003, 5, 1920), (262144, 8, 4032), (262144, 8, 192 * 1365), (53687 * 5 + 2, 5, 192 * 7),
    (1 << 20, 5, 192 * 128), (1 << 20, 5, 192 * 5462)])
def test_chunk_schedule_matches_one_shot(S, N, chunk):
    data = np.random.default_rng(S + N).integers(0, 256, S, dtype=np.uint8).tobytes()
    fid, fd, fb = replay(data, N, chunk)
    assert fid == hashlib.sha256(data).digest()
    for i, (o, n) in enumerate(O.py_split(S, N)):
        assert fd[i] == hashlib.sha256(data[o:o + n]).digest(), i
        assert fb[i] == base64.b64encode(data[o:o + n]), i


def test_chunk_must_be_grain_multiple():
    with pytest.raises(ValueError):
        ChunkSchedule(1000, 5, 100)


@pytest.mark.gpu
def test_streaming_upload_gpu(engine):
    """Three files of 3 MiB + 12,345 B, N=5, 196,608-byte chunks (17 chunks):
    fileId / fragment digests and Base64 bit-exact vs the oracle."""
    import torch
    from dfs_amd.streaming import StreamingUpload, synth_fill_at
    F, S, N, chunk = 3, 3 * (1 << 20) + 12345, 5, 192 * 1024
    dev = torch.device("cuda", 0)
    up = StreamingUpload(engine, F, S, N, chunk, dev)
    got_b64 = [[bytearray() for _ in range(N)] for _ in range(F)]

    def fill(ptr, lo, hi):
        spans = np.array([(f * up.stride, hi - lo) for f in range(F)], dtype=np.uint64)
        synth_fill_at(engine, ptr, spans, 100, O.SYNTH_SEED, lo)

    def emit(c, items, out_off):
        host = up.d_b64[:int(out_off[-1])].cpu().numpy().tobytes()
        m = len(items)
        for f in range(F):
            for j, (k, a, n, begin, final) in enumerate(items):
                got_b64[f][k - 1] += host[int(out_off[f * m + j]):int(out_off[f * m + j + 1])]

    up.run(fill, emit)
    torch.cuda.synchronize()
    for f in range(F):
        data = O.c_synth(100 + f, 0, S)
        assert up.file_digest(f) == hashlib.sha256(data).digest()
        for i, (o, n) in enumerate(O.py_split(S, N)):
            assert up.frag_digest(f, i) == hashlib.sha256(data[o:o + n]).digest(), (f, i)
            assert bytes(got_b64[f][i]) == base64.b64encode(data[o:o + n]), (f, i)


@pytest.mark.gpu
def test_synth_fill_at_matches_oracle(engine):
    import torch
    from dfs_amd.streaming import synth_fill_at
    dev = torch.device("cuda", 0)
    buf = torch.zeros(3 * 5000, dtype=torch.uint8, device=dev)
    spans = np.array([(0, 4999), (5000, 1), (10000, 4096)], dtype=np.uint64)
    for off in (0, 8, 1 << 30):
        synth_fill_at(engine, buf.data_ptr(), spans, 7, O.SYNTH_SEED, off)
        h = buf.cpu().numpy().tobytes()
        for f, (o, n) in enumerate(spans):
            assert h[int(o):int(o + n)] == O.c_synth(7 + f, off, int(n)), (off, f)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [9000, 20000])
def test_sha256_update_many_messages_in_parts(engine, n):
    """dfs_sha256_update_batch over thousands of messages in three parts (the
    first two multiples of 64 bytes, states carried in HBM between launches):
    9,000 messages run the pair-lane latency kernel with two wave pairs per
    workgroup, 20,000 the one-lane kernel with two pairs; against hashlib."""
    rng = np.random.default_rng(n)
    cuts = [(64 * int(a), 64 * int(b), int(c)) for a, b, c in
            zip(rng.integers(1, 4, n), rng.integers(0, 3, n), rng.integers(0, 130, n))]
    msgs = [rng.integers(0, 256, a + b + c, dtype=np.uint8).tobytes() for a, b, c in cuts]
    state = np.zeros((n, 8), dtype=np.uint32)
    total = [len(m) for m in msgs]
    assert engine.sha256_update([m[:a] for m, (a, b, c) in zip(msgs, cuts)], state, True, False) is None
    assert engine.sha256_update([m[a:a + b] for m, (a, b, c) in zip(msgs, cuts)], state, False, False) is None
    got = engine.sha256_update([m[a + b:] for m, (a, b, c) in zip(msgs, cuts)], state, False, True, total)
    assert all(bytes(g) == hashlib.sha256(m).digest() for g, m in zip(got, msgs))
