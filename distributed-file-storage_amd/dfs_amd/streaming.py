"""Chunked upload of files larger than HBM — BASELINE config 4 ("long-fragment
skew": 1,024 files x 256 MiB, N = 5; 256 GiB of input plus 341 GiB of Base64
exceed one GPU's 288 GB).

Same pipeline as handleUpload (StorageNode.java, SN:line): the fileId is the
SHA-256 of the whole file (SN:127), every fragment of the N-way split
(SN:138-157) is hashed (SN:159) and Base64-encoded (SN:636) — but the files
pass through HBM in chunks.  Every SHA-256 message carries its 8-word state
from chunk to chunk (dfs_sha256_update_parts: per-part state slots, so a
fragment can begin and end in other chunks than its file's fileId message)
and every fragment's Base64 is produced part by part (a part whose length is a
multiple of 3 encodes to exactly the next 4n/3 characters, no padding).

Fragment starts are arbitrary (53,687,092 x i at 256 MiB), so a part ends on
a GRAIN = lcm(64, 3) = 192-byte boundary relative to its fragment and the
< 192 bytes left over are re-read from the next chunk's window, which starts
GRAIN bytes before the chunk itself.

ChunkSchedule is pure host planning (CPU-testable against hashlib/base64);
StreamingUpload drives libdfsgpu.so on device buffers.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Iterator, List, Optional, Tuple

import numpy as np

from . import _lib as L
from ._lib import check, lib
from .engine import FragmentEngine, _ptr, split_plan

GRAIN = 192  # lcm(64, 3)
PART_DTYPE = np.dtype([("off", "<u8"), ("len", "<u8"), ("total", "<u8"), ("slot", "<u4"), ("flags", "<u4")])
assert PART_DTYPE.itemsize == 32  # dfs_part (include/dfs_gpu.h)

# (message kind, absolute file offset, length, begin, final); kind 0 = the
# fileId message (whole file), kind 1 + i = fragment i.
Item = Tuple[int, int, int, bool, bool]


class ChunkSchedule:
    """Which bytes of every message each chunk feeds (identical for every
    file of one length).  Chunk c holds file bytes [lo, hi) with
    lo = max(0, c*chunk - GRAIN), hi = min(S, (c+1)*chunk)."""

    def __init__(self, file_len: int, nfrag: int, chunk: int):
        if chunk <= 0 or chunk % GRAIN:
            raise ValueError(f"chunk must be a positive multiple of {GRAIN}")
        self.S, self.N, self.chunk = int(file_len), int(nfrag), int(chunk)
        fr = split_plan(self.S, self.N)
        self.msg_start = [0] + [o for o, _ in fr]
        self.msg_len = [self.S] + [n for _, n in fr]
        self.nchunks = max(1, -(-self.S // self.chunk))

    def window(self, c: int) -> Tuple[int, int]:
        return max(0, c * self.chunk - GRAIN), min(self.S, (c + 1) * self.chunk)

    def plan(self) -> Iterator[Tuple[int, int, int, List[Item]]]:
        pos = [0] * (self.N + 1)
        done = [False] * (self.N + 1)
        for c in range(self.nchunks):
            lo, hi = self.window(c)
            items: List[Item] = []
            for k in range(self.N + 1):
                if done[k]:
                    continue
                s, ln = self.msg_start[k], self.msg_len[k]
                a = s + pos[k]
                if s + ln <= hi:  # the message ends in this chunk
                    assert a >= lo, "carry exceeds the chunk window"
                    items.append((k, a, s + ln - a, pos[k] == 0, True))
                    done[k] = True
                elif a < hi:
                    assert a >= lo, "carry exceeds the chunk window"
                    n = (hi - a) // GRAIN * GRAIN
                    if n:
                        items.append((k, a, n, pos[k] == 0, False))
                        pos[k] += n
            yield c, lo, hi, items
        assert all(done)


class StreamingUpload:
    """Config-4 upload of `nfiles` files of `file_len` bytes on one GPU.

    Digest slots: slot f = fileId of file f; slot nfiles + f*nfrag + i =
    fragment i of file f (32 bytes each, big-endian, in `digests`)."""

    def __init__(self, engine: FragmentEngine, nfiles: int, file_len: int, nfrag: int, chunk: int, device):
        import torch
        self.engine, self.nfiles, self.N = engine, int(nfiles), int(nfrag)
        self.sched = ChunkSchedule(file_len, nfrag, chunk)
        self.stride = (chunk + GRAIN + 255) // 256 * 256  # per-file window in the chunk buffer
        self.nslots = self.nfiles * (1 + self.N)
        self.device = device
        self.d_chunk = torch.empty(self.nfiles * self.stride, dtype=torch.uint8, device=device)
        self.d_state = torch.empty(self.nslots * 8, dtype=torch.int32, device=device)
        self.digests = torch.zeros(self.nslots * 32, dtype=torch.uint8, device=device)
        self.b64_cap = self.nfiles * ((chunk + GRAIN) * 4 // 3 + 8 * (self.N + 1))
        self.d_b64 = torch.empty(self.b64_cap, dtype=torch.uint8, device=device)

    def slot(self, f: int, kind: int) -> int:
        return f if kind == 0 else self.nfiles + f * self.N + kind - 1

    def _parts(self, lo: int, items: List[Item]) -> np.ndarray:
        F = self.nfiles
        parts = np.zeros(F * len(items), dtype=PART_DTYPE)
        fo = np.arange(F, dtype=np.uint64) * np.uint64(self.stride)
        for j, (k, a, n, begin, final) in enumerate(items):
            sl = parts[j::len(items)]
            sl["off"] = fo + np.uint64(a - lo)
            sl["len"] = n
            sl["total"] = self.sched.msg_len[k]
            sl["slot"] = (np.arange(F, dtype=np.uint32) if k == 0 else
                          np.uint32(F) + np.arange(F, dtype=np.uint32) * np.uint32(self.N) + np.uint32(k - 1))
            sl["flags"] = (L.DFS_SHA_BEGIN if begin else 0) | (L.DFS_SHA_FINAL if final else 0)
        return parts

    def run(self, fill: Callable[[int, int, int], None],
            emit_b64: Optional[Callable[[int, List[Item], np.ndarray], None]] = None) -> dict:
        """fill(d_chunk_ptr, lo, hi) writes every file's bytes [lo, hi) at
        d_chunk + f*stride.  emit_b64(c, fragment_items, out_off) sees each
        chunk's Base64 (d_b64 at out_off[f*m + j] for file f, item j).
        Returns per-run kernel times (ms)."""
        ctx = self.engine.ctx
        sha_ms = b64_ms = 0.0
        for c, lo, hi, items in self.sched.plan():
            fill(self.d_chunk.data_ptr(), lo, hi)
            parts = self._parts(lo, items)
            self.engine.set_profiling(True)
            check(lib().dfs_sha256_update_parts(ctx, ctypes.c_void_p(self.d_chunk.data_ptr()), _ptr(parts),
                                                len(parts), ctypes.c_void_p(self.d_state.data_ptr()),
                                                ctypes.c_void_p(self.digests.data_ptr()), L.DFS_DEVICE_PTRS),
                  "dfs_sha256_update_parts")
            sha_ms += self.engine.timings()["sha"]
            fitems = [it for it in items if it[0] > 0]
            if fitems:
                fp = parts.reshape(self.nfiles, len(items))[:, [j for j, it in enumerate(items) if it[0] > 0]]
                spans = np.ascontiguousarray(np.stack([fp["off"].ravel(), fp["len"].ravel()], axis=1),
                                             dtype=np.uint64)
                out_off = np.zeros(len(spans) + 1, dtype=np.uint64)
                check(lib().dfs_b64_encode_batch(ctx, ctypes.c_void_p(self.d_chunk.data_ptr()), _ptr(spans),
                                                 len(spans), ctypes.c_void_p(self.d_b64.data_ptr()), self.b64_cap,
                                                 _ptr(out_off), L.DFS_DEVICE_PTRS), "dfs_b64_encode_batch")
                b64_ms += self.engine.timings()["b64enc"]
                if emit_b64:
                    emit_b64(c, fitems, out_off)
            self.engine.set_profiling(False)
        return {"sha_ms": sha_ms, "b64_ms": b64_ms}

    def file_digest(self, f: int) -> bytes:
        return self.digests[32 * f:32 * f + 32].cpu().numpy().tobytes()

    def frag_digest(self, f: int, i: int) -> bytes:
        s = self.slot(f, i + 1)
        return self.digests[32 * s:32 * s + 32].cpu().numpy().tobytes()


def synth_fill_at(engine: FragmentEngine, d_dst: int, spans: np.ndarray, first_file: int, seed: int,
                  file_off: int) -> None:
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    check(lib().dfs_synth_fill_at(engine.ctx, ctypes.c_void_p(d_dst), _ptr(spans), len(spans), first_file, seed,
                                  file_off), "dfs_synth_fill_at")
