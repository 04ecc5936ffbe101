"""Python face of the fragment pipeline over libdfsgpu.so.

Mirrors the reference's fragment-pipeline operations (StorageNode.java, cited
SN:line) batch-wise; every byte of data-path work runs in the gfx950 kernels
behind the C ABI.  Host buffers are numpy arrays; device buffers are torch
tensors (PyTorch is plumbing here: device memory, streams, distributed).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import check, dfs_span, lib


class IllegalArgumentException(ValueError):
    """java.util.Base64.Decoder's IllegalArgumentException (SN:281)."""


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _pack(messages: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate byte strings into one buffer + span array."""
    n = len(messages)
    spans = np.zeros((n, 2), dtype=np.uint64)
    total = sum(len(m) for m in messages)
    buf = np.empty(max(total, 1), dtype=np.uint8)
    o = 0
    for i, m in enumerate(messages):
        ln = len(m)
        spans[i] = (o, ln)
        if ln:
            buf[o:o + ln] = np.frombuffer(m, dtype=np.uint8)
        o += ln
    return buf, spans


def split_plan(file_len: int, nfrag: int) -> List[Tuple[int, int]]:
    """handleUpload's split (SN:138-171) as computed by the library."""
    out = (dfs_span * nfrag)()
    check(lib().dfs_split_plan(file_len, nfrag, out), "dfs_split_plan")
    return [(s.off, s.len) for s in out]


def fragment_holders(frag: int, nfrag: int) -> Tuple[int, int]:
    """0-based nodes holding fragment `frag` (SN:143-145, 427-428)."""
    h = (ctypes.c_uint32 * 2)()
    check(lib().dfs_fragment_holders(frag, nfrag, h), "dfs_fragment_holders")
    return h[0], h[1]


def b64_encoded_len(n: int) -> int:
    return lib().dfs_b64_encoded_len(n)


@dataclass
class Fragment:
    """StorageNode.Fragment (SN:779-789) plus its split offset and Base64."""
    index: int
    offset: int
    length: int
    hash: str
    b64: Optional[bytes] = None


@dataclass
class UploadResult:
    file_id: str
    fragments: List[Fragment]


class FragmentEngine:
    """One dfs_ctx on one gfx950 device."""

    def __init__(self, device: int = 0):
        self._ctx = ctypes.c_void_p()
        check(lib().dfs_open(ctypes.byref(self._ctx), device), "dfs_open")
        self.device = device

    # -- context -------------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            lib().dfs_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self) -> ctypes.c_void_p:
        return self._ctx

    def set_stream(self, stream_handle: int) -> None:
        check(lib().dfs_set_stream(self._ctx, ctypes.c_void_p(stream_handle or None)), "dfs_set_stream")

    def set_profiling(self, on: bool) -> None:
        check(lib().dfs_set_profiling(self._ctx, int(on)), "dfs_set_profiling")

    def timings(self) -> dict:
        ms = (ctypes.c_float * L.DFS_T_COUNT)()
        check(lib().dfs_get_timings(self._ctx, ms, L.DFS_T_COUNT), "dfs_get_timings")
        names = ["sha", "b64enc", "b64dec", "gather", "total"]
        return {k: (v if v >= 0 else None) for k, v in zip(names, ms)}

    def stats(self) -> dict:
        """ctx counters (dfs_get_stats): ovl_redo = decode-ahead downloads
        whose SHA launch was redone after an in-kernel wait timed out;
        recv_one_pass = dfs_receive_fragments_batch calls that decoded and
        hashed in one pass."""
        v = (ctypes.c_uint64 * L.DFS_S_COUNT)()
        check(lib().dfs_get_stats(self._ctx, v, L.DFS_S_COUNT), "dfs_get_stats")
        return {"ovl_redo": int(v[L.DFS_S_OVL_REDO]), "recv_one_pass": int(v[L.DFS_S_RECV_ONE_PASS])}

    # -- sha256Hex (SN:603-613) ----------------------------------------------
    def sha256(self, messages: Sequence[bytes]) -> List[bytes]:
        buf, spans = _pack(messages)
        n = len(messages)
        out = np.zeros((max(n, 1), 32), dtype=np.uint8)
        check(lib().dfs_sha256_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), 0), "dfs_sha256_batch")
        return [out[i].tobytes() for i in range(n)]

    def sha256_spans(self, buf: np.ndarray, spans: np.ndarray) -> np.ndarray:
        n = len(spans)
        out = np.zeros((max(n, 1), 32), dtype=np.uint8)
        spans = np.ascontiguousarray(spans, dtype=np.uint64)
        check(lib().dfs_sha256_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), 0), "dfs_sha256_batch")
        return out[:n]

    def sha256_hex(self, data: bytes) -> str:
        return self.sha256([data])[0].hex()

    def sha256_update(self, parts: Sequence[bytes], state: np.ndarray, begin: bool, final: bool,
                      total_len: Optional[Sequence[int]] = None) -> Optional[List[bytes]]:
        """One streaming step (dfs_sha256_update_batch): hash the next part of
        every message; `state` is an (n, 8) uint32 array updated in place.
        Returns the digests when final."""
        buf, spans = _pack(parts)
        n = len(parts)
        assert state.shape == (n, 8) and state.dtype == np.uint32 and state.flags.c_contiguous
        flags = (L.DFS_SHA_BEGIN if begin else 0) | (L.DFS_SHA_FINAL if final else 0)
        tl = np.array(list(total_len) if total_len is not None else [0] * n, dtype=np.uint64)
        out = np.zeros((max(n, 1), 32), dtype=np.uint8)
        check(lib().dfs_sha256_update_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(state), _ptr(tl),
                                            _ptr(out), flags), "dfs_sha256_update_batch")
        return [out[i].tobytes() for i in range(n)] if final else None

    def receive_fragments(self, texts: Sequence[bytes]) -> List[Tuple[Optional[bytes], Optional[str]]]:
        """handleInternalStoreFragments (SN:265-293): per received Base64
        fragment, (decoded bytes, sha256 hex) or (None, None) where the JDK
        decoder throws."""
        buf, spans = _pack(texts)
        n = len(texts)
        caps = [lib().dfs_b64_decoded_cap(len(t)) for t in texts]
        out_off = np.zeros(max(n, 1), dtype=np.uint64)
        o = 0
        for i, cp in enumerate(caps):
            out_off[i] = o
            o += cp
        out = np.zeros(max(o, 1), dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.int32)
        dig = np.zeros((max(n, 1), 32), dtype=np.uint8)
        rc = lib().dfs_receive_fragments_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), _ptr(out_off),
                                              _ptr(out_len), _ptr(dig), _ptr(status), 0)
        if rc not in (L.DFS_OK, L.DFS_E_DECODE):
            check(rc, "dfs_receive_fragments_batch")
        res = []
        for i in range(n):
            if status[i]:
                res.append((None, None))
            else:
                a = int(out_off[i])
                res.append((out[a:a + int(out_len[i])].tobytes(), dig[i].tobytes().hex()))
        return res

    # -- Base64 (SN:636 encode, SN:281 decode) --------------------------------
    def b64_encode(self, messages: Sequence[bytes]) -> List[bytes]:
        buf, spans = _pack(messages)
        n = len(messages)
        total = sum(b64_encoded_len(len(m)) for m in messages)
        out = np.zeros(max(total, 1), dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.uint64)
        check(lib().dfs_b64_encode_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), total, _ptr(off), 0),
              "dfs_b64_encode_batch")
        return [out[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]

    def b64_decode(self, texts: Sequence[bytes], out_offsets: Optional[Sequence[int]] = None
                   ) -> List[Optional[bytes]]:
        """Decoded bytes per message, None where the JDK would throw."""
        buf, spans = _pack(texts)
        n = len(texts)
        caps = [lib().dfs_b64_decoded_cap(len(t)) for t in texts]
        if out_offsets is None:
            out_off = np.zeros(max(n, 1), dtype=np.uint64)
            o = 0
            for i, c in enumerate(caps):
                out_off[i] = o
                o += c
        else:
            out_off = np.array(list(out_offsets) + [0] * (n == 0), dtype=np.uint64)
        end = max([int(out_off[i]) + caps[i] for i in range(n)] + [1])
        out = np.zeros(end, dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.int32)
        rc = lib().dfs_b64_decode_batch(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), _ptr(out_off),
                                       _ptr(out_len), _ptr(status), 0)
        if rc not in (L.DFS_OK, L.DFS_E_DECODE):
            check(rc, "dfs_b64_decode_batch")
        res: List[Optional[bytes]] = []
        for i in range(n):
            if status[i] != 0:
                res.append(None)
            else:
                o = int(out_off[i])
                res.append(out[o:o + int(out_len[i])].tobytes())
        return res

    def b64_decode_one(self, text: bytes) -> bytes:
        r = self.b64_decode([text])[0]
        if r is None:
            raise IllegalArgumentException("Illegal base64 input")
        return r

    # -- handleUpload (SN:118-189) ---------------------------------------------
    def upload(self, files: Sequence[bytes], nfrag: int, with_b64: bool = True) -> List[UploadResult]:
        buf, spans = _pack(files)
        nf = len(files)
        fd = np.zeros((max(nf, 1), 32), dtype=np.uint8)
        frd = np.zeros((max(nf * nfrag, 1), 32), dtype=np.uint8)
        b64_off = np.zeros(nf * nfrag + 1, dtype=np.uint64)
        total = sum(b64_encoded_len(ln) for f in files for (_, ln) in split_plan(len(f), nfrag))
        b64 = np.zeros(max(total, 1), dtype=np.uint8)
        flags = 0 if with_b64 else L.DFS_NO_B64
        check(lib().dfs_upload_batch(self._ctx, _ptr(buf), _ptr(spans), nf, nfrag, _ptr(fd), _ptr(frd),
                                     _ptr(b64), total, _ptr(b64_off), flags), "dfs_upload_batch")
        out = []
        for f in range(nf):
            frags = []
            for i, (off, ln) in enumerate(split_plan(len(files[f]), nfrag)):
                k = f * nfrag + i
                data = b64[int(b64_off[k]):int(b64_off[k + 1])].tobytes() if with_b64 else None
                frags.append(Fragment(i, off, ln, frd[k].tobytes().hex(), data))
            out.append(UploadResult(fd[f].tobytes().hex(), frags))
        return out

    # -- sendFragmentsToPeers + buildFragmentsJson (SN:195-205, 629-642) ----------
    def store_bodies(self, files: Sequence[bytes], nfrag: int, uploader: int,
                     file_ids: Sequence[str]) -> List[List[Tuple[int, bytes]]]:
        """storeFragments request bodies built on the device: per file, one
        (peer node k, body) per peer k != uploader (0-based, ascending), each
        carrying fragments k and k+1 mod nfrag (SN:199-200)."""
        buf, spans = _pack(files)
        nf = len(files)
        peers = nfrag - 1
        body_off = np.zeros(nf * peers + 1, dtype=np.uint64)
        dig = np.frombuffer(b"".join(bytes.fromhex(h) for h in file_ids) or b"\0", dtype=np.uint8).copy()
        check(lib().dfs_store_bodies_build(self._ctx, _ptr(buf), _ptr(spans), nf, nfrag, uploader, _ptr(dig), None,
                                           _ptr(body_off), 0), "dfs_store_bodies_build (layout)")
        out = np.zeros(max(int(body_off[-1]), 1), dtype=np.uint8)
        check(lib().dfs_store_bodies_build(self._ctx, _ptr(buf), _ptr(spans), nf, nfrag, uploader, _ptr(dig),
                                           _ptr(out), _ptr(body_off), 0), "dfs_store_bodies_build")
        res = []
        for f in range(nf):
            peers_k = [k for k in range(nfrag) if k != uploader]
            row = []
            for j, k in enumerate(peers_k):
                o = int(body_off[f * peers + j])
                n = int(lib().dfs_store_body_len(len(files[f]), nfrag, k, (k + 1) % nfrag))
                row.append((k, out[o:o + n].tobytes()))
            res.append(row)
        return res

    def store_receive(self, bodies: Sequence[bytes]):
        """handleInternalStoreFragments (SN:265-293) on the device for bodies in
        buildFragmentsJson form.  Per body: (status, fileId or None,
        [(index, bytes, sha256 hex)] for both entries or [])."""
        n = len(bodies)
        buf, spans = _pack(bodies)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        cap = sum((3 * ((len(b) + 3) // 4) + 16 + 15) & ~15 for b in bodies)  # dfs_store_bodies_receive's slots
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        idx = np.zeros(max(2 * n, 1), dtype=np.uint32)
        foff = np.zeros(max(2 * n, 1), dtype=np.uint64)
        flen = np.zeros(max(2 * n, 1), dtype=np.uint64)
        dig = np.zeros((max(n, 1), 2, 32), dtype=np.uint8)
        ids = np.zeros((max(n, 1), 64), dtype=np.uint8)
        status = np.zeros(max(n, 1), dtype=np.int32)
        check(lib().dfs_store_bodies_receive(self._ctx, _ptr(buf), _ptr(spans), n, _ptr(out), _ptr(out_off),
                                             _ptr(idx), _ptr(foff), _ptr(flen), _ptr(dig), _ptr(ids), _ptr(status), 0),
              "dfs_store_bodies_receive")
        res = []
        for i in range(n):
            st = int(status[i])
            if st == L.DFS_E_WIRE:
                res.append((st, None, []))
                continue
            frags = []
            for q in range(2):
                o, ln = int(foff[2 * i + q]), int(flen[2 * i + q])
                frags.append((int(idx[2 * i + q]), out[o:o + ln].tobytes(), dig[i, q].tobytes().hex()))
            res.append((st, ids[i].tobytes().decode("latin-1"), frags))
        return res

    # -- handleDownload gather + verify (SN:419-458) ------------------------------
    def reassemble_verify(self, frags: Sequence[Sequence[Optional[bytes]]],
                          expected_file_ids: Optional[Sequence[str]] = None
                          ) -> List[Tuple[int, Optional[bytes], str]]:
        """Per file: (status, rebuilt bytes or None, sha256 hex of rebuilt bytes)."""
        nfiles = len(frags)
        nfrag = len(frags[0]) if nfiles else 1
        keep = []
        ptrs = (ctypes.c_void_p * max(nfiles * nfrag, 1))()
        lens = np.zeros(max(nfiles * nfrag, 1), dtype=np.uint64)
        file_off = np.zeros(max(nfiles, 1), dtype=np.uint64)
        o = 0
        for f in range(nfiles):
            file_off[f] = o
            for i in range(nfrag):
                d = frags[f][i]
                k = f * nfrag + i
                if d is None:
                    ptrs[k] = None
                    lens[k] = 1  # a missing fragment: SN:443-446
                else:
                    a = np.frombuffer(d, dtype=np.uint8).copy() if d else np.zeros(1, np.uint8)
                    keep.append(a)
                    ptrs[k] = a.ctypes.data
                    lens[k] = len(d)
            o += int(sum(lens[f * nfrag:(f + 1) * nfrag]))
        out = np.zeros(max(o, 1), dtype=np.uint8)
        exp = None
        if expected_file_ids is not None:
            exp = np.frombuffer(b"".join(bytes.fromhex(h) for h in expected_file_ids), dtype=np.uint8).copy()
        dig = np.zeros((max(nfiles, 1), 32), dtype=np.uint8)
        status = np.zeros(max(nfiles, 1), dtype=np.int32)
        rc = lib().dfs_reassemble_verify(self._ctx, ptrs, _ptr(lens), nfiles, nfrag, _ptr(out), _ptr(file_off),
                                        _ptr(exp) if exp is not None else None, _ptr(dig), _ptr(status), 0)
        if rc not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_CORRUPT):
            check(rc, "dfs_reassemble_verify")
        res = []
        for f in range(nfiles):
            st = int(status[f])
            ln = int(sum(lens[f * nfrag:(f + 1) * nfrag]))
            body = None if st == L.DFS_E_MISSING else out[int(file_off[f]):int(file_off[f]) + ln].tobytes()
            res.append((st, body, dig[f].tobytes().hex()))
        return res

    def download(self, b64_frags: Sequence[Sequence[Optional[bytes]]], file_lens: Sequence[int],
                 frag_hashes: Optional[Sequence[Sequence[str]]] = None,
                 file_ids: Optional[Sequence[str]] = None) -> List[Tuple[int, Optional[bytes]]]:
        """Base64 download path: decode into place, per-fragment verify, fileId verify."""
        nfiles = len(b64_frags)
        nfrag = len(b64_frags[0]) if nfiles else 1
        texts, spans = [], np.zeros((max(nfiles * nfrag, 1), 2), dtype=np.uint64)
        o = 0
        for f in range(nfiles):
            for i in range(nfrag):
                t = b64_frags[f][i]
                k = f * nfrag + i
                if t is None:
                    spans[k] = (0, L.DFS_SPAN_MISSING)
                else:
                    spans[k] = (o, len(t))
                    texts.append(t)
                    o += len(t)
        buf = np.frombuffer(b"".join(texts) or b"\0", dtype=np.uint8).copy()
        flen = np.array(list(file_lens) or [0], dtype=np.uint64)
        file_off = np.zeros(max(nfiles, 1), dtype=np.uint64)
        if nfiles > 1:
            file_off[1:nfiles] = np.cumsum(flen[:nfiles])[:-1]
        out = np.zeros(max(int(flen[:nfiles].sum()), 1), dtype=np.uint8)
        ef = None
        if frag_hashes is not None:
            ef = np.frombuffer(b"".join(bytes.fromhex(h) for fh in frag_hashes for h in fh), dtype=np.uint8).copy()
        ei = None
        if file_ids is not None:
            ei = np.frombuffer(b"".join(bytes.fromhex(h) for h in file_ids), dtype=np.uint8).copy()
        status = np.zeros(max(nfiles, 1), dtype=np.int32)
        rc = lib().dfs_download_batch(self._ctx, _ptr(buf), _ptr(spans), nfiles, nfrag, _ptr(flen),
                                     _ptr(ef) if ef is not None else None, _ptr(ei) if ei is not None else None,
                                     _ptr(out), _ptr(file_off), _ptr(status), 0)
        if rc not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH, L.DFS_E_CORRUPT):
            check(rc, "dfs_download_batch")
        res = []
        for f in range(nfiles):
            st = int(status[f])
            o = int(file_off[f])
            res.append((st, out[o:o + int(flen[f])].tobytes() if st == 0 else None))
        return res


def sha256_device(engine: "FragmentEngine", d_base: int, spans: np.ndarray) -> np.ndarray:
    """dfs_sha256_batch over device memory (spans into d_base); returns the
    (n, 32) digests on the host after the engine's stream finished."""
    import torch
    spans = np.ascontiguousarray(spans, dtype=np.uint64).reshape(-1, 2)
    n = len(spans)
    dig = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=f"cuda:{engine.device}")
    check(lib().dfs_sha256_batch(engine.ctx, ctypes.c_void_p(d_base), _ptr(spans), n, ctypes.c_void_p(dig.data_ptr()),
                                 L.DFS_DEVICE_PTRS), "dfs_sha256_batch")
    torch.cuda.synchronize(engine.device)  # device-wide: the ctx stream too
    return dig.view(-1, 32).cpu().numpy()[:n]


def sha256_static_device(engine: "FragmentEngine", d_base: int, d_spans: int, n: int, d_digests: int,
                         d_status: int = 0) -> int:
    """dfs_sha256_batch_static: every argument a device address (spans
    included); asynchronous on the engine's stream.  Returns the DFS_* code
    (DFS_E_TOOBIG beyond DFS_STATIC_MAX_MSGS) instead of raising."""
    return lib().dfs_sha256_batch_static(engine.ctx, ctypes.c_void_p(d_base or None), ctypes.c_void_p(d_spans or None),
                                         n, ctypes.c_void_p(d_digests or None), ctypes.c_void_p(d_status or None))


def download_device(engine: "FragmentEngine", d_b64: int, spans: np.ndarray, nfiles: int, nfrag: int,
                    file_len: np.ndarray, d_exp_frag: int, d_exp_file: int, d_out: int,
                    file_off: np.ndarray) -> np.ndarray:
    """dfs_download_batch on device buffers; returns the per-file status."""
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    file_len = np.ascontiguousarray(file_len, dtype=np.uint64)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    status = np.zeros(max(nfiles, 1), dtype=np.int32)
    rc = lib().dfs_download_batch(engine.ctx, ctypes.c_void_p(d_b64), _ptr(spans), nfiles, nfrag, _ptr(file_len),
                                 ctypes.c_void_p(d_exp_frag or None), ctypes.c_void_p(d_exp_file or None),
                                 ctypes.c_void_p(d_out), _ptr(file_off), _ptr(status), L.DFS_DEVICE_PTRS)
    if rc not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH, L.DFS_E_CORRUPT):
        check(rc, "dfs_download_batch")
    return status[:nfiles]


def reassemble_device(engine: "FragmentEngine", frag_addr: np.ndarray, frag_len: np.ndarray, nfiles: int,
                      nfrag: int, d_out: int, file_off: np.ndarray,
                      expected: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """dfs_reassemble_verify with device fragments and output (raw-fragment
    download, SN:419-458): frag_addr[k] = device address of fragment k (0 =
    missing); expected = host (nfiles, 32) fileId digests or None.  Returns
    (per-file status, (nfiles, 32) digests of the rebuilt files)."""
    addr = np.ascontiguousarray(frag_addr, dtype=np.uint64)
    frag_len = np.ascontiguousarray(frag_len, dtype=np.uint64)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    exp = None if expected is None else np.ascontiguousarray(expected, dtype=np.uint8)
    status = np.zeros(max(nfiles, 1), dtype=np.int32)
    dig = np.zeros((max(nfiles, 1), 32), dtype=np.uint8)
    rc = lib().dfs_reassemble_verify(engine.ctx, _ptr(addr), _ptr(frag_len), nfiles, nfrag, ctypes.c_void_p(d_out),
                                    _ptr(file_off), _ptr(exp) if exp is not None else None, _ptr(dig),
                                    _ptr(status), L.DFS_DEVICE_PTRS)
    if rc not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_CORRUPT):
        check(rc, "dfs_reassemble_verify")
    return status[:nfiles], dig[:nfiles]


def store_bodies_layout(engine: "FragmentEngine", spans: np.ndarray, nfrag: int, uploader: int) -> np.ndarray:
    """body_off of dfs_store_bodies_build for `spans` (layout query, no launch)."""
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    nf = len(spans)
    body_off = np.zeros(nf * (nfrag - 1) + 1, dtype=np.uint64)
    check(lib().dfs_store_bodies_build(engine.ctx, None, _ptr(spans), nf, nfrag, uploader, None, None,
                                       _ptr(body_off), L.DFS_DEVICE_PTRS), "dfs_store_bodies_build (layout)")
    return body_off


def store_bodies_device(engine: "FragmentEngine", d_files: int, spans: np.ndarray, nfrag: int, uploader: int,
                        d_file_digest: int, d_bodies: int, body_off: np.ndarray) -> None:
    """dfs_store_bodies_build on device buffers (asynchronous on the engine's stream)."""
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    check(lib().dfs_store_bodies_build(engine.ctx, ctypes.c_void_p(d_files), _ptr(spans), len(spans), nfrag,
                                       uploader, ctypes.c_void_p(d_file_digest), ctypes.c_void_p(d_bodies),
                                       _ptr(body_off), L.DFS_DEVICE_PTRS), "dfs_store_bodies_build")


def store_receive_device(engine: "FragmentEngine", d_bodies: int, spans: np.ndarray, d_out: int):
    """dfs_store_bodies_receive on device buffers.  Returns (status,
    frag_index (n, 2), frag_off (n, 2), frag_len (n, 2), digests (n, 2, 32),
    file_ids (n, 64) uint8).  d_out must hold store_receive_out_bytes(spans)."""
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    n = len(spans)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    idx = np.zeros((max(n, 1), 2), dtype=np.uint32)
    foff = np.zeros((max(n, 1), 2), dtype=np.uint64)
    flen = np.zeros((max(n, 1), 2), dtype=np.uint64)
    dig = np.zeros((max(n, 1), 2, 32), dtype=np.uint8)
    ids = np.zeros((max(n, 1), 64), dtype=np.uint8)
    status = np.zeros(max(n, 1), dtype=np.int32)
    check(lib().dfs_store_bodies_receive(engine.ctx, ctypes.c_void_p(d_bodies), _ptr(spans), n,
                                         ctypes.c_void_p(d_out), _ptr(out_off), _ptr(idx), _ptr(foff), _ptr(flen),
                                         _ptr(dig), _ptr(ids), _ptr(status), L.DFS_DEVICE_PTRS),
          "dfs_store_bodies_receive")
    return status[:n], idx[:n], foff[:n], flen[:n], dig[:n], ids[:n]


def store_receive_out_bytes(spans: np.ndarray) -> int:
    """Bytes dfs_store_bodies_receive needs in `out`: per body 3*ceil(len/4) +
    16, rounded up to a multiple of 16 (both payloads decode to 16-byte
    aligned places)."""
    return int(sum((3 * ((int(ln) + 3) // 4) + 16 + 15) & ~15 for ln in np.asarray(spans)[:, 1]))


class UploadPlan:
    """dfs_upload_plan over device-resident (torch) buffers — the bench path."""

    def __init__(self, engine: FragmentEngine, spans: np.ndarray, nfrag: int, frag_major: bool = False,
                 align128: bool = False):
        self.engine = engine
        spans = np.ascontiguousarray(spans, dtype=np.uint64)
        self.nfiles = len(spans)
        self.nfrag = nfrag
        self.frag_major = frag_major
        self.align128 = align128
        self._plan = ctypes.c_void_p()
        total = ctypes.c_uint64(0)
        flags = (L.DFS_LAYOUT_FRAG_MAJOR if frag_major else 0) | (L.DFS_LAYOUT_ALIGN128 if align128 else 0)
        check(lib().dfs_upload_plan_create(engine.ctx, _ptr(spans), self.nfiles, nfrag, flags,
                                           ctypes.byref(self._plan), ctypes.byref(total)), "dfs_upload_plan_create")
        self.b64_total = total.value

    def b64_offsets(self) -> np.ndarray:
        """nfiles*nfrag+1 offsets (fragment start; last = total)."""
        off = np.zeros(self.nfiles * self.nfrag + 1, dtype=np.uint64)
        check(lib().dfs_upload_plan_b64_offsets(self._plan, _ptr(off)), "dfs_upload_plan_b64_offsets")
        return off

    def b64_spans(self, file_lens) -> np.ndarray:
        """(start, length) of every fragment's Base64 in [file][fragment]
        order; lengths come from the split, so they are exact with the
        align128 gaps too."""
        off = self.b64_offsets()
        fl = np.asarray(file_lens, dtype=np.uint64).reshape(-1, 1)
        i = np.arange(self.nfrag, dtype=np.uint64).reshape(1, -1)
        n = np.uint64(self.nfrag)
        frag = fl // n + (i < fl % n).astype(np.uint64)  # the split of SN:138-171 (dfs_split_plan)
        lens = (np.uint64(4) * ((frag + np.uint64(2)) // np.uint64(3))).reshape(-1)
        return np.stack([off[:-1], lens], axis=1).astype(np.uint64)

    def run(self, d_files: int, d_file_digest: int, d_frag_digest: int, d_b64: int, flags: int = 0) -> None:
        check(lib().dfs_upload_plan_run(self.engine.ctx, self._plan, ctypes.c_void_p(d_files),
                                        ctypes.c_void_p(d_file_digest or None), ctypes.c_void_p(d_frag_digest),
                                        ctypes.c_void_p(d_b64 or None), flags), "dfs_upload_plan_run")

    def close(self) -> None:
        if self._plan:
            lib().dfs_upload_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DownloadPlan:
    """dfs_download_plan: the descriptor tables of one download shape built
    once and kept in HBM (handleDownload with Base64 transport, SN:399-461 +
    281-282); run() as download_device."""

    def __init__(self, engine: FragmentEngine, spans: np.ndarray, nfiles: int, nfrag: int, file_len: np.ndarray,
                 file_off: np.ndarray):
        self.engine = engine
        self.nfiles = nfiles
        spans = np.ascontiguousarray(spans, dtype=np.uint64)
        file_len = np.ascontiguousarray(file_len, dtype=np.uint64)
        file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
        self._plan = ctypes.c_void_p()
        check(lib().dfs_download_plan_create(engine.ctx, _ptr(spans), nfiles, nfrag, _ptr(file_len), _ptr(file_off),
                                             ctypes.byref(self._plan)), "dfs_download_plan_create")

    def run(self, d_b64: int, d_exp_frag: int, d_exp_file: int, d_out: int) -> np.ndarray:
        status = np.zeros(max(self.nfiles, 1), dtype=np.int32)
        rc = lib().dfs_download_plan_run(self.engine.ctx, self._plan, ctypes.c_void_p(d_b64 or None),
                                        ctypes.c_void_p(d_exp_frag or None), ctypes.c_void_p(d_exp_file or None),
                                        ctypes.c_void_p(d_out), _ptr(status))
        if rc not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH, L.DFS_E_CORRUPT):
            check(rc, "dfs_download_plan_run")
        return status[:self.nfiles]

    def close(self) -> None:
        if self._plan:
            lib().dfs_download_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_fill(engine: FragmentEngine, d_dst: int, spans: np.ndarray, first_file: int, seed: int) -> None:
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    check(lib().dfs_synth_fill(engine.ctx, ctypes.c_void_p(d_dst), _ptr(spans), len(spans), first_file, seed),
          "dfs_synth_fill")
