"""Request batcher (dfs_batcher_* / dfs_submit_*): StorageNode's
thread-per-connection handlers (SN:28-31) each submit ONE file; the library
coalesces concurrent submissions into one launch.  Calls release the GIL
(ctypes), so Python threads stand in for the Java handler threads."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import check, dfs_batcher_opts, lib


class PinnedBuffer:
    """A dfs_host_alloc buffer (page-locked host memory) viewed as a uint8
    numpy array.  Requests whose buffers all lie in such buffers are "direct":
    the batcher's DMA reads / writes them, no staging copy on the handler."""

    def __init__(self, nbytes: int):
        self._p = ctypes.c_void_p()
        check(lib().dfs_host_alloc(nbytes, ctypes.byref(self._p)), "dfs_host_alloc")
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self._p.value))[:nbytes]

    def free(self) -> None:
        if self._p:
            self.array = None
            check(lib().dfs_host_free(self._p), "dfs_host_free")
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Batcher:
    def __init__(self, device: int, nfrag: int, max_wait_us: int = 0, max_files: int = 0, max_bytes: int = 0,
                 depth: int = 0):
        self.nfrag = nfrag
        self._b = ctypes.c_void_p()
        o = dfs_batcher_opts(max_wait_us, max_files, max_bytes, depth, 0)
        check(lib().dfs_batcher_create(device, nfrag, ctypes.byref(o), ctypes.byref(self._b)), "dfs_batcher_create")

    def upload_into(self, data: np.ndarray, fd: np.ndarray, frd: np.ndarray, b64: np.ndarray,
                    b64_off: np.ndarray) -> int:
        """handleUpload's pipeline for one file into caller buffers (no copies
        on the Python side): fd (32,), frd (nfrag, 32), b64, b64_off
        (nfrag + 1,) uint8/uint64 arrays.  Returns the DFS status."""
        return lib().dfs_submit_upload(self._b, data.ctypes.data if data.size else None, data.size, fd.ctypes.data,
                                       frd.ctypes.data, b64.ctypes.data if b64.size else None, b64.size,
                                       b64_off.ctypes.data)

    def upload(self, data: bytes) -> Tuple[bytes, list, list]:
        """(fileId digest, fragment digests, fragment Base64 strings)."""
        a = np.frombuffer(data, dtype=np.uint8)
        n = len(data)
        cap = sum(4 * ((n // self.nfrag + 1 + 2) // 3) for _ in range(self.nfrag)) + 16
        fd = np.zeros(32, np.uint8)
        frd = np.zeros((self.nfrag, 32), np.uint8)
        b64 = np.zeros(cap, np.uint8)
        off = np.zeros(self.nfrag + 1, np.uint64)
        check(self.upload_into(a, fd, frd, b64, off), "dfs_submit_upload")
        return (fd.tobytes(), [frd[i].tobytes() for i in range(self.nfrag)],
                [b64[int(off[i]):int(off[i + 1])].tobytes() for i in range(self.nfrag)])

    def upload_view(self, data: np.ndarray, keep: bool = False):
        """dfs_submit_upload_view for one file (a uint8 array; read in place
        when it lies in a PinnedBuffer): (fileId digest, fragment digests,
        fragment Base64 strings), the Base64 copied out of the view, which is
        then released.  keep=True returns (..., view handle) unreleased, for
        tests of the buffer life cycle: give it to release_view."""
        fd = np.zeros(32, np.uint8)
        frd = np.zeros((self.nfrag, 32), np.uint8)
        off = np.zeros(self.nfrag + 1, np.uint64)
        ptr, view = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().dfs_submit_upload_view(self._b, data.ctypes.data if data.size else None, data.size, fd.ctypes.data,
                                           frd.ctypes.data, ctypes.byref(ptr), off.ctypes.data, ctypes.byref(view)),
              "dfs_submit_upload_view")
        total = int(off[self.nfrag])
        text = ctypes.string_at(ptr.value, total) if total else b""
        res = (fd.tobytes(), [frd[i].tobytes() for i in range(self.nfrag)],
               [text[int(off[i]):int(off[i + 1])] for i in range(self.nfrag)])
        if keep:
            return res + (view,)
        self.release_view(view)
        return res

    @staticmethod
    def release_view(view) -> None:
        if view:
            check(lib().dfs_view_release(view), "dfs_view_release")

    def download_view(self, text: np.ndarray, spans, file_len: int, ef: Optional[np.ndarray],
                      ei: Optional[np.ndarray]) -> Tuple[int, Optional[bytes]]:
        """dfs_submit_download_view: (status, the file's bytes copied out of
        the view or None); the view is released."""
        ptr, view = ctypes.c_void_p(), ctypes.c_void_p()
        st = lib().dfs_submit_download_view(self._b, text.ctypes.data, spans, file_len,
                                            ef.ctypes.data if ef is not None else None,
                                            ei.ctypes.data if ei is not None else None, ctypes.byref(ptr),
                                            ctypes.byref(view))
        if st not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH, L.DFS_E_CORRUPT):
            check(st, "dfs_submit_download_view")
        out = None
        if st == L.DFS_OK:
            out = ctypes.string_at(ptr.value, file_len) if file_len else b""
        self.release_view(view)
        return st, out

    def download_into(self, text: np.ndarray, spans, file_len: int, ef: Optional[np.ndarray],
                      ei: Optional[np.ndarray], out: np.ndarray) -> int:
        """handleDownload's pipeline for one file from / into caller buffers:
        text (uint8 Base64 chars), spans (dfs_span * nfrag into text), out
        (>= file_len bytes).  Returns the DFS status."""
        return lib().dfs_submit_download(self._b, text.ctypes.data, spans, file_len,
                                         ef.ctypes.data if ef is not None else None,
                                         ei.ctypes.data if ei is not None else None, out.ctypes.data)

    def download(self, b64_frags: Sequence[Optional[bytes]], file_len: int, frag_digests: Optional[Sequence[bytes]],
                 file_digest: Optional[bytes]) -> Tuple[int, Optional[bytes]]:
        """Base64 download of one file: (status, bytes or None)."""
        texts = [t for t in b64_frags if t is not None]
        buf = np.frombuffer(b"".join(texts) or b"\0", dtype=np.uint8)
        spans = (L.dfs_span * self.nfrag)()
        o = 0
        for i, t in enumerate(b64_frags):
            if t is None:
                spans[i].off, spans[i].len = 0, L.DFS_SPAN_MISSING
            else:
                spans[i].off, spans[i].len = o, len(t)
                o += len(t)
        ef = np.frombuffer(b"".join(frag_digests), np.uint8) if frag_digests is not None else None
        ei = np.frombuffer(file_digest, np.uint8) if file_digest is not None else None
        out = np.zeros(max(file_len, 1), np.uint8)
        st = lib().dfs_submit_download(self._b, buf.ctypes.data, spans, file_len,
                                       ef.ctypes.data if ef is not None else None,
                                       ei.ctypes.data if ei is not None else None, out.ctypes.data)
        if st not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH, L.DFS_E_CORRUPT):
            check(st, "dfs_submit_download")
        return st, (out[:file_len].tobytes() if st == 0 else None)

    def reassemble(self, frags: Sequence[Optional[bytes]], file_digest: Optional[bytes]
                   ) -> Tuple[int, Optional[bytes], Optional[bytes]]:
        """Raw-fragment download of one file (handleDownload as the reference
        has it, SN:419-458): (status, rebuilt bytes or None, SHA-256 of the
        rebuilt bytes or None)."""
        assert len(frags) == self.nfrag
        keep = [np.frombuffer(f, np.uint8).copy() if f else None for f in frags]
        ptrs = (ctypes.c_void_p * self.nfrag)(*[a.ctypes.data if a is not None and a.size else None for a in keep])
        lens = (ctypes.c_uint64 * self.nfrag)(*[1 if f is None else len(f) for f in frags])  # None: a missing fragment
        for i, f in enumerate(frags):
            if f is not None and not f:
                lens[i] = 0
        total = sum(len(f) for f in frags if f is not None)
        out = np.zeros(max(total, 1), np.uint8)
        dig = np.zeros(32, np.uint8)
        ei = np.frombuffer(file_digest, np.uint8) if file_digest is not None else None
        st = lib().dfs_submit_reassemble(self._b, ptrs, lens, ei.ctypes.data if ei is not None else None,
                                         out.ctypes.data, dig.ctypes.data)
        if st not in (L.DFS_OK, L.DFS_E_MISSING, L.DFS_E_CORRUPT):
            check(st, "dfs_submit_reassemble")
        return st, (out[:total].tobytes() if st == 0 else None), (dig.tobytes() if st != L.DFS_E_MISSING else None)

    def stats(self) -> dict:
        st = L.dfs_batcher_stats_t()
        check(lib().dfs_batcher_stats(self._b, ctypes.byref(st)), "dfs_batcher_stats")
        return {k: getattr(st, k) for k, _ in L.dfs_batcher_stats_t._fields_}

    def close(self) -> None:
        if self._b:
            lib().dfs_batcher_destroy(self._b)
            self._b = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
