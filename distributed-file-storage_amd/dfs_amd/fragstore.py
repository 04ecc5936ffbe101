"""A storage node's on-disk fragment store over libdfsgpu.so
(dfs_store_write_fragments / dfs_store_read_fragments, include/dfs_gpu.h).

Mirrors StorageNode.java's fragment files (cited SN:line): dataRoot =
data/node-<id> (SN:20), <dataRoot>/<fileId>/fragments/<i>.frag written with
the raw fragment bytes on upload (SN:147-149, 163-166) and by the replica
receiver (SN:273-285), read back by tryLoadFragmentLocal (SN:463-469).  The
file I/O is native (a C++ thread pool); device buffers move through the
library's pinned staging ring, so fragments go HBM -> disk and disk -> HBM
without a Python copy.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import FRAG_REF_DTYPE, check, lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _order_after_torch(engine) -> None:
    """Device-mode store calls copy on the engine's ctx stream, which nothing
    orders after torch's current stream: finish the producer (or consumer
    fill) queued on torch's stream first.  A caller that set the
    ctx stream to torch's own stream (engine.set_stream) is ordered already."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.current_stream(engine.device).synchronize()


def make_refs(off: Sequence[int], length: Sequence[int], file: Sequence[int], index: Sequence[int]) -> np.ndarray:
    """dfs_frag_ref array: fragment `index[i]` of file `file[i]` at data + off[i]."""
    refs = np.zeros(len(off), dtype=FRAG_REF_DTYPE)
    refs["off"], refs["len"], refs["file"], refs["index"] = off, length, file, index
    return refs


class FragmentStore:
    """One node's data directory (the reference's dataRoot)."""

    def __init__(self, node_id: int, data_dir: str = "data", engine=None):
        self.node_id = node_id
        self.root = os.path.join(data_dir, f"node-{node_id}")  # SN:20
        os.makedirs(self.root, exist_ok=True)  # SN:24
        self.engine = engine

    def fragment_path(self, file_id_hex: str, index: int) -> str:
        return os.path.join(self.root, file_id_hex, "fragments", f"{index}.frag")  # SN:165, 284, 464

    def _ctx(self, device: bool):
        if device:
            if self.engine is None:
                raise ValueError("device buffers need a FragmentEngine")
            return self.engine.ctx
        return self.engine.ctx if self.engine is not None else None

    def write(self, file_digests: np.ndarray, data, refs: np.ndarray, device: bool = False) -> np.ndarray:
        """Write every ref (Files.write, SN:166 / 285).  data: a host uint8
        array, or with device=True a device address.  Returns per-ref status;
        raises only on argument / HIP errors."""
        dig = np.ascontiguousarray(file_digests, dtype=np.uint8).reshape(-1, 32)
        refs = np.ascontiguousarray(refs, dtype=FRAG_REF_DTYPE)
        n = len(refs)
        status = np.zeros(max(n, 1), dtype=np.int32)
        dptr = ctypes.c_void_p(int(data)) if device else (ctypes.c_void_p(_ptr(data)) if data is not None else None)
        if device:
            _order_after_torch(self.engine)
        rc = lib().dfs_store_write_fragments(self._ctx(device), self.root.encode(), _ptr(dig), len(dig), dptr,
                                             _ptr(refs), n,
                                             _ptr(status), L.DFS_DEVICE_PTRS if device else 0)
        if rc not in (L.DFS_OK, L.DFS_E_IO):
            check(rc, "dfs_store_write_fragments")
        return status[:n]

    def read(self, file_digests: np.ndarray, data, refs: np.ndarray, device: bool = False
             ) -> Tuple[np.ndarray, np.ndarray]:
        """Load every ref into data + off (capacity len).  Returns (status,
        out_len): status DFS_E_MISSING where tryLoadFragmentLocal returns null."""
        dig = np.ascontiguousarray(file_digests, dtype=np.uint8).reshape(-1, 32)
        refs = np.ascontiguousarray(refs, dtype=FRAG_REF_DTYPE)
        n = len(refs)
        status = np.zeros(max(n, 1), dtype=np.int32)
        out_len = np.zeros(max(n, 1), dtype=np.uint64)
        dptr = ctypes.c_void_p(int(data)) if device else (ctypes.c_void_p(_ptr(data)) if data is not None else None)
        if device:
            _order_after_torch(self.engine)
        rc = lib().dfs_store_read_fragments(self._ctx(device), self.root.encode(), _ptr(dig), len(dig), dptr,
                                            _ptr(refs), n,
                                            _ptr(out_len), _ptr(status), L.DFS_DEVICE_PTRS if device else 0)
        if rc not in (L.DFS_OK, L.DFS_E_IO, L.DFS_E_MISSING, L.DFS_E_ARG):
            check(rc, "dfs_store_read_fragments")
        return status[:n], out_len[:n]

    def try_load_fragment_local(self, file_id_hex: str, index: int) -> Optional[bytes]:
        """tryLoadFragmentLocal (SN:463-469) for one fragment: bytes or None."""
        dig = np.frombuffer(bytes.fromhex(file_id_hex), dtype=np.uint8)
        path = self.fragment_path(file_id_hex, index)
        size = os.path.getsize(path) if os.path.isfile(path) else 0
        buf = np.zeros(max(size, 1), dtype=np.uint8)
        st, ln = self.read(dig, buf, make_refs([0], [max(size, 0)], [0], [index]))
        if st[0] == L.DFS_E_MISSING:
            return None
        if st[0] != L.DFS_OK:
            raise L.DfsError(int(st[0]), "tryLoadFragmentLocal")
        return buf[: int(ln[0])].tobytes()
