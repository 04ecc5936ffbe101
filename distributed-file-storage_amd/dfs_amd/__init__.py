"""dfs_amd — MI355X (gfx950) fragment pipeline for hiagoluansilva/distributed-file-storage.

The data path (SHA-256, Base64, reassembly gather) runs only in the HIP
kernels of libdfsgpu.so behind the C ABI in include/dfs_gpu.h.  This package
is the Python face of that ABI (ctypes), used by tests/ and bench.py.
"""
from ._lib import (DFS_LAYOUT_ALIGN128, DFS_LAYOUT_FRAG_MAJOR, DFS_DEVICE_PTRS, DFS_E_ARG, DFS_E_CORRUPT, DFS_E_DECODE, DFS_E_FRAG_MISMATCH, DFS_E_HIP,
                   DFS_E_MISSING, DFS_E_NODEV, DFS_E_NOMEM, DFS_NO_B64, DFS_NO_FILEID, DFS_OK, DFS_SERIAL, DFS_B64_ONLY,
                   DFS_SPAN_MISSING, DfsError, LIB_PATH, SIGNATURES, lib)
from .engine import (DownloadPlan, Fragment, FragmentEngine, IllegalArgumentException, UploadPlan, UploadResult, b64_encoded_len,
                     fragment_holders, split_plan, synth_fill)

__all__ = [
    "FragmentEngine", "UploadPlan", "DownloadPlan", "UploadResult", "Fragment", "IllegalArgumentException", "DfsError",
    "split_plan", "fragment_holders", "b64_encoded_len", "synth_fill", "lib", "LIB_PATH", "SIGNATURES",
    "DFS_OK", "DFS_E_ARG", "DFS_E_HIP", "DFS_E_NOMEM", "DFS_E_DECODE", "DFS_E_MISSING", "DFS_E_CORRUPT",
    "DFS_E_FRAG_MISMATCH", "DFS_E_NODEV", "DFS_DEVICE_PTRS", "DFS_NO_FILEID", "DFS_NO_B64", "DFS_SERIAL", "DFS_B64_ONLY",
    "DFS_SPAN_MISSING", "DFS_LAYOUT_FRAG_MAJOR", "DFS_LAYOUT_ALIGN128",
]
