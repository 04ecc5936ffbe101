"""ctypes binding of libdfsgpu.so (include/dfs_gpu.h).

The library is built in-tree (``make -C distributed-file-storage_amd``) and is
the only implementation of the data path: there is no Python or CPU fallback.
Importing this module without the built library raises immediately.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DFS_LIB_PATH: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("DFS_LIB_PATH") or os.path.join(PKG_DIR, "libdfsgpu.so")
REPO_ROOT = os.path.dirname(PKG_DIR)
HEADER_PATH = os.path.join(REPO_ROOT, "include", "dfs_gpu.h")

# Return codes / flags (mirrors include/dfs_gpu.h).
DFS_OK = 0
DFS_E_ARG = -1
DFS_E_HIP = -2
DFS_E_NOMEM = -3
DFS_E_DECODE = -4
DFS_E_MISSING = -5
DFS_E_CORRUPT = -6
DFS_E_FRAG_MISMATCH = -7
DFS_E_NODEV = -8
DFS_E_WIRE = -9
DFS_E_IO = -10
DFS_E_COMM = -11
DFS_E_TOOBIG = -12
DFS_STATIC_MAX_MSGS = 65536

DFS_DEVICE_PTRS = 0x1
DFS_NO_FILEID = 0x2
DFS_NO_B64 = 0x4
DFS_SERIAL = 0x8
DFS_B64_ONLY = 0x80
DFS_LAYOUT_FRAG_MAJOR = 0x10
DFS_LAYOUT_ALIGN128 = 0x100
DFS_SHA_BEGIN = 0x20
DFS_SHA_FINAL = 0x40

DFS_SPAN_MISSING = (1 << 64) - 1

DFS_COMM_ID_BYTES = 128
DFS_PLACE_RING, DFS_PLACE_STAR, DFS_PLACE_FETCH = 0, 1, 2
DFS_XFER_SEND, DFS_XFER_RECV, DFS_XFER_COPY = 0, 1, 2

DFS_T_SHA, DFS_T_B64ENC, DFS_T_B64DEC, DFS_T_GATHER, DFS_T_TOTAL, DFS_T_COUNT = range(6)
DFS_S_OVL_REDO, DFS_S_RECV_ONE_PASS, DFS_S_COUNT = range(3)


class dfs_span(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint64)]


class dfs_batcher_stats_t(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("requests", ctypes.c_uint64), ("max_batch", ctypes.c_uint64),
                ("queue_s", ctypes.c_double), ("stage_in_s", ctypes.c_double), ("device_s", ctypes.c_double),
                ("stage_out_s", ctypes.c_double), ("enqueue_s", ctypes.c_double), ("return_s", ctypes.c_double),
                ("direct", ctypes.c_uint64), ("views", ctypes.c_uint64)]


class dfs_batcher_opts(ctypes.Structure):
    _fields_ = [("max_wait_us", ctypes.c_uint32), ("max_files", ctypes.c_uint32), ("max_bytes", ctypes.c_uint64),
                ("depth", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


# dfs_frag_ref as a numpy record (24 bytes: off, len, file, index).
FRAG_REF_DTYPE = [("off", "<u8"), ("len", "<u8"), ("file", "<u4"), ("index", "<u4")]
# dfs_xfer (48 bytes).
XFER_DTYPE = [("phase", "<u4"), ("kind", "<u4"), ("peer", "<i4"), ("frag", "<u4"), ("from_dst", "<u4"),
              ("reserved", "<u4"), ("src_off", "<u8"), ("dst_off", "<u8"), ("len", "<u8")]


# dfs_held_frag (48 bytes).
HELD_FRAG_DTYPE = [("rank", "<u4"), ("file", "<u4"), ("frag", "<u4"), ("reserved", "<u4"), ("b64_off", "<u8"),
                   ("b64_len", "<u8"), ("raw_off", "<u8"), ("raw_len", "<u8")]

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_int = ctypes.c_int

# name -> (restype, argtypes); every symbol include/dfs_gpu.h declares.
SIGNATURES = {
    "dfs_open": (_int, [ctypes.POINTER(_vp), _int]),
    "dfs_close": (_int, [_vp]),
    "dfs_strerror": (ctypes.c_char_p, [_int]),
    "dfs_abi_version": (_int, []),
    "dfs_set_stream": (_int, [_vp, _vp]),
    "dfs_set_profiling": (_int, [_vp, _int]),
    "dfs_get_timings": (_int, [_vp, _vp, _int]),
    "dfs_get_stats": (_int, [_vp, _vp, _int]),
    "dfs_split_plan": (_int, [_u64, _u32, _vp]),
    "dfs_b64_encoded_len": (_u64, [_u64]),
    "dfs_b64_decoded_cap": (_u64, [_u64]),
    "dfs_fragment_holders": (_int, [_u32, _u32, _vp]),
    "dfs_sha256_batch": (_int, [_vp, _vp, _vp, _u32, _vp, _u32]),
    "dfs_sha256_batch_static": (_int, [_vp, _vp, _vp, _u32, _vp, _vp]),
    "dfs_sha256_update_batch": (_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _u32]),
    "dfs_receive_fragments_batch": (_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32]),
    "dfs_b64_encode_batch": (_int, [_vp, _vp, _vp, _u32, _vp, _u64, _vp, _u32]),
    "dfs_b64_decode_batch": (_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32]),
    "dfs_upload_batch": (_int, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _u64, _vp, _u32]),
    "dfs_reassemble_verify": (_int, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _u32]),
    "dfs_download_batch": (_int, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    "dfs_download_plan_create": (_int, [_vp, _vp, _u32, _u32, _vp, _vp, ctypes.POINTER(_vp)]),
    "dfs_download_plan_run": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dfs_download_plan_destroy": (_int, [_vp]),
    "dfs_upload_plan_create": (_int, [_vp, _vp, _u32, _u32, _u32, ctypes.POINTER(_vp), ctypes.POINTER(_u64)]),
    "dfs_upload_plan_b64_offsets": (_int, [_vp, _vp]),
    "dfs_upload_plan_run": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    "dfs_upload_plan_destroy": (_int, [_vp]),
    "dfs_synth_fill": (_int, [_vp, _vp, _vp, _u32, _u64, _u64]),
    "dfs_sha256_update_parts": (_int, [_vp, _vp, _vp, _u32, _vp, _vp, _u32]),
    "dfs_synth_fill_at": (_int, [_vp, _vp, _vp, _u32, _u64, _u64, _u64]),
    "dfs_store_body_len": (_u64, [_u64, _u32, _u32, _u32]),
    "dfs_store_bodies_build": (_int, [_vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _u32]),
    "dfs_store_bodies_receive": (_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    "dfs_store_write_fragments": (_int, [_vp, ctypes.c_char_p, _vp, _u32, _vp, _vp, _u32, _vp, _u32]),
    "dfs_store_read_fragments": (_int, [_vp, ctypes.c_char_p, _vp, _u32, _vp, _vp, _u32, _vp, _vp, _u32]),
    "dfs_batcher_create": (_int, [_int, _u32, _vp, ctypes.POINTER(_vp)]),
    "dfs_batcher_destroy": (_int, [_vp]),
    "dfs_batcher_stats": (_int, [_vp, _vp]),
    "dfs_host_alloc": (_int, [_u64, ctypes.POINTER(_vp)]),
    "dfs_host_free": (_int, [_vp]),
    "dfs_submit_upload": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _u64, _vp]),
    "dfs_submit_download": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "dfs_submit_reassemble": (_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "dfs_submit_upload_view": (_int, [_vp, _vp, _u64, _vp, _vp, ctypes.POINTER(_vp), _vp, ctypes.POINTER(_vp)]),
    "dfs_submit_download_view": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "dfs_view_release": (_int, [_vp]),
    "dfs_store_hash_response_cap": (_u64, []),
    "dfs_store_hash_responses_build": (_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _u64, _vp]),
    "dfs_store_hash_responses_check": (_int, [_vp, _vp, ctypes.c_uint32, _vp, _vp, _vp]),
    "dfs_comm_unique_id": (_int, [_vp]),
    "dfs_comm_init_rank": (_int, [_vp, _vp, _u32, _u32, ctypes.POINTER(_vp)]),
    "dfs_comm_init_all": (_int, [_vp, _u32, _vp]),
    "dfs_comm_destroy": (_int, [_vp]),
    "dfs_comm_info": (_int, [_vp, _vp, _vp]),
    "dfs_comm_counters": (_int, [_vp, _vp]),
    "dfs_comm_last_error": (ctypes.c_char_p, []),
    "dfs_place_sizes": (_int, [_vp, _u32, _vp, _u32, _vp]),
    "dfs_place_plan": (_int, [_u32, _u32, _u32, _vp, _u32, _u64, _vp, _vp, _vp, _vp]),
    "dfs_place_ring": (_int, [_vp, _u32, _u32, _vp, _vp, _vp]),
    "dfs_place_star": (_int, [_vp, _u32, _u32, _vp, _vp, _vp]),
    "dfs_fetch_degraded": (_int, [_vp, _u32, _u32, _vp, _u64, _vp, _vp, _vp]),
    "dfs_place_simulate": (_int, [_u32, _u32, _vp, _u32, _u64, _vp, _vp, _vp]),
    "dfs_replica_layout": (_int, [_u32, _u32, _u32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "dfs_replica_plan_create": (_int, [_vp, _u32, _u32, _vp, _vp, _u32, _vp]),
    "dfs_replica_plan_info": (_int, [_vp, _vp, _vp, _vp, _vp]),
    "dfs_replica_plan_one_pass": (_int, [_vp]),
    "dfs_replica_plan_frags": (_int, [_vp, _vp]),
    "dfs_replica_verify": (_int, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dfs_replica_exchange": (_int, [_vp, _u32, _vp, _vp]),
    "dfs_replica_check": (_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "dfs_replica_report": (_int, [_vp, _u32, _vp]),
    "dfs_replica_plan_destroy": (_int, [_vp]),
}

_LIB = None


class DfsError(RuntimeError):
    """A DFS_E_* return code (RuntimeException in the Java mapping)."""

    def __init__(self, code: int, where: str = ""):
        self.code = code
        msg = lib().dfs_strerror(code).decode(errors="replace")
        super().__init__(f"{where}: {msg} ({code})" if where else f"{msg} ({code})")


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built; run `make -C {PKG_DIR}` (hipcc, gfx950). "
                "There is no CPU fallback for the fragment pipeline.")
        # One HIP runtime per process: torch ships its own libamdhip64.so
        # (soname libamdhip64.so.7, the same soname libdfsgpu.so needs).  If
        # torch is importable, load it first so libdfsgpu.so binds to the
        # runtime already in the process instead of pulling in a second copy
        # from /opt/rocm (two runtimes make torch report "No HIP GPUs").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("DFS_LIB_PATH") and not hasattr(L, name):
                continue  # an older A/B build: its missing entry points stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc: int, where: str = "") -> int:
    if rc != DFS_OK:
        raise DfsError(rc, where)
    return rc
