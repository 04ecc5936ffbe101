"""The C-ABI library loads and exports every symbol include/dfs_gpu.h declares
(no compute calls: these run without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

import dfs_amd
import oracle as O
from dfs_amd import _lib


def declared_functions():
    text = open(_lib.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dfs_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding():
    assert declared_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    L = dfs_amd.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (dfs_[a-z0-9_]+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_abi_version_and_strerror():
    L = dfs_amd.lib()
    assert L.dfs_abi_version() == 3
    assert L.dfs_strerror(dfs_amd.DFS_E_CORRUPT) == b"File corrupted"
    assert L.dfs_strerror(dfs_amd.DFS_E_MISSING) == b"Could not retrieve fragment"


def test_host_helpers_match_oracle():
    for S in [0, 1, 2, 3, 4, 5, 7, 28, 467, 2154, 9506, (1 << 20), (1 << 28) + 3]:
        for N in [1, 3, 5, 8, 13]:
            assert dfs_amd.split_plan(S, N) == O.c_split(S, N)
    for N in [2, 5, 8]:
        for f in range(N):
            assert dfs_amd.fragment_holders(f, N) == O.py_fragment_holders(f, N)
    for n in range(0, 50):
        assert dfs_amd.b64_encoded_len(n) == len(O.c_b64_encode(b"x" * n))
    assert dfs_amd.lib().dfs_b64_decoded_cap(8) == 6


def test_bad_arguments_fail_loudly():
    L = dfs_amd.lib()
    assert L.dfs_split_plan(10, 0, None) == dfs_amd.DFS_E_ARG
    h = (ctypes.c_uint32 * 2)()
    assert L.dfs_fragment_holders(5, 5, h) == dfs_amd.DFS_E_ARG
    assert L.dfs_sha256_batch(None, None, None, 0, None, 0) == dfs_amd.DFS_E_ARG


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dfs_amd.DfsError) as ei:
        dfs_amd.FragmentEngine(0)
    assert ei.value.code == dfs_amd.DFS_E_NODEV


def test_product_path_never_imports_oracle():
    pkg = os.path.dirname(dfs_amd.__file__)
    for root, _, files in os.walk(os.path.dirname(pkg)):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h", ".hpp")):
                src = open(os.path.join(root, fn), errors="ignore").read()
                assert "oracle" not in src.replace("no oracle", ""), os.path.join(root, fn)
