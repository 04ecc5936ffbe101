"""CPU oracle for the StorageNode fragment pipeline — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product path (``dfs_amd`` over ``libdfsgpu.so``) never
imports it and has no CPU fallback.

Two independent restatements live here:

* ``liboracle.so`` (oracle/dfs_oracle.c), a plain-C restatement of
  StorageNode.java's split / hash / encode / decode / reassemble path, used
  for bulk parity checks and the CPU baseline;
* pure-Python functions built on ``hashlib`` / ``base64`` (OpenSSL-backed),
  used to cross-check the C restatement and to generate tests/golden/.

Citations: SN = storage-node/src/StorageNode.java in the reference.
"""
from __future__ import annotations

import base64
import ctypes
import hashlib
import os
from typing import List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SYNTH_SEED = 0x5EED5EED


def lib() -> ctypes.CDLL:
    """Load (building on first use if needed) oracle/liboracle.so."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(_HERE, "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", _HERE])
    L = ctypes.CDLL(path)
    u8p, u64p = ctypes.c_void_p, ctypes.c_void_p
    L.oracle_sha256.argtypes = [u8p, ctypes.c_uint64, u8p]
    L.oracle_sha256.restype = None
    L.oracle_b64_encode.argtypes = [u8p, ctypes.c_uint64, ctypes.c_void_p]
    L.oracle_b64_encode.restype = ctypes.c_uint64
    L.oracle_b64_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u8p, ctypes.POINTER(ctypes.c_uint64)]
    L.oracle_b64_decode.restype = ctypes.c_int
    L.oracle_split.argtypes = [ctypes.c_uint64, ctypes.c_uint32, u64p, u64p]
    L.oracle_split.restype = None
    L.oracle_fragment_holders.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    L.oracle_fragment_holders.restype = None
    L.oracle_upload_batch.argtypes = [u8p, u64p, u64p, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p,
                                      ctypes.c_void_p, u64p, ctypes.c_int]
    L.oracle_upload_batch.restype = ctypes.c_uint64
    L.oracle_reassemble_verify.argtypes = [ctypes.c_void_p, u64p, ctypes.c_uint32, u8p, u8p]
    L.oracle_reassemble_verify.restype = ctypes.c_int
    L.oracle_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p]
    L.oracle_synth.restype = None
    L.oracle_cpu_upload_bench.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_int, ctypes.c_int, u8p, u8p]
    L.oracle_cpu_upload_bench.restype = ctypes.c_double
    L.oracle_synth_digests.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_int, ctypes.c_int, u8p, u8p, u8p]
    L.oracle_synth_digests.restype = ctypes.c_int
    L.oracle_cpu_download_bench.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_int, ctypes.c_int]
    L.oracle_cpu_download_bench.restype = ctypes.c_double
    _LIB = L
    return L


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else ctypes.c_char_p(b"\0")


# --------------------------------------------------------------------------
# C restatement wrappers
# --------------------------------------------------------------------------
def c_sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(_buf(data), len(data), out)
    return out.raw


def c_b64_encode(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(4 * ((len(data) + 2) // 3) + 1)
    n = lib().oracle_b64_encode(_buf(data), len(data), out)
    return out.raw[:n]


def c_b64_decode(text: bytes) -> Optional[bytes]:
    """Returns decoded bytes, or None where the JDK throws IllegalArgumentException."""
    out = ctypes.create_string_buffer(3 * ((len(text) + 3) // 4) + 1)
    n = ctypes.c_uint64(0)
    rc = lib().oracle_b64_decode(_buf(text), len(text), out, ctypes.byref(n))
    return None if rc != 0 else out.raw[: n.value]


def c_split(total: int, parts: int) -> List[Tuple[int, int]]:
    off = (ctypes.c_uint64 * parts)()
    ln = (ctypes.c_uint64 * parts)()
    lib().oracle_split(total, parts, off, ln)
    return [(off[i], ln[i]) for i in range(parts)]


def c_synth(file_index: int, start: int, length: int, seed: int = SYNTH_SEED) -> bytes:
    out = ctypes.create_string_buffer(max(length, 1))
    lib().oracle_synth(seed, file_index, start, length, out)
    return out.raw[:length]


def c_upload_batch(files: Sequence[bytes], nfrag: int, threads: int = 1):
    """Upload half for a list of files: (file_digests, frag_digests, b64 blob, b64_off)."""
    import numpy as np
    lens = np.array([len(f) for f in files], dtype=np.uint64)
    offs = np.zeros(len(files), dtype=np.uint64)
    if len(files) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    blob = b"".join(files)
    nf = len(files)
    fd = np.zeros((nf, 32), np.uint8)
    frd = np.zeros((nf, nfrag, 32), np.uint8)
    b64_off = np.zeros(nf * nfrag + 1, np.uint64)
    cap = int(sum(4 * ((int(l) // nfrag + 1 + 2) // 3) for l in lens) * nfrag + 16)
    b64 = ctypes.create_string_buffer(max(cap, 1))
    total = lib().oracle_upload_batch(_buf(blob), offs.ctypes.data, lens.ctypes.data, nf, nfrag,
                                      fd.ctypes.data, frd.ctypes.data, b64, b64_off.ctypes.data, threads)
    return fd, frd, b64.raw[:total], b64_off


def cpu_upload_bench(nfiles: int, file_len: int, nfrag: int, threads: int, use_openssl: bool,
                     seed: int = SYNTH_SEED):
    """Seconds spent hashing + encoding `nfiles` synthetic files (generation excluded)."""
    import numpy as np
    fd = np.zeros((nfiles, 32), np.uint8)
    frd = np.zeros((nfiles, nfrag, 32), np.uint8)
    secs = lib().oracle_cpu_upload_bench(seed, nfiles, file_len, nfrag, threads, int(use_openssl),
                                         fd.ctypes.data, frd.ctypes.data)
    return secs, fd, frd


def synth_digests(first: int, nfiles: int, file_len: int, nfrag: int, threads: int, use_openssl: bool = True,
                  with_b64: bool = True, seed: int = SYNTH_SEED):
    """(file digests (n, 32), fragment digests (n, N, 32), SHA-256 of every
    fragment's Base64 (n, N, 32) or None) of synthetic files [first, first+n):
    the checker for a whole batch.  Falls back to the scalar SHA-256 when
    libcrypto is not loadable."""
    import numpy as np
    fd = np.zeros((nfiles, 32), np.uint8)
    frd = np.zeros((nfiles, nfrag, 32), np.uint8)
    b64d = np.zeros((nfiles, nfrag, 32), np.uint8) if with_b64 else None
    args = (seed, first, nfiles, file_len, nfrag, threads)
    tail = (fd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), frd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
            b64d.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if with_b64 else None)
    rc = lib().oracle_synth_digests(*args, int(use_openssl), *tail)
    if rc == -1:
        rc = lib().oracle_synth_digests(*args, 0, *tail)
    if rc != 0:
        raise RuntimeError(f"oracle_synth_digests failed ({rc})")
    return fd, frd, b64d


def cpu_download_bench(nfiles: int, file_len: int, nfrag: int, threads: int, use_openssl: bool,
                       seed: int = SYNTH_SEED) -> float:
    """Seconds spent on the download path (decode + fragment SHA-256 verify +
    ordered append + fileId SHA-256 verify) for `nfiles` synthetic files;
    < 0 on error."""
    return lib().oracle_cpu_download_bench(seed, nfiles, file_len, nfrag, threads, int(use_openssl))


# --------------------------------------------------------------------------
# Pure-Python restatement (hashlib / base64) — independent cross-check
# --------------------------------------------------------------------------
def py_sha256_hex(data: bytes) -> str:
    """sha256Hex (SN:603-613)."""
    return hashlib.sha256(data).hexdigest()


def py_split(total: int, parts: int) -> List[Tuple[int, int]]:
    """handleUpload split loop (SN:138-171)."""
    base, rem = divmod(total, parts)
    out, off = [], 0
    for i in range(parts):
        n = base + (1 if i < rem else 0)
        out.append((off, n))
        off += n
    return out


def py_b64_encode(data: bytes) -> bytes:
    """Base64.getEncoder().encodeToString (SN:636)."""
    return base64.b64encode(data)


_ALPHA = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
_VAL = {c: i for i, c in enumerate(_ALPHA)}


def py_b64_decode_jdk(text: bytes) -> Optional[bytes]:
    """Base64.getDecoder().decode (SN:281), JDK basic-decoder semantics.

    Returns None where the JDK throws IllegalArgumentException.  A separate
    restatement from the C one (written as a grammar, not a state machine):
    body of complete 4-char units, then an optional final unit of 2 or 3
    alphabet chars, optionally padded to 4 with '=' (exactly "xx==" or
    "xxx="), nothing after the padding.
    """
    n = len(text)
    if n == 0:
        return b""
    if n < 2:
        return None
    p = 0
    while p < n and text[p] in _VAL:
        p += 1
    r = p % 4
    if p < n:
        if text[p] != ord("="):
            return None
        if r == 2:
            if p + 1 >= n or text[p + 1] != ord("=") or p + 2 != n:
                return None
        elif r == 3:
            if p + 1 != n:
                return None
        else:
            return None
    elif r == 1:
        return None
    body = text[:p]
    pad = (-len(body)) % 4
    # base64 module with validate=True cannot decode unpadded or non-canonical
    # tails the JDK accepts, so decode unit by unit.
    out = bytearray()
    for i in range(0, len(body), 4):
        unit = body[i:i + 4]
        bits, shift = 0, 18
        for c in unit:
            bits |= _VAL[c] << shift
            shift -= 6
        k = len(unit) - 1  # output bytes for a 2/3/4-char unit: 1/2/3
        out += bytes([(bits >> 16) & 255, (bits >> 8) & 255, bits & 255][:k])
    del pad
    return bytes(out)


def py_fragment_holders(f: int, n: int) -> Tuple[int, int]:
    """0-based holders of fragment f: node f (SN:144/427) and node f-1 (SN:145/428)."""
    return f, (f - 1 + n) % n


def py_node_fragments(k: int, n: int) -> Tuple[int, int]:
    """Fragments stored by 0-based node k: {k, k+1 mod N} (SN:143-145, 199-200)."""
    return k, (k + 1) % n


def py_build_fragments_json(file_id: str, frags: Sequence[Tuple[int, bytes]]) -> str:
    """buildFragmentsJson (SN:629-642): the storeFragments body."""
    parts = ['{"index":"%d","data":"%s"}' % (i, py_b64_encode(d).decode("ascii")) for i, d in frags]
    return '{"fileId":"' + file_id + '","fragments":[' + ",".join(parts) + "]}"


def py_manifest_json(file_id: str, name: str, total: int) -> str:
    """buildManifestJson (SN:620-626)."""
    return '{"fileId":"%s","originalName":"%s","totalFragments":%d}' % (file_id, name, total)


def py_download_plan(my_node: int, n: int, local: Sequence[int], down: Sequence[int] = ()) -> List[str]:
    """Source of each fragment in handleDownload (SN:422-449), 1-based node ids.

    `local` = fragment indices present on this node; `down` = 1-based nodes
    that fail to answer.  Returns "local", "node<k>" or "missing" per fragment.
    """
    plan = []
    for i in range(n):
        if i in local:
            plan.append("local")
            continue
        src = "missing"
        for node in (i + 1, ((i - 1 + n) % n) + 1):
            if node == my_node:
                continue
            if node in down:
                continue
            src = "node%d" % node
            break
        plan.append(src)
    return plan


# ---------------------------------------------------------------------------
# storeFragments wire codec (SN:629-753), restated with java.lang.String
# semantics: indexOf clamps a negative fromIndex to 0, trim() strips chars
# <= U+0020 at both ends, split(regex) drops trailing empty strings (and
# returns [s] when nothing matches), split(regex, 2) keeps them.

class JavaException(Exception):
    """A RuntimeException the reference would throw (kind = Java class name)."""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def j_index_of(s: str, sub: str, start: int = 0) -> int:
    return s.find(sub, max(start, 0))


def j_trim(s: str) -> str:
    a, b = 0, len(s)
    while a < b and ord(s[a]) <= 0x20:
        a += 1
    while b > a and ord(s[b - 1]) <= 0x20:
        b -= 1
    return s[a:b]


def j_split(s: str, sep: str, limit: int = 0) -> List[str]:
    """String.split for a literal separator (the reference's regexes are
    literal: "\\},\\{", ",", ":")."""
    if sep not in s:
        return [s]
    parts = s.split(sep) if limit <= 0 else s.split(sep, limit - 1)
    if limit == 0:
        while parts and parts[-1] == "":
            parts.pop()
    return parts


def j_parse_int(s: str) -> int:
    """Integer.parseInt (ASCII digits; NumberFormatException otherwise)."""
    body = s[1:] if s[:1] in ("-", "+") else s
    if not body or not all("0" <= c <= "9" for c in body):
        raise JavaException("NumberFormatException")
    v = int(s)
    if v < -2 ** 31 or v > 2 ** 31 - 1:
        raise JavaException("NumberFormatException")
    return v


def py_parse_json(json: str):
    """parseJson (SN:704-753): (fileId or None, [{"index": str, "data": str}])."""
    file_id = None
    frags = []
    i = j_index_of(json, '"fileId"')
    if i != -1:
        colon = j_index_of(json, ":", i)
        q1 = j_index_of(json, '"', colon + 1)
        q2 = j_index_of(json, '"', q1 + 1)
        if q1 != -1 and q2 != -1:
            file_id = json[q1 + 1:q2]
    k = j_index_of(json, '"fragments"')
    if k != -1:
        a = j_index_of(json, "[", k)
        b = j_index_of(json, "]", a)
        if a != -1 and b != -1:
            arr = j_trim(json[a + 1:b])
            if arr:
                for item in j_split(arr, "},{"):
                    item = j_trim(item.replace("{", "").replace("}", ""))
                    frag = {}
                    for field in j_split(item, ","):
                        kv = j_split(field, ":", 2)
                        if len(kv) != 2:
                            continue
                        key = j_trim(kv[0]).replace('"', "")
                        val = j_trim(kv[1]).replace('"', "")
                        if key in ("index", "data"):
                            frag[key] = val
                    if "index" in frag and "data" in frag:
                        frags.append(frag)
    return file_id, frags


def py_java_hashmap_order(keys: Sequence[int]) -> List[int]:
    """Iteration order of a java.util.HashMap<Integer, ?> after put(k) for k
    in `keys` (duplicates keep their first position): buckets ascending
    under the final table size, insertion order within a bucket."""
    uniq = []
    for k in keys:
        if k not in uniq:
            uniq.append(k)
    cap = 16
    while len(uniq) > cap * 3 // 4:
        cap *= 2

    def bucket(k):
        h = k & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)

    return sorted(uniq, key=lambda k: (bucket(k), uniq.index(k)))


def py_build_hash_response(file_id: str, pairs: Sequence[Tuple[int, str]]) -> str:
    """buildHashResponse (SN:644-655) over the HashMap filled by put(index, hash)."""
    m = {}
    for k, h in pairs:
        m[k] = h
    items = ['{"index":"%d","hash":"%s"}' % (k, m[k]) for k in py_java_hashmap_order([k for k, _ in pairs])]
    return '{"fileId":"' + file_id + '","received":[' + ",".join(items) + "]}"


def py_parse_response_hashes(json: str) -> dict:
    """parseResponseHashes (SN:657-701): {index: hash}."""
    out = {}
    json = j_trim(json)
    start = j_index_of(json, '"received"')
    if start == -1:
        return out
    start = j_index_of(json, "[", start)
    end = j_index_of(json, "]", start)
    if start == -1 or end == -1:
        return out
    if end < start + 1:
        raise JavaException("StringIndexOutOfBoundsException")
    arr = j_trim(json[start + 1:end])
    if not arr:
        return out
    for item in j_split(arr, "},{"):
        item = j_trim(item.replace("{", "").replace("}", "").replace('"', ""))
        index = None
        h = None
        for field in j_split(item, ","):
            kv = j_split(field, ":", 2)
            if len(kv) != 2:
                continue
            key, value = j_trim(kv[0]), j_trim(kv[1])
            if key == "index":
                index = j_parse_int(value)
            elif key == "hash":
                h = value
        if index is not None and h is not None:
            out[index] = h
    return out


def py_store_fragments(body: bytes):
    """handleInternalStoreFragments (SN:265-293) on one request body.

    Returns (status, file_id, done, response): status None or the Java
    exception class that ends the handler; `done` = [(index, data, hash)]
    for the fragments processed (written to <index>.frag, SN:284-285) before
    it; `response` = buildHashResponse JSON when status is None.
    """
    text = body.decode("utf-8", errors="replace")
    file_id, frags = py_parse_json(text)
    if file_id is None:
        return "NullPointerException", None, [], None  # dataRoot.resolve(null), SN:273
    done = []
    for fr in frags:
        try:
            index = j_parse_int(fr["index"])
        except JavaException as e:
            return e.kind, file_id, done, None
        data = py_b64_decode_jdk(fr["data"].encode("utf-8"))
        if data is None:
            return "IllegalArgumentException", file_id, done, None
        done.append((index, data, py_sha256_hex(data)))
    return None, file_id, done, py_build_hash_response(file_id, [(i, h) for i, _, h in done])


# ---- on-disk fragment store (SN:20, 147-149, 163-166, 273-285, 463-469) ----
def py_fragment_path(data_root: str, file_id: str, index: int) -> str:
    """dataRoot.resolve(fileId).resolve("fragments").resolve(i + ".frag")
    (SN:147-148, 165, 464); dataRoot = data/node-<id> (SN:20)."""
    return os.path.join(data_root, file_id, "fragments", f"{index}.frag")


def py_store_write(data_root: str, file_id: str, index: int, data: bytes) -> None:
    """Files.createDirectories(fragmentsDir) + Files.write(fragPath, fragment)
    (SN:149, 166; 275, 285): create or truncate, raw bytes."""
    path = py_fragment_path(data_root, file_id, index)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(data)


def py_try_load_fragment_local(data_root: str, file_id: str, index: int) -> Optional[bytes]:
    """tryLoadFragmentLocal (SN:463-469): the bytes, or None if absent."""
    path = py_fragment_path(data_root, file_id, index)
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        return f.read()


def py_tree(root: str) -> dict:
    """{relative path: bytes} of every file under root (tree comparison)."""
    out = {}
    for d, _, names in os.walk(root):
        for nm in names:
            p = os.path.join(d, nm)
            with open(p, "rb") as f:
                out[os.path.relpath(p, root)] = f.read()
    return out
