"""The CPU oracle pinned against the golden vectors (no GPU).

Golden vectors: FIPS 180-4 / RFC 4648 known answers, the reference's own
examples/ files, edge sizes on synthetic data, the JDK decoder's accept/reject
cases (restated semantics: parity unpinned, no JDK here to run them on).
"""
import base64
import hashlib
import os
import random

import numpy as np
import pytest

import oracle as O


def kat_bytes(inp):
    if inp["kind"] == "ascii":
        return inp["text"].encode()
    return bytes([inp["byte"]]) * inp["count"]


def test_sha256_kats(golden):
    for k in golden["sha256_kat"]:
        assert O.c_sha256(kat_bytes(k["input"])).hex() == k["digest"]


def test_b64_rfc4648(golden):
    for v in golden["b64_rfc4648"]:
        assert O.c_b64_encode(v["input"].encode()).decode() == v["output"]
        assert O.c_b64_decode(v["output"].encode()) == v["input"].encode()


def test_b64_decode_jdk_cases(golden):
    for d in golden["b64_decode_jdk"]:
        t = bytes.fromhex(d["input_hex"])
        want = None if d["output_hex"] is None else bytes.fromhex(d["output_hex"])
        assert O.c_b64_decode(t) == want, t
        assert O.py_b64_decode_jdk(t) == want, t


def test_survey_appendix_a_values(golden):
    # A few values of the reference's example files, computed independently
    # with hashlib and cross-checked with sha256sum / openssl dgst.
    ex = {e["name"]: e for e in golden["examples"]}
    assert ex["teste.txt"]["fileId"] == "3915569114252388ab0ede1637a7ca2c871d7785311389a22d10a13a71d662a3"
    assert ex["id.jpg"]["fileId"] == "020122de5ef7472f33fb6bc9c9b5fe49377f96f0cb37180a58a48b04b5bfdff2"
    assert ex["pl.png"]["fragments"][4]["sha256"] == \
        "855884a258a74bf17c0e09a38660f7ee907a95e7e52465c2a357f5900c664451"
    assert [f["b64"] for f in ex["teste.txt"]["fragments"]] == \
        ["VGVzdGUg", "cGFyYSBl", "bnZpbyBk", "ZSBhcnE=", "dWl2by4="]
    assert ex["teste.txt"]["store_fragments_from_node1"]["5"] == (
        '{"fileId":"3915569114252388ab0ede1637a7ca2c871d7785311389a22d10a13a71d662a3",'
        '"fragments":[{"index":"4","data":"dWl2by4="},{"index":"0","data":"VGVzdGUg"}]}')
    plan = golden["download_plan_node3_down"]
    assert plan["1"] == ["local", "local", "node2", "node4", "node5"]
    assert plan["4"] == ["node1", "node2", "node2", "local", "local"]


def test_examples_upload(golden, example_bytes):
    for e in golden["examples"]:
        data = example_bytes[e["name"]]
        assert O.c_sha256(data).hex() == e["fileId"]
        fd, frd, b64, off = O.c_upload_batch([data], e["nfrag"])
        assert fd[0].tobytes().hex() == e["fileId"]
        for f in e["fragments"]:
            assert frd[0, f["index"]].tobytes().hex() == f["sha256"]
            seg = b64[int(off[f["index"]]):int(off[f["index"] + 1])]
            assert len(seg) == f["b64_len"]
            assert hashlib.sha256(seg).hexdigest() == f["b64_sha256"]
        assert [(f["offset"], f["length"]) for f in e["fragments"]] == O.c_split(len(data), e["nfrag"])


def test_edge_sizes(golden):
    for e in golden["edge"]:
        data = O.c_synth(e["synth_file_index"], 0, e["size"])
        assert O.c_sha256(data).hex() == e["fileId"]
        for f in e["fragments"]:
            frag = data[f["offset"]:f["offset"] + f["length"]]
            assert O.c_sha256(frag).hex() == f["sha256"]
            enc = O.c_b64_encode(frag)
            assert hashlib.sha256(enc).hexdigest() == f["b64_sha256"]
            if "b64" in f:
                assert enc.decode() == f["b64"]
            assert O.c_b64_decode(enc) == frag


def test_synth_pins(golden):
    for s in golden["synth"]:
        assert O.c_synth(s["file"], 0, 16, s["seed"]).hex() == s["head_hex"]
        assert O.c_synth(s["file"], 1000, 16, s["seed"]).hex() == s["at1000_hex"]
    for e in golden["synth_1mib"]:
        data = O.c_synth(e["synth_file_index"], 0, e["size"])
        assert O.c_sha256(data).hex() == e["fileId"]


def test_c_vs_python_random():
    rng = random.Random(1234)
    for _ in range(300):
        n = rng.choice([0, 1, 2, 3, 55, 56, 63, 64, 65, rng.randrange(0, 5000)])
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.c_sha256(d) == hashlib.sha256(d).digest()
        e = O.c_b64_encode(d)
        assert e == base64.b64encode(d)
        assert O.c_b64_decode(e) == d


def test_decode_fuzz_c_vs_py():
    rng = random.Random(99)
    alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/="
    for _ in range(3000):
        n = rng.randrange(0, 14)
        t = bytes(rng.choice(alphabet + b"-_ \n\xff") for _ in range(n))
        assert O.c_b64_decode(t) == O.py_b64_decode_jdk(t), t
    # The JDK accepts everything Python's strict decoder accepts, with the same bytes.
    for _ in range(500):
        d = os.urandom(rng.randrange(0, 40))
        e = base64.b64encode(d)
        assert O.py_b64_decode_jdk(e) == base64.b64decode(e, validate=True) == d


def test_split_and_placement():
    for S in [0, 1, 2, 4, 5, 6, 28, 9506, 1 << 20, (1 << 28)]:
        for N in [1, 2, 5, 8]:
            sp = O.c_split(S, N)
            assert sp == O.py_split(S, N)
            assert sum(l for _, l in sp) == S
            assert max(l for _, l in sp) - min(l for _, l in sp) <= 1
    # node k holds {k, k+1}; fragment f lives on nodes {f, f-1}
    for N in [5, 8]:
        for f in range(N):
            a, b = O.py_fragment_holders(f, N)
            assert f in O.py_node_fragments(a, N) and f in O.py_node_fragments(b, N)


def test_reassemble_verify_oracle():
    import ctypes
    L = O.lib()
    data = O.c_synth(5, 0, 1000)
    parts = [data[o:o + l] for o, l in O.c_split(len(data), 5)]
    bufs = [ctypes.create_string_buffer(p, len(p) or 1) for p in parts]
    ptrs = (ctypes.c_void_p * 5)(*[ctypes.addressof(b) for b in bufs])
    lens = np.array([len(p) for p in parts], dtype=np.uint64)
    out = ctypes.create_string_buffer(1000)
    exp = ctypes.create_string_buffer(hashlib.sha256(data).digest(), 32)
    assert L.oracle_reassemble_verify(ptrs, lens.ctypes.data, 5, exp, out) == 0
    assert out.raw == data
    bad = ctypes.create_string_buffer(b"\0" * 32, 32)
    assert L.oracle_reassemble_verify(ptrs, lens.ctypes.data, 5, bad, out) == -6


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_bench_matches_oracle(threads):
    secs, fd, frd = O.cpu_upload_bench(6, 4096 + 3, 5, threads, use_openssl=False)
    assert secs >= 0
    for f in range(6):
        data = O.c_synth(f, 0, 4096 + 3)
        assert fd[f].tobytes() == hashlib.sha256(data).digest()
        for i, (o, l) in enumerate(O.c_split(len(data), 5)):
            assert frd[f, i].tobytes() == hashlib.sha256(data[o:o + l]).digest()
    s2, fd2, frd2 = O.cpu_upload_bench(6, 4096 + 3, 5, threads, use_openssl=True)
    if s2 >= 0:  # libcrypto present
        assert (fd2 == fd).all() and (frd2 == frd).all()


def test_cpu_download_baseline_verifies():
    """The download-side CPU baseline decodes, hashes and reassembles every
    file and checks every digest itself (< 0 on any mismatch)."""
    for n in (0, 1, 2, 7, 100, 4097, 1000003):
        for ossl in (False, True):
            secs = O.cpu_download_bench(3, n, 5, 2, ossl)
            assert secs >= 0 or (ossl and secs == -1.0), (n, ossl, secs)


def test_synth_digests_checker_matches_hashlib():
    """oracle_synth_digests (the whole-batch checker of bench.py and the GPU
    tests): fileId, fragment digests and the SHA-256 of each fragment's Base64
    for synthetic files, libcrypto and scalar SHA-256 alike, against hashlib /
    base64 on the same bytes — including files shorter than N (empty fragments)."""
    import base64
    import hashlib
    for first, n, S, N in [(0, 5, 1000, 5), (77, 3, 3, 5), (9, 2, 0, 8), (1234, 4, 262144, 8), (5, 2, (1 << 20) + 1, 5)]:
        for ossl in (True, False):
            fd, frd, b64d = O.synth_digests(first, n, S, N, 3, use_openssl=ossl)
            for f in range(n):
                d = O.c_synth(first + f, 0, S)
                assert fd[f].tobytes() == hashlib.sha256(d).digest()
                for i, (o, ln) in enumerate(O.py_split(S, N)):
                    assert frd[f, i].tobytes() == hashlib.sha256(d[o:o + ln]).digest()
                    assert b64d[f, i].tobytes() == hashlib.sha256(base64.b64encode(d[o:o + ln])).digest()
    fd, frd, none = O.synth_digests(0, 2, 100, 5, 1, with_b64=False)
    assert none is None and fd.shape == (2, 32) and frd.shape == (2, 5, 32)
