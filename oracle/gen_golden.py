#!/usr/bin/env python3
"""Generate tests/golden/golden.json — TEST INFRASTRUCTURE ONLY.

Uses only the Python standard library (hashlib / base64 are OpenSSL-backed
implementations of FIPS 180-4 and RFC 4648) plus oracle.py's pure-Python
JDK-decoder restatement.  The C oracle is NOT used here, so the fixtures are an
independent check on it.

Inputs: the reference's own data files (examples/*, copied byte-for-byte to
tests/golden/examples/), FIPS 180-4 / RFC 4648 known answers, edge sizes and
the synthetic generator.  There is no JDK in this image, so the reference
itself could not be run: digests and Base64 are pinned by the standards the
JDK classes implement; decoder error cases are restated JDK semantics
(java.util.Base64.Decoder, basic) and are "parity unpinned": never run on a JDK.

Run:  python oracle/gen_golden.py   (rewrites tests/golden/golden.json)
"""
import base64
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402

EX_DIR = os.path.join(ROOT, "tests", "golden", "examples")
N_REF = 5  # TOTAL_NODES, StorageNode.java:15


def splitmix64(x):
    m = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def synth(f, start, length, seed=O.SYNTH_SEED):
    out = bytearray()
    for o in range(start, start + length):
        v = splitmix64(seed ^ ((f << 40) | (o >> 3)))
        out.append((v >> (8 * (o & 7))) & 255)
    return bytes(out)


def frag_record(data, off, ln, full_b64):
    frag = data[off:off + ln]
    b = base64.b64encode(frag)
    rec = {"index": None, "offset": off, "length": ln, "sha256": hashlib.sha256(frag).hexdigest(),
           "b64_len": len(b), "b64_sha256": hashlib.sha256(b).hexdigest()}
    if full_b64:
        rec["b64"] = b.decode()
    return rec


def file_record(name, data, nfrag, full_b64=False):
    fid = hashlib.sha256(data).hexdigest()
    frags = []
    for i, (off, ln) in enumerate(O.py_split(len(data), nfrag)):
        r = frag_record(data, off, ln, full_b64)
        r["index"] = i
        frags.append(r)
    return {"name": name, "size": len(data), "nfrag": nfrag, "fileId": fid, "fragments": frags}


def main():
    g = {"generator": "oracle/gen_golden.py", "n_ref": N_REF}

    # FIPS 180-4 examples (SHA-256).
    g["sha256_kat"] = [
        {"input": {"kind": "ascii", "text": ""},
         "digest": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"},
        {"input": {"kind": "ascii", "text": "abc"},
         "digest": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"},
        {"input": {"kind": "ascii", "text": "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"},
         "digest": "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"},
        {"input": {"kind": "repeat", "byte": 97, "count": 1000000},
         "digest": "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"},
    ]
    for k in g["sha256_kat"]:  # the standard's answers must agree with hashlib
        inp = k["input"]
        data = inp["text"].encode() if inp["kind"] == "ascii" else bytes([inp["byte"]]) * inp["count"]
        assert hashlib.sha256(data).hexdigest() == k["digest"], k

    # RFC 4648 §10 test vectors.
    g["b64_rfc4648"] = [{"input": s, "output": o} for s, o in [
        ("", ""), ("f", "Zg=="), ("fo", "Zm8="), ("foo", "Zm9v"), ("foob", "Zm9vYg=="),
        ("fooba", "Zm9vYmE="), ("foobar", "Zm9vYmFy")]]
    for v in g["b64_rfc4648"]:
        assert base64.b64encode(v["input"].encode()).decode() == v["output"]

    # Decoder cases: JDK basic-decoder semantics (None = IllegalArgumentException).
    dec_inputs = [b"", b"Zg==", b"Zm8=", b"Zm9v", b"Zm9vYg==", b"Zm9vYmE=", b"Zm9vYmFy",
                  b"Zg", b"Zm8", b"Zm9vYg", b"Zm9vYmE", b"Zh==", b"Zm9=",  # accepted by the JDK
                  b"Z", b"=", b"Z===", b"Zg=", b"Zg=x", b"Zm9v=", b"Zm9v====", b"Zg==Zg==",
                  b"Zm8==", b"Zm 9v", b"Zm9v\n", b"Zm-v", b"Zm_v", b"Zm9\xff", b"====", b"Zm9vY"]
    g["b64_decode_jdk"] = []
    for t in dec_inputs:
        r = O.py_b64_decode_jdk(t)
        g["b64_decode_jdk"].append({"input_hex": t.hex(), "output_hex": None if r is None else r.hex()})

    # The reference's examples/ files at N=5.
    g["examples"] = []
    for name in ["teste.txt", "id.jpg", "pl.png", "pag1.html"]:
        data = open(os.path.join(EX_DIR, name), "rb").read()
        rec = file_record(name, data, N_REF, full_b64=(name == "teste.txt"))
        rec["manifest"] = O.py_manifest_json(rec["fileId"], name, N_REF)
        # storeFragments bodies sent by uploader node 1 (SN:195-205, 629-642).
        bodies = {}
        for node in range(N_REF):
            if node == 0:
                continue
            f1, f2 = O.py_node_fragments(node, N_REF)
            frags = [(f1, data[rec["fragments"][f1]["offset"]:][:rec["fragments"][f1]["length"]]),
                     (f2, data[rec["fragments"][f2]["offset"]:][:rec["fragments"][f2]["length"]])]
            body = O.py_build_fragments_json(rec["fileId"], frags)
            bodies[str(node + 1)] = body if name == "teste.txt" else hashlib.sha256(body.encode()).hexdigest()
        rec["store_fragments_from_node1"] = bodies
        # The log line the reference prints per fragment (SN:160), uploader node 1.
        rec["log_lines"] = ["[1] Fragment %d: %d bytes, hash=%s" % (f["index"], f["length"], f["sha256"])
                            for f in rec["fragments"]]
        g["examples"].append(rec)

    # Degraded download plan with node 3 down (SN:422-449), every other node downloading.
    g["download_plan_node3_down"] = {}
    for me in [1, 2, 4, 5]:
        local = O.py_node_fragments(me - 1, N_REF)
        g["download_plan_node3_down"][str(me)] = O.py_download_plan(me, N_REF, local, down=[3])

    # Edge sizes (SHA padding boundaries, Base64 padding, S < N) on synthetic data.
    g["edge"] = []
    for nfrag in (5, 8):
        for S in [0, 1, 2, 3, 4, 5, 7, 8, 9, 54, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129,
                  191, 192, 255, 256, 319, 320, 321, 447, 448, 449, 1000, 4097]:
            data = synth(S, 0, S)
            rec = file_record("synth-%d" % S, data, nfrag, full_b64=(S <= 64))
            rec["synth_file_index"] = S
            g["edge"].append(rec)

    # Synthetic generator pins: first 16 bytes and bytes 1000..1015 of a few files.
    g["synth"] = []
    for f in [0, 1, 7, 65535, 1 << 20]:
        g["synth"].append({"file": f, "seed": O.SYNTH_SEED,
                           "head_hex": synth(f, 0, 16).hex(), "at1000_hex": synth(f, 1000, 16).hex()})

    # Config-2-shaped digests for a couple of 1 MiB synthetic files (N=5).
    g["synth_1mib"] = []
    for f in [0, 3]:
        data = synth_fast(f, 1 << 20)
        g["synth_1mib"].append(file_record("synth-1MiB-%d" % f, data, N_REF))
        g["synth_1mib"][-1]["synth_file_index"] = f

    path = os.path.join(ROOT, "tests", "golden", "golden.json")
    with open(path, "w") as fh:
        json.dump(g, fh, indent=1, sort_keys=True)
    print("wrote", path)


def synth_fast(f, length, seed=O.SYNTH_SEED):
    words = [splitmix64(seed ^ ((f << 40) | j)) for j in range((length + 7) // 8)]
    return b"".join(struct.pack("<Q", w) for w in words)[:length]


if __name__ == "__main__":
    main()
