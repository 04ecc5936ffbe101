"""storeFragments wire codec, sender side: dfs_store_bodies_build vs the
oracle's buildFragmentsJson restatement (SN:629-642) and the golden bodies of
the reference's examples (uploaded at node 1).

Bar: byte-identical request bodies.  The CPU test covers the length helper;
the GPU tests build the bodies on the device through the C ABI."""
import hashlib
import random

import numpy as np
import pytest

import oracle as O


def _expected(data: bytes, nfrag: int, uploader: int):
    fid = hashlib.sha256(data).hexdigest()
    parts = [data[o:o + n] for o, n in O.py_split(len(data), nfrag)]
    out = []
    for k in range(nfrag):
        if k == uploader:  # SN:197
            continue
        a, b = k, (k + 1) % nfrag  # SN:199-200
        out.append((k, O.py_build_fragments_json(fid, [(a, parts[a]), (b, parts[b])]).encode()))
    return out


def test_store_body_len_matches_oracle():
    from dfs_amd._lib import lib
    rng = random.Random(5)
    for _ in range(300):
        n = rng.choice([0, 1, 2, 7, 28, 467, 2154, 9506, rng.randrange(0, 100000)])
        nfrag = rng.randrange(2, 11)
        k = rng.randrange(nfrag)
        data = bytes(n)
        parts = [data[o:o + m] for o, m in O.py_split(n, nfrag)]
        b = (k + 1) % nfrag
        want = len(O.py_build_fragments_json("0" * 64, [(k, parts[k]), (b, parts[b])]))
        assert lib().dfs_store_body_len(n, nfrag, k, b) == want


@pytest.mark.gpu
def test_store_bodies_examples_golden(engine, golden, example_bytes):
    for ex in golden["examples"]:
        data = example_bytes[ex["name"]]
        got = engine.store_bodies([data], 5, 0, [ex["fileId"]])[0]
        assert [k for k, _ in got] == [1, 2, 3, 4]
        for k, body in got:
            want = ex["store_fragments_from_node1"][str(k + 1)]  # the body, or its SHA-256 for large files
            assert (body.decode() if want.startswith("{") else hashlib.sha256(body).hexdigest()) == want


@pytest.mark.gpu
def test_store_bodies_vs_oracle_random(engine):
    rng = random.Random(11)
    for nfrag in (2, 3, 5, 8, 10):
        files = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 5, 11, 12, 13, 100, 777, 4099])))
                 for _ in range(12)]
        uploader = rng.randrange(nfrag)
        ids = [hashlib.sha256(d).hexdigest() for d in files]
        got = engine.store_bodies(files, nfrag, uploader, ids)
        for d, row in zip(files, got):
            assert row == _expected(d, nfrag, uploader)


@pytest.mark.gpu
def test_store_bodies_device_buffers(engine):
    """Device pointers (the bench path): 96 synthetic files of mixed sizes,
    fileIds from the device upload, bodies checked against the oracle."""
    import torch
    import dfs_amd
    from dfs_amd.engine import store_bodies_layout, store_bodies_device
    rng = np.random.default_rng(3)
    sizes = rng.integers(0, 300_000, 96).astype(np.uint64)
    sizes[:4] = [0, 1, 1 << 20, 209_716 * 5 + 3]
    offs = np.concatenate([[0], np.cumsum((sizes + 63) // 64 * 64)[:-1]]).astype(np.uint64)
    spans = np.stack([offs, sizes], axis=1)
    nf, nfrag, up = len(sizes), 5, 2
    dev = torch.device("cuda", 0)
    files = torch.empty(int(offs[-1] + sizes[-1]) + 64, dtype=torch.uint8, device=dev)
    dfs_amd.synth_fill(engine, files.data_ptr(), spans, 0, 0x5EED5EED)
    digests = torch.frombuffer(bytearray(b"".join(hashlib.sha256(O.c_synth(f, 0, int(sizes[f]))).digest()
                                                  for f in range(nf))), dtype=torch.uint8).to(dev)
    body_off = store_bodies_layout(engine, spans, nfrag, up)
    bodies = torch.zeros(int(body_off[-1]), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    store_bodies_device(engine, files.data_ptr(), spans, nfrag, up, digests.data_ptr(), bodies.data_ptr(), body_off)
    torch.cuda.synchronize(dev)
    host = bodies.cpu().numpy()
    for f in range(nf):
        want = _expected(O.c_synth(f, 0, int(sizes[f])), nfrag, up)
        for j, (k, body) in enumerate(want):
            o = int(body_off[f * (nfrag - 1) + j])
            assert host[o:o + len(body)].tobytes() == body, (f, k)


def _oracle_receive(body: bytes):
    st, fid, done, _resp = O.py_store_fragments(body)
    return st, fid, done


@pytest.mark.gpu
def test_store_receive_roundtrip_vs_oracle(engine):
    """Bodies from the device builder, received on the device: parse, decode,
    hash == the oracle's handleInternalStoreFragments restatement."""
    rng = random.Random(21)
    files = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 2, 3, 4, 5, 47, 48, 49, 1000, 70001])))
             for _ in range(10)]
    ids = [hashlib.sha256(d).hexdigest() for d in files]
    for nfrag in (2, 5, 10):
        built = engine.store_bodies(files, nfrag, nfrag - 1, ids)
        bodies = [b for row in built for _, b in row]
        got = engine.store_receive(bodies)
        for body, (st, fid, frags) in zip(bodies, got):
            ost, ofid, done = _oracle_receive(body)
            assert ost is None and st == 0
            assert fid == ofid
            assert [(i, d, h) for i, d, h in frags] == done


@pytest.mark.gpu
def test_store_receive_examples_and_bad_bodies(engine, golden, example_bytes):
    from dfs_amd._lib import DFS_E_DECODE, DFS_E_WIRE
    teste = golden["examples"][0]
    good = teste["store_fragments_from_node1"]["5"].encode()  # {4, 0}
    bad_b64 = good.replace(b"VGVzdGUg", b"VGVzd*Ug")      # entry 2 not Base64 -> IAE after entry 1
    bad_pad = good.replace(b"dWl2by4=", b"dWl2b")          # 5 chars: dangling char -> IAE on entry 1
    spaced = good.replace(b'","data"', b'", "data"', 1)  # parseJson accepts it, the device form does not
    three = good.replace(b"]}", b',{"index":"1","data":"Zm9v"}]}')
    got = engine.store_receive([good, bad_b64, bad_pad, spaced, three, b"", b"{}"])
    st, fid, frags = got[0]
    assert st == 0 and fid == teste["fileId"]
    assert [(i, h) for i, _, h in frags] == [(4, teste["fragments"][4]["sha256"]), (0, teste["fragments"][0]["sha256"])]
    assert got[1][0] == DFS_E_DECODE and _oracle_receive(bad_b64)[0] == "IllegalArgumentException"
    assert got[1][2][0][2] == teste["fragments"][4]["sha256"]  # entry 1 was processed, as SN:280-285 does
    assert got[2][0] == DFS_E_DECODE and _oracle_receive(bad_pad)[0] == "IllegalArgumentException"
    for k in (3, 4, 5, 6):
        assert got[k][0] == DFS_E_WIRE
    assert _oracle_receive(spaced)[0] is None  # the host parser's case
