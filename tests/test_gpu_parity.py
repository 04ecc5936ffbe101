"""HIP path vs the CPU oracle and the golden vectors (needs a gfx950 GPU).

Bar: bit-exact digests and bytes (integer/byte work).  Every call goes through
the C ABI of libdfsgpu.so; the oracle is only the checker.
"""
import base64
import os
import hashlib
import random

import numpy as np
import pytest

import dfs_amd
import oracle as O

pytestmark = pytest.mark.gpu


def kat_bytes(inp):
    if inp["kind"] == "ascii":
        return inp["text"].encode()
    return bytes([inp["byte"]]) * inp["count"]


def test_sha256_kats(engine, golden):
    msgs = [kat_bytes(k["input"]) for k in golden["sha256_kat"]]
    got = engine.sha256(msgs)
    assert [g.hex() for g in got] == [k["digest"] for k in golden["sha256_kat"]]


def test_sha256_every_length_and_alignment(engine):
    # lengths 0..300 (every padding case) at every start offset mod 4
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    spans = np.array([(a, n) for n in range(0, 301) for a in (0, 1, 2, 3, 517)], dtype=np.uint64)
    got = engine.sha256_spans(buf, spans)
    raw = buf.tobytes()
    for i, (a, n) in enumerate(spans):
        assert got[i].tobytes() == hashlib.sha256(raw[a:a + n]).digest(), (a, n)


def test_sha256_random_messages_vs_oracle(engine):
    rng = random.Random(11)
    msgs = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 20000))) for _ in range(40)]
    msgs += [b"", b"a" * 64, b"b" * 55, b"c" * 56]
    got = engine.sha256(msgs)
    for m, g in zip(msgs, got):
        assert g == O.c_sha256(m)


def test_b64_encode_rfc_and_edges(engine, golden):
    vec = golden["b64_rfc4648"]
    got = engine.b64_encode([v["input"].encode() for v in vec])
    assert [g.decode() for g in got] == [v["output"] for v in vec]
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    msgs = [raw[a:a + n] for n in list(range(0, 40)) + [12287, 12288, 12289, 24577, 65536]
            for a in (0, 1, 2, 3)]
    got = engine.b64_encode(msgs)
    for m, g in zip(msgs, got):
        assert g == base64.b64encode(m)
        assert g == O.c_b64_encode(m)


def test_b64_encode_every_source_and_destination_phase(engine):
    """Messages packed back to back: the source of a message starts at any
    byte phase mod 4 and its Base64 at any dword phase mod 16 (0, 4, 8, 12).
    Every one of the 16 combinations is steered to (a short filler message
    before it) for each length: one partial group, a wave, a tile of 12 KiB
    more or less a group, several tiles — so a lane's 16 chars straddle
    16-byte chunks inside waves, across waves, across tiles and at a
    message's last group.  Against Python's base64."""
    rng = random.Random(77)
    msgs, want = [], []
    s = o = 0  # source bytes / Base64 chars before the next message

    def add(m):
        nonlocal s, o
        msgs.append(m)
        s += len(m)
        o += 4 * ((len(m) + 2) // 3)

    for n in [5, 13, 767, 769, 12287, 12288, 12289, 12301, 24576 + 7, 40001, 100003]:
        for sp in range(4):
            for dp in (0, 4, 8, 12):
                # one or two fillers reach every phase (one alone reaches 12 of the 16)
                fill = next((a, b) for a in range(1, 14) for b in range(0, 14)
                            if (s + a + b) % 4 == sp and (o + 4 * ((a + 2) // 3) + 4 * ((b + 2) // 3)) % 16 == dp)
                for k in fill:
                    if k:
                        add(rng.randbytes(k))
                want.append((n, sp, dp, len(msgs)))
                assert (s % 4, o % 16) == (sp, dp)
                add(rng.randbytes(n))
    got = engine.b64_encode(msgs)
    for k, m in enumerate(msgs):
        assert got[k] == base64.b64encode(m), (k, len(m), [w for w in want if w[3] == k])


def test_b64_decode_jdk_cases(engine, golden):
    cases = golden["b64_decode_jdk"]
    got = engine.b64_decode([bytes.fromhex(d["input_hex"]) for d in cases])
    for d, g in zip(cases, got):
        want = None if d["output_hex"] is None else bytes.fromhex(d["output_hex"])
        assert g == want, d["input_hex"]
    with pytest.raises(dfs_amd.IllegalArgumentException):
        engine.b64_decode_one(b"Zm9v=")


def test_b64_decode_alignments_and_lengths(engine):
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes()
             for n in list(range(0, 60)) + [4095, 4096, 12288, 12289, 50001]]
    texts = [base64.b64encode(d) for d in datas]
    for pad_in in (0, 1, 2, 3):
        # misalign inputs by prefixing the packed buffer, and outputs by offsets
        for out_shift in (0, 1, 2, 3):
            offs, o = [], out_shift
            for d in datas:
                offs.append(o)
                o += len(d) + 5 + out_shift
            msgs = [b"x" * pad_in + t for t in texts]
            # decode the prefixed texts: the prefix makes them invalid, so build spans by hand
            buf = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
            spans, p = [], 0
            for t in msgs:
                spans.append((p + pad_in, len(t) - pad_in))
                p += len(t)
            got = _decode_spans(engine, buf, spans, offs)
            for d, g in zip(datas, got):
                assert g == d


def test_b64_decode_multitile_every_output_phase(engine):
    """The LDS-staged decode (tiles of 16 or 32 KiB of chars, 16-byte aligned output
    chunks cut at byte offset h mod 3): messages spanning 1-5 tiles at every
    output address mod 16 and every input address mod 4, incl. lengths that
    end one char before / after a tile and every final-unit form."""
    rng = np.random.default_rng(23)
    sizes = [12287, 12288, 12289, 24575, 24576, 24577, 49150, 61441, 65536 + 7]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    texts = [base64.b64encode(d) for d in datas]
    texts += [t.rstrip(b"=") for t in texts]  # unpadded final units decode too (JDK basic decoder)
    datas += datas
    for pad_in in (0, 1, 2, 3):
        buf = np.frombuffer(b"".join(b"#" * pad_in + t for t in texts), dtype=np.uint8).copy()
        spans, p = [], 0
        for t in texts:
            spans.append((p + pad_in, len(t)))
            p += len(t) + pad_in
        for out_phase in range(16):
            offs, o = [], out_phase
            for d in datas:
                offs.append(o)
                o += (len(d) + 16 + 15) // 16 * 16 + out_phase
            got = _decode_spans(engine, buf, spans, offs)
            for d, g in zip(datas, got):
                assert g == d, (pad_in, out_phase, len(d))


def test_reassemble_multitile_every_alignment(engine):
    """gather_kernel: fragments of 16 KiB tiles and more, every destination
    phase mod 16 (via the file size mod 16 shifting later fragments) and
    every source phase (host fragments are staged back to back)."""
    files = [O.c_synth(40 + k, 0, 5 * 16384 * 3 + k) for k in range(16)] + [O.c_synth(60, 0, 1 << 20)]
    ups = engine.upload(files, 5)
    frags = [[d[g.offset:g.offset + g.length] for g in u.fragments] for d, u in zip(files, ups)]
    res = engine.reassemble_verify(frags, [u.file_id for u in ups])
    for d, (st, body, h) in zip(files, res):
        assert st == 0 and body == d and h == hashlib.sha256(d).hexdigest()


def _decode_spans(engine, buf, spans, out_off):
    import ctypes
    n = len(spans)
    spans = np.array(spans, dtype=np.uint64)
    caps = [int(dfs_amd.lib().dfs_b64_decoded_cap(int(s[1]))) for s in spans]
    out_off = np.array(out_off, dtype=np.uint64)
    out = np.zeros(int(max(out_off + np.array(caps, dtype=np.uint64))) + 1, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    rc = dfs_amd.lib().dfs_b64_decode_batch(engine.ctx, buf.ctypes.data, spans.ctypes.data, n, out.ctypes.data,
                                            out_off.ctypes.data, out_len.ctypes.data, status.ctypes.data, 0)
    assert rc in (0, dfs_amd.DFS_E_DECODE)
    return [None if status[i] else out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes()
            for i in range(n)]


def test_b64_decode_fuzz_vs_oracle(engine):
    rng = random.Random(17)
    alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/="
    texts = []
    for _ in range(2000):
        n = rng.randrange(0, 40)
        texts.append(bytes(rng.choice(alphabet + b"-_ \n\xff") for _ in range(n)))
    # long valid texts with one corrupted char somewhere
    for _ in range(40):
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(100, 30000)))
        t = bytearray(base64.b64encode(d))
        t[rng.randrange(len(t))] = rng.choice(b"*-_= \n")
        texts.append(bytes(t))
    got = engine.b64_decode(texts)
    for t, g in zip(texts, got):
        assert g == O.c_b64_decode(t), t[:40]


def test_examples_upload_matches_golden(engine, golden, example_bytes):
    names = [e["name"] for e in golden["examples"]]
    res = engine.upload([example_bytes[n] for n in names], 5)
    for e, r in zip(golden["examples"], res):
        assert r.file_id == e["fileId"]
        for f, g in zip(e["fragments"], r.fragments):
            assert (g.index, g.offset, g.length, g.hash) == (f["index"], f["offset"], f["length"], f["sha256"])
            assert len(g.b64) == f["b64_len"]
            assert hashlib.sha256(g.b64).hexdigest() == f["b64_sha256"]
            if "b64" in f:
                assert g.b64.decode() == f["b64"]
        # the reference's per-fragment log line (SN:160), uploader node 1
        lines = ["[1] Fragment %d: %d bytes, hash=%s" % (g.index, g.length, g.hash) for g in r.fragments]
        assert lines == e["log_lines"]


def test_edge_sizes_upload(engine, golden):
    for nfrag in (5, 8):
        recs = [e for e in golden["edge"] if e["nfrag"] == nfrag]
        files = [O.c_synth(e["synth_file_index"], 0, e["size"]) for e in recs]
        res = engine.upload(files, nfrag)
        for e, r in zip(recs, res):
            assert r.file_id == e["fileId"]
            for f, g in zip(e["fragments"], r.fragments):
                assert g.hash == f["sha256"]
                assert hashlib.sha256(g.b64).hexdigest() == f["b64_sha256"]


def test_upload_batch_vs_oracle_mixed_sizes(engine):
    rng = random.Random(23)
    sizes = [rng.choice([0, 1, 4, 63, 64, 65, 999, 4096, 70001, 1 << 18]) for _ in range(60)] + [1 << 20] * 4
    files = [O.c_synth(1000 + i, 0, s) for i, s in enumerate(sizes)]
    for nfrag in (5, 8):
        res = engine.upload(files, nfrag)
        fd, frd, b64, off = O.c_upload_batch(files, nfrag, threads=4)
        for f, r in enumerate(res):
            assert r.file_id == fd[f].tobytes().hex()
            for i, g in enumerate(r.fragments):
                k = f * nfrag + i
                assert g.hash == frd[f, i].tobytes().hex()
                assert g.b64 == b64[int(off[k]):int(off[k + 1])]


def _check_upload(res, files, nfrag):
    fd, frd, b64, off = O.c_upload_batch(files, nfrag, threads=4)
    for f, r in enumerate(res):
        assert r.file_id == fd[f].tobytes().hex()
        for i, g in enumerate(r.fragments):
            k = f * nfrag + i
            assert g.hash == frd[f, i].tobytes().hex(), (len(files[f]), i)
            assert g.b64 == b64[int(off[k]):int(off[k + 1])], (len(files[f]), i)


def test_fused_encode_every_block_phase(monkeypatch):
    """DFS_UPLOAD_MODE=fused (Base64 written by the SHA fragment lanes):
    fragments of 0..7 full 64-byte blocks (every block phase k mod 3 and
    carry) plus every tail class, at the byte alignments the batch packing
    produces; then mixed lengths inside one wave (lanes leaving the block
    loop at different blocks park their state)."""
    monkeypatch.setenv("DFS_UPLOAD_MODE", "fused")
    eng = dfs_amd.FragmentEngine(0)
    try:
        sizes = [64 * k + r for k in range(8) for r in (0, 1, 2, 3, 5, 55, 56, 63)]
        for nfrag in (1, 3, 5):
            files = [O.c_synth(3000 + i, 0, s * nfrag + (i % nfrag)) for i, s in enumerate(sizes)]
            _check_upload(eng.upload(files, nfrag), files, nfrag)
        rng = random.Random(17)
        files = [O.c_synth(3500 + i, 0, rng.randrange(0, 6000)) for i in range(200)]
        _check_upload(eng.upload(files, 5), files, 5)
        sizes = [rng.choice([0, 7, 64, 200, 4099, 65536, 300001]) for _ in range(40)]
        files = [O.c_synth(3800 + i, 0, s) for i, s in enumerate(sizes)]
        _check_upload(eng.upload(files, 4), files, 4)
    finally:
        eng.close()


def test_upload_two_kernel_mode(monkeypatch):
    """DFS_UPLOAD_MODE=kernels (the library default): SHA-256 and the Base64
    encode kernel on two streams."""
    monkeypatch.setenv("DFS_UPLOAD_MODE", "kernels")
    eng = dfs_amd.FragmentEngine(0)
    try:
        rng = random.Random(5)
        sizes = [rng.choice([0, 7, 64, 200, 4099, 65536, 300001]) for _ in range(40)]
        files = [O.c_synth(4000 + i, 0, s) for i, s in enumerate(sizes)]
        _check_upload(eng.upload(files, 5), files, 5)
    finally:
        eng.close()


def test_reassemble_verify(engine, example_bytes):
    files = [example_bytes["id.jpg"], example_bytes["teste.txt"], O.c_synth(9, 0, 100003)]
    ups = engine.upload(files, 5)
    frags = [[d[g.offset:g.offset + g.length] for g in u.fragments] for d, u in zip(files, ups)]
    res = engine.reassemble_verify(frags, [u.file_id for u in ups])
    for d, (st, body, h) in zip(files, res):
        assert st == 0 and body == d and h == hashlib.sha256(d).hexdigest()
    # corrupted fragment -> "File corrupted" (SN:455-458); missing -> SN:443-446
    bad = [list(f) for f in frags]
    bad[0][2] = bytes([bad[0][2][0] ^ 1]) + bad[0][2][1:]
    bad[1][4] = None
    res = engine.reassemble_verify(bad, [u.file_id for u in ups])
    assert res[0][0] == dfs_amd.DFS_E_CORRUPT
    assert res[1][0] == dfs_amd.DFS_E_MISSING
    assert res[2][0] == 0


def test_download_base64_path(engine, example_bytes):
    files = [example_bytes[n] for n in ("id.jpg", "pl.png", "pag1.html", "teste.txt")] + \
        [O.c_synth(77, 0, 262144), O.c_synth(78, 0, 3), b""]
    for nfrag in (5, 8):
        ups = engine.upload(files, nfrag)
        b64 = [[g.b64 for g in u.fragments] for u in ups]
        hashes = [[g.hash for g in u.fragments] for u in ups]
        ids = [u.file_id for u in ups]
        res = engine.download(b64, [len(f) for f in files], hashes, ids)
        for d, (st, body) in zip(files, res):
            assert st == 0 and body == d
        # failure modes, first failure in pipeline order
        b2 = [list(x) for x in b64]
        b2[0][1] = None                                   # missing
        b2[1][0] = b2[1][0][:-1] + b"*"                    # IllegalArgumentException
        h2 = [list(x) for x in hashes]
        h2[2][3] = "00" * 32                               # per-fragment mismatch
        i2 = list(ids)
        i2[3] = "11" * 32                                  # fileId mismatch
        res = engine.download(b2, [len(f) for f in files], h2, i2)
        assert [r[0] for r in res[:4]] == [dfs_amd.DFS_E_MISSING, dfs_amd.DFS_E_DECODE,
                                           dfs_amd.DFS_E_FRAG_MISMATCH, dfs_amd.DFS_E_CORRUPT]
        assert all(r[0] == 0 for r in res[4:])


def test_device_plan_and_synth_vs_oracle(engine):
    import torch
    nfiles, S, nfrag = 96, (1 << 16) + 5, 5
    spans = np.array([(f * S, S) for f in range(nfiles)], dtype=np.uint64)
    files = torch.empty(nfiles * S + 16, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(engine, files.data_ptr(), spans, 0, O.SYNTH_SEED)
    torch.cuda.synchronize()
    host = files.cpu().numpy()
    for f in (0, 1, 95):
        assert host[f * S:(f + 1) * S].tobytes() == O.c_synth(f, 0, S)
    plan = dfs_amd.UploadPlan(engine, spans, nfrag)
    fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
    frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
    b64 = torch.zeros(plan.b64_total, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    engine.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        for flags in (0, dfs_amd.DFS_SERIAL):
            fd.zero_(); frd.zero_(); b64.zero_()
            plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
            torch.cuda.synchronize()
            files_b = [host[f * S:(f + 1) * S].tobytes() for f in range(nfiles)]
            efd, efrd, eb64, eoff = O.c_upload_batch(files_b, nfrag, threads=8)
            assert (fd.cpu().numpy().reshape(nfiles, 32) == efd).all()
            assert (frd.cpu().numpy().reshape(nfiles, nfrag, 32) == efrd).all()
            assert b64.cpu().numpy().tobytes() == eb64
            assert (plan.b64_offsets() == eoff).all()
    finally:
        engine.set_stream(0)
        plan.close()


@pytest.mark.parametrize("mode", ["kernels", "fused"])
def test_align128_plan(monkeypatch, mode):
    """DFS_LAYOUT_ALIGN128: fragment Base64 starts on 128-byte boundaries,
    bytes identical to the oracle, gap bytes untouched, and the download path
    reads the fragments back through b64_spans."""
    import torch
    from dfs_amd.engine import download_device
    monkeypatch.setenv("DFS_UPLOAD_MODE", mode)
    eng = dfs_amd.FragmentEngine(0)
    nfiles, nfrag = 60, 5
    rng = random.Random(128)
    lens = [rng.choice([0, 1, 100, 4096, 70001, 123457]) for _ in range(nfiles)]
    offs_f = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    spans = np.stack([offs_f[:-1], np.array(lens, dtype=np.uint64)], axis=1)
    files = torch.empty(int(offs_f[-1]) + 64, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(eng, files.data_ptr(), spans, 900, O.SYNTH_SEED)
    plan = dfs_amd.UploadPlan(eng, spans, nfrag, align128=True)
    try:
        fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
        frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
        b64 = torch.full((plan.b64_total,), 0xAA, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
        torch.cuda.synchronize()
        bsp = plan.b64_spans(lens)
        assert (bsp[:, 0] % 128 == 0).all()
        host = files.cpu().numpy()
        blob = b64.cpu().numpy().tobytes()
        files_b = [host[int(o):int(o) + ln].tobytes() for o, ln in zip(offs_f[:-1], lens)]
        efd, efrd, _, _ = O.c_upload_batch(files_b, nfrag)
        assert (fd.cpu().numpy().reshape(nfiles, 32) == efd).all()
        assert (frd.cpu().numpy().reshape(nfiles, nfrag, 32) == efrd).all()
        covered = np.zeros(len(blob), dtype=bool)
        for f, d in enumerate(files_b):
            for i, (o, ln) in enumerate(O.c_split(len(d), nfrag)):
                so, sl = (int(x) for x in bsp[f * nfrag + i])
                assert blob[so:so + sl] == O.c_b64_encode(d[o:o + ln])
                covered[so:so + sl] = True
        gaps = np.frombuffer(blob, dtype=np.uint8)[~covered]
        assert (gaps == 0xAA).all()
        out = torch.zeros(int(offs_f[-1]) + 1, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        st = download_device(eng, b64.data_ptr(), bsp, nfiles, nfrag, np.array(lens, dtype=np.uint64),
                             frd.data_ptr(), fd.data_ptr(), out.data_ptr(), offs_f[:-1].copy())
        torch.cuda.synchronize()
        assert (st == 0).all()
        assert torch.equal(out[:int(offs_f[-1])], files[:int(offs_f[-1])])
    finally:
        plan.close()
        eng.close()


def test_frag_major_plan_and_device_download(engine):
    """The single-GPU half of bench.py's placement leg: a fragment-major
    upload plan, then dfs_download_batch on device pointers over the
    concatenated groups (what dfs_fetch_degraded hands back)."""
    import torch
    from dfs_amd import placement as P
    from dfs_amd.engine import download_device
    nfiles, S, nfrag = 40, 70001, 5
    spans = np.array([(f * S, S) for f in range(nfiles)], dtype=np.uint64)
    files = torch.empty(nfiles * S + 8, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(engine, files.data_ptr(), spans, 500, O.SYNTH_SEED)
    plan = dfs_amd.UploadPlan(engine, spans, nfrag, frag_major=True)
    fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
    frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
    b64 = torch.zeros(plan.b64_total, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
    torch.cuda.synchronize()
    offs = plan.b64_offsets()
    msp = P.frag_major_spans([S] * nfiles, nfrag)
    assert (msp[:, 0] == offs[:-1]).all()
    host = files.cpu().numpy()
    blob = b64.cpu().numpy().tobytes()
    for f in (0, 17, 39):
        d = host[f * S:(f + 1) * S].tobytes()
        for i, (o, ln) in enumerate(O.c_split(S, nfrag)):
            k = f * nfrag + i
            assert blob[int(msp[k, 0]):int(msp[k, 0] + msp[k, 1])] == O.c_b64_encode(d[o:o + ln])
    out = torch.zeros(nfiles * S, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    st = download_device(engine, b64.data_ptr(), msp, nfiles, nfrag, np.full(nfiles, S, np.uint64),
                         frd.data_ptr(), fd.data_ptr(), out.data_ptr(),
                         np.arange(nfiles, dtype=np.uint64) * np.uint64(S))
    assert (st == 0).all()
    assert torch.equal(out, files[:nfiles * S])
    plan.close()


def test_rccl_placement_single_rank(engine):
    """The RCCL path of the C-ABI placement on one GPU (world 1: every node on
    rank 0): comm init from a unique id, the size all-gather, ring and star
    placement, then the degraded fetch hands back the rank's own groups in
    source layout and dfs_download_batch rebuilds and verifies every file.
    Multi-rank schedules are checked on the CPU (tests/test_placement_plan.py,
    tests/test_dist.py); the driver's 8-GPU bench runs them over xGMI."""
    import torch
    from dfs_amd import placement as P
    from dfs_amd.engine import download_device
    nfiles, S, nfrag = 33, 40007, 5
    spans = np.array([(f * S, S) for f in range(nfiles)], dtype=np.uint64)
    files = torch.empty(nfiles * S + 8, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(engine, files.data_ptr(), spans, 900, O.SYNTH_SEED)
    plan = dfs_amd.UploadPlan(engine, spans, nfrag, frag_major=True)
    fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
    frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
    b64 = torch.zeros(plan.b64_total, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
    torch.cuda.synchronize()
    offs = plan.b64_offsets()
    grp = [int(offs[f]) for f in range(nfrag)] + [int(offs[-1])]  # group f starts with file 0's fragment f
    comm = P.Comm(engine, P.unique_id(), 1, 0)
    try:
        table = comm.sizes([grp[f + 1] - grp[f] for f in range(nfrag)])
        assert table.tolist() == [[grp[f + 1] - grp[f] for f in range(nfrag)]]
        lay = P.held_layout(1, 0, nfrag, table)
        held = {}
        for mode in ("ring", "star"):
            h = torch.zeros(int(lay[nfrag]), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
            comm.place(mode, table, b64.data_ptr(), h.data_ptr())
            torch.cuda.synchronize()
            held[mode] = h
        assert torch.equal(held["ring"], held["star"])
        assert torch.equal(held["star"], b64[:int(lay[nfrag])])  # one rank holds every group as uploaded
        back = torch.zeros_like(b64)
        st = comm.fetch(table, held["star"].data_ptr(), back.data_ptr())
        torch.cuda.synchronize()
        assert (st == 0).all() and torch.equal(back, b64)
        out = torch.zeros(nfiles * S, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        status = download_device(engine, back.data_ptr(), plan.b64_spans([S] * nfiles), nfiles, nfrag,
                                 np.full(nfiles, S, np.uint64), frd.data_ptr(), fd.data_ptr(), out.data_ptr(),
                                 np.arange(nfiles, dtype=np.uint64) * np.uint64(S))
        assert (status == 0).all() and torch.equal(out, files[:nfiles * S])
        # the only rank offline: every fragment is missing (SN:443-446)
        assert (comm.fetch(table, held["star"].data_ptr(), back.data_ptr(), offline=[0]) ==
                dfs_amd.DFS_E_MISSING).all()
    finally:
        comm.close()
        plan.close()


def test_comm_init_all_one_gpu(engine):
    """dfs_comm_init_all (one process, one communicator per GPU through
    ncclCommInitAll) with the one GPU present: the comm reports world 1 /
    rank 0, gathers sizes and places like one made from a unique id."""
    import ctypes
    import torch
    from dfs_amd import _lib as L
    from dfs_amd import placement as P
    (comm,) = P.Comm.init_all([engine])
    try:
        nr, rk = ctypes.c_uint32(9), ctypes.c_uint32(9)
        assert L.lib().dfs_comm_info(comm._c, ctypes.byref(nr), ctypes.byref(rk)) == 0 and (nr.value, rk.value) == (1, 0)
        sizes = [1000, 0, 77, 4096, 5]
        table = comm.sizes(sizes)
        assert table.tolist() == [sizes]
        src = torch.randint(0, 256, (sum(sizes),), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        lay = P.held_layout(1, 0, len(sizes), table)
        held = torch.zeros(int(lay[len(sizes)]), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        comm.place("ring", table, src.data_ptr(), held.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(held, src)
        assert comm.counters() == {"sends": 0, "recvs": 0, "copies": 4}  # the empty group is skipped
    finally:
        comm.close()


def test_sha256_update_streaming(engine, golden):
    """Chunked SHA-256 with carried state == one-shot digest (skew config's
    streaming path), for several chunkings, message lengths and alignments."""
    rng = np.random.default_rng(9)
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            for n in (0, 1, 63, 64, 65, 191, 192, 1000, 4096, 100003, 262144 + 7)]
    for chunk in (64, 192, 4096, 65536):
        state = np.zeros((len(msgs), 8), dtype=np.uint32)
        nparts = max((len(m) + chunk - 1) // chunk for m in msgs)
        digests = None
        for p in range(max(nparts, 1)):
            final = p == max(nparts, 1) - 1
            parts = []
            for m in msgs:
                l64 = len(m) - len(m) % 64  # non-final parts stop at a block boundary
                a = min(p * chunk, l64)
                b = len(m) if final else min((p + 1) * chunk, l64)
                parts.append(m[a:b])
            digests = engine.sha256_update(parts, state, begin=(p == 0), final=final,
                                           total_len=[len(m) for m in msgs])
        assert [d.hex() for d in digests] == [hashlib.sha256(m).hexdigest() for m in msgs], chunk
    # a non-final part that is not a multiple of 64 is rejected
    with pytest.raises(dfs_amd.DfsError):
        engine.sha256_update([b"x" * 65], np.zeros((1, 8), np.uint32), begin=True, final=False)
    # million-'a' KAT in 4 streamed parts
    kat = golden["sha256_kat"][3]
    st = np.zeros((1, 8), np.uint32)
    parts = [b"a" * 262144] * 3 + [b"a" * (1000000 - 3 * 262144)]
    for i, part in enumerate(parts):
        d = engine.sha256_update([part], st, begin=(i == 0), final=(i == 3), total_len=[1000000])
    assert d[0].hex() == kat["digest"]


def test_receive_fragments(engine, golden, example_bytes):
    """handleInternalStoreFragments: decode + hash each received fragment; the
    digests are what the sender compares with its own (SN:248-257)."""
    ex = golden["examples"][1]  # id.jpg
    data = example_bytes[ex["name"]]
    ups = engine.upload([data], 5)[0]
    texts = [g.b64 for g in ups.fragments] + [b"Zm9v=", b"", b"Zg"]
    got = engine.receive_fragments(texts)
    for g, f, (body, h) in zip(ups.fragments, ex["fragments"], got):
        assert h == f["sha256"] == g.hash
        assert body == data[f["offset"]:f["offset"] + f["length"]]
    assert got[5] == (None, None)
    assert got[6] == (b"", hashlib.sha256(b"").hexdigest())
    assert got[7] == (b"f", hashlib.sha256(b"f").hexdigest())


def test_profiling_timings(engine):
    engine.set_profiling(True)
    try:
        engine.upload([O.c_synth(3, 0, 1 << 20)] * 8, 5)
        t = engine.timings()
        assert t["sha"] is not None and t["sha"] > 0
        assert t["total"] is not None and t["total"] >= t["sha"] * 0.99
        if t["b64enc"] is not None:  # two-kernel upload (the fused mode has no separate encode)
            assert t["b64enc"] > 0
    finally:
        engine.set_profiling(False)


@pytest.mark.parametrize("handlers", ["threads", "serial"])
def test_storage_node_sim_config1(golden, tmp_path, handlers):
    """BASELINE config 1 replayed through the C++ host mirror: 5 nodes, upload
    examples/* at node 1, node 3 down, download at nodes 1, 2, 4, 5.  The
    fragment log lines must equal the golden ones and the fetch plans the
    reference's (SN:422-440); every node's data directory
    holds exactly its pair as raw .frag files (SN:143-145, 163-166, 284-285).
    threads (the default): one handler thread per request as in the reference
    (SN:28-31), the four uploads at once and then each node's four downloads
    at once, every handler through the request batcher (dfs_submit_upload /
    dfs_submit_reassemble); serial: one handler at a time through the per-call
    ABI.  Both print the same log."""
    import subprocess
    from conftest import EXAMPLES, PKG
    names = [e["name"] for e in golden["examples"]]
    exe = os.path.join(PKG, "host", "storage_node_sim")
    env = dict(os.environ, DFS_SIM_DATA=str(tmp_path / "data"))
    flag = ["--serial"] if handlers == "serial" else []
    r = subprocess.run([exe] + flag + [os.path.join(EXAMPLES, n) for n in names], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    if handlers == "threads":
        stats = [l for l in r.stdout.splitlines() if l.startswith("[sim] batcher: ")]
        assert len(stats) == 1 and stats[0].startswith("[sim] batcher: 20 requests in "), stats  # 4 uploads + 16 downloads
        env2 = dict(os.environ, DFS_SIM_DATA=str(tmp_path / "data_serial"))
        r2 = subprocess.run([exe, "--serial"] + [os.path.join(EXAMPLES, n) for n in names], capture_output=True,
                            text=True, timeout=120, env=env2)
        assert r2.returncode == 0
        assert [l for l in r.stdout.splitlines() if not l.startswith("[sim] batcher: ")] == r2.stdout.splitlines()
    lines = r.stdout.splitlines()
    frag_lines = [l for l in lines if l.startswith("[1] Fragment ")]
    assert frag_lines == [l for e in golden["examples"] for l in e["log_lines"]]
    ids = [l.split("= ")[1] for l in lines if l.startswith("[1] FileId = ")]
    assert ids == [e["fileId"] for e in golden["examples"]]
    plans = golden["download_plan_node3_down"]
    for me in (1, 2, 4, 5):
        for e in golden["examples"]:
            want = "[%d] Download %s fileId=%s plan=%s -> %d bytes OK" % (
                me, e["name"], e["fileId"], ",".join(plans[str(me)]), e["size"])
            assert want in lines, want
    assert "[1] Download with nodes 2,3 down -> 500 Could not retrieve fragment 2" in lines
    for e in golden["examples"]:
        data = open(os.path.join(EXAMPLES, e["name"]), "rb").read()
        spans = O.py_split(len(data), 5)
        for k in range(5):
            fdir = tmp_path / "data" / f"node-{k + 1}" / e["fileId"] / "fragments"
            held = sorted(os.listdir(fdir))
            assert held == sorted(f"{i}.frag" for i in O.py_node_fragments(k, 5))
            for i in O.py_node_fragments(k, 5):
                o, l = spans[i]
                assert (fdir / f"{i}.frag").read_bytes() == data[o:o + l]


def test_concurrent_handlers_share_one_ctx(engine):
    """StorageNode runs one thread per connection (SN:30) and the ABI promises
    that one ctx serialises its calls: 8 threads upload / download / receive
    through the same engine at once (ctypes drops the GIL), every result
    bit-exact against the oracle."""
    import threading
    errors = []

    def worker(k):
        try:
            rng = random.Random(100 + k)
            for it in range(6):
                files = [O.c_synth(1000 * k + it * 10 + j, 0, rng.randrange(0, 300_000)) for j in range(3)]
                ups = engine.upload(files, 5)
                fd, frd, b64, off = O.c_upload_batch(files, 5)
                for f, u in enumerate(ups):
                    assert u.file_id == fd[f].tobytes().hex()
                    for i, g in enumerate(u.fragments):
                        assert g.hash == frd[f, i].tobytes().hex()
                        assert g.b64 == b64[int(off[f * 5 + i]):int(off[f * 5 + i + 1])]
                res = engine.download([[g.b64 for g in u.fragments] for u in ups], [len(x) for x in files],
                                      [[g.hash for g in u.fragments] for u in ups], [u.file_id for u in ups])
                assert all(st == 0 and body == x for x, (st, body) in zip(files, res))
                bodies = [b for _, b in engine.store_bodies(files[:1], 5, k % 5, [ups[0].file_id])[0]]
                got = engine.store_receive(bodies)
                assert all(st == 0 and fid == ups[0].file_id for st, fid, _ in got)
        except Exception as e:  # reported below
            import traceback
            errors.append(traceback.format_exc())

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors[0]
    assert not any(t.is_alive() for t in threads)


def test_sha256_both_kernels_large_and_small_launches(engine):
    """Launches up to dfs::kChainMaxLanes lanes run the owner/helper latency
    kernels, larger ones the persistent throughput kernel: the same random
    messages (every alignment, lengths around the padding boundaries) through
    both, against hashlib."""
    rng = np.random.default_rng(77)
    n_big = 33000  # > kChainMaxLanes (32768)
    lens = rng.integers(0, 700, n_big)
    lens[:64] = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129] + list(range(191, 242))
    buf = rng.integers(0, 256, int(lens.sum()) + 8 * n_big, dtype=np.uint8)
    offs, o = [], 0
    for i, ln in enumerate(lens):
        o += i % 4  # every alignment
        offs.append(o)
        o += int(ln)
    spans = np.stack([np.array(offs, np.uint64), lens.astype(np.uint64)], axis=1)
    raw = buf.tobytes()
    want = [hashlib.sha256(raw[a:a + int(n)]).digest() for a, n in spans]
    big = engine.sha256_spans(buf, spans)
    assert all(big[i].tobytes() == want[i] for i in range(n_big))
    small = engine.sha256_spans(buf, spans[:5000])
    assert all(small[i].tobytes() == want[i] for i in range(5000))
    # Launches up to half of kChainMaxLanes take the pair-lane latency kernel
    # (two owner lanes per message, 32 messages per workgroup), the rest of the
    # range the one-lane kernel (64 per workgroup): one launch in the upper
    # range, and message counts around the workgroup sizes.
    mid = engine.sha256_spans(buf, spans[:20000])
    assert all(mid[i].tobytes() == want[i] for i in range(20000))
    for k in (1, 2, 31, 32, 33, 63, 64, 65, 16384, 16385):
        got = engine.sha256_spans(buf, spans[100:100 + k])
        assert all(got[i].tobytes() == want[100 + i] for i in range(k)), k


_ONE_LANE_CHILD = r"""
import hashlib, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "distributed-file-storage_amd"))
import dfs_amd
rng = np.random.default_rng(5)
n = 700
lens = rng.integers(0, 900, n)
lens[:13] = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129]
buf = rng.integers(0, 256, int(lens.sum()) + 4 * n, dtype=np.uint8)
offs, o = [], 0
for i, ln in enumerate(lens):
    o += i % 4
    offs.append(o)
    o += int(ln)
spans = np.stack([np.array(offs, np.uint64), lens.astype(np.uint64)], axis=1)
raw = buf.tobytes()
eng = dfs_amd.FragmentEngine(0)
for k in (1, 63, 64, 65, n):
    got = eng.sha256_spans(buf, spans[:k])
    assert all(got[i].tobytes() == hashlib.sha256(raw[a:a + int(m)]).digest() for i, (a, m) in enumerate(spans[:k])), k
up = eng.upload([raw[:100003]], 5)
assert up[0].file_id == hashlib.sha256(raw[:100003]).hexdigest()
eng.close()
print("one-lane ok")
"""


def test_sha256_one_lane_chain_kernel_forced():
    """DFS_SHA_CHAIN=1 (read once per process) sends small launches to the
    one-lane latency kernel, which otherwise only runs launches above half of
    dfs::kChainMaxLanes: the same checks against hashlib in a child process."""
    import subprocess
    import sys
    env = dict(os.environ, DFS_SHA_CHAIN="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ONE_LANE_CHILD, root], capture_output=True, text=True, env=env,
                       timeout=150)
    assert r.returncode == 0 and "one-lane ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("mode", ["overlap", "pipelined", "serial", "overlap-timeout"])
def test_download_overlapped_large_batch(engine, mode, monkeypatch):
    """A download above dfs::kChainMaxLanes SHA lanes.  6,000 files (36,000
    lanes): every file rebuilt and verified, plus the failure statuses on a
    few files — missing fragment (SN:443-446), invalid Base64 (SN:281), wrong
    fragment digest (SN:250-257), wrong fileId (SN:455-458), a Base64 char
    changed to another alphabet char (decodes, digest differs) — and their
    neighbours unaffected.  Default (overlap): fragment 0 of every file
    decoded first, then the other fragments in order beside one SHA launch
    whose lanes wait in-kernel for each fragment group;
    DFS_DOWNLOAD_MODE=pipelined: passes by fragment group (pass i decodes its
    group while the fileIds advance over group i - 1, their states in HBM
    between launches); DFS_DOWNLOAD_MODE=serial: the whole decode, then one
    SHA launch.  One unpadded fragment (valid for the JDK
    decoder) shifts every later Base64 offset off dword alignment.
    overlap-timeout: the same overlapped download with the in-kernel waits
    forced to time out from the host (DFS_SHA_WAIT_FORCE_TIMEOUT: the lanes
    wait for a count the decode never reaches and give up after 10 us; every
    kernel still exits), so the SHA launch is redone after the decode: the
    results must be the same and the redo counted."""
    if mode == "overlap-timeout":
        monkeypatch.setenv("DFS_SHA_WAIT_FORCE_TIMEOUT", "1")
        engine = dfs_amd.FragmentEngine(0)
    elif mode != "overlap":
        monkeypatch.setenv("DFS_DOWNLOAD_MODE", mode)
        engine = dfs_amd.FragmentEngine(0)
    import base64
    rng = np.random.default_rng(31)
    nfiles, nfrag = 6000, 5
    sizes = rng.integers(0, 20000, nfiles)
    sizes[:7] = [0, 1, 2, 4, 5, 6, 7]
    files = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in sizes]
    texts, frag_h, file_h = [], [], []
    for d in files:
        parts = [d[o:o + n] for o, n in O.c_split(len(d), nfrag)]
        texts.append([base64.b64encode(p) for p in parts])
        frag_h.append([hashlib.sha256(p).hexdigest() for p in parts])
        file_h.append(hashlib.sha256(d).hexdigest())
    want = [0] * nfiles
    texts[100][2] = None
    want[100] = dfs_amd.DFS_E_MISSING
    t = bytearray(texts[2000][1]); t[3] = ord("!"); texts[2000][1] = bytes(t)
    want[2000] = dfs_amd.DFS_E_DECODE
    frag_h[3000] = list(frag_h[3000]); frag_h[3000][4] = "0" * 64
    want[3000] = dfs_amd.DFS_E_FRAG_MISMATCH
    t = bytearray(texts[4000][3]); t[len(t) // 2] = ord("A") if t[len(t) // 2] != ord("A") else ord("B")
    texts[4000][3] = bytes(t)
    want[4000] = dfs_amd.DFS_E_FRAG_MISMATCH
    file_h[5999] = "f" * 64
    want[5999] = dfs_amd.DFS_E_CORRUPT
    f = next(f for f in range(7, nfiles) if texts[f][0].endswith(b"="))
    texts[f][0] = texts[f][0].rstrip(b"=")
    try:
        res = engine.download(texts, [len(d) for d in files], frag_h, file_h)
        if mode == "overlap-timeout":
            assert engine.stats()["ovl_redo"] == 1  # the forced timeout was seen and the launch redone once
        else:
            assert engine.stats()["ovl_redo"] == 0  # no decode-ahead wait timed out
    finally:
        if mode != "overlap":
            engine.close()
    for f, (st, body) in enumerate(res):
        assert st == want[f], (f, st, want[f])
        if want[f] == 0:
            assert body == files[f], f


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["overlap", "pipelined"])
def test_download_pipelined_many_fragments_small_files(engine, mode, monkeypatch):
    """The pipelined / overlapped download with nfrag = 12 and small files:
    fileId parts of 0 bytes in most passes (files under 64 B per fragment),
    parts ending on every 64-byte boundary case, empty files and fragments;
    fileId lanes whose wait points (each fragment's first block) coincide
    (several fragments start inside one block); 3,000 files x 13 lanes =
    39,000 (above dfs::kChainMaxLanes, so the large-batch paths)."""
    if mode != "overlap":
        monkeypatch.setenv("DFS_DOWNLOAD_MODE", mode)
        engine = dfs_amd.FragmentEngine(0)
    import base64
    rng = np.random.default_rng(77)
    nfiles, nfrag = 3000, 12
    sizes = rng.integers(0, 4000, nfiles)
    edge = [0, 1, 11, 12, 13, 63, 64, 65, 767, 768, 769, 64 * 12, 64 * 12 + 1, 64 * 13 - 1]
    sizes[:len(edge)] = edge
    files = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in sizes]
    texts, frag_h, file_h = [], [], []
    for d in files:
        parts = [d[o:o + n] for o, n in O.c_split(len(d), nfrag)]
        texts.append([base64.b64encode(p) for p in parts])
        frag_h.append([hashlib.sha256(p).hexdigest() for p in parts])
        file_h.append(hashlib.sha256(d).hexdigest())
    try:
        res = engine.download(texts, [len(d) for d in files], frag_h, file_h)
        if mode == "overlap-timeout":
            assert engine.stats()["ovl_redo"] == 1  # the forced timeout was seen and the launch redone once
        else:
            assert engine.stats()["ovl_redo"] == 0  # no decode-ahead wait timed out
    finally:
        if mode != "overlap":
            engine.close()
    for f, (st, body) in enumerate(res):
        assert st == 0, (f, st)
        assert body == files[f], f


@pytest.mark.parametrize("mode", ["overlap", "serial", "overlap-timeout"])
def test_reassemble_large_batch_overlap(engine, mode, monkeypatch):
    """dfs_reassemble_verify above dfs::kChainMaxLanes files (SN:419-458, raw
    fragments): default (overlap) gathers fragment 0 of every file first, then
    the other fragments beside one fileId SHA-256 launch whose lanes wait for
    each fragment group; serial: gather, then SHA.  Every file rebuilt and
    verified against hashlib, plus a corrupted fragment ("File corrupted",
    SN:455-458), a missing one (SN:443-446), empty and tiny files (fragments
    of 0 bytes, several fragments starting inside one block), and a batch
    whose fragment lengths are not the split's (a fetched fragment one byte
    longer: the serial path, still verified).  overlap-timeout: the in-kernel
    waits forced to time out from the host, the fileId launch redone."""
    if mode == "overlap-timeout":
        monkeypatch.setenv("DFS_SHA_WAIT_FORCE_TIMEOUT", "1")
        engine = dfs_amd.FragmentEngine(0)
    elif mode != "overlap":
        monkeypatch.setenv("DFS_DOWNLOAD_MODE", mode)
        engine = dfs_amd.FragmentEngine(0)
    try:
        rng = np.random.default_rng(91)
        nfiles, nfrag = 34000, 5
        sizes = rng.integers(0, 3000, nfiles)
        sizes[:6] = [0, 1, 4, 5, 63, 64 * 5 + 3]
        sizes[100] = sizes[200] = 1000
        blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
        files, o = [], 0
        for n in sizes:
            files.append(blob[o:o + int(n)])
            o += int(n)
        frags = [[d[a:a + n] for a, n in O.c_split(len(d), nfrag)] for d in files]
        ids = [hashlib.sha256(d).hexdigest() for d in files]
        want = [0] * nfiles
        frags[100][2] = bytes([frags[100][2][0] ^ 1]) + frags[100][2][1:]
        want[100] = dfs_amd.DFS_E_CORRUPT
        frags[200][3] = None
        want[200] = dfs_amd.DFS_E_MISSING
        res = engine.reassemble_verify(frags, ids)
        assert engine.stats()["ovl_redo"] == (1 if mode == "overlap-timeout" else 0)
        for f, (st, body, h) in enumerate(res):
            assert st == want[f], (f, st, want[f])
            if want[f] == 0:
                assert body == files[f] and h == ids[f], f
        frags2 = [list(x) for x in frags[:34000]]
        frags2[7][1] = frags2[7][1] + b"\x00"  # not the split's length: whole batch serial
        res2 = engine.reassemble_verify(frags2, ids)
        assert res2[7][0] == dfs_amd.DFS_E_CORRUPT and res2[8][0] == 0 and res2[8][1] == files[8]
    finally:
        if mode != "overlap":
            engine.close()


@pytest.mark.parametrize("mode", ["overlap", "serial"])
def test_device_download_verdicts(engine, mode, monkeypatch):
    """dfs_download_batch on device buffers with the expected digests in HBM:
    the per-file verdict is computed on the device (verdict_kernel) — a Base64
    char outside the alphabet (SN:281 -> DFS_E_DECODE), a wrong expected
    fragment digest (SN:250-257 -> DFS_E_FRAG_MISMATCH), a wrong fileId
    (SN:454-458 -> DFS_E_CORRUPT), a fragment no holder had (SN:443-446 ->
    DFS_E_MISSING) — and every other file rebuilt bit-exact.  6,000 files x 6
    lanes: above kChainMaxLanes, so the overlap (default) or serial path."""
    import torch
    from dfs_amd import placement as P
    from dfs_amd.engine import download_device
    if mode != "overlap":
        monkeypatch.setenv("DFS_DOWNLOAD_MODE", mode)
        engine = dfs_amd.FragmentEngine(0)
    try:
        nfiles, S, nfrag = 6000, 3001, 5
        spans = np.array([(f * S, S) for f in range(nfiles)], dtype=np.uint64)
        files = torch.empty(nfiles * S + 8, dtype=torch.uint8, device="cuda")
        dfs_amd.synth_fill(engine, files.data_ptr(), spans, 77, O.SYNTH_SEED)
        plan = dfs_amd.UploadPlan(engine, spans, nfrag, frag_major=True)
        fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
        frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
        b64 = torch.zeros(plan.b64_total, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
        torch.cuda.synchronize()
        msp = P.frag_major_spans([S] * nfiles, nfrag).copy()
        want = np.zeros(nfiles, dtype=np.int32)
        k = 7 * nfrag + 3
        b64[int(msp[k, 0]) + 5] = ord("!")
        want[7] = dfs_amd.DFS_E_DECODE
        frd[(3 * nfrag + 2) * 32] ^= 1
        want[3] = dfs_amd.DFS_E_FRAG_MISMATCH
        fd[5 * 32 + 31] ^= 0x80
        want[5] = dfs_amd.DFS_E_CORRUPT
        msp[9 * nfrag + 4, 1] = np.uint64(dfs_amd.DFS_SPAN_MISSING)
        want[9] = dfs_amd.DFS_E_MISSING
        out = torch.zeros(nfiles * S, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        st = download_device(engine, b64.data_ptr(), msp, nfiles, nfrag, np.full(nfiles, S, np.uint64),
                             frd.data_ptr(), fd.data_ptr(), out.data_ptr(),
                             np.arange(nfiles, dtype=np.uint64) * np.uint64(S))
        assert engine.stats()["ovl_redo"] == 0
        assert st.tolist() == want.tolist()
        good = np.nonzero(want == 0)[0]
        o, f0 = out.view(nfiles, S), files[:nfiles * S].view(nfiles, S)
        assert torch.equal(o[torch.as_tensor(good)], f0[torch.as_tensor(good)])
        # the same download through a prepared plan (tables built once, in HBM),
        # run three times: same verdicts and bytes every time; then with the
        # corruptions repaired it is clean
        flen, foff = np.full(nfiles, S, np.uint64), np.arange(nfiles, dtype=np.uint64) * np.uint64(S)
        dplan = dfs_amd.DownloadPlan(engine, msp, nfiles, nfrag, flen, foff)
        for rep in range(3):
            out.zero_()
            torch.cuda.synchronize()
            st = dplan.run(b64.data_ptr(), frd.data_ptr(), fd.data_ptr(), out.data_ptr())
            assert st.tolist() == want.tolist(), rep
            assert torch.equal(out.view(nfiles, S)[torch.as_tensor(good)], f0[torch.as_tensor(good)]), rep
        b64[int(msp[k, 0]) + 5] = ord("A")  # a valid char, but not the encoder's: the fragment digest differs
        torch.cuda.synchronize()
        st = dplan.run(b64.data_ptr(), frd.data_ptr(), fd.data_ptr(), out.data_ptr())
        want2 = want.copy()
        want2[7] = dfs_amd.DFS_E_FRAG_MISMATCH
        assert st.tolist() == want2.tolist()
        assert dplan.run(b64.data_ptr(), 0, 0, out.data_ptr()).tolist() == \
            [dfs_amd.DFS_E_MISSING if f == 9 else 0 for f in range(nfiles)]  # nothing to compare with
        # an output that is not 16-byte aligned is not what the plan was tiled for
        import ctypes as C
        rc = dfs_amd.lib().dfs_download_plan_run(engine.ctx, dplan._plan, C.c_void_p(b64.data_ptr()), None, None,
                                                 C.c_void_p(out.data_ptr() + 4), np.zeros(nfiles, np.int32).ctypes.data)
        assert rc == dfs_amd.DFS_E_ARG
        dplan.close()
        assert engine.stats()["ovl_redo"] == 0
        plan.close()
    finally:
        if mode != "overlap":
            engine.close()
