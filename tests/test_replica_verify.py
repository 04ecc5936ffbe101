"""dfs_replica_verify on the GPU (one-rank communicator: every node on rank 0,
so the held buffer is the upload's own Base64): the holders' decode + SHA-256
of every held fragment (SN:281-282) and the comparison with the uploader's
digests (SN:248-257), through the C ABI, against the oracle."""
import hashlib

import numpy as np
import pytest

import dfs_amd
import oracle as O
from dfs_amd import _lib as L
from dfs_amd import placement as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    with dfs_amd.FragmentEngine(0) as e:
        yield e


def _run(engine, lens, nfrag, align128, seed):
    import torch
    dev = torch.device("cuda", 0)
    nfiles = len(lens)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    spans = np.stack([offs, np.array(lens, dtype=np.uint64)], axis=1)
    total = int(sum(lens))
    files = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    dfs_amd.synth_fill(engine, files.data_ptr(), spans, seed, O.SYNTH_SEED)
    plan = dfs_amd.UploadPlan(engine, spans, nfrag, frag_major=True, align128=align128)
    fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device=dev)
    frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device=dev)
    b64 = torch.zeros(max(plan.b64_total, 1), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), 0)
    torch.cuda.synchronize()
    comm = P.Comm(engine, P.unique_id(), 1, 0)
    rp = P.ReplicaPlan(comm, nfrag, lens, align128)
    return dict(torch=torch, dev=dev, files=files, plan=plan, frd=frd, b64=b64, comm=comm, rp=rp, nfiles=nfiles,
                host=files.cpu().numpy(), offs=offs)


# how the holders' check runs: "two" = decode kernel, then SHA lanes over the decoded bytes; "slices" = that in
# three slices (DFS_REPLICA_SLICES), slice i hashed while slice i + 1 is decoded on the second stream; "fused" =
# one pass, every lane decodes, stores and hashes its own fragment (the default from 128-byte fragments up)
@pytest.mark.parametrize("how", ["two", "slices", "fused"])
@pytest.mark.parametrize("align128", [False, True])
@pytest.mark.parametrize("shape", ["ragged", "uniform-large"])
def test_replica_verify_single_rank(engine, align128, shape, how, monkeypatch):
    slices = 3 if how == "slices" else 0
    monkeypatch.setenv("DFS_REPLICA_FUSED", "1" if how == "fused" else "0")
    if slices:
        monkeypatch.setenv("DFS_REPLICA_SLICES", str(slices))
    rng = np.random.default_rng(5 + align128)
    nfrag = 5 if shape == "ragged" else 8
    if shape == "ragged":
        lens = [int(x) for x in rng.choice([0, 1, 4, 5, 63, 320, 4097, 20000, 65537], 300)]
    else:
        lens = [4096] * 9000  # 72,000 held fragments: the persistent SHA kernel
    c = _run(engine, lens, nfrag, align128, 4200)
    torch, dev, rp, comm = c["torch"], c["dev"], c["rp"], c["comm"]
    try:
        offs = c["plan"].b64_offsets()
        grp = [int(offs[f]) for f in range(nfrag)] + [int(offs[-1])]
        assert rp.table.tolist() == [[grp[f + 1] - grp[f] for f in range(nfrag)]]
        assert rp.table.tolist() == comm.sizes([grp[f + 1] - grp[f] for f in range(nfrag)]).tolist()
        assert rp.nheld == len(lens) * nfrag and rp.held_bytes == grp[-1]
        held = torch.zeros(max(rp.held_bytes, 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        comm.place("star", rp.table, c["b64"].data_ptr(), held.data_ptr())
        raw = torch.zeros(rp.raw_bytes + 16, dtype=torch.uint8, device=dev)
        verdict = torch.full((rp.nheld,), 99, dtype=torch.int32, device=dev)
        failed = torch.full((1,), 99, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
        assert rp.one_pass == (how == "fused")
        print(f"replica verify {shape} align128={align128} {how}: {rp.nheld} held fragments", flush=True)
        rp.verify(c["frd"].data_ptr(), held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
        torch.cuda.synchronize()
        assert int(failed[0]) == 0 and bool((verdict == 0).all())
        frags = rp.frags()
        rawh = raw.cpu().numpy()
        for k in list(range(0, rp.nheld, max(1, rp.nheld // 97))) + [rp.nheld - 1]:
            x = frags[k]
            fo = int(c["offs"][int(x["file"])])
            o, n = O.c_split(lens[int(x["file"])], nfrag)[int(x["frag"])]
            assert int(x["raw_len"]) == n
            assert rawh[int(x["raw_off"]):int(x["raw_off"]) + n].tobytes() == c["host"][fo + o:fo + o + n].tobytes(), k
        # one held byte changed to another alphabet char: that fragment's digest differs (SN:250-257)
        big = [k for k in range(rp.nheld) if int(frags[k]["b64_len"]) >= 8]
        k1, k2 = big[len(big) // 3], big[2 * len(big) // 3]
        p1 = int(frags[k1]["b64_off"]) + 5
        old = int(held[p1])
        held[p1] = ord("B") if old == ord("A") else ord("A")
        torch.cuda.synchronize()
        rp.verify(c["frd"].data_ptr(), held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
        torch.cuda.synchronize()
        v = verdict.cpu().numpy()
        assert np.nonzero(v)[0].tolist() == [k1] and v[k1] == L.DFS_E_FRAG_MISMATCH and int(failed[0]) == 1
        # and one byte outside the alphabet in another fragment: the decoder's IllegalArgumentException (SN:281)
        held[int(frags[k2]["b64_off"]) + 2] = ord("!")
        torch.cuda.synchronize()
        rp.verify(c["frd"].data_ptr(), held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
        torch.cuda.synchronize()
        v = verdict.cpu().numpy()
        assert sorted(np.nonzero(v)[0].tolist()) == sorted([k1, k2])
        assert v[k1] == L.DFS_E_FRAG_MISMATCH and v[k2] == L.DFS_E_DECODE and int(failed[0]) == 2
        # a wrong sender digest is a mismatch too; verdict may be NULL (counts only)
        held[p1] = old
        held[int(frags[k2]["b64_off"]) + 2] = ord("A")
        frd2 = c["frd"].clone()
        frd2[32 * 7 + 3] ^= 1  # file 1, fragment 2 of [file][fragment] (nfrag >= 5)
        torch.cuda.synchronize()
        rp.verify(frd2.data_ptr(), held.data_ptr(), raw.data_ptr(), 0, failed.data_ptr())
        torch.cuda.synchronize()
        assert int(failed[0]) >= 1
    finally:
        rp.close()
        comm.close()
        c["plan"].close()


def test_replica_verify_digest_is_the_oracles(engine):
    """The digests compared are the oracle's: SHA-256(decode(encode(fragment)))
    == SHA-256(fragment) per held fragment (the reference's own invariant)."""
    lens = [28, 9506, 2154, 467]  # the reference's examples' sizes
    c = _run(engine, lens, 5, False, 77)
    try:
        frd = c["frd"].cpu().numpy().reshape(len(lens), 5, 32)
        for f, n in enumerate(lens):
            d = c["host"][int(c["offs"][f]):int(c["offs"][f]) + n].tobytes()
            for i, (o, ln) in enumerate(O.c_split(n, 5)):
                assert frd[f, i].tobytes() == hashlib.sha256(d[o:o + ln]).digest()
    finally:
        c["rp"].close()
        c["comm"].close()
        c["plan"].close()


@pytest.mark.parametrize("align128", [False, True])
def test_fused_check_every_length_and_final_unit_rule(engine, align128, monkeypatch):
    """The one-pass check (a lane decodes, stores and hashes its fragment) on
    fragments of every length 0..450 and a few long ones: block boundaries at
    every phase of the 3-byte unit, tails of every size, final units "xxxx",
    "xxx=" and "xx==".  Decoded bytes, digests and verdicts against the oracle;
    then damaged replicas: a char outside the alphabet in the first block, in
    the last whole block and in the final unit, padding where a char belongs and
    a char where padding belongs (java.util.Base64's IllegalArgumentException,
    SN:281, or a decoded length / digest that differs, SN:250-257) - each with
    the verdict the two-kernel check gives for the same bytes."""
    nfrag = 5
    lens = [nfrag * n + r for n in range(0, 451, 3) for r in (0, 2)] + [nfrag * n for n in (1000, 4096, 4097, 65536 + 7)]
    monkeypatch.setenv("DFS_REPLICA_FUSED", "1")
    c = _run(engine, lens, nfrag, align128, 9100)
    monkeypatch.setenv("DFS_REPLICA_FUSED", "0")
    rp2 = P.ReplicaPlan(c["comm"], nfrag, lens, align128)
    torch, dev, rp, comm = c["torch"], c["dev"], c["rp"], c["comm"]
    assert rp.one_pass and not rp2.one_pass
    try:
        held = torch.zeros(max(rp.held_bytes, 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        comm.place("star", rp.table, c["b64"].data_ptr(), held.data_ptr())
        torch.cuda.synchronize()
        frags = rp.frags()

        def run(plan):
            raw = torch.full((plan.raw_bytes + 16,), 0xEE, dtype=torch.uint8, device=dev)
            verdict = torch.full((plan.nheld,), 99, dtype=torch.int32, device=dev)
            failed = torch.full((1,), 99, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            plan.verify(c["frd"].data_ptr(), held.data_ptr(), raw.data_ptr(), verdict.data_ptr(), failed.data_ptr())
            torch.cuda.synchronize()
            return raw.cpu().numpy(), verdict.cpu().numpy(), int(failed[0])

        raw, v, failed = run(rp)
        assert failed == 0 and not v.any()
        for k, x in enumerate(frags):  # every decoded fragment, byte for byte (SN:281)
            fo = int(c["offs"][int(x["file"])])
            o, n = O.c_split(lens[int(x["file"])], nfrag)[int(x["frag"])]
            a = int(x["raw_off"])
            assert raw[a:a + n].tobytes() == c["host"][fo + o:fo + o + n].tobytes(), (k, n)
            assert (raw[a + n:a + ((n + 15) & ~15)] == 0xEE).all(), (k, n)  # nothing written past the fragment
        # damaged replicas: same verdicts from both checks
        by_len = {}
        for k, x in enumerate(frags):
            by_len.setdefault(int(x["raw_len"]), k)
        edits = []
        for n, k in sorted(by_len.items()):
            if n < 6:
                continue
            b0, bl = int(frags[k]["b64_off"]), int(frags[k]["b64_len"])
            where = {0: 1, 1: bl - 6 if bl >= 12 else 2, 2: bl - 3, 3: bl - 1, 4: bl - 2}[len(edits) % 5]
            newc = ord("=") if len(edits) % 5 == 3 else ord("!") if len(edits) % 5 < 3 else ord("A")
            edits.append((b0 + where, newc))
        for pos, ch in edits:
            held[pos] = ch
        torch.cuda.synchronize()
        _, v1, f1 = run(rp)
        _, v2, f2 = run(rp2)
        assert f1 == f2 and f1 > 0 and v1.tolist() == v2.tolist()
        assert set(np.unique(v1).tolist()) <= {0, L.DFS_E_DECODE, L.DFS_E_FRAG_MISMATCH} and L.DFS_E_DECODE in v1
    finally:
        rp2.close()
        c["rp"].close()
        comm.close()
        c["plan"].close()
