"""The library's own placement runner under a simulated RCCL, and the replica
receiver's layout (CPU only).

dfs_place_simulate drives placement.cpp's run_plans — the code that issues
ncclSend / ncclRecv on GPUs — for every rank at once, with an in-process
transport that pairs rank a's sends to b with b's receives from a in posting
order per group, and rejects unequal counts or sizes (what would hang or
corrupt over RCCL).  dfs_replica_layout says where every held fragment's
Base64 lies after a placement and where its digest lands in the digest table
exchange of dfs_replica_verify (SN:248-257, 265-293): both are checked against
buffers built from the oracle's split / Base64 / SHA-256."""
import hashlib

import numpy as np
import pytest

import oracle as O
from dfs_amd import _lib as L
from dfs_amd import placement as P
from test_placement_plan import _groups


@pytest.fixture(params=[False, True], ids=["copies", "loopback"])
def loopback(request, monkeypatch):
    """With DFS_COMM_LOOPBACK=1 the runner posts a rank's local copies as a
    send to itself paired with a receive from itself inside the phase's group
    (what a one-rank RCCL run uses to drive ncclSend / ncclRecv); the simulated
    transport then also checks that no such pair reads bytes the same group
    writes."""
    if request.param:
        monkeypatch.setenv("DFS_COMM_LOOPBACK", "1")
    else:
        monkeypatch.delenv("DFS_COMM_LOOPBACK", raising=False)
    return request.param


@pytest.mark.parametrize("world,nfrag", [(2, 5), (2, 8), (4, 4), (4, 8), (8, 8), (8, 5), (3, 8), (5, 5), (1, 5)])
@pytest.mark.parametrize("mode", ["ring", "star"])
def test_native_runner_places_like_the_reference(world, nfrag, mode, loopback):
    rng = np.random.default_rng(world * 131 + nfrag)
    table, src = _groups(world, nfrag, rng)
    blobs = [b"".join(g) for g in src]
    held, st = P.simulate_native(world, nfrag, table, mode, blobs)
    assert (st == 0).all()
    assert held == P.simulate(world, nfrag, table, mode, blobs)  # the Python model of the same plans
    for r in range(world):
        lay = P.held_layout(world, r, nfrag, table)
        for f in P.gpu_fragments(r, nfrag, world):  # node k stores {k, k+1}, SN:143-145
            exp = b"".join(src[q][f] for q in range(world))
            assert held[r][int(lay[f]):int(lay[f]) + len(exp)] == exp, (r, f)


@pytest.mark.parametrize("world,nfrag", [(2, 5), (4, 4), (4, 8), (8, 8), (8, 5), (5, 5)])
def test_native_runner_degraded_fetch(world, nfrag, loopback):
    rng = np.random.default_rng(world + 11 * nfrag)
    table, src = _groups(world, nfrag, rng)
    held, _ = P.simulate_native(world, nfrag, table, "star", [b"".join(g) for g in src])
    for off in [()] + [(g,) for g in range(world)] + ([(0, 1)] if world > 2 else []):
        out, st = P.simulate_native(world, nfrag, table, "fetch", held, offline=off)
        for q in range(world):
            srcs = P.download_sources(nfrag, world, q, off)
            _, dst_off, _ = P.plan(world, q, nfrag, table, "fetch", off)
            for f in range(nfrag):
                if q in off or srcs[f] is None:
                    assert st[q, f] == L.DFS_E_MISSING  # "Could not retrieve fragment i", SN:443-446
                    continue
                assert st[q, f] == 0
                o = int(dst_off[f])
                assert out[q][o:o + len(src[q][f])] == src[q][f], (off, q, f)


def _frag_major_b64(files, nfrag, align):
    """A rank's fragment-major Base64 buffer as an upload plan lays it out:
    [fragment][file], every fragment start rounded up to `align`."""
    buf = bytearray()
    starts = []
    for f in range(nfrag):
        for j, d in enumerate(files):
            buf += b"\0" * (-len(buf) % align)
            if j == 0:
                starts.append(len(buf))
            o, n = O.c_split(len(d), nfrag)[f]
            buf += O.c_b64_encode(d[o:o + n])
        if not files:
            starts.append(len(buf))
    return bytes(buf), starts + [len(buf)]


@pytest.mark.parametrize("world,nfrag", [(1, 5), (2, 5), (2, 8), (3, 8), (4, 4), (8, 8), (8, 5)])
@pytest.mark.parametrize("align128", [False, True])
def test_replica_layout_and_digest_exchange(world, nfrag, align128):
    rng = np.random.default_rng(world * 17 + nfrag + (1000 if align128 else 0))
    counts = [int(rng.integers(0, 6)) for _ in range(world)]
    counts[0] = max(counts[0], 2)
    files = [[O.c_synth(100 * r + j, 0, int(rng.choice([0, 1, 3, nfrag - 1, nfrag, 64 * nfrag, 777, 2048, 5000])))
              for j in range(counts[r])] for r in range(world)]
    lens = [[len(d) for d in fs] for fs in files]
    align = 128 if align128 else 1
    blobs, tables = [], []
    for r in range(world):
        b, st = _frag_major_b64(files[r], nfrag, align)
        blobs.append(b)
        tables.append([st[f + 1] - st[f] for f in range(nfrag)])
    # digest tables: [fragment][file] x 32 bytes (what dfs_replica_verify sends)
    digs = [b"".join(hashlib.sha256(d[o:o + n]).digest() for f in range(nfrag) for d in files[r]
                     for o, n in [O.c_split(len(d), nfrag)[f]]) for r in range(world)]
    dig_table = np.array([[32 * counts[r]] * nfrag for r in range(world)], dtype=np.uint64)
    first = None
    for me in range(world):
        frags, table, held_bytes, raw_bytes = P.replica_layout(world, me, nfrag, lens, align128)
        assert table.tolist() == tables  # == the group sizes dfs_place_sizes would gather
        if first is None:
            held, _ = P.simulate_native(world, nfrag, table, "star", blobs)
            exp_dig, _ = P.simulate_native(world, nfrag, dig_table, "star", digs)
            first = True
        assert held_bytes == len(held[me])
        assert len(exp_dig[me]) == 32 * len(frags)
        raw_end = 0
        want_order = [(f, r, j) for f in P.gpu_fragments(me, nfrag, world) for r in range(world) for j in range(counts[r])]
        assert [(int(x["frag"]), int(x["rank"]), int(x["file"])) for x in frags] == want_order
        for k, x in enumerate(frags):
            d = files[int(x["rank"])][int(x["file"])]
            o, n = O.c_split(len(d), nfrag)[int(x["frag"])]
            part = d[o:o + n]
            a, ln = int(x["b64_off"]), int(x["b64_len"])
            assert held[me][a:a + ln] == O.c_b64_encode(part), (me, k)            # SN:636 bytes, where they landed
            assert int(x["raw_len"]) == n and int(x["raw_off"]) % 16 == 0 and int(x["raw_off"]) >= raw_end
            raw_end = int(x["raw_off"]) + n
            assert exp_dig[me][32 * k:32 * k + 32] == hashlib.sha256(part).digest(), (me, k)  # SN:159 == SN:282
        assert raw_bytes >= raw_end


def test_replica_layout_bad_arguments():
    import ctypes
    n = ctypes.c_uint64(0)
    nf = np.array([1, 1], dtype=np.uint32)
    ln = np.array([10, 10], dtype=np.uint64)
    lib = L.lib()
    assert lib.dfs_replica_layout(0, 0, 5, nf.ctypes.data, ln.ctypes.data, 0, None, ctypes.byref(n), None, None, None) == L.DFS_E_ARG
    assert lib.dfs_replica_layout(2, 2, 5, nf.ctypes.data, ln.ctypes.data, 0, None, ctypes.byref(n), None, None, None) == L.DFS_E_ARG
    assert lib.dfs_replica_layout(2, 0, 5, nf.ctypes.data, None, 0, None, ctypes.byref(n), None, None, None) == L.DFS_E_ARG
    assert lib.dfs_replica_layout(2, 0, 5, nf.ctypes.data, ln.ctypes.data, 0x8, None, ctypes.byref(n), None, None, None) == L.DFS_E_ARG
    assert lib.dfs_replica_layout(2, 0, 5, nf.ctypes.data, ln.ctypes.data, 0, None, ctypes.byref(n), None, None, None) == L.DFS_OK
    assert n.value == 10  # rank 0 of 2 hosts nodes 0, 2, 4 = all five fragments, of one file per rank
