"""Multi-rank placement (gloo on CPU, world 2, 4 and 8; 8 ranks x 5 nodes is
the bench's 8-GPU replication leg, GPUs 5-7 hosting no node).

Checks that the replication exchange leaves every rank holding exactly the
fragments of the nodes it hosts (node k stores {k, k+1}, SN:143-145,
196-205), bit-exact, and that a degraded read with one rank offline fetches
every fragment from the surviving holder (SN:422-446).  The Base64 payloads
come from the CPU oracle; the exchange code is the same module bench.py runs
over RCCL on GPUs.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_files(rank, nfiles):
    import oracle as O
    sizes = [(1000 + 37 * (rank * nfiles + i)) % 3000 + i for i in range(nfiles)]
    return [O.c_synth(rank * 1000 + i, 0, s) for i, s in enumerate(sizes)]


def _frag_major(files, nfrag):
    """Fragment-major Base64 buffer + group offsets (what a frag_major plan writes)."""
    import oracle as O
    groups = []
    for f in range(nfrag):
        parts = []
        for d in files:
            o, ln = O.c_split(len(d), nfrag)[f]
            parts.append(O.c_b64_encode(d[o:o + ln]))
        groups.append(b"".join(parts))
    off = np.cumsum([0] + [len(g) for g in groups]).tolist()
    return b"".join(groups), off, groups


def _worker(rank, world, port, nfrag, nfiles, offline, q):
    try:
        sys.path[:0] = [os.path.join(ROOT, "distributed-file-storage_amd"), os.path.join(ROOT, "oracle")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dfs_amd import placement as P
        files = _rank_files(rank, nfiles)
        blob, off, _ = _frag_major(files, nfrag)
        t = torch.frombuffer(bytearray(blob or b"\0"), dtype=torch.uint8)[:len(blob)]
        held, table = P.exchange_upload(t, off, nfrag)
        # expected: group f of every rank in rank order, for my fragments
        want = P.gpu_fragments(rank, nfrag, world)
        assert sorted(held) == want, (sorted(held), want)
        for f in want:
            exp = b"".join(_frag_major(_rank_files(r, nfiles), nfrag)[2][f] for r in range(world))
            got = held[f][0].numpy().tobytes()
            assert got == exp, (rank, f)
            assert held[f][1] == [table[r][f] for r in range(world)]
        # the star fan-out as one all-to-all yields the same holdings
        star, table2 = P.exchange_upload_star(t, off, nfrag)
        assert table2 == table and sorted(star) == want
        for f in want:
            assert torch.equal(star[f][0], held[f][0]) and star[f][1] == held[f][1], (rank, f)
        # degraded read: my own fragments back from the holders
        got = P.exchange_download(held, table, nfrag, offline=offline)
        if rank not in offline:
            mine = _frag_major(files, nfrag)[2]
            for f in range(nfrag):
                assert got[f] is not None and got[f].numpy().tobytes() == mine[f], (rank, f)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,nfrag,offline", [(2, 5, ()), (2, 5, (1,)), (4, 4, ()), (4, 4, (2,)), (4, 8, (0,)),
                                                       (4, 3, (3,)), (8, 5, (7,))])
def test_placement_exchange(world, nfrag, offline):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nfrag, 7, offline, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] == "ok", res[r]


def test_pure_maps():
    sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))
    from dfs_amd import placement as P
    import oracle as O
    # W == N: GPU g holds {g, g+1}; fetch plan with node 3 down == SURVEY §3.2 table
    for n in (5, 8):
        for g in range(n):
            assert P.gpu_fragments(g, n, n) == sorted({g, (g + 1) % n})
    table = {1: ["local", "local", "node2", "node4", "node5"], 2: ["node1", "local", "local", "node4", "node5"],
             4: ["node1", "node2", "node2", "local", "local"], 5: ["local", "node2", "node2", "node4", "local"]}
    for me1, row in table.items():
        src = P.download_sources(5, 5, me1 - 1, offline=[2])
        got = ["local" if s == me1 - 1 else "node%d" % (s + 1) for s in src]
        assert got == row
        assert got == O.py_download_plan(me1, 5, O.py_node_fragments(me1 - 1, 5), down=[3])
    # two adjacent GPUs down: fragment between them is lost
    assert P.download_sources(5, 5, 0, offline=[2, 3])[3] is None


def test_file_owner_digest_prefix():
    """Owner of a fileId = first 8 digest bytes (big-endian) mod world, the
    same from raw digests (device-side path) and from the hex string."""
    import hashlib
    import torch
    from dfs_amd.placement import file_owner, file_owner_hex
    ids = [hashlib.sha256(bytes([i]) * i).digest() for i in range(200)] + [b"\xff" * 32, b"\x00" * 32]
    dig = torch.tensor([list(x) for x in ids], dtype=torch.uint8)
    for world in (1, 2, 3, 5, 8):
        got = file_owner(dig, world).tolist()
        want = [int.from_bytes(x[:8], "big") % world for x in ids]
        assert got == want == [file_owner_hex(x.hex(), world) for x in ids]
