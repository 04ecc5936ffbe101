"""The RCCL placement schedules (dfs_place_plan, csrc/placement.cpp) checked on
the CPU by simulating every rank in one process: ring and star uploads leave
every rank holding exactly the fragments of the nodes it hosts (node k stores
{k, k+1}, SN:143-145, 195-224), and the degraded fetch returns every live
rank's own groups from the first live holder in SN:427-428 order, or
"Could not retrieve fragment i" (SN:443-446)."""
import itertools

import numpy as np
import pytest

from dfs_amd import _lib as L
from dfs_amd import placement as P


def _groups(world, nfrag, rng, zero_frac=0.2):
    table = rng.integers(0, 400, (world, nfrag)).astype(np.uint64)
    table[rng.random((world, nfrag)) < zero_frac] = 0
    src = [[rng.integers(0, 256, int(table[r, f]), dtype=np.uint8).tobytes() for f in range(nfrag)]
           for r in range(world)]
    return table, src


CASES = [(w, n) for w in (1, 2, 3, 4, 5, 8) for n in (2, 3, 4, 5, 8)] + [(8, 10), (16, 8), (7, 5)]


@pytest.mark.parametrize("world,nfrag", CASES)
@pytest.mark.parametrize("mode", ["ring", "star"])
def test_upload_placement_holdings(world, nfrag, mode):
    rng = np.random.default_rng(world * 100 + nfrag)
    table, src = _groups(world, nfrag, rng)
    held = P.simulate(world, nfrag, table, mode, [b"".join(g) for g in src])
    for r in range(world):
        lay = P.held_layout(world, r, nfrag, table)
        want = P.gpu_fragments(r, nfrag, world)
        assert [f for f in range(nfrag) if lay[f] != np.uint64(2**64 - 1)] == want
        for f in want:
            exp = b"".join(src[q][f] for q in range(world))
            o = int(lay[f])
            assert held[r][o:o + len(exp)] == exp, (r, f)
        assert len(held[r]) == sum(int(table[:, f].sum()) for f in want)


@pytest.mark.parametrize("world,nfrag", [(2, 5), (4, 4), (4, 8), (5, 5), (8, 8), (8, 5), (3, 8)])
def test_ring_and_star_traffic(world, nfrag):
    """W == N: the ring's replica step uses one link per rank (every rank
    forwards to rank g-1 only); the star sends each group straight to both
    holders.  Both move the same held bytes."""
    rng = np.random.default_rng(3)
    table, _ = _groups(world, nfrag, rng, zero_frac=0.0)
    for r in range(world):
        ops, _, _ = P.plan(world, r, nfrag, table, "ring")
        fwd = ops[(ops["phase"] == 1) & (ops["kind"] == L.DFS_XFER_SEND)]
        if world == nfrag:
            assert set(fwd["peer"].tolist()) <= {(r - 1) % world}
        sops, _, _ = P.plan(world, r, nfrag, table, "star")
        assert (sops["phase"] == 0).all()


@pytest.mark.parametrize("world,nfrag", [(2, 5), (4, 4), (4, 8), (5, 5), (8, 8), (8, 5), (3, 2), (1, 5)])
def test_degraded_fetch(world, nfrag):
    rng = np.random.default_rng(world + 7 * nfrag)
    table, src = _groups(world, nfrag, rng)
    held = P.simulate(world, nfrag, table, "star", [b"".join(g) for g in src])
    offs = [()] + [(g,) for g in range(world)] + ([(0, 1)] if world > 2 else [])
    for off in offs:
        out = P.simulate(world, nfrag, table, "fetch", None, dst_in=held, offline=off)
        for q in range(world):
            ops, dst_off, st = P.plan(world, q, nfrag, table, "fetch", off)
            srcs = P.download_sources(nfrag, world, q, off)
            for f in range(nfrag):
                if q in off or srcs[f] is None:
                    assert st[f] == L.DFS_E_MISSING, (off, q, f)
                    continue
                assert st[f] == 0
                o = int(dst_off[f])
                assert out[q][o:o + len(src[q][f])] == src[q][f], (off, q, f)
            # fetched from the holder SN:427-428 names (or locally)
            for x in ops[ops["kind"] == L.DFS_XFER_RECV]:
                assert int(x["peer"]) == srcs[int(x["frag"])]


def test_node3_down_plan_matches_reference_table():
    """The reference's fetch plan (SN:422-440) for 5 nodes on 5 ranks with node 3 (rank 2) down."""
    table = np.full((5, 5), 10, dtype=np.uint64)
    want = {0: [None, None, 1, 3, 4], 1: [0, None, None, 3, 4], 3: [0, 1, 1, None, None], 4: [None, 1, 1, 3, None]}
    for q, row in want.items():
        ops, _, st = P.plan(5, q, 5, table, "fetch", (2,))
        got = [None] * 5
        for x in ops[ops["kind"] == L.DFS_XFER_RECV]:
            got[int(x["frag"])] = int(x["peer"])
        assert got == row and (st == 0).all()


def test_plan_bad_arguments():
    t = np.zeros((2, 5), dtype=np.uint64)
    import ctypes
    n = ctypes.c_uint32(0)
    lib = L.lib()
    assert lib.dfs_place_plan(0, 0, 5, t.ctypes.data, 0, 0, None, ctypes.byref(n), None, None) == L.DFS_E_ARG
    assert lib.dfs_place_plan(2, 2, 5, t.ctypes.data, 0, 0, None, ctypes.byref(n), None, None) == L.DFS_E_ARG
    assert lib.dfs_place_plan(2, 0, 5, t.ctypes.data, 9, 0, None, ctypes.byref(n), None, None) == L.DFS_E_ARG
    assert lib.dfs_place_plan(2, 0, 5, None, 0, 0, None, ctypes.byref(n), None, None) == L.DFS_E_ARG
    # capacity too small
    assert lib.dfs_place_plan(2, 0, 5, np.ones((2, 5), dtype=np.uint64).ctypes.data, 1, 0,
                              np.zeros(1, dtype=L.XFER_DTYPE).ctypes.data, ctypes.byref(ctypes.c_uint32(1)), None,
                              None) == L.DFS_E_ARG
