"""Fragment placement across GPUs — StorageNode's replication and fetch plan,
over the C-ABI (libdfsgpu.so: dfs_comm_* / dfs_place_* / dfs_fetch_degraded,
RCCL send/recv over xGMI).

Reference (StorageNode.java, SN:line):
  * node k (0-based) stores fragments {k, (k+1) mod N}            SN:143-145, 199-200
  * the uploader sends every peer its pair (star fan-out)          SN:195-224
  * download takes fragment i locally, else from node i, else from
    node i-1 (candidates nodeA = i+1, nodeB = ((i-1+N)%N)+1 1-based) SN:422-440

MI355X mapping: one process per GPU; node k is hosted by GPU k mod W (W = world
size; with W == N, GPU g *is* node g).  Files are sharded by index over the
ranks; each rank hashes and Base64-encodes its shard on its own GPU with the
Base64 laid out fragment-major (DFS_LAYOUT_FRAG_MAJOR), so group f (fragment f
of every file of the rank) is one span.  After a placement every rank holds,
for each fragment f it hosts, group f of every rank in rank order.

Everything that moves bytes is in the library: the schedule is
`dfs_place_plan` (pure host, also used by the CPU tests, which simulate every
rank), the transfers are ncclSend / ncclRecv inside RCCL groups
(`dfs_place_ring`, `dfs_place_star`, `dfs_fetch_degraded`).  This module only
holds the pure maps, the comm setup and thin wrappers.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import check, lib


# ---------------------------------------------------------------------------
# Pure maps
# ---------------------------------------------------------------------------
def node_fragments(k: int, n: int) -> Tuple[int, int]:
    """Fragments stored by 0-based node k (SN:143-145, 199-200)."""
    return k, (k + 1) % n


def fragment_holders(f: int, n: int) -> Tuple[int, int]:
    """0-based nodes holding fragment f: (nodeA, nodeB) of SN:427-428."""
    return f, (f - 1 + n) % n


def node_gpu(k: int, world: int) -> int:
    return k % world


def gpu_fragments(g: int, n: int, world: int) -> List[int]:
    """Fragment indices GPU g must hold after placement."""
    out = set()
    for k in range(n):
        if node_gpu(k, world) == g:
            out.update(node_fragments(k, n))
    return sorted(out)


def download_sources(n: int, world: int, me: int, offline: Iterable[int] = ()) -> List[Optional[int]]:
    """GPU to fetch each fragment from, in SN:422-440's order: the local copy
    first, then node i's GPU, then node i-1's GPU, skipping offline GPUs.
    None = "Could not retrieve fragment i" (SN:443-446)."""
    off = set(offline)
    mine = set(gpu_fragments(me, n, world)) if me not in off else set()
    src: List[Optional[int]] = []
    for f in range(n):
        if f in mine:
            src.append(me)
            continue
        pick = None
        for node in fragment_holders(f, n):
            g = node_gpu(node, world)
            if g not in off:
                pick = g
                break
        src.append(pick)
    return src


def file_owner(file_digest, world: int):
    """Lookup rank of files after the upload (BASELINE configs[2], "sharded by fileId"): files are
    sharded by index for hashing, but a later GET /download?fileId=<hex>
    (SN:399-403) only knows the fileId, so the owner is the digest's first 8
    bytes (big-endian, the first 16 hex chars) mod world.  file_digest:
    (n, 32) uint8 raw digests (torch tensor on any device); returns (n,) int64
    ranks, computed where the digests live (no host round trip)."""
    import torch
    d = file_digest.reshape(-1, 32)[:, :8].to(torch.int64)
    acc = torch.zeros(d.shape[0], dtype=torch.int64, device=d.device)
    for j in range(8):  # prefix mod world, one byte at a time
        acc = (acc * 256 + d[:, j]) % world
    return acc


def file_owner_hex(file_id: str, world: int) -> int:
    """file_owner for one lowercase-hex fileId (the HTTP side)."""
    return int(file_id[:16], 16) % world


def offline_mask(offline: Iterable[int]) -> int:
    m = 0
    for g in offline:
        m |= 1 << int(g)
    return m


# ---------------------------------------------------------------------------
# Schedules (pure host, dfs_place_plan)
# ---------------------------------------------------------------------------
MODES = {"ring": L.DFS_PLACE_RING, "star": L.DFS_PLACE_STAR, "fetch": L.DFS_PLACE_FETCH}


def plan(world: int, rank: int, nfrag: int, table: np.ndarray, mode: str, offline: Iterable[int] = ()
         ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(ops as an XFER_DTYPE array, dst_off (nfrag+1), frag_status (nfrag)) of
    rank `rank`'s transfer schedule; table = (world, nfrag) group bytes."""
    t = np.ascontiguousarray(table, dtype=np.uint64).reshape(world, nfrag)
    n = ctypes.c_uint32(0)
    dst_off = np.zeros(nfrag + 1, dtype=np.uint64)
    status = np.zeros(nfrag, dtype=np.int32)
    m = offline_mask(offline)
    check(lib().dfs_place_plan(world, rank, nfrag, t.ctypes.data, MODES[mode], m, None, ctypes.byref(n),
                               dst_off.ctypes.data, status.ctypes.data), "dfs_place_plan")
    ops = np.zeros(max(n.value, 1), dtype=L.XFER_DTYPE)
    check(lib().dfs_place_plan(world, rank, nfrag, t.ctypes.data, MODES[mode], m, ops.ctypes.data, ctypes.byref(n),
                               None, None), "dfs_place_plan")
    return ops[:n.value], dst_off, status


def held_layout(world: int, rank: int, nfrag: int, table: np.ndarray) -> np.ndarray:
    """Offsets of the held groups on `rank` after a placement (UINT64_MAX =
    not hosted); last entry = bytes of the held buffer."""
    return plan(world, rank, nfrag, table, "star")[1]


def bytes_sent(ops: np.ndarray) -> int:
    return int(ops["len"][ops["kind"] == L.DFS_XFER_SEND].sum())


# ---------------------------------------------------------------------------
# RCCL comms and transfers (device buffers; asynchronous on the ctx stream)
# ---------------------------------------------------------------------------
def _comm_error(rc: int, where: str):
    if rc == L.DFS_E_COMM:
        raise L.DfsError(rc, f"{where}: {lib().dfs_comm_last_error().decode(errors='replace')}")
    check(rc, where)


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * L.DFS_COMM_ID_BYTES)()
    _comm_error(lib().dfs_comm_unique_id(buf), "dfs_comm_unique_id")
    return bytes(buf)


class Comm:
    """One RCCL communicator bound to a FragmentEngine (its device and
    stream).  Rank-per-process: Comm(engine, uid, world, rank), uid from
    unique_id() on one rank shared out of band (e.g. torch.distributed)."""

    def __init__(self, engine, uid: bytes, world: int, rank: int):
        assert len(uid) == L.DFS_COMM_ID_BYTES
        self.engine = engine
        self.world, self.rank = world, rank
        self._c = ctypes.c_void_p()
        idb = (ctypes.c_uint8 * L.DFS_COMM_ID_BYTES).from_buffer_copy(uid)
        _comm_error(lib().dfs_comm_init_rank(engine.ctx, idb, world, rank, ctypes.byref(self._c)),
                    "dfs_comm_init_rank")

    @classmethod
    def init_all(cls, engines) -> "List[Comm]":
        """dfs_comm_init_all: one process driving one communicator per engine
        (one engine per GPU; ncclCommInitAll), rank i on engines[i]."""
        n = len(engines)
        ctxs = (ctypes.c_void_p * n)(*[e.ctx for e in engines])
        out = (ctypes.c_void_p * n)()
        _comm_error(lib().dfs_comm_init_all(ctxs, n, out), "dfs_comm_init_all")
        comms = []
        for i, e in enumerate(engines):
            c = cls.__new__(cls)
            c.engine, c.world, c.rank, c._c = e, n, i, ctypes.c_void_p(out[i])
            comms.append(c)
        return comms

    def _arr(self):
        return (ctypes.c_void_p * 1)(self._c.value)

    def counters(self) -> dict:
        """Transfers issued on this comm so far: sends, receives, local copies."""
        c = np.zeros(3, dtype=np.uint64)
        _comm_error(lib().dfs_comm_counters(self._c, c.ctypes.data), "dfs_comm_counters")
        return {"sends": int(c[0]), "recvs": int(c[1]), "copies": int(c[2])}

    def sizes(self, grp_len: Sequence[int]) -> np.ndarray:
        """(world, nfrag) table of every rank's group bytes (synchronous)."""
        g = np.ascontiguousarray(grp_len, dtype=np.uint64)
        nfrag = len(g)
        table = np.zeros((self.world, nfrag), dtype=np.uint64)
        _comm_error(lib().dfs_place_sizes(self._arr(), 1, g.ctypes.data, nfrag, table.ctypes.data), "dfs_place_sizes")
        return table

    def place(self, mode: str, table: np.ndarray, d_src: int, d_dst: int) -> None:
        """Upload placement ("ring" or "star") of the fragment-major groups
        at d_src into the held buffer d_dst (held_layout)."""
        nfrag = table.shape[1]
        t = np.ascontiguousarray(table, dtype=np.uint64)
        src = (ctypes.c_void_p * 1)(d_src)
        dst = (ctypes.c_void_p * 1)(d_dst)
        fn = lib().dfs_place_ring if mode == "ring" else lib().dfs_place_star
        _comm_error(fn(self._arr(), 1, nfrag, t.ctypes.data, src, dst), f"dfs_place_{mode}")

    def fetch(self, table: np.ndarray, d_held: int, d_out: int, offline: Iterable[int] = ()) -> np.ndarray:
        """Degraded read: this rank's groups back into d_out (source layout)
        from the live holders; returns per-fragment status."""
        nfrag = table.shape[1]
        t = np.ascontiguousarray(table, dtype=np.uint64)
        st = np.zeros(nfrag, dtype=np.int32)
        src = (ctypes.c_void_p * 1)(d_held)
        dst = (ctypes.c_void_p * 1)(d_out)
        _comm_error(lib().dfs_fetch_degraded(self._arr(), 1, nfrag, t.ctypes.data, offline_mask(offline), src, dst,
                                             st.ctypes.data), "dfs_fetch_degraded")
        return st

    def close(self) -> None:
        if self._c:
            lib().dfs_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def simulate_native(world: int, nfrag: int, table: np.ndarray, mode: str, src: Sequence[bytes],
                    offline: Iterable[int] = ()) -> Tuple[List[bytes], np.ndarray]:
    """dfs_place_simulate: the library's own runner (the code that issues the
    RCCL calls) for every rank at once over host buffers and an in-process
    stand-in for RCCL's group matching.  Returns (every rank's destination
    buffer, (world, nfrag) fragment status); raises DfsError(DFS_E_COMM) when
    sends and receives do not pair up."""
    t = np.ascontiguousarray(table, dtype=np.uint64).reshape(world, nfrag)
    sizes = [int(plan(world, r, nfrag, t, mode, offline)[1][nfrag]) for r in range(world)]
    srcs = [np.frombuffer(bytes(s) or b"\0", dtype=np.uint8).copy() for s in src]
    dsts = [np.zeros(max(n, 1), dtype=np.uint8) for n in sizes]
    sp = (ctypes.c_void_p * world)(*[a.ctypes.data for a in srcs])
    dp = (ctypes.c_void_p * world)(*[a.ctypes.data for a in dsts])
    st = np.zeros((world, nfrag), dtype=np.int32)
    _comm_error(lib().dfs_place_simulate(world, nfrag, t.ctypes.data, MODES[mode], offline_mask(offline), sp, dp,
                                         st.ctypes.data), "dfs_place_simulate")
    return [d[:n].tobytes() for d, n in zip(dsts, sizes)], st


def replica_layout(world: int, rank: int, nfrag: int, file_lens: Sequence[Sequence[int]], align128: bool = False):
    """dfs_replica_layout (pure host): what `rank` holds after a placement of
    fragment-major uploads, file_lens[r] = rank r's file lengths.  Returns
    (frags as a HELD_FRAG_DTYPE array in held order, (world, nfrag) Base64
    group table, held_bytes, raw_bytes)."""
    nfiles = np.array([len(x) for x in file_lens], dtype=np.uint32)
    lens = np.array([int(v) for x in file_lens for v in x] or [0], dtype=np.uint64)
    flags = L.DFS_LAYOUT_FRAG_MAJOR | (L.DFS_LAYOUT_ALIGN128 if align128 else 0)
    n = ctypes.c_uint64(0)
    table = np.zeros((world, nfrag), dtype=np.uint64)
    held, raw = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(lib().dfs_replica_layout(world, rank, nfrag, nfiles.ctypes.data, lens.ctypes.data, flags, None,
                                   ctypes.byref(n), table.ctypes.data, ctypes.byref(held), ctypes.byref(raw)),
          "dfs_replica_layout")
    frags = np.zeros(max(n.value, 1), dtype=L.HELD_FRAG_DTYPE)
    check(lib().dfs_replica_layout(world, rank, nfrag, nfiles.ctypes.data, lens.ctypes.data, flags, frags.ctypes.data,
                                   ctypes.byref(n), None, None, None), "dfs_replica_layout")
    return frags[:n.value], table, held.value, raw.value


class ReplicaPlan:
    """dfs_replica_plan of one batch shape on one Comm: the replica receiver's
    verify (SN:265-293 + 248-257) over the held buffer a placement filled."""

    def __init__(self, comm: "Comm", nfrag: int, file_lens: Sequence[int], align128: bool = False):
        self.comm = comm
        lens = np.ascontiguousarray(file_lens, dtype=np.uint64)
        nf = (ctypes.c_uint32 * 1)(len(lens))
        lp = (ctypes.c_void_p * 1)(lens.ctypes.data if len(lens) else None)
        out = (ctypes.c_void_p * 1)()
        flags = L.DFS_LAYOUT_FRAG_MAJOR | (L.DFS_LAYOUT_ALIGN128 if align128 else 0)
        _comm_error(lib().dfs_replica_plan_create(comm._arr(), 1, nfrag, nf, lp, flags, out), "dfs_replica_plan_create")
        self._p = ctypes.c_void_p(out[0])
        n, held, raw = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self.table = np.zeros((comm.world, nfrag), dtype=np.uint64)
        check(lib().dfs_replica_plan_info(self._p, ctypes.byref(n), ctypes.byref(held), ctypes.byref(raw),
                                          self.table.ctypes.data), "dfs_replica_plan_info")
        self.nheld, self.held_bytes, self.raw_bytes = n.value, held.value, raw.value

    @property
    def one_pass(self) -> bool:
        """True if the check decodes, stores and hashes in one kernel."""
        return lib().dfs_replica_plan_one_pass(self._p) == 1

    def frags(self) -> np.ndarray:
        out = np.zeros(max(self.nheld, 1), dtype=L.HELD_FRAG_DTYPE)
        check(lib().dfs_replica_plan_frags(self._p, out.ctypes.data), "dfs_replica_plan_frags")
        return out[:self.nheld]

    def verify(self, d_frag_digest: int, d_held: int, d_raw: int, d_verdict: int, d_failed: int) -> None:
        """Asynchronous on the comm's engine stream (dfs_replica_verify)."""
        one = lambda v: (ctypes.c_void_p * 1)(v or None)  # noqa: E731
        plans = (ctypes.c_void_p * 1)(self._p.value)
        _comm_error(lib().dfs_replica_verify(self.comm._arr(), 1, plans, one(d_frag_digest), one(d_held), one(d_raw),
                                             one(d_verdict), one(d_failed)), "dfs_replica_verify")

    def exchange(self, d_frag_digest: int) -> None:
        """Stage 1 (comm stream): this rank's digests to the holders."""
        plans = (ctypes.c_void_p * 1)(self._p.value)
        _comm_error(lib().dfs_replica_exchange(self.comm._arr(), 1, plans, (ctypes.c_void_p * 1)(d_frag_digest or None)),
                    "dfs_replica_exchange")

    def check(self, engine, d_held: int, d_raw: int, d_verdict: int, d_failed: int) -> None:
        """Stage 2 (engine's stream, no communication): decode, hash, compare."""
        c = ctypes.c_void_p
        check(lib().dfs_replica_check(engine.ctx, self._p, c(d_held or None), c(d_raw or None), c(d_verdict or None),
                                      c(d_failed or None)), "dfs_replica_check")

    def report(self, d_failed: int) -> None:
        """Stage 3 (comm stream): failures per uploader summed over the holders."""
        _comm_error(lib().dfs_replica_report(self.comm._arr(), 1, (ctypes.c_void_p * 1)(d_failed or None)),
                    "dfs_replica_report")

    def close(self) -> None:
        if self._p:
            lib().dfs_replica_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def frag_major_spans(file_lens: Sequence[int], nfrag: int):
    """(nfiles*nfrag, 2) uint64 spans of each (file, fragment) Base64 inside a
    fragment-major buffer ([fragment][file], the layout of a frag_major upload
    plan and of the groups dfs_fetch_degraded hands back)."""
    nf = len(file_lens)
    enc = np.zeros((nf, nfrag), dtype=np.uint64)
    for f, S in enumerate(file_lens):
        b, rem = divmod(int(S), nfrag)
        for i in range(nfrag):
            n = b + (1 if i < rem else 0)
            enc[f, i] = 4 * ((n + 2) // 3)
    spans = np.zeros((nf * nfrag, 2), dtype=np.uint64)
    o = 0
    for i in range(nfrag):
        col = enc[:, i]
        starts = o + np.concatenate([[0], np.cumsum(col)[:-1]]).astype(np.uint64) if nf else col
        spans[i::nfrag, 0] = starts
        spans[i::nfrag, 1] = col
        o += int(col.sum())
    return spans


def simulate(world: int, nfrag: int, table: np.ndarray, mode: str, src: Sequence[bytes],
             dst_in: Optional[Sequence[bytes]] = None, offline: Iterable[int] = ()) -> List[bytes]:
    """Run every rank's dfs_place_plan schedule in one process over host
    bytes (the matching RCCL does: per phase, rank a's sends to b pair with
    b's receives from a in issue order).  Returns every rank's destination
    buffer.  Used by the CPU tests and the bench's --dry-run harness check to
    prove the schedules before they run over RCCL."""
    plans = [plan(world, r, nfrag, table, mode, offline) for r in range(world)]
    dst = [bytearray(int(p[1][nfrag])) for p in plans]
    srcb = [bytes(s) for s in (dst_in if mode == "fetch" else src)]
    phases = max([int(p[0]["phase"].max()) + 1 if len(p[0]) else 0 for p in plans] + [0])
    for ph in range(phases):
        snapshot = [bytes(d) for d in dst]  # a phase reads what earlier phases wrote
        for r, (ops, _, _) in enumerate(plans):
            for x in ops[(ops["phase"] == ph) & (ops["kind"] == L.DFS_XFER_COPY)]:
                s = snapshot[r] if x["from_dst"] else srcb[r]
                a, n, o = int(x["src_off"]), int(x["len"]), int(x["dst_off"])
                dst[r][o:o + n] = s[a:a + n]
        for a_r in range(world):
            for b_r in range(world):
                if a_r == b_r:
                    continue
                sa = plans[a_r][0]
                sends = sa[(sa["phase"] == ph) & (sa["kind"] == L.DFS_XFER_SEND) & (sa["peer"] == b_r)]
                rb = plans[b_r][0]
                recvs = rb[(rb["phase"] == ph) & (rb["kind"] == L.DFS_XFER_RECV) & (rb["peer"] == a_r)]
                if len(sends) != len(recvs):
                    raise AssertionError(f"phase {ph}: {a_r}->{b_r} {len(sends)} sends vs {len(recvs)} recvs")
                for x, y in zip(sends, recvs):
                    if int(x["len"]) != int(y["len"]):
                        raise AssertionError(f"phase {ph}: {a_r}->{b_r} send {x['len']} vs recv {y['len']}")
                    s = snapshot[a_r] if x["from_dst"] else srcb[a_r]
                    a, n, o = int(x["src_off"]), int(x["len"]), int(y["dst_off"])
                    dst[b_r][o:o + n] = s[a:a + n]
    return [bytes(d) for d in dst]


def run_plan_torch(ops: np.ndarray, src, dst) -> None:
    """Execute one rank's dfs_place_plan schedule with torch.distributed
    point-to-point ops on CPU tensors (gloo): the multi-process CPU check of
    the schedules (tests/test_dist.py, bench.py --dry-run).  GPU buffers go
    through the library's RCCL runner (Comm.place / Comm.fetch), never here."""
    import torch.distributed as dist
    phases = int(ops["phase"].max()) + 1 if len(ops) else 0
    for ph in range(phases):
        cur = ops[ops["phase"] == ph]
        for x in cur[cur["kind"] == L.DFS_XFER_COPY]:
            s = dst if x["from_dst"] else src
            a, n, o = int(x["src_off"]), int(x["len"]), int(x["dst_off"])
            dst[o:o + n].copy_(s[a:a + n])
        p2p = []
        for x in cur[cur["kind"] != L.DFS_XFER_COPY]:
            n = int(x["len"])
            if x["kind"] == L.DFS_XFER_SEND:
                s = dst if x["from_dst"] else src
                a = int(x["src_off"])
                p2p.append(dist.P2POp(dist.isend, s[a:a + n].contiguous(), int(x["peer"])))
            else:
                o = int(x["dst_off"])
                p2p.append(dist.P2POp(dist.irecv, dst[o:o + n], int(x["peer"])))
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()
