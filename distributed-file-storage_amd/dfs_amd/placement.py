"""Fragment placement across GPUs — StorageNode's replication and fetch plan.

Reference (StorageNode.java, SN:line):
  * node k (0-based) stores fragments {k, (k+1) mod N}            SN:143-145, 199-200
  * the uploader sends every peer its pair (star fan-out)          SN:195-224
  * download takes fragment i locally, else from node i, else from
    node i-1 (candidates nodeA = i+1, nodeB = ((i-1+N)%N)+1 1-based) SN:422-440

MI355X mapping: one process per GPU; node k is hosted by GPU k mod W (W = world
size; with W == N, GPU g *is* node g).  Files are sharded by index over the
ranks; each rank hashes and Base64-encodes its shard on its own GPU
(libdfsgpu.so), with the Base64 laid out fragment-major
(DFS_LAYOUT_FRAG_MAJOR) so the bytes bound for one node are one span.

The exchange realises the reference's pair set in two steps:
  1. primary scatter: fragment f of every file goes to GPU(f) (point-to-point
     sends of whole fragment groups, RCCL over xGMI on GPUs, gloo on CPU);
  2. replica step: the primary GPU of fragment f forwards its group to the
     GPU hosting node f-1.  With W == N this is the ring g -> g-1 of
     BASELINE.json's north_star ("GPU g sends to g+1" under the relabelling
     node k <-> GPU k+1), one xGMI link per GPU.
After both steps every GPU holds exactly the fragments of the nodes it hosts.

`exchange_upload_star` realises the reference's star fan-out itself as one
all-to-all (every link busy at once); it yields the same holdings.

`download_sources` mirrors SN:427-440's candidate order for a degraded fetch
(one GPU offline) and `exchange_download` moves each requester's fragments back
from the holders for decode + verify + reassembly (dfs_download_batch).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


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


# ---------------------------------------------------------------------------
# Exchanges (torch.distributed point-to-point; RCCL on GPU, gloo on CPU)
# ---------------------------------------------------------------------------
def file_owner(file_digest: torch.Tensor, world: int) -> torch.Tensor:
    """Lookup rank of files after the upload: files are
    sharded by index for hashing, but a later GET /download?fileId=<hex>
    (SN:399-403) only knows the fileId, so the owner is the digest's first 8
    bytes (big-endian, the first 16 hex chars) mod world.  file_digest:
    (n, 32) uint8 raw digests on any device; returns (n,) int64 ranks, computed
    where the digests live (no host round trip)."""
    d = file_digest.reshape(-1, 32)[:, :8].to(torch.int64)
    # prefix mod world, one byte at a time: (acc * 256 + byte) mod world
    acc = torch.zeros(d.shape[0], dtype=torch.int64, device=d.device)
    for j in range(8):
        acc = (acc * 256 + d[:, j]) % world
    return acc


def file_owner_hex(file_id: str, world: int) -> int:
    """file_owner for one lowercase-hex fileId (the HTTP side)."""
    return int(file_id[:16], 16) % world


def _all_sizes(local: Sequence[int], device) -> torch.Tensor:
    """[world, len(local)] int64 table of every rank's sizes."""
    world = dist.get_world_size()
    t = torch.tensor(list(local), dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.stack(out)


def _p2p(ops: List[dist.P2POp]) -> None:
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()


def exchange_upload(b64: torch.Tensor, group_off: Sequence[int], nfrag: int
                    ) -> Tuple[Dict[int, Tuple[torch.Tensor, List[int]]], List[List[int]]]:
    """Place this rank's fragment-major Base64 on the GPUs that host its nodes.

    b64        uint8 tensor, fragment-major ([fragment][file]) Base64 of the
               rank's files (an upload plan built with frag_major=True)
    group_off  nfrag+1 byte offsets of each fragment group inside `b64`
    Returns (held, table): held = {f: (bytes of group f of every rank,
    concatenated in rank order, [per-source-rank byte counts])} for every
    fragment this GPU must hold (gpu_fragments); table[r][f] = bytes of rank
    r's group f.
    """
    world, me, dev = dist.get_world_size(), dist.get_rank(), b64.device
    sizes = [int(group_off[f + 1] - group_off[f]) for f in range(nfrag)]
    table = _all_sizes(sizes, dev).cpu().tolist()  # table[rank][f]

    def group(f):
        return b64[int(group_off[f]):int(group_off[f + 1])]

    # 1. primary scatter: fragment f -> GPU(f)
    prim: Dict[int, torch.Tensor] = {}
    ops = []
    for f in range(nfrag):
        dst = node_gpu(f, world)
        if dst == me:
            buf = torch.empty(sum(table[r][f] for r in range(world)), dtype=torch.uint8, device=dev)
            o = 0
            for r in range(world):
                n = table[r][f]
                if r == me:
                    buf[o:o + n].copy_(group(f))
                elif n:
                    ops.append(dist.P2POp(dist.irecv, buf[o:o + n], r))
                o += n
            prim[f] = buf
        elif sizes[f]:
            ops.append(dist.P2POp(dist.isend, group(f).contiguous(), dst))
    _p2p(ops)

    # 2. replica step: GPU(f) -> GPU(node f-1)
    held: Dict[int, Tuple[torch.Tensor, List[int]]] = {}
    per_src = {f: [table[r][f] for r in range(world)] for f in range(nfrag)}
    ops = []
    for f in range(nfrag):
        src = node_gpu(f, world)
        dst = node_gpu(fragment_holders(f, nfrag)[1], world)
        total = sum(per_src[f])
        if src == me:
            held[f] = (prim[f], per_src[f])
            if dst != me and total:
                ops.append(dist.P2POp(dist.isend, prim[f], dst))
        elif dst == me:
            buf = torch.empty(total, dtype=torch.uint8, device=dev)
            if total:
                ops.append(dist.P2POp(dist.irecv, buf, src))
            held[f] = (buf, per_src[f])
    _p2p(ops)
    return held, table


def exchange_upload_star(b64: torch.Tensor, group_off: Sequence[int], nfrag: int
                         ) -> Tuple[Dict[int, Tuple[torch.Tensor, List[int]]], List[List[int]]]:
    """The reference's own fan-out (SN:195-205: the uploader sends every peer
    its pair directly) as ONE all-to-all: rank r sends GPU g the groups of
    every fragment g must hold (gpu_fragments), so each fragment group leaves
    its source once per holder and every xGMI link carries traffic at once
    (SURVEY §8f rank 3), instead of the ring's scatter + forward over one
    link.  Same result format as exchange_upload."""
    world, me, dev = dist.get_world_size(), dist.get_rank(), b64.device
    sizes = [int(group_off[f + 1] - group_off[f]) for f in range(nfrag)]
    table = _all_sizes(sizes, dev).cpu().tolist()  # table[rank][f]
    need = [gpu_fragments(g, nfrag, world) for g in range(world)]
    parts, in_split = [], []
    for g in range(world):
        in_split.append(sum(sizes[f] for f in need[g]))
        parts += [b64[int(group_off[f]):int(group_off[f + 1])] for f in need[g]]
    send = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device=dev)
    out_split = [sum(table[r][f] for f in need[me]) for r in range(world)]
    flat = torch.empty(sum(out_split), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(flat, send, out_split, in_split)
    starts = [sum(out_split[:r]) for r in range(world)]
    recv = [flat[starts[r]:starts[r] + out_split[r]] for r in range(world)]
    held: Dict[int, Tuple[torch.Tensor, List[int]]] = {}
    pos = [0] * world
    for f in need[me]:
        per = [table[r][f] for r in range(world)]
        pieces = []
        for r in range(world):
            pieces.append(recv[r][pos[r]:pos[r] + per[r]])
            pos[r] += per[r]
        held[f] = (torch.cat(pieces), per)
    return held, table


def exchange_download(held: Dict[int, Tuple[torch.Tensor, List[int]]], table: List[List[int]], nfrag: int,
                      offline: Iterable[int] = (), device=None) -> Dict[int, Optional[torch.Tensor]]:
    """Fetch this rank's fragments back from the holders (degraded read).

    Each fragment f is served by the first online holder in SN:427-428 order
    (download_sources); the server cuts the requester's slice out of its
    group f.  Returns {f: this rank's group-f bytes or None if no holder is
    online}.  Offline ranks neither serve nor request.
    """
    world, me = dist.get_world_size(), dist.get_rank()
    off = set(offline)
    dev = device if device is not None else (next(iter(held.values()))[0].device if held else torch.device("cpu"))
    out: Dict[int, Optional[torch.Tensor]] = {}
    ops = []
    for q in range(world):  # requester q
        if q in off:
            continue
        srcs = download_sources(nfrag, world, q, off)
        for f in range(nfrag):
            s = srcs[f]
            if s is None:
                if q == me:
                    out[f] = None
                continue
            if s == me:
                buf, per = held[f]
                lo = sum(per[:q])
                piece = buf[lo:lo + per[q]]
                if q == me:
                    out[f] = piece
                elif per[q]:
                    ops.append(dist.P2POp(dist.isend, piece.contiguous(), q))
            elif q == me:
                n = table[me][f]
                buf = torch.empty(n, dtype=torch.uint8, device=dev)
                if n:
                    ops.append(dist.P2POp(dist.irecv, buf, s))
                out[f] = buf
    _p2p(ops)
    return out


def frag_major_spans(file_lens: Sequence[int], nfrag: int):
    """(nfiles*nfrag, 2) uint64 spans of each (file, fragment) Base64 inside a
    fragment-major buffer ([fragment][file], the layout of a frag_major upload
    plan and of the groups exchange_download returns concatenated in order)."""
    import numpy as np
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


def group_sizes_table(group_off: Sequence[int], nfrag: int, device) -> List[List[int]]:
    sizes = [int(group_off[f + 1] - group_off[f]) for f in range(nfrag)]
    return _all_sizes(sizes, device).cpu().tolist()
