#!/usr/bin/env python3
"""bench.py — StorageNode upload fragment pipeline on MI355X (BASELINE.json metric).

One step = one pass of handleUpload's fragment pipeline (StorageNode.java
:118-189) over one batch of synthetic files resident in HBM: fileId SHA-256
(:127), N-way split (:138-157), per-fragment SHA-256 (:159) and the Base64 of
every fragment (:636) — all in the gfx950 kernels of libdfsgpu.so.

Default workload = BASELINE.json configs[1]: 65,536 files x 1 MiB per GPU,
N = 5 fragments.  With --gpus N (launched one rank per GPU by
torch.distributed.run) every rank processes its own shard of files (weak
scaling, no data-path collective); `value` = file bytes of all ranks / the
slowest rank's time.  Rank 0 prints ONE JSON line.

Extra objects on the line:
  roofline      dominant kernel (multi-message SHA-256) vs the int32-VALU peak,
                timed with HIP events on its own stream inside the timed loop
  roofline_b64  the Base64 encode kernel vs the HBM peak
  cpu_baseline  CPU restatement (OpenSSL SHA-NI SHA-256 + scalar Base64, one
                file per thread) on a bounded sample, rank 0, N = 1 only
  download      handleDownload over the same files: Base64 decode into place +
                fragment / fileId SHA-256 verify, and the raw-fragment gather
  wire          storeFragments request bodies built on the device, then
                received (parse + decode + SHA-256) on the device
  store         on-disk fragment store: node 1's fragments HBM -> disk -> HBM
  replication   N > 1: ring and all-to-all placement over RCCL, degraded read
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))

METRIC = "SHA-256+Base64 fragment GB/s per node at 1/8 GPUs; % of int-VALU peak"
SEED = 0x5EED5EED
# canonical int32 VALU ops per 64-byte SHA-256 block (gfx950
# ISA without v_xor3).  The shipped kernel issues 1,405 (v_bitop3 folds the
# three-input XORs), so `frac` below is algorithmic, not issue utilisation;
# `valu_issue_frac` gives the executed-instruction view.
OPS_PER_BLOCK_CANON = 1688
OPS_PER_BLOCK_ISSUED = 1405
# Peaks: MI355X_MICROARCH.md — 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32
# (the FP32 vector rate without FMA doubling), HBM 8 TB/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0


def sha_blocks(n: int) -> int:
    return n // 64 + (1 if n % 64 < 56 else 2)


def split(S: int, N: int):
    base, rem = divmod(S, N)
    return [base + (1 if i < rem else 0) for i in range(N)]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--files", type=int, default=65536, help="files per GPU")
    ap.add_argument("--file-size", type=int, default=1 << 20)
    ap.add_argument("--nfrag", type=int, default=5)
    ap.add_argument("--mode", choices=("fused", "kernels", "serial"), default="kernels",
                    help="kernels: SHA and Base64 kernels on two streams (default); fused: Base64 "
                         "written by the SHA fragment lanes; serial: the two kernels on one stream")
    ap.add_argument("--serial", action="store_true", help="alias of --mode serial")
    ap.add_argument("--align128", action=argparse.BooleanOptionalAction, default=True,
                    help="DFS_LAYOUT_ALIGN128: every fragment's Base64 starts on a 128-byte boundary")
    ap.add_argument("--b64-steps", type=int, default=3, help="steps of the standalone Base64 leg")
    ap.add_argument("--frag-only-steps", type=int, default=3, help="steps of the fragment-only (no fileId) leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--verify", type=int, default=8, help="files spot-checked against the oracle (rank 0)")
    ap.add_argument("--no-replicate", action="store_true", help="N>1: skip the placement / degraded-read leg")
    ap.add_argument("--rep-files", type=int, default=8192, help="files per GPU in the placement leg")
    ap.add_argument("--rep-steps", type=int, default=3)
    ap.add_argument("--no-download", action="store_true", help="skip the download/verify leg")
    ap.add_argument("--dl-steps", type=int, default=2)
    ap.add_argument("--dl-chunks", type=int, default=0,
                    help="> 0: also time the chunked 2-context download (slower: see DESIGN §9)")
    ap.add_argument("--wire-files", type=int, default=16384, help="files in the storeFragments body leg")
    ap.add_argument("--no-wire", action="store_true", help="skip the storeFragments body leg")
    ap.add_argument("--store-files", type=int, default=2048, help="files in the on-disk fragment store leg")
    ap.add_argument("--no-store", action="store_true", help="skip the on-disk fragment store leg")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4),
                    help="2: BASELINE configs[1] (default bench line); 3: configs[2]'s per-GPU shard "
                         "(131,072 x 256 KiB, N=8 per GPU; 1M files on 8 GPUs); 4: configs[3], the long-fragment "
                         "skew (1,024 x 256 MiB, N=5) streamed through HBM in chunks, its own JSON line")
    ap.add_argument("--long-files", type=int, default=1024)
    ap.add_argument("--long-size", type=int, default=256 << 20)
    ap.add_argument("--long-chunk", type=int, default=192 * 87381, help="bytes per file per chunk (x192)")
    args = ap.parse_args()
    if args.config == 3:  # BASELINE configs[2]: 1M files x 256 KiB sharded by file over 8 GPUs, N = 8
        args.files, args.file_size, args.nfrag = 131072, 256 << 10, 8
        args.wire_files = min(args.wire_files, 65536)
    return args


def cpu_baseline(args, log):
    """Oracle leg: C restatement on the host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure, checker/baseline only)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    S, N = args.file_size, args.nfrag
    # calibrate: 2 files per thread
    secs, _, _ = O.cpu_upload_bench(2 * threads, S, N, threads, use_openssl=True)
    kind_sha = "openssl"
    if secs < 0:
        secs, _, _ = O.cpu_upload_bench(2 * threads, S, N, threads, use_openssl=False)
        kind_sha = "scalar"
    per_file = max(secs, 1e-6) / 2.0  # seconds per file per thread
    nfiles = int(max(threads, min(200000, args.cpu_seconds / per_file * threads)))
    secs, _, _ = O.cpu_upload_bench(nfiles, S, N, threads, use_openssl=(kind_sha == "openssl"))
    gbs = nfiles * S / secs / 1e9
    log(f"cpu baseline: {nfiles} files x {S} B on {threads} threads: {secs:.2f} s -> {gbs:.3f} GB/s")
    # one connection-handler thread alone (1-thread and all-core)
    n1 = int(max(1, min(20000, 3.0 / per_file)))
    secs1, _, _ = O.cpu_upload_bench(n1, S, N, 1, use_openssl=(kind_sha == "openssl"))
    gbs1 = n1 * S / secs1 / 1e9
    log(f"cpu baseline: {n1} files on 1 thread: {secs1:.2f} s -> {gbs1:.3f} GB/s")
    return {"value": round(gbs, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{nfiles} synthetic files x {S} B, N={N}: fileId + fragment SHA-256 "
                      f"({'OpenSSL SHA256 (SHA-NI), approximating HotSpot intrinsic' if kind_sha == 'openssl' else 'scalar C'})"
                      f" + scalar Base64, one file per thread (thread-per-connection, SN:30); "
                      f"CPU proxy, not Java (no JDK on the box)",
            "seconds": round(secs, 3), "single_thread_value": round(gbs1, 4), "single_thread_files": n1}


def replication_leg(args, eng, files, S, N, dev, log):
    """N>1 only: place a bounded sample of this rank's fragments on the GPUs
    hosting their nodes (primary scatter + replica step over RCCL/xGMI,
    dfs_amd.placement), then run config 5's degraded download with the last
    rank offline: fetch from the surviving holders, Base64-decode into place,
    per-fragment and fileId SHA-256 verify (dfs_download_batch).  Timed
    separately from the compute steps; returns a dict for the JSON line."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import dfs_amd
    from dfs_amd import placement as P
    from dfs_amd.engine import download_device
    world, me = dist.get_world_size(), dist.get_rank()
    R = min(args.files, args.rep_files)
    spans = np.stack([np.arange(R, dtype=np.uint64) * np.uint64(S), np.full(R, S, dtype=np.uint64)], axis=1)
    plan = dfs_amd.UploadPlan(eng, spans, N, frag_major=True)
    fd = torch.empty(R * 32, dtype=torch.uint8, device=dev)
    frd = torch.empty(R * N * 32, dtype=torch.uint8, device=dev)
    b64 = torch.empty(plan.b64_total, dtype=torch.uint8, device=dev)
    plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), dfs_amd.DFS_SERIAL)
    torch.cuda.synchronize(dev)
    offs = plan.b64_offsets()
    group_off = [int(offs[i]) for i in range(N)] + [int(offs[-1])]

    def timed(fn, reps):
        fn()  # warm-up
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return r, float(tt.item()) / reps

    (held, table), t_up = timed(lambda: P.exchange_upload(b64, group_off, N), args.rep_steps)
    sent = sum(table[me][f] for f in range(N) if P.node_gpu(f, world) != me)
    sent += sum(sum(table[r][f] for r in range(world)) for f in range(N)
                if P.node_gpu(f, world) == me and P.node_gpu(P.fragment_holders(f, N)[1], world) != me)
    sent_t = torch.tensor([sent], dtype=torch.float64, device=dev)
    dist.all_reduce(sent_t)
    ok_ex = all(len(held[f][0]) == sum(table[r][f] for r in range(world)) for f in P.gpu_fragments(me, N, world))

    # The reference's star fan-out (SN:195-205) as one all-to-all: every link busy at once.
    (held_s, _t), t_star = timed(lambda: P.exchange_upload_star(b64, group_off, N), args.rep_steps)
    ok_ex = ok_ex and all(torch.equal(held_s[f][0], held[f][0]) for f in P.gpu_fragments(me, N, world))
    need = [P.gpu_fragments(g, N, world) for g in range(world)]
    sent_s = sum(table[me][f] for g in range(world) if g != me for f in need[g])
    sent_st = torch.tensor([sent_s], dtype=torch.float64, device=dev)
    dist.all_reduce(sent_st)
    del held_s

    offline = {world - 1}
    fetched, t_fetch = timed(lambda: P.exchange_download(held, table, N, offline=offline, device=dev), args.rep_steps)
    result = {"files_per_gpu": R, "nodes": N, "node_to_gpu": "node k on GPU k mod W",
              "upload_exchange_ms": round(t_up * 1e3, 3),
              "upload_exchange_gbps_per_gpu": round(sent_t.item() / world / t_up / 1e9, 2),
              "star_exchange_ms": round(t_star * 1e3, 3),
              "star_exchange_gbps_per_gpu": round(sent_st.item() / world / t_star / 1e9, 2),
              "exchange_sizes_ok": bool(ok_ex), "offline_gpu": world - 1,
              "degraded_fetch_ms": round(t_fetch * 1e3, 3)}
    status_ok = True
    if me not in offline:
        # one contiguous Base64 buffer, spans per (file, fragment)
        groups = [fetched[f] for f in range(N)]
        status_ok = all(g is not None for g in groups)
        if status_ok:
            blob = torch.cat(groups)
            msp = P.frag_major_spans([S] * R, N)
            out = torch.empty(R * S, dtype=torch.uint8, device=dev)
            file_len = np.full(R, S, dtype=np.uint64)
            file_off = np.arange(R, dtype=np.uint64) * np.uint64(S)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            status = download_device(eng, blob.data_ptr(), msp, R, N, file_len, frd.data_ptr(), fd.data_ptr(),
                                     out.data_ptr(), file_off)
            t_dl = time.perf_counter() - t0
            status_ok = bool((status == 0).all()) and bool(torch.equal(out, files[:R * S]))
            result["degraded_download_ms"] = round(t_dl * 1e3, 3)
            result["degraded_download_gbps"] = round(R * S / t_dl / 1e9, 2)
    flag = torch.tensor([1 if status_ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    result["degraded_download_ok"] = bool(flag.item())
    plan.close()
    return result


def download_leg(args, eng, files, plan, fd, frd, b64, S, N, F, dev, log):
    """handleDownload's verify path (SN:399-461) plus north_star's per-fragment
    check, over this GPU's whole upload: Base64-decode every fragment straight
    into its file offset (fused gather, SN:448-451), per-fragment SHA-256 vs the
    upload-time digests, fileId SHA-256 re-verify (SN:454-458) — one
    dfs_download_batch on device buffers.  Returns a dict for the JSON line."""
    import numpy as np
    import torch
    from dfs_amd.engine import download_device
    msp = plan.b64_spans([S] * F)
    file_len = np.full(F, S, dtype=np.uint64)
    file_off = np.arange(F, dtype=np.uint64) * np.uint64(S)
    out = torch.empty(F * S, dtype=torch.uint8, device=dev)
    reps = max(1, args.dl_steps)

    def once():
        return download_device(eng, b64.data_ptr(), msp, F, N, file_len, frd.data_ptr(), fd.data_ptr(),
                               out.data_ptr(), file_off)

    once()
    torch.cuda.synchronize(dev)
    eng.set_profiling(True)
    dec, sha, tot, wall = [], [], [], []
    ok = True
    for _ in range(reps):
        t0 = time.perf_counter()
        st = once()
        wall.append(time.perf_counter() - t0)
        t = eng.timings()
        dec.append(t["b64dec"]); sha.append(t["sha"]); tot.append(t["total"])
        ok = ok and bool((st == 0).all())
    eng.set_profiling(False)
    ok = ok and bool(torch.equal(out, files[:F * S]))
    pipe = None
    if args.dl_chunks > 0:
        pipe = pipelined_download(args, eng, files, fd, frd, b64, msp, out, S, N, F, dev)
        ok = ok and pipe.get("ok", False)
    # Raw-fragment reassembly (SN:419-451, fragments fetched as raw bytes,
    # :513-514): gather the fragments of every file (spans of the upload
    # buffer) into `out`, then the fileId re-verify (:454-458).
    from dfs_amd.engine import reassemble_device
    out.zero_()
    lens = np.array(split(S, N), dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    addr = (np.uint64(files.data_ptr()) + file_off[:, None] + offs[None, :]).reshape(-1)
    flen = np.tile(lens, F)
    exp = fd[:F * 32].cpu().numpy().reshape(F, 32)
    reassemble_device(eng, addr, flen, F, N, out.data_ptr(), file_off, exp)
    torch.cuda.synchronize(dev)
    eng.set_profiling(True)
    gat = []
    for _ in range(reps):
        st, _dig = reassemble_device(eng, addr, flen, F, N, out.data_ptr(), file_off, exp)
        gat.append(eng.timings()["gather"])
        ok = ok and bool((st == 0).all())
    eng.set_profiling(False)
    ok = ok and bool(torch.equal(out, files[:F * S]))
    del out
    gat_ms = float(np.mean(gat))
    gat_gbs = 2 * F * S / (gat_ms / 1e3) / 1e9
    dev_ms = float(np.mean(tot))
    dec_ms = float(np.mean(dec))
    dec_bytes = int(msp[:, 1].sum()) + F * S  # Base64 read + bytes written
    log(f"download: {F} files, device {dev_ms:.1f} ms (decode {dec_ms:.1f}, sha {np.mean(sha):.1f}), "
        f"raw gather {gat_ms:.1f} ms, ok={ok}")
    return {"files_per_gpu": F, "device_ms": round(dev_ms, 3), "wall_ms": round(float(np.mean(wall)) * 1e3, 3),
            "gbps": round(F * S / (dev_ms / 1e3) / 1e9, 2),
            "decode_ms": round(dec_ms, 3), "decode_gbs": round(dec_bytes / (dec_ms / 1e3) / 1e9, 1),
            "decode_frac_hbm": round(dec_bytes / (dec_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "sha_ms": round(float(np.mean(sha)), 3),
            "gather_ms": round(gat_ms, 3), "gather_gbs": round(gat_gbs, 1),
            "gather_frac_hbm": round(gat_gbs / HBM_PEAK_GBS, 4), "ok": ok, **({"pipelined": pipe} if pipe else {}),
            "note": "wall_ms includes host-side job planning per call; gbps = file bytes / device time"}


def pipelined_download(args, eng, files, fd, frd, b64, msp, out, S, N, F, dev):
    """Server-style download: the same F files as chunks over two contexts on
    two host threads (two connection handlers, SN:30, sharing a GPU), so one
    chunk's verify SHA-256 runs beside the next chunk's Base64 decode.  The
    second thread starts with a half chunk so the two do not run in lockstep.
    Wall clock over the whole set, host planning included."""
    import threading
    import numpy as np
    import torch
    import dfs_amd
    from dfs_amd.engine import download_device
    K = max(2, args.dl_chunks)
    step = F // K
    bounds = [0, step // 2] + [step // 2 + step * i for i in range(1, K)] + [F]
    bounds = sorted(set(b for b in bounds if 0 <= b <= F))
    chunks = list(zip(bounds[:-1], bounds[1:]))
    file_len = np.full(F, S, dtype=np.uint64)
    file_off = np.arange(F, dtype=np.uint64) * np.uint64(S)
    eng2 = dfs_amd.FragmentEngine(dev.index or 0)
    engines = [eng, eng2]
    ok = [True]

    def run(t):
        for c, (a, b) in enumerate(chunks):
            if c % 2 != t:
                continue
            st = download_device(engines[t], b64.data_ptr(), msp[a * N:b * N], b - a, N, file_len[a:b],
                                 frd.data_ptr() + a * N * 32, fd.data_ptr() + a * 32, out.data_ptr(), file_off[a:b])
            ok[0] = ok[0] and bool((st == 0).all())

    def once():
        ths = [threading.Thread(target=run, args=(t,)) for t in (0, 1)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0

    try:
        once()
        out.zero_()
        torch.cuda.synchronize(dev)
        walls = [once() for _ in range(max(1, args.dl_steps))]
        torch.cuda.synchronize(dev)
        good = ok[0] and bool(torch.equal(out, files[:F * S]))
    finally:
        eng2.close()
    ms = float(np.mean(walls)) * 1e3
    return {"chunks": len(chunks), "contexts": 2, "wall_ms": round(ms, 3),
            "gbps": round(F * S / (ms / 1e3) / 1e9, 2), "ok": good}


def wire_leg(args, eng, files, fd, frd, S, N, F, dev, log):
    """storeFragments request bodies on the device (SN:195-205 + 629-642):
    node 1 (0-based 0) uploads; for each sampled file the N-1 peer bodies
    {"fileId":..,"fragments":[{k},{k+1}]} with the Base64 encoded straight
    from the file bytes into the body.  Timed with HIP events; the first and
    last files are checked byte-for-byte against the oracle's
    buildFragmentsJson.  Returns a dict for the JSON line."""
    import numpy as np
    import torch
    from dfs_amd.engine import store_bodies_layout, store_bodies_device
    R = min(F, args.wire_files)
    spans = np.stack([np.arange(R, dtype=np.uint64) * np.uint64(S), np.full(R, S, dtype=np.uint64)], axis=1)
    body_off = store_bodies_layout(eng, spans, N, 0)
    bodies = torch.empty(int(body_off[-1]) + 16, dtype=torch.uint8, device=dev)

    def once():
        store_bodies_device(eng, files.data_ptr(), spans, N, 0, fd.data_ptr(), bodies.data_ptr(), body_off)

    once()
    torch.cuda.synchronize(dev)
    eng.set_profiling(True)
    tot, enc = [], []
    for _ in range(max(1, args.dl_steps)):
        once()
        t = eng.timings()
        tot.append(t["total"]); enc.append(t["b64enc"])
    eng.set_profiling(False)
    torch.cuda.synchronize(dev)
    ok = True
    if args.verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import hashlib
        import oracle as O  # checker only
        host = None
        for f in sorted({0, R - 1}):
            data = files[f * S:(f + 1) * S].cpu().numpy().tobytes()
            fid = hashlib.sha256(data).hexdigest()
            parts = [data[o:o + n] for o, n in O.py_split(S, N)]
            for j, k in enumerate(range(1, N)):
                want = O.py_build_fragments_json(fid, [(k, parts[k]), (((k + 1) % N), parts[(k + 1) % N])]).encode()
                o = int(body_off[f * (N - 1) + j])
                ok &= bodies[o:o + len(want)].cpu().numpy().tobytes() == want
    # Receiver side (handleInternalStoreFragments, SN:265-293) over the same
    # bodies: device parse, decode of both entries, SHA-256 of each; the
    # digests must equal the upload-time fragment digests (the sender's check,
    # SN:248-257).  Synchronous call, wall-clock timed.
    from dfs_amd.engine import store_receive_device, store_receive_out_bytes
    lens = split(S, N)
    blen = np.array([139 + 4 * ((lens[k] + 2) // 3) + 4 * ((lens[(k + 1) % N] + 2) // 3) for k in range(1, N)],
                    dtype=np.uint64)
    bspans = np.stack([body_off[:-1], np.tile(blen, R)], axis=1)
    rout = torch.empty(store_receive_out_bytes(bspans) + 16, dtype=torch.uint8, device=dev)
    store_receive_device(eng, bodies.data_ptr(), bspans, rout.data_ptr())
    torch.cuda.synchronize(dev)
    rw = []
    for _ in range(max(1, args.dl_steps)):
        t0 = time.perf_counter()
        st, idx, foff, flen, rdig, ids = store_receive_device(eng, bodies.data_ptr(), bspans, rout.data_ptr())
        rw.append(time.perf_counter() - t0)
    frdh = frd[:R * N * 32].view(R, N, 32).cpu().numpy()
    want_idx = np.tile(np.array([[k, (k + 1) % N] for k in range(1, N)], dtype=np.uint32), (R, 1))
    rok = bool((st == 0).all()) and bool((idx == want_idx).all())
    fi = np.repeat(np.arange(R), N - 1)
    rok = rok and bool((rdig == frdh[fi[:, None], want_idx]).all())
    fdh = fd[:R * 32].view(R, 32).cpu().numpy()
    hexes = np.frombuffer(b"".join(fdh[f].tobytes().hex().encode() for f in range(R)), dtype=np.uint8).reshape(R, 64)
    rok = rok and bool((ids == hexes[fi]).all())
    del rout
    recv_ms = float(np.mean(rw)) * 1e3
    body_bytes = int(blen.sum())
    raw_read = sum(lens[k] + lens[(k + 1) % N] for k in range(1, N))
    moved = R * (body_bytes + raw_read)
    ms = float(np.mean(tot))
    log(f"wire: {R} files x {N - 1} storeFragments bodies, {ms:.1f} ms, ok={ok}")
    del bodies
    return {"files": R, "bodies": R * (N - 1), "uploader_node": 1, "ms": round(ms, 3),
            "encode_ms": round(float(np.mean(enc)), 3), "body_gbs": round(R * body_bytes / (ms / 1e3) / 1e9, 1),
            "hbm_gbs": round(moved / (ms / 1e3) / 1e9, 1), "hbm_frac": round(moved / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "ok": bool(ok),
            "receive_wall_ms": round(recv_ms, 3), "receive_body_gbs": round(R * body_bytes / (recv_ms / 1e3) / 1e9, 1),
            "receive_ok": rok,
            "note": "bodies byte-identical to buildFragmentsJson (SN:629-642); hbm_gbs = raw fragment bytes read "
                    "+ body bytes written per second; receive = device parse + decode + SHA-256 of every entry "
                    "(synchronous call, wall clock incl. host job planning), digests == upload-time fragment "
                    "digests"}


def store_leg(args, eng, files, fd, S, N, F, dev, log):
    """On-disk fragment store (SN:147-166 upload save, SN:463-469 local load):
    node 1 (0-based 0) keeps fragments {0, 1} of every sampled file; they go
    HBM -> pinned ring -> <tmp>/node-1/<fileId>/fragments/<i>.frag and back
    into HBM (dfs_store_write_fragments / dfs_store_read_fragments).  The
    read follows the write, so it is a page-cache rate (the box gives no way
    to drop caches).  Checked: every byte read back equals the file bytes."""
    import shutil
    import tempfile
    import numpy as np
    import torch
    from dfs_amd.fragstore import FragmentStore, make_refs
    R = min(F, args.store_files)
    lens = split(S, N)
    offs = [sum(lens[:i]) for i in range(N)]
    keep = (0, 1)  # SN:143-145 for node 1
    off = [f * S + offs[i] for f in range(R) for i in keep]
    ln = [lens[i] for _ in range(R) for i in keep]
    fi = [f for f in range(R) for _ in keep]
    ix = [i for _ in range(R) for i in keep]
    # fileId directory names: the upload's device-computed fileIds
    dig = fd[:R * 32].view(R, 32).cpu().numpy()
    tmp = tempfile.mkdtemp(prefix="dfs_store_")
    try:
        store = FragmentStore(1, tmp, engine=eng)
        refs = make_refs(off, ln, fi, ix)
        # allocate the pinned staging ring outside the timed region (a 1-byte
        # write of fragment 0 of file 0, truncated by the timed write)
        store.write(dig, files.data_ptr(), make_refs([off[0]], [1], [0], [0]),
                    device=True)
        t0 = time.perf_counter()
        st = store.write(dig, files.data_ptr(), refs, device=True)
        t_w = time.perf_counter() - t0
        total = int(sum(ln))
        pos = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
        back = torch.empty(total, dtype=torch.uint8, device=dev)
        rrefs = make_refs(pos, ln, fi, ix)
        t0 = time.perf_counter()
        st2, got = store.read(dig, back.data_ptr(), rrefs, device=True)
        t_r = time.perf_counter() - t0
        want = torch.cat([files[o:o + n] for o, n in zip(off, ln)])
        ok = bool((st == 0).all()) and bool((st2 == 0).all()) and bool((got == np.array(ln)).all()) \
            and bool(torch.equal(want, back))
        del want, back
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    log(f"store: {2 * R} fragments, {total / 1e9:.2f} GB: write {t_w * 1e3:.0f} ms, read {t_r * 1e3:.0f} ms, ok={ok}")
    return {"files": R, "fragments": 2 * R, "bytes": total, "node": 1,
            "write_ms": round(t_w * 1e3, 2), "write_gbs": round(total / t_w / 1e9, 2),
            "read_ms": round(t_r * 1e3, 2), "read_gbs": round(total / t_r / 1e9, 2), "ok": ok,
            "threads": int(os.environ.get("DFS_STORE_THREADS", "0")) or "min(16, cores)",
            "note": "HBM -> pinned staging ring -> <tmp>/node-1/<fileId>/fragments/<i>.frag (raw bytes, "
                    "SN:166) and back (SN:466); wall clock, page cache (no fsync, as Files.write)"}


def long_leg(args):
    """BASELINE configs[3]: files larger than HBM (dfs_amd.streaming).  Every
    chunk: synthesize the files' window on device (stands for bytes arriving
    from the TCP upload, not timed as pipeline work), one SHA-256 update
    launch over all fileId + fragment parts (states carried in HBM), one
    Base64 launch over the fragment parts.  Prints one JSON line."""
    import numpy as np
    import torch
    import dfs_amd
    from dfs_amd.streaming import StreamingUpload, synth_fill_at
    F, S, N, chunk = args.long_files, args.long_size, args.nfrag, args.long_chunk
    dev = torch.device("cuda", 0)
    eng = dfs_amd.FragmentEngine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    up = StreamingUpload(eng, F, S, N, chunk, dev)

    def fill(ptr, lo, hi):
        spans = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(up.stride),
                          np.full(F, hi - lo, dtype=np.uint64)], axis=1)
        synth_fill_at(eng, ptr, spans, 0, SEED, lo)

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    k = up.run(fill)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ok = True
    if args.verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import hashlib
        import oracle as O  # checker only
        for f in sorted({0, F - 1}):
            data = O.c_synth(f, 0, S)
            ok &= up.file_digest(f) == hashlib.sha256(data).digest()
            for i, (o, n) in enumerate(O.py_split(S, N)):
                ok &= up.frag_digest(f, i) == hashlib.sha256(data[o:o + n]).digest()
    dev_s = (k["sha_ms"] + k["b64_ms"]) / 1e3
    lens = split(S, N)
    blocks = F * (sha_blocks(S) + sum(sha_blocks(x) for x in lens))
    tops = blocks * OPS_PER_BLOCK_CANON / (k["sha_ms"] / 1e3) / 1e12
    lanes = F * (N + 1)
    b64_bytes = F * S + 4 * F * sum((x + 2) // 3 for x in lens)
    res = {"metric": METRIC, "value": round(F * S / dev_s / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": 1,
           "warmup": 0, "ms_per_step": round(dev_s * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic (splitmix64, seed 0x5EED5EED), generated on "
           "device chunk by chunk",
           "config": {"workload": f"long-fragment skew (BASELINE configs[3]): {F} files x {S} B, N={N}, streamed "
                                  f"in {up.sched.nchunks} chunks of {chunk} B per file", "files": F,
                      "file_bytes": S, "nfrag": N, "chunk": chunk},
           "roofline": {"bound": "valu (lane-limited)", "achieved": round(tops, 3), "peak": round(VALU_PEAK_TOPS, 3),
                        "unit": "Tops/s (int32)", "frac": round(tops / VALU_PEAK_TOPS, 4), "kernel": "sha256_lanes",
                        "ms": round(k["sha_ms"], 3), "lanes": lanes, "lane_occupancy": round(lanes / 65536, 4),
                        "note": "one message per lane and SHA-256 is sequential within a message: the fileId "
                                "chains (4.19M blocks each) bound the run"},
           "roofline_b64": {"bound": "hbm", "ms": round(k["b64_ms"], 3),
                            "achieved": round(b64_bytes / (k["b64_ms"] / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s"},
           "wall_ms_incl_synth": round(wall * 1e3, 3), "verified": bool(ok)}
    print(json.dumps(res), flush=True)
    eng.close()


def main():
    args = parse()
    if args.config == 4:
        return long_leg(args)
    if args.serial:
        args.mode = "serial"
    # read by dfs_open: two-kernel mode vs the fused SHA+Base64 kernel
    os.environ["DFS_UPLOAD_MODE"] = "kernels" if args.mode != "fused" else "fused"
    import numpy as np
    import torch
    import torch.distributed as dist
    import dfs_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # A stuck exchange in the side legs must raise (and be reported in the
        # JSON line) rather than hang or abort the job: blocking waits with a
        # bounded timeout, communicator cleanup without process teardown.
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        import datetime
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=240))
    dev = torch.device("cuda", local if world > 1 else 0)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    S, N, F = args.file_size, args.nfrag, args.files
    eng = dfs_amd.FragmentEngine(dev.index)
    spans = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(S), np.full(F, S, dtype=np.uint64)], axis=1)
    first_file = rank * F  # this rank's shard of the global file set
    files = torch.empty(F * S + 64, dtype=torch.uint8, device=dev)
    dfs_amd.synth_fill(eng, files.data_ptr(), spans, first_file, SEED)
    plan = dfs_amd.UploadPlan(eng, spans, N, align128=args.align128)
    fd = torch.empty(F * 32, dtype=torch.uint8, device=dev)
    frd = torch.empty(F * N * 32, dtype=torch.uint8, device=dev)
    b64 = torch.empty(plan.b64_total, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    flags = dfs_amd.DFS_SERIAL if args.mode == "serial" else 0
    torch.cuda.synchronize(dev)
    log(f"rank0: {F} files x {S} B, N={N}, b64 {plan.b64_total / 1e9:.2f} GB, world {world}")

    for _ in range(args.warmup):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
    torch.cuda.synchronize(dev)

    # ---- timed region ---------------------------------------------------------
    eng.set_profiling(True)
    sha_ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
        t = eng.timings()  # waits on this step's last HIP event; per-kernel ms
        sha_ms.append(t["sha"])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- fragment-only variant: the same step without the fileId
    # SHA-256 (SN:127), e.g. for a caller that already knows the content address.
    frag_only = None
    if args.frag_only_steps:
        eng.set_profiling(True)
        fo_ms, fo_sha = [], []
        for _ in range(args.frag_only_steps):
            plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags | dfs_amd.DFS_NO_FILEID)
            t = eng.timings()
            fo_ms.append(t["total"]); fo_sha.append(t["sha"])
        eng.set_profiling(False)
        fo = float(np.mean(fo_ms))
        frag_only = {"ms_per_step": round(fo, 3), "gbps": round(F * S / (fo / 1e3) / 1e9, 3),
                     "sha_ms": round(float(np.mean(fo_sha)), 3),
                     "note": "fragment SHA-256 + Base64 only (no fileId SHA-256), HIP-event device time, this GPU"}

    # ---- the HBM-bound Base64 encode pass alone (roofline_b64) -----------------
    # Outside the timed steps (in the default fused mode the upload writes the
    # Base64 from the SHA kernel); same plan, same buffers, own HIP events.
    eng.set_profiling(True)
    b64_ms = []
    for _ in range(max(1, args.b64_steps)):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), dfs_amd.DFS_B64_ONLY)
        b64_ms.append(eng.timings()["b64enc"])
    eng.set_profiling(False)
    torch.cuda.synchronize(dev)

    # ---- spot-check against the oracle (outside the timed region) -------------
    ok = True
    if rank == 0 and args.verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # checker only
        idx = sorted(set([0, F - 1] + list(np.random.default_rng(1).integers(0, F, args.verify))))
        bsp = plan.b64_spans([S] * F)
        fdh = fd.view(F, 32).cpu().numpy()
        frdh = frd.view(F, N, 32).cpu().numpy()
        for f in idx:
            data = O.c_synth(first_file + f, 0, S)
            efd, efrd, eb64, eoff = O.c_upload_batch([data], N)
            k0 = f * N
            got_b64 = b"".join(b64[int(o):int(o + n)].cpu().numpy().tobytes() for o, n in bsp[k0:k0 + N])
            if not ((fdh[f] == efd[0]).all() and (frdh[f] == efrd[0]).all() and got_b64 == eb64):
                ok = False
        log(f"oracle spot-check of {len(idx)} files: {'OK' if ok else 'MISMATCH'}")

    # ---- numbers -----------------------------------------------------------------
    total_bytes = F * S * world * args.steps  # file bytes all ranks pushed through the timed steps
    value = total_bytes / elapsed / 1e9
    lens = split(S, N)
    blocks = F * (sha_blocks(S) + sum(sha_blocks(x) for x in lens))
    sha_avg = float(np.mean(sha_ms)) / 1e3
    b64_avg = float(np.mean(b64_ms)) / 1e3
    achieved_tops = blocks * OPS_PER_BLOCK_CANON / sha_avg / 1e12
    issued_tops = blocks * OPS_PER_BLOCK_ISSUED / sha_avg / 1e12
    b64_bytes = F * S + 4 * F * sum((x + 2) // 3 for x in lens)  # read + Base64 written
    b64_gbs = b64_bytes / b64_avg / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("workload") == f"{F}x{S}/N{N}":
                traffic = pmc.get("sha_hbm_bytes_per_launch")
        except Exception:
            traffic = None
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64, seed 0x5EED5EED), resident in HBM",
        "config": {"workload": f"upload: {F} files x {S} B per GPU, N={N} fragments: fileId SHA-256 + "
                               f"fragment SHA-256 + fragment Base64",
                   "files_per_gpu": F, "file_bytes": S, "nfrag": N,
                   "mode": {"fused": "Base64 fused into the SHA-256 fragment lanes (one kernel)",
                            "kernels": "SHA-256 || Base64 kernels on two streams",
                            "serial": "SHA-256 then Base64 kernel, one stream"}[args.mode],
                   "b64_layout": "128-byte aligned fragment starts" if args.align128 else "packed"},
        "roofline": {"bound": "valu", "achieved": round(achieved_tops, 3), "peak": round(VALU_PEAK_TOPS, 3),
                     "unit": "Tops/s (int32)", "frac": round(achieved_tops / VALU_PEAK_TOPS, 4),
                     "traffic": traffic, "kernel": "sha256_lanes" + (" (+ fused Base64)" if args.mode == "fused" else ""),
                     "ms": round(sha_avg * 1e3, 3),
                     "blocks_per_launch": blocks, "ops_per_block": OPS_PER_BLOCK_CANON,
                     "valu_issue_frac": round(issued_tops / VALU_PEAK_TOPS, 4)},
        "roofline_b64": {"bound": "hbm", "achieved": round(b64_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(b64_gbs / HBM_PEAK_GBS, 4), "kernel": "b64_encode_kernel",
                         "ms": round(b64_avg * 1e3, 3), "bytes_per_launch": b64_bytes,
                         "note": "standalone encode pass over the same fragments (DFS_B64_ONLY), outside "
                                 "the timed steps"},
        "verified": ok,
    }
    if frag_only:
        result["fragment_only"] = frag_only
    if not args.no_download:
        try:
            result["download"] = download_leg(args, eng, files, plan, fd, frd, b64, S, N, F, dev, log)
        except Exception as e:
            result["download"] = {"error": repr(e)[:300]}
    if not args.no_wire:
        try:
            result["wire"] = wire_leg(args, eng, files, fd, frd, S, N, F, dev, log)
        except Exception as e:
            result["wire"] = {"error": repr(e)[:300]}
    if not args.no_store:
        try:
            result["store"] = store_leg(args, eng, files, fd, S, N, F, dev, log)
        except Exception as e:
            result["store"] = {"error": repr(e)[:300]}
    if world > 1 and not args.no_replicate:
        # The upload's Base64 (91.6 GB at config 2) is not needed any more: free
        # it so the placement buffers (held groups of every rank, all-to-all
        # send / receive copies) fit beside the files in HBM.
        b64 = None
        torch.cuda.empty_cache()
        try:
            result["replication"] = replication_leg(args, eng, files, S, N, dev, log)
        except Exception as e:  # never lose the main line to the side measurement
            result["replication"] = {"error": repr(e)[:300]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, log)
    if rank == 0:
        print(json.dumps(result), flush=True)
    plan.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
