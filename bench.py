#!/usr/bin/env python3
"""bench.py — StorageNode upload fragment pipeline on MI355X (BASELINE.json metric).

One step = one pass of handleUpload's fragment pipeline (StorageNode.java
:118-189) over one batch of synthetic files resident in HBM: fileId SHA-256
(:127), N-way split (:138-157), per-fragment SHA-256 (:159) and the Base64 of
every fragment (:636) — all in the gfx950 kernels of libdfsgpu.so — and, on
N > 1 GPUs, the replica placement of that Base64 (sendFragmentsToPeers,
:195-224) over RCCL / xGMI.

Workloads (BASELINE.json configs):
  N = 1  configs[1]: 65,536 files x 1 MiB, N = 5 fragments (default).
  N > 1  configs[2]: its per-GPU shard, 131,072 files x 256 KiB, N = 8
         fragments per GPU (1M files on 8 GPUs), node k hosted by GPU k mod W.
         The step is upload + placement: the files are processed in chunks
         and chunk c's placement runs on a comm stream beside chunk c+1's
         hashing (--placement star: the reference's own fan-out as one
         all-to-all; ring: primary scatter + replica step g -> g-1).
`python bench.py --gpus N` launches its own N ranks (torch.distributed.run)
when WORLD_SIZE is not set; rank 0 prints ONE JSON line and the exit code is
non-zero if any leg failed or mismatched.  `--gpus N --comm host --files F`
rehearses the N > 1 step with N rank processes on fewer GPUs (the library's
host-staged communicator instead of RCCL): a functional check, the line says so.

Extra objects on the line:
  roofline      dominant kernel (multi-message SHA-256) vs the int32-VALU peak,
                timed with HIP events on its own stream inside the timed loop
  roofline_b64  the Base64 encode kernel vs the HBM peak
  cpu_baseline  CPU restatement (OpenSSL SHA-NI SHA-256 + scalar Base64, one
                file per thread) on a bounded sample, rank 0, N = 1 only;
                `download` inside it: the download path on the CPU
  download      handleDownload over the same files: Base64 decode into place +
                fragment / fileId SHA-256 verify, and the raw-fragment gather
  wire          storeFragments request bodies built on the device, then
                received (parse + decode + SHA-256) on the device
  store         on-disk fragment store: node 1's fragments HBM -> disk -> HBM
  placement     N > 1: ring and star xGMI rates, compute-only rate, the
                degraded read (config 5: last GPU offline, fetch + decode +
                verify + reassembly)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))

METRIC = "SHA-256+Base64 fragment GB/s per node at 1/8 GPUs; % of int-VALU peak"
SEED = 0x5EED5EED
# Canonical int32 VALU ops per 64-byte SHA-256 block, the count the roofline is priced with (gfx950
# ISA without v_xor3).  The shipped kernel issues 1,405 (v_bitop3 folds the
# three-input XORs), so `frac` below is algorithmic, not issue utilisation;
# `valu_issue_frac` gives the executed-instruction view.
OPS_PER_BLOCK_CANON = 1688
OPS_PER_BLOCK_ISSUED = 1405
# Peaks: MI355X_MICROARCH.md — 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32
# (the FP32 vector rate without FMA doubling), HBM 8 TB/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0


class LegError(RuntimeError):
    pass


def sha_blocks(n: int) -> int:
    return n // 64 + (1 if n % 64 < 56 else 2)


def split(S: int, N: int):
    base, rem = divmod(S, N)
    return [base + (1 if i < rem else 0) for i in range(N)]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=0, choices=(0, 2, 3, 4),
                    help="0 (default): configs[1] at N=1, configs[2]'s per-GPU shard at N>1; 2: BASELINE "
                         "configs[1]; 3: configs[2]'s per-GPU shard (131,072 x 256 KiB, N=8); 4: configs[3], the "
                         "long-fragment skew (1,024 x 256 MiB, N=5) streamed through HBM, its own JSON line")
    ap.add_argument("--files", type=int, default=0, help="files per GPU (0 = the config's)")
    ap.add_argument("--file-size", type=int, default=0)
    ap.add_argument("--nfrag", type=int, default=0)
    ap.add_argument("--mode", choices=("fused", "kernels", "serial", "hybrid"), default="kernels",
                    help="kernels: SHA and Base64 kernels on two streams (default); fused: Base64 "
                         "written by the SHA fragment lanes; hybrid: the fragment lanes write their own Base64, the "
                         "encode kernel only that of the fragments hashed as twins inside their fileId lane; serial: "
                         "the two kernels on one stream")
    ap.add_argument("--serial", action="store_true", help="alias of --mode serial")
    ap.add_argument("--align128", action=argparse.BooleanOptionalAction, default=True,
                    help="DFS_LAYOUT_ALIGN128: every fragment's Base64 starts on a 128-byte boundary")
    ap.add_argument("--b64-steps", type=int, default=3, help="steps of the standalone Base64 leg")
    ap.add_argument("--frag-only-steps", type=int, default=3, help="steps of the fragment-only (no fileId) leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work (upload leg)")
    ap.add_argument("--verify", type=int, default=8,
                    help="files whose Base64 text is compared byte by byte with the oracle's (0: no verification at all)")
    ap.add_argument("--verify-all", action=argparse.BooleanOptionalAction, default=True,
                    help="check EVERY file of the timed batch against the oracle's C path: every fileId, every "
                         "fragment digest, and every fragment's Base64 through its SHA-256 (outside the timed region)")
    ap.add_argument("--placement", choices=("star", "ring"), default="star",
                    help="N>1: placement inside the timed step (the other one is timed beside it)")
    ap.add_argument("--comm", choices=("rccl", "host"), default="rccl",
                    help="N > 1 transport: RCCL over xGMI (one rank per GPU), or 'host': the library's host-staged "
                         "communicator (shared-memory mailboxes, synchronous) with rank r on GPU r mod <GPUs present> "
                         "- a functional rehearsal of the N > 1 step on fewer GPUs than ranks, never a measurement")
    ap.add_argument("--chunks", type=int, default=2,
                    help="N>1: file chunks pipelined through compute + placement (2: 65,536-file launches keep the "
                         "SHA twin lanes; chunk c of step k+1 waits only for chunk c's placement of step k)")
    ap.add_argument("--placement-step", action="store_true",
                    help="run the N>1 step (upload + RCCL placement, degraded read) at N=1 too: a one-rank "
                         "communicator, every node on this GPU (checks that code path on a one-GPU box)")
    ap.add_argument("--no-download", action="store_true", help="skip the download/verify leg")
    ap.add_argument("--dl-steps", type=int, default=2)
    ap.add_argument("--wire-files", type=int, default=16384, help="files in the storeFragments body leg")
    ap.add_argument("--no-wire", action="store_true", help="skip the storeFragments body leg")
    ap.add_argument("--store-files", type=int, default=2048, help="files in the on-disk fragment store leg")
    ap.add_argument("--no-store", action="store_true", help="skip the on-disk fragment store leg")
    ap.add_argument("--no-batcher", action="store_true", help="skip the concurrent-clients (batcher) leg")
    ap.add_argument("--no-rehearsal", action="store_true",
                    help="skip the 8-rank rehearsal of the N > 1 step on this GPU (host-staged communicator; part of "
                         "the scaling-reference leg, so --no-scaling-ref skips it too)")
    ap.add_argument("--no-scaling-ref", action="store_true",
                    help="N=1: skip the leg that runs the N>1 step (upload + placement + holders' verify on BASELINE "
                         "configs[2]'s shard) on this one GPU, the equal-workload reference for the N>1 lines")
    ap.add_argument("--clients", default="1,512,2048,4096", help="batcher leg: concurrent handler threads")
    ap.add_argument("--client-seconds", type=float, default=2.0, help="batcher leg: seconds per concurrency")
    ap.add_argument("--long-files", type=int, default=1024)
    ap.add_argument("--long-size", type=int, default=256 << 20)
    ap.add_argument("--long-chunk", type=int, default=192 * 87381, help="bytes per file per chunk (x192)")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check without a GPU (gloo, CPU tensors): launcher, rendezvous, timing and the "
                         "placement schedules; prints a line marked dry_run, never a measurement")
    return ap.parse_args(argv)


def resolve_config(args, world: int) -> None:
    cfg = args.config or (2 if world == 1 and not args.placement_step else 3)
    args.config = cfg
    if cfg == 3:  # BASELINE configs[2]: 1M files x 256 KiB sharded by file over 8 GPUs, N = 8
        F, S, N = 131072, 256 << 10, 8
        args.wire_files = min(args.wire_files, 65536)
    else:
        F, S, N = 65536, 1 << 20, 5
    args.files = args.files or F
    args.file_size = args.file_size or S
    args.nfrag = args.nfrag or N


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_RESULT_OUT = None


def emit(obj) -> None:
    """The run's one JSON line, on the original stdout (see main)."""
    out = _RESULT_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def relaunch(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks (one per GPU) with
    torch.distributed.run as a child process.  Runs before this process
    touches the GPU; returns the child's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle's C restatement on the host cores
# ---------------------------------------------------------------------------
def host_cpu_info():
    """Cores this process may use and what they are: nproc (the machine),
    the affinity set, the cgroup CPU quota (a GPU box gives a process a
    share of the machine), the lscpu model name."""
    info = {"nproc": os.cpu_count()}
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    info["affinity"] = aff
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    info["cgroup_cpu_quota"] = quota
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    info["model"] = model
    # physical cores lscpu reports (sockets x cores per socket): the box may
    # show only its share of the machine
    try:
        sockets = cores_per = None
        for line in out.splitlines():
            if line.startswith("Socket(s)"):
                sockets = int(line.split(":", 1)[1])
            elif line.startswith("Core(s) per socket"):
                cores_per = int(line.split(":", 1)[1])
        info["physical_cores"] = sockets * cores_per if sockets and cores_per else None
    except (NameError, ValueError):
        info["physical_cores"] = None
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return info, usable


def cpu_baseline(args, log):
    """Oracle leg: C restatement on the host cores, bounded sample, on every
    core this process may use (one file per thread, thread-per-connection
    SN:30), plus one connection handler alone and the download path."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure, checker/baseline only)
    info, threads = host_cpu_info()
    S, N = args.file_size, args.nfrag
    secs, _, _ = O.cpu_upload_bench(2 * threads, S, N, threads, use_openssl=True)
    kind_sha = "openssl"
    if secs < 0:
        secs, _, _ = O.cpu_upload_bench(2 * threads, S, N, threads, use_openssl=False)
        kind_sha = "scalar"
    ossl = kind_sha == "openssl"
    per_file = max(secs, 1e-6) / 2.0  # seconds per file per thread
    nfiles = int(max(threads, min(400000, args.cpu_seconds / per_file * threads)))
    secs, _, _ = O.cpu_upload_bench(nfiles, S, N, threads, use_openssl=ossl)
    if secs <= 0:
        raise LegError(f"cpu upload baseline failed ({secs})")
    gbs = nfiles * S / secs / 1e9
    log(f"cpu baseline: {nfiles} files x {S} B on {threads} threads ({info}): {secs:.2f} s -> {gbs:.3f} GB/s")
    n1 = int(max(1, min(20000, 3.0 / per_file)))
    secs1, _, _ = O.cpu_upload_bench(n1, S, N, 1, use_openssl=ossl)
    gbs1 = n1 * S / secs1 / 1e9
    # download path: decode + fragment verify + ordered append + fileId verify
    d_cal = O.cpu_download_bench(threads, S, N, threads, ossl)
    if d_cal <= 0:
        raise LegError(f"cpu download baseline failed ({d_cal})")
    nd = int(max(threads, min(400000, 0.5 * args.cpu_seconds / max(d_cal, 1e-6) * threads)))
    d_secs = O.cpu_download_bench(nd, S, N, threads, ossl)
    if d_secs <= 0:
        raise LegError(f"cpu download baseline failed ({d_secs})")
    d_gbs = nd * S / d_secs / 1e9
    log(f"cpu baseline download: {nd} files on {threads} threads: {d_secs:.2f} s -> {d_gbs:.3f} GB/s")
    sha_txt = "OpenSSL SHA256 (SHA-NI), approximating the HotSpot intrinsic" if ossl else "scalar C SHA-256"
    return {"value": round(gbs, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{nfiles} synthetic files x {S} B, N={N}: fileId + fragment SHA-256 ({sha_txt}) + scalar "
                      f"Base64, one file per thread (thread-per-connection, SN:30), {threads} threads; CPU proxy, "
                      f"not Java (no JDK on the box)",
            "host": info, "seconds": round(secs, 3),
            "single_thread_value": round(gbs1, 4), "single_thread_files": n1,
            "download": {"value": round(d_gbs, 4), "unit": "GB/s", "cores": threads, "files": nd,
                         "seconds": round(d_secs, 3),
                         "sample": "per file: table-driven Base64 decode of each fragment (SN:281), SHA-256 vs the "
                                   "upload digest (SN:282, 250-257), ordered append (SN:448), SHA-256 vs fileId "
                                   "(SN:454); same files, one file per thread"}}


# ---------------------------------------------------------------------------
# Side legs (N = 1)
# ---------------------------------------------------------------------------
def download_leg(args, eng, files, plan, fd, frd, b64, S, N, F, dev, log):
    """handleDownload's verify path (SN:399-461) plus north_star's per-fragment
    check, over this GPU's whole upload: Base64-decode every fragment straight
    into its file offset (fused gather, SN:448-451), per-fragment SHA-256 vs the
    upload-time digests, fileId SHA-256 re-verify (SN:454-458) — one
    dfs_download_batch on device buffers."""
    import numpy as np
    import torch
    import dfs_amd
    from dfs_amd.engine import download_device, reassemble_device
    msp = plan.b64_spans([S] * F)
    file_len = np.full(F, S, dtype=np.uint64)
    file_off = np.arange(F, dtype=np.uint64) * np.uint64(S)
    out = torch.empty(F * S, dtype=torch.uint8, device=dev)
    reps = max(1, args.dl_steps)
    # the per-call entry point once (its wall clock includes the host planning) ...
    t0 = time.perf_counter()
    st0 = download_device(eng, b64.data_ptr(), msp, F, N, file_len, frd.data_ptr(), fd.data_ptr(), out.data_ptr(),
                          file_off)
    batch_wall = time.perf_counter() - t0
    # ... then the prepared plan: tables built once, kept in HBM
    t0 = time.perf_counter()
    dplan = dfs_amd.DownloadPlan(eng, msp, F, N, file_len, file_off)
    dl_plan_ms = (time.perf_counter() - t0) * 1e3

    def once():
        return dplan.run(b64.data_ptr(), frd.data_ptr(), fd.data_ptr(), out.data_ptr())

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
    ok = ok and bool((st0 == 0).all()) and bool(torch.equal(out, files[:F * S]))
    dplan.close()
    redo = eng.stats()["ovl_redo"]
    # The same download with the decode alone, then one SHA launch
    # (DFS_DOWNLOAD_MODE=serial on a second ctx): the decode kernel's
    # standalone HBM rate, and the serial device time beside the default's.
    os.environ["DFS_DOWNLOAD_MODE"] = "serial"
    try:
        eng_s = dfs_amd.FragmentEngine(eng.device)
    finally:
        del os.environ["DFS_DOWNLOAD_MODE"]
    s_dec, s_sha, s_tot = [], [], []
    try:
        download_device(eng_s, b64.data_ptr(), msp, F, N, file_len, frd.data_ptr(), fd.data_ptr(), out.data_ptr(),
                        file_off)
        eng_s.set_profiling(True)
        for _ in range(reps):
            st = download_device(eng_s, b64.data_ptr(), msp, F, N, file_len, frd.data_ptr(), fd.data_ptr(),
                                 out.data_ptr(), file_off)
            t = eng_s.timings()
            s_dec.append(t["b64dec"]); s_sha.append(t["sha"]); s_tot.append(t["total"])
            ok = ok and bool((st == 0).all())
    finally:
        eng_s.close()
    ok = ok and bool(torch.equal(out, files[:F * S]))
    # Raw-fragment reassembly (SN:419-451, fragments fetched as raw bytes,
    # :513-514): gather the fragments of every file into `out`, then the
    # fileId re-verify (:454-458).
    out.zero_()
    lens = np.array(split(S, N), dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    addr = (np.uint64(files.data_ptr()) + file_off[:, None] + offs[None, :]).reshape(-1)
    flen = np.tile(lens, F)
    exp = fd[:F * 32].cpu().numpy().reshape(F, 32)
    reassemble_device(eng, addr, flen, F, N, out.data_ptr(), file_off, exp)
    torch.cuda.synchronize(dev)
    eng.set_profiling(True)
    gat, rtot = [], []
    for _ in range(reps):
        st, _dig = reassemble_device(eng, addr, flen, F, N, out.data_ptr(), file_off, exp)
        t = eng.timings()
        gat.append(t["gather"]); rtot.append(t["total"])
        ok = ok and bool((st == 0).all())
    eng.set_profiling(False)
    ok = ok and bool(torch.equal(out, files[:F * S]))
    # the same reassembly gather-then-SHA (serial ctx): the gather kernel's
    # standalone rate and the serial time beside the default's
    os.environ["DFS_DOWNLOAD_MODE"] = "serial"
    try:
        eng_s = dfs_amd.FragmentEngine(eng.device)
    finally:
        del os.environ["DFS_DOWNLOAD_MODE"]
    s_gat, s_rtot = [], []
    try:
        out.zero_()
        torch.cuda.synchronize(dev)  # torch's stream; the library runs on the engine's
        reassemble_device(eng_s, addr, flen, F, N, out.data_ptr(), file_off, exp)
        eng_s.set_profiling(True)
        for _ in range(reps):
            st, _dig = reassemble_device(eng_s, addr, flen, F, N, out.data_ptr(), file_off, exp)
            t = eng_s.timings()
            s_gat.append(t["gather"]); s_rtot.append(t["total"])
            ok = ok and bool((st == 0).all())
    finally:
        eng_s.close()
    ok = ok and bool(torch.equal(out, files[:F * S]))
    redo = eng.stats()["ovl_redo"]
    del out
    gat_ms = float(np.mean(s_gat))  # standalone gather (serial ctx)
    gat_gbs = 2 * F * S / (gat_ms / 1e3) / 1e9
    dev_ms = float(np.mean(tot))
    dec_ms = float(np.mean(s_dec))  # standalone decode (serial ctx)
    dec_bytes = int(msp[:, 1].sum()) + F * S  # Base64 read + bytes written
    log(f"download: {F} files, device {dev_ms:.1f} ms (decode span {np.mean(dec):.1f}, sha span {np.mean(sha):.1f}); "
        f"serial {np.mean(s_tot):.1f} ms (decode {dec_ms:.1f}, sha {np.mean(s_sha):.1f}); raw reassembly + verify "
        f"{np.mean(rtot):.1f} ms (serial {np.mean(s_rtot):.1f}, gather {gat_ms:.1f}), "
        f"ok={ok}, redo={redo}")
    if not ok:
        raise LegError("download leg: status or bytes differ")
    if redo:
        raise LegError(f"download leg: {redo} decode-ahead SHA launches redone (in-kernel wait timed out)")
    return {"files_per_gpu": F, "mode": "overlap: fragment 0 decoded, then fragments 1.. decoded beside one "
                                        "SHA-256 launch that waits per fragment group",
            "device_ms": round(dev_ms, 3), "wall_ms": round(float(np.mean(wall)) * 1e3, 3),
            "plan_ms": round(dl_plan_ms, 2), "batch_call_wall_ms": round(batch_wall * 1e3, 3),
            "gbps": round(F * S / (dev_ms / 1e3) / 1e9, 2),
            "decode_span_ms": round(float(np.mean(dec)), 3), "sha_span_ms": round(float(np.mean(sha)), 3),
            "serial": {"device_ms": round(float(np.mean(s_tot)), 3), "decode_ms": round(dec_ms, 3),
                       "sha_ms": round(float(np.mean(s_sha)), 3)},
            "decode_ms": round(dec_ms, 3), "decode_gbs": round(dec_bytes / (dec_ms / 1e3) / 1e9, 1),
            "decode_frac_hbm": round(dec_bytes / (dec_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "sha_ms": round(float(np.mean(s_sha)), 3),
            "reassemble_ms": round(float(np.mean(rtot)), 3), "reassemble_serial_ms": round(float(np.mean(s_rtot)), 3),
            "gather_ms": round(gat_ms, 3), "gather_gbs": round(gat_gbs, 1),
            "gather_frac_hbm": round(gat_gbs / HBM_PEAK_GBS, 4), "ok": ok, "ovl_redo": redo,
            "note": "device_ms / wall_ms: dfs_download_plan_run (tables prebuilt in HBM, plan_ms once per shape); "
                    "batch_call_wall_ms: one dfs_download_batch call, which plans on the host every time; gbps = file "
                    "bytes / device time; decode_* "
                    "and sha_ms are the standalone kernels of the serial run; reassemble = the reference's raw-fragment "
                    "download (SN:419-458: ordered gather + fileId verify), gather fragment by fragment beside the "
                    "fileId SHA-256 (serial: gather, then SHA)"}


def wire_leg(args, eng, files, fd, frd, S, N, F, dev, log):
    """storeFragments request bodies on the device (SN:195-205 + 629-642):
    node 1 (0-based 0) uploads; for each sampled file the N-1 peer bodies
    {"fileId":..,"fragments":[{k},{k+1}]} with the Base64 encoded straight
    from the file bytes into the body; then received on the device."""
    import numpy as np
    import torch
    from dfs_amd.engine import (store_bodies_device, store_bodies_layout, store_receive_device,
                                store_receive_out_bytes)
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
        for f in sorted({0, R - 1}):
            data = files[f * S:(f + 1) * S].cpu().numpy().tobytes()
            fid = hashlib.sha256(data).hexdigest()
            parts = [data[o:o + n] for o, n in O.py_split(S, N)]
            for j, k in enumerate(range(1, N)):
                want = O.py_build_fragments_json(fid, [(k, parts[k]), (((k + 1) % N), parts[(k + 1) % N])]).encode()
                o = int(body_off[f * (N - 1) + j])
                ok &= bodies[o:o + len(want)].cpu().numpy().tobytes() == want
    # Receiver side (handleInternalStoreFragments, SN:265-293) over the same
    # bodies; the digests must equal the upload-time fragment digests (the
    # sender's check, SN:248-257).  Synchronous call, wall-clock timed.
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
    log(f"wire: {R} files x {N - 1} storeFragments bodies, {ms:.1f} ms, ok={ok}, receive ok={rok}")
    del bodies
    if not (ok and rok):
        raise LegError(f"wire leg: bodies ok={ok} receive ok={rok}")
    return {"files": R, "bodies": R * (N - 1), "uploader_node": 1, "ms": round(ms, 3),
            "encode_ms": round(float(np.mean(enc)), 3), "body_gbs": round(R * body_bytes / (ms / 1e3) / 1e9, 1),
            "hbm_gbs": round(moved / (ms / 1e3) / 1e9, 1), "hbm_frac": round(moved / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "ok": bool(ok), "receive_wall_ms": round(recv_ms, 3),
            "receive_body_gbs": round(R * body_bytes / (recv_ms / 1e3) / 1e9, 1), "receive_ok": rok,
            "receive_one_pass_calls": eng.stats()["recv_one_pass"],
            "note": "bodies byte-identical to buildFragmentsJson (SN:629-642); hbm_gbs = raw fragment bytes read "
                    "+ body bytes written per second; receive = device parse + decode + SHA-256 of every entry "
                    "(synchronous call, wall clock incl. host job planning), digests == upload-time fragment "
                    "digests"}


def store_leg(args, eng, files, fd, S, N, F, dev, log):
    """On-disk fragment store (SN:147-166 upload save, SN:463-469 local load):
    node 1 (0-based 0) keeps fragments {0, 1} of every sampled file; they go
    HBM -> pinned ring -> <tmp>/node-1/<fileId>/fragments/<i>.frag and back
    into HBM.  The read follows the write, so it is a page-cache rate."""
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
    dig = fd[:R * 32].view(R, 32).cpu().numpy()
    tmp = tempfile.mkdtemp(prefix="dfs_store_")
    try:
        store = FragmentStore(1, tmp, engine=eng)
        refs = make_refs(off, ln, fi, ix)
        store.write(dig, files.data_ptr(), make_refs([off[0]], [1], [0], [0]), device=True)  # staging ring alloc
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
    if not ok:
        raise LegError("store leg: status or bytes differ")
    return {"files": R, "fragments": 2 * R, "bytes": total, "node": 1,
            "write_ms": round(t_w * 1e3, 2), "write_gbs": round(total / t_w / 1e9, 2),
            "read_ms": round(t_r * 1e3, 2), "read_gbs": round(total / t_r / 1e9, 2), "ok": ok,
            "threads": int(os.environ.get("DFS_STORE_THREADS", "0")) or "min(16, cores)",
            "note": "HBM -> pinned staging ring -> <tmp>/node-1/<fileId>/fragments/<i>.frag (raw bytes, "
                    "SN:166) and back (SN:466); wall clock, page cache (no fsync, as Files.write)"}


def batcher_leg(args, log):
    """Thread-per-connection clients (SN:28-31), one 1 MiB file per request,
    through the library's batcher (dfs_submit_upload / dfs_submit_download,
    host buffers: PCIe in and out) at each concurrency in --clients, closed
    loop for --client-seconds, in four buffer modes: "staged" (pageable
    handler buffers: each handler copies its bytes into and out of the
    worker's pinned staging), "pinned" (handler buffers from
    dfs_host_alloc: the worker's DMA reads / writes them, no host copies) and
    "view" (pinned inputs; the answer stays in the batch's pinned result
    buffer and the handler gets a pointer: dfs_submit_*_view, one DMA out per
    batch instead of one per request) and "staged_view" (pageable inputs
    copied into the staging, the answer as a view: one DMA each way).
    The clients are native threads (tools/batcher_load, a child process); the
    fileIds it reports are checked here.  Beside it the CPU proxy at the same
    concurrency (min(C, cores) threads, one file per thread), upload and
    download."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker + cpu_baseline leg only
    S, N = 1 << 20, 5
    tool = os.path.join(ROOT, "tools", "batcher_load")
    _, cores = host_cpu_info()
    want = [hashlib.sha256(O.c_synth(f, 0, S)).hexdigest() for f in (0, 1)]
    rows, ok, cpu_one = [], True, None
    for C in [int(x) for x in args.clients.split(",") if x]:
        row = {"clients": C}
        for pinned in (0, 1, 2, 3):
            for kind in ("upload", "download"):
                p = subprocess.run([tool, str(C), str(args.client_seconds), kind, str(S), str(N), "2000", "3",
                                    str(pinned)], capture_output=True, text=True, timeout=300)
                if p.returncode != 0:
                    raise LegError(f"batcher_load {C} {kind} pinned={pinned}: rc {p.returncode}: {p.stderr[-300:]} "
                                   f"{p.stdout[-300:]}")
                r = json.loads(p.stdout.strip().splitlines()[-1])
                ok &= r["ok"] and [r["file0_id"], r["file1_id"]] == want
                key = kind + ("", "_pinned", "_view", "_staged_view")[pinned]
                row[key] = {k: r[k] for k in ("requests", "gbps", "p50_ms", "p99_ms")}
                st = r["stats"]
                row[key]["batches"] = st["batches"]
                row[key]["direct"] = st["direct"]
                if pinned >= 2:
                    row[key]["views"] = st["views"]
                row[key]["mean_batch"] = round(st["requests"] / max(st["batches"], 1), 1)
                row[key]["device_ms_per_batch"] = round(st["device_s"] / max(st["batches"], 1) * 1e3, 2)
                row[key]["client_cpu_us_per_req"] = round(r["client_cpu_us_per_req"]["in_submit"], 1)
                row[key]["cgroup_throttled_s"] = r["throttled_s"]
                log(f"batcher: {C} clients {key}: {r['gbps']} GB/s p50 {r['p50_ms']} ms")  # progress per run
        th_cpu = min(C, cores)
        nf = max(th_cpu, int(th_cpu / 0.0012))  # ~1 s of work
        secs, _, _ = O.cpu_upload_bench(nf, S, N, th_cpu, use_openssl=True)
        cpu = nf * S / secs / 1e9 if secs > 0 else None
        if C == 1 and secs > 0:
            cpu_one = secs / nf
        nd = max(th_cpu, int(th_cpu / 0.0012))
        dsecs = O.cpu_download_bench(nd, S, N, th_cpu, True)
        row["cpu_upload_gbps"] = round(cpu, 3) if cpu else None
        row["cpu_download_gbps"] = round(nd * S / dsecs / 1e9, 3) if dsecs > 0 else None
        row["cpu_threads"] = th_cpu
        if cpu_one:  # one handler's file, queued behind C / threads others
            row["cpu_latency_est_ms"] = round(cpu_one * 1e3 * ((C + th_cpu - 1) // th_cpu), 2)
        rows.append(row)
        log(f"batcher: {C} clients: upload {row['upload']['gbps']} / pinned {row['upload_pinned']['gbps']} / view "
            f"{row['upload_view']['gbps']} GB/s p50 {row['upload_view']['p50_ms']} ms (batch "
            f"{row['upload_view']['mean_batch']}), download {row['download']['gbps']} / pinned "
            f"{row['download_pinned']['gbps']} / view {row['download_view']['gbps']} GB/s; cpu "
            f"{row['cpu_upload_gbps']} / {row['cpu_download_gbps']}")

    def cross(key, cpu_key):
        return next((r["clients"] for r in rows if r[cpu_key] and r[key]["gbps"] > r[cpu_key]), None)
    # What the CPU path would reach on a whole host, as a projection: the
    # measured single-thread rate x physical cores, linear scaling assumed
    # (an upper bound: memory bandwidth and turbo are ignored).
    info, _ = host_cpu_info()
    one_up = next((r["cpu_upload_gbps"] for r in rows if r["cpu_threads"] == 1 and r["cpu_upload_gbps"]), None)
    one_dn = next((r["cpu_download_gbps"] for r in rows if r["cpu_threads"] == 1 and r["cpu_download_gbps"]), None)
    modes = ("", "_pinned", "_view", "_staged_view")
    best_up = max((max(r["upload" + m]["gbps"] for m in modes) for r in rows), default=None)
    best_dn = max((max(r["download" + m]["gbps"] for m in modes) for r in rows), default=None)
    proj = None
    if one_up and one_dn:
        proj = {"single_thread_upload_gbps": one_up, "single_thread_download_gbps": one_dn, "hosts": []}
        for label, ncores in (("this box as lscpu shows it", info.get("physical_cores")),
                              ("a 2 x 64-core host (e.g. EPYC 9575F x2)", 128)):
            if ncores:
                proj["hosts"].append({"host": label, "cores": ncores, "upload_gbps": round(one_up * ncores, 1),
                                      "download_gbps": round(one_dn * ncores, 1)})
        proj["gpu_serving_best_gbps"] = {"upload": best_up, "download": best_dn}
        proj["note"] = ("PROJECTION, not a measurement: single-thread CPU-proxy rate x cores.  The serving path moves "
                        "every request over PCIe (1 MiB in + 1.33 MiB of Base64 out per upload: at most ~42 GB/s of "
                        "file bytes on a 56 GB/s link), so a host with all its cores free would outrun it; the GPU wins "
                        "where data is already in HBM (the headline step) or the host's cores are needed elsewhere")
    if not ok:
        raise LegError("batcher leg: a client result is wrong")
    return {"file_bytes": S, "nfrag": N, "rows": rows,
            "crossover_clients": {"upload": cross("upload", "cpu_upload_gbps"),
                                  "download": cross("download", "cpu_download_gbps"),
                                  "upload_pinned": cross("upload_pinned", "cpu_upload_gbps"),
                                  "download_pinned": cross("download_pinned", "cpu_download_gbps"),
                                  "upload_view": cross("upload_view", "cpu_upload_gbps"),
                                  "download_view": cross("download_view", "cpu_download_gbps"),
                                  "upload_staged_view": cross("upload_staged_view", "cpu_upload_gbps"),
                                  "download_staged_view": cross("download_staged_view", "cpu_download_gbps")},
            "ok": ok, "cpu_cores": cores, "full_host_cpu_projection": proj,
            "note": "native client threads (tools/batcher_load, 3 workers, 2 ms window), host buffers: each request "
                    "crosses PCIe in and out; staged = pageable handler buffers copied by the handler into / out of "
                    "pinned staging, pinned = dfs_host_alloc buffers moved by DMA directly (direct = such requests), view = pinned "
                    "inputs, the answer left in the batch's pinned result buffer and handed out as a pointer "
                    "(dfs_submit_*_view: one DMA out per batch), staged_view = pageable inputs copied by the handler into "
                    "the staging (one DMA in) with the answer as a view (one DMA out, no copy back); "
                    "latency = one handler's blocking call; cpu = the oracle's C proxy with min(C, cores) threads "
                    "(OpenSSL SHA-256 + scalar Base64, upload and download sequences); cpu_latency_est = one file's "
                    "single-thread time x ceil(C / threads); crossover = fewest clients where the GPU path beats the "
                    "CPU proxy"}


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
    F, S, N, chunk = args.long_files, args.long_size, 5, args.long_chunk
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
                        "unit": "Tops/s (int32)", "frac": round(tops / VALU_PEAK_TOPS, 4),
                        "kernel": "sha256_chain2 (pair-lane latency kernel)" if lanes <= 16384 else
                                  ("sha256_chain" if lanes <= 32768 else "sha256_lanes"),
                        "ms": round(k["sha_ms"], 3), "lanes": lanes, "lane_occupancy": round(lanes / 65536, 4),
                        "note": "one message per lane and SHA-256 is sequential within a message: the fileId "
                                "chains (4.19M blocks each) bound the run"},
           "roofline_b64": {"bound": "hbm", "ms": round(k["b64_ms"], 3),
                            "achieved": round(b64_bytes / (k["b64_ms"] / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s"},
           "wall_ms_incl_synth": round(wall * 1e3, 3), "verified": bool(ok)}
    emit(res)
    eng.close()
    return 0 if ok else 3


# ---------------------------------------------------------------------------
# N > 1: upload + placement pipeline over RCCL
# ---------------------------------------------------------------------------
class Shard:
    """This rank's files in `chunks` upload plans (fragment-major Base64, so
    group f of a chunk is one span) with their Base64, held and digest
    buffers; `table[c]` = every rank's group sizes of chunk c."""

    def __init__(self, args, eng, comm, files, dev):
        import numpy as np
        import torch
        import dfs_amd
        from dfs_amd import placement as P
        F, S, N = args.files, args.file_size, args.nfrag
        C = max(1, min(args.chunks, F))
        bounds = [F * c // C for c in range(C + 1)]
        self.chunks = []
        raw_max = 0
        self.replica_plan_ms = 0.0
        for c in range(C):
            a, b = bounds[c], bounds[c + 1]
            spans = np.stack([np.arange(a, b, dtype=np.uint64) * np.uint64(S),
                              np.full(b - a, S, dtype=np.uint64)], axis=1)
            plan = dfs_amd.UploadPlan(eng, spans, N, frag_major=True, align128=args.align128)
            offs = plan.b64_offsets()
            grp = [int(offs[f]) for f in range(N)] + [int(offs[-1])]
            # replica receiver's plan of this chunk (a collective: every rank's
            # file lengths are gathered); its table is what dfs_place_sizes gathers
            t0 = time.perf_counter()
            rp = P.ReplicaPlan(comm, N, [S] * (b - a), align128=args.align128)
            self.replica_plan_ms += (time.perf_counter() - t0) * 1e3
            table = rp.table
            if table[comm.rank].tolist() != [grp[f + 1] - grp[f] for f in range(N)]:
                raise LegError("replica plan: group sizes differ from the upload plan's")
            lay = P.held_layout(comm.world, comm.rank, N, table)
            if int(lay[N]) != rp.held_bytes:
                raise LegError("replica plan: held bytes differ from the placement's")
            raw_max = max(raw_max, rp.raw_bytes)
            ch = {"a": a, "b": b, "plan": plan, "grp": grp, "table": table, "lay": lay, "rp": rp,
                  "b64": torch.empty(max(grp[-1], 1), dtype=torch.uint8, device=dev),
                  "held": torch.empty(max(int(lay[N]), 1), dtype=torch.uint8, device=dev),
                  "verdict": torch.zeros(max(rp.nheld, 1), dtype=torch.int32, device=dev),
                  "failed": torch.zeros(comm.world, dtype=torch.int32, device=dev),
                  "ev_up": torch.cuda.Event(), "ev_placed": torch.cuda.Event(), "ev_checked": torch.cuda.Event()}
            for mode in ("ring", "star"):
                ops, _, _ = P.plan(comm.world, comm.rank, N, table, mode)
                ch["sent_" + mode] = P.bytes_sent(ops)
            self.chunks.append(ch)
        # decoded replicas of one chunk (what a holder would write as .frag
        # files, SN:284-285): one buffer, the chunks' checks run in order
        self.raw = torch.empty(raw_max + 16, dtype=torch.uint8, device=dev)
        self.fd = torch.empty(F * 32, dtype=torch.uint8, device=dev)
        self.frd = torch.empty(F * N * 32, dtype=torch.uint8, device=dev)
        self.files, self.N = files, N

    def upload(self, c, flags=0):
        ch = self.chunks[c]
        ch["plan"].run(self.files.data_ptr(), self.fd.data_ptr() + 32 * ch["a"],
                       self.frd.data_ptr() + 32 * self.N * ch["a"], ch["b64"].data_ptr(), flags)


def multi_gpu(args, world, rank, local, log):
    """N > 1 step: upload (compute stream) + placement (comm stream), chunk c's
    placement beside chunk c+1's hashing.  Returns (result dict, ok)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import dfs_amd
    from dfs_amd import placement as P
    from dfs_amd.engine import download_device
    dev = torch.device("cuda", local)
    # the harness's own collectives: device tensors over nccl, host tensors over gloo (--comm host)
    hdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    F, S, N = args.files, args.file_size, args.nfrag
    eng = dfs_amd.FragmentEngine(local)   # compute ctx
    eng_c = dfs_amd.FragmentEngine(local)  # comm ctx (RCCL on its own stream)
    s_comp, s_comm = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    eng.set_stream(s_comp.cuda_stream)
    eng_c.set_stream(s_comm.cuda_stream)
    uid = [P.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = P.Comm(eng_c, uid[0], world, rank)
    files = torch.empty(F * S + 64, dtype=torch.uint8, device=dev)
    spans = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(S), np.full(F, S, dtype=np.uint64)], axis=1)
    dfs_amd.synth_fill(eng, files.data_ptr(), spans, rank * F, SEED)
    sh = Shard(args, eng, comm, files, dev)
    C = len(sh.chunks)
    flags = dfs_amd.DFS_SERIAL if args.mode == "serial" else 0
    torch.cuda.synchronize(dev)
    log(f"{world} ranks x {F} files x {S} B, N={N}, {C} chunks, placement {args.placement}")

    def frd_ptr(ch):
        return sh.frd.data_ptr() + 32 * N * ch["a"]

    pending = []  # the chunk whose holders' check is still to be enqueued

    def check(ch):
        """The holder's half of the upload (SN:281-282 + 248-257) on the
        compute stream: decode + SHA-256 of every held fragment of the chunk,
        compared with the digests the uploaders sent; then the failure counts
        back to the uploaders (comm stream)."""
        s_comp.wait_event(ch["ev_placed"])
        ch["rp"].check(eng, ch["held"].data_ptr(), sh.raw.data_ptr(), ch["verdict"].data_ptr(),
                       ch["failed"].data_ptr())
        ch["ev_checked"].record(s_comp)
        s_comm.wait_event(ch["ev_checked"])
        ch["rp"].report(ch["failed"].data_ptr())

    def flush():
        while pending:
            check(pending.pop(0))

    def step(mode, compute=True, place=True, verify=True):
        """One upload of the shard as the reference completes it: hash + encode
        (compute stream), placement + the digest tables (comm stream), the
        holders' decode + hash + compare (compute stream) and the failure
        counts back to the uploaders (comm stream).  The check of a chunk is
        enqueued one chunk behind the hashing — after the next chunk's upload,
        which for the last chunk is the next step's first — so its placement
        hides behind that upload; flush() enqueues what is still pending."""
        verify = verify and place
        for c, ch in enumerate(sh.chunks):
            if compute:
                s_comp.wait_event(ch["ev_placed"])  # chunk c's Base64 is free again
                sh.upload(c, flags)
                ch["ev_up"].record(s_comp)
            if place:
                if pending and pending[0] is ch:  # its held buffer is about to be overwritten
                    flush()
                s_comm.wait_event(ch["ev_up"])
                s_comm.wait_event(ch["ev_checked"])  # chunk c's held buffer is free again
                comm.place(mode, ch["table"], ch["b64"].data_ptr(), ch["held"].data_ptr())
                if verify:
                    ch["rp"].exchange(frd_ptr(ch))
                ch["ev_placed"].record(s_comm)
            if verify:
                flush()
                pending.append(ch)

    def full_steps(mode, n):
        for _ in range(n):
            step(mode)
        flush()  # inside the timed region: the last chunk's check and report

    def verify_only():
        for ch in sh.chunks:
            ch["rp"].exchange(frd_ptr(ch))
            ch["ev_placed"].record(s_comm)
            check(ch)

    def verify_clean():
        return all(int(ch["failed"].sum().item()) == 0 and not bool(ch["verdict"].any().item()) for ch in sh.chunks)

    def timed(fn, reps):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=hdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item()) / reps

    full_steps(args.placement, args.warmup)
    t_step = timed(lambda: full_steps(args.placement, args.steps), 1) / max(args.steps, 1)
    torch.cuda.synchronize(dev)
    verify_ok = verify_clean()  # every replica of every step's last run checked good on its holder
    side = max(1, min(args.steps, 3))
    # the same step without the holders' verify, without any
    # exchange, the verify alone, and each placement alone
    t_noverify = timed(lambda: step(args.placement, verify=False), side)
    t_comp = timed(lambda: step(args.placement, place=False), side)
    t_verify = timed(verify_only, side)
    verify_ok = verify_ok and verify_clean()
    # A corrupted replica must be caught, by the right holder, for the right
    # uploader, and every rank must learn of it: rank 0 flips one Base64 char
    # of one held fragment (to another alphabet char), every rank re-runs the
    # verify, then the placement restores the held buffer.
    ch0 = sh.chunks[0]
    probe = torch.zeros(2, dtype=torch.int64, device=hdev)
    if rank == 0 and ch0["rp"].nheld:
        fr = ch0["rp"].frags()
        k = int(ch0["rp"].nheld * 2 // 3)
        pos = int(fr[k]["b64_off"]) + 5
        ch0["held"][pos] = ord("B") if int(ch0["held"][pos]) == ord("A") else ord("A")
        probe[0], probe[1] = k, int(fr[k]["rank"])
        torch.cuda.synchronize(dev)  # the flipped char is in place before the library's stream reads it
    dist.broadcast(probe, src=0)
    probe = probe.cpu()  # the broadcast is complete before the library's own communicator is used again
    verify_only()
    torch.cuda.synchronize(dev)
    want_failed = torch.zeros(world, dtype=torch.int32, device=dev)
    want_failed[int(probe[1])] = 1
    probe_ok = bool(torch.equal(ch0["failed"], want_failed))
    if rank == 0:
        bad = torch.nonzero(ch0["verdict"]).flatten().tolist()
        probe_ok = probe_ok and bad == [int(probe[0])] and int(ch0["verdict"][bad[0]]) == dfs_amd.DFS_E_FRAG_MISMATCH
    else:
        probe_ok = probe_ok and not bool(ch0["verdict"].any().item())
    step(args.placement, compute=False, verify=False)  # restore the held buffer
    verify_only()
    torch.cuda.synchronize(dev)
    verify_ok = verify_ok and probe_ok and verify_clean()
    # SHA-256 kernel time per launch (one launch per chunk), HIP events on
    # the compute stream, outside the timed steps
    eng.set_profiling(True)
    sha_ms = []
    for c in range(C):
        sh.upload(c, flags)
        sha_ms.append(eng.timings()["sha"])
    eng.set_profiling(False)
    # Every file this rank uploaded against the oracle (outside the timing):
    # fileIds, fragment digests and, through a device SHA-256 of each
    # fragment's Base64, the Base64 (as the N = 1 line does); mismatches are
    # summed over the ranks.
    oracle_check, oracle_ok = None, True
    if args.verify and args.verify_all:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # checker only
        from dfs_amd.engine import sha256_device
        _, threads = host_cpu_info()
        threads = max(1, threads // world)  # the ranks share the host's cores
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        efd, efrd, eb64 = O.synth_digests(rank * F, F, S, N, threads)
        t_cpu = time.perf_counter() - t0
        bad_fd = int((sh.fd.view(F, 32).cpu().numpy() != efd).any(axis=1).sum())
        bad_frd = int((sh.frd.view(F, N, 32).cpu().numpy() != efrd).any(axis=2).sum())
        bad_b64 = 0
        for ch in sh.chunks:
            nf = ch["b"] - ch["a"]
            got = sha256_device(eng, ch["b64"].data_ptr(), ch["plan"].b64_spans([S] * nf)).reshape(nf, N, 32)
            bad_b64 += int((got != eb64[ch["a"]:ch["b"]]).any(axis=2).sum())
        bad = torch.tensor([bad_fd, bad_frd, bad_b64], dtype=torch.int64, device=hdev)
        dist.all_reduce(bad)
        oracle_check = {"files_per_rank": F, "ranks": world, "file_digests_checked": F * world,
                        "fragment_digests_checked": F * N * world, "base64_fragments_checked": F * N * world,
                        "mismatches": int(bad.sum().item()), "oracle_seconds": round(t_cpu, 2), "oracle_threads": threads,
                        "how": "every rank checks its own shard: oracle C path (libcrypto SHA-256, scalar Base64) over "
                               "each synthetic file; the device Base64 through a per-fragment SHA-256 on the device"}
        oracle_ok = oracle_check["mismatches"] == 0
        log(f"oracle check of every rank's {F} files: {oracle_check['mismatches']} mismatches ({t_cpu:.1f} s, {threads} threads per rank)")
    t_place = {}
    for mode in ("star", "ring"):
        step(mode, compute=False, verify=False)
        t_place[mode] = timed(lambda m=mode: step(m, compute=False, verify=False), side)
    # held buffers after ring == after star: SHA-256 of every held group
    # (the library's own kernel as a checksum of checksums)
    def held_digests():
        from dfs_amd.engine import sha256_device
        out = []
        for ch in sh.chunks:
            n = int(ch["lay"][N])
            piece = 1 << 20
            sp = np.array([(o, min(piece, n - o)) for o in range(0, n, piece)], dtype=np.uint64)
            out.append(sha256_device(eng_c, ch["held"].data_ptr(), sp).tobytes() if n else b"")
        return out
    torch.cuda.synchronize(dev)
    dig_ring = held_digests()
    step("star", compute=False, verify=False)
    torch.cuda.synchronize(dev)
    ok = dig_ring == held_digests() and verify_ok and oracle_ok
    # Degraded read (BASELINE configs[4]): the last GPU offline; every other
    # rank fetches its groups back from the live holders (SN:422-446), then
    # Base64-decodes them into place with per-fragment and fileId verify.
    # (One rank alone: nobody offline, the fetch is local.)
    offline = [world - 1] if world > 1 else []
    fetch_ms = dl_ms = dl_dev_ms = dl_plan_ms = 0.0
    dl_ok = True
    held_frags = sum(ch["rp"].nheld for ch in sh.chunks)
    raw_bytes = sum(ch["rp"].raw_bytes for ch in sh.chunks)
    sh.raw = None  # hand the replica buffer back before the read leg's buffers
    out = torch.empty(max(sh.chunks[0]["b"] - sh.chunks[0]["a"], 1) * S, dtype=torch.uint8, device=dev)
    back = torch.empty(max(ch["grp"][-1] for ch in sh.chunks), dtype=torch.uint8, device=dev)
    for ch in sh.chunks:
        nf = ch["b"] - ch["a"]
        spans_c = ch["plan"].b64_spans([S] * nf)
        # the read's descriptor tables depend only on the batch shape: built once (plan_ms), kept in HBM
        t0 = time.perf_counter()
        dplan = dfs_amd.DownloadPlan(eng_c, spans_c, nf, N, np.full(nf, S, np.uint64),
                                     np.arange(nf, dtype=np.uint64) * np.uint64(S))
        dl_plan_ms += (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        st = comm.fetch(ch["table"], ch["held"].data_ptr(), back.data_ptr(), offline)
        torch.cuda.synchronize(dev)
        fetch_ms += (time.perf_counter() - t0) * 1e3
        if rank in offline:
            dplan.close()
            continue
        dl_ok &= bool((st == 0).all()) and bool(torch.equal(back[:ch["grp"][-1]], ch["b64"][:ch["grp"][-1]]))
        eng_c.set_profiling(True)
        t0 = time.perf_counter()
        status = dplan.run(back.data_ptr(), sh.frd.data_ptr() + 32 * N * ch["a"], sh.fd.data_ptr() + 32 * ch["a"],
                           out.data_ptr())
        dl_ms += (time.perf_counter() - t0) * 1e3
        dl_dev_ms += eng_c.timings()["total"] or 0.0
        eng_c.set_profiling(False)
        dplan.close()
        dl_ok &= bool((status == 0).all()) and bool(torch.equal(out[:nf * S], files[ch["a"] * S:ch["b"] * S]))
    flag = torch.tensor([1 if (ok and dl_ok) else 0], dtype=torch.int32, device=hdev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    ok_all = bool(flag.item())
    sent = {m: sum(ch["sent_" + m] for ch in sh.chunks) for m in ("ring", "star")}
    sent_t = torch.tensor([sent["ring"], sent["star"]], dtype=torch.float64, device=hdev)
    dist.all_reduce(sent_t)
    held_bytes = sum(int(ch["lay"][N]) for ch in sh.chunks)
    res = {
        "step_s": t_step,
        "placement": {
            "mode_in_step": args.placement, "chunks": C, "node_to_gpu": "node k on GPU k mod W",
            "compute_only_ms": round(t_comp * 1e3, 3),
            "compute_only_gbps": round(F * S * world / t_comp / 1e9, 3),
            "receive_verify_ms": round(t_verify * 1e3, 3),
            "step_without_verify_ms": round(t_noverify * 1e3, 3),
            "receive_verify": {"held_fragments_per_gpu": held_frags, "decoded_bytes_per_gpu": raw_bytes,
                               "plan_ms": round(sh.replica_plan_ms, 2),
                               "kernels": "one pass (each lane decodes, stores and hashes its fragment)"
                               if sh.chunks[0]["rp"].one_pass else "decode kernel, then SHA-256 lanes",
                               "all_replicas_good": verify_ok, "corrupt_probe_caught": probe_ok,
                               "note": "inside the timed step: every rank's fragment digests to the holders "
                                       "(dfs_replica_exchange, RCCL), each holder Base64-decodes and SHA-256s every "
                                       "held fragment and compares (dfs_replica_check; SN:281-282, 248-257), failure "
                                       "counts per uploader summed over the holders (dfs_replica_report); "
                                       "receive_verify_ms = those three alone; the probe flips one held Base64 char on "
                                       "rank 0 and expects exactly that fragment's DFS_E_FRAG_MISMATCH, counted for its "
                                       "uploader on every rank"},
            "star_ms": round(t_place["star"] * 1e3, 3),
            "star_xgmi_gbps_per_gpu": round(sent_t[1].item() / world / t_place["star"] / 1e9, 2),
            "ring_ms": round(t_place["ring"] * 1e3, 3),
            "ring_xgmi_gbps_per_gpu": round(sent_t[0].item() / world / t_place["ring"] / 1e9, 2),
            "bytes_sent_per_gpu": {"star": int(sent_t[1].item() / world), "ring": int(sent_t[0].item() / world)},
            "held_bytes_per_gpu": held_bytes, "ring_equals_star": ok,
            "transfers_issued": dict(comm.counters(), loopback=os.environ.get("DFS_COMM_LOOPBACK") == "1",
                                     note="this rank's sends / receives / local copies over the whole run; with "
                                          "DFS_COMM_LOOPBACK=1 the local copies travel as ncclSend / ncclRecv to itself"),
            "degraded": {"offline_gpu": offline[0] if offline else None, "fetch_ms": round(fetch_ms, 3),
                         "download_ms": round(dl_ms, 3), "download_device_ms": round(dl_dev_ms, 3),
                         "download_plan_ms": round(dl_plan_ms, 2),
                         "download_gbps": round(F * S / (dl_ms / 1e3) / 1e9, 2) if dl_ms else None,
                         "download_device_gbps": round(F * S / (dl_dev_ms / 1e3) / 1e9, 2) if dl_dev_ms else None,
                         "ok": ok_all},
            "note": "xgmi_gbps = bytes this GPU sends / placement time (RCCL send/recv, dfs_place_ring / "
                    "dfs_place_star); download = Base64 decode into place + fragment and fileId SHA-256 verify of "
                    "the fetched groups (dfs_download_plan_run: tables prebuilt, download_plan_ms once per shape), wall "
                    "clock and HIP-event device time"},
        "sha_ms_per_launch": float(np.mean(sha_ms)), "files_per_launch": F / C, "ok": ok_all, "verify": oracle_check}
    for ch in sh.chunks:
        ch["plan"].close()
        ch["rp"].close()
    comm.close()
    eng.close()
    eng_c.close()
    return res, ok_all


def roofline_n(res, S, N):
    """SHA-256 kernel roofline at N > 1 (rank 0's compute ctx, one launch per
    chunk of files_per_launch files)."""
    blocks = res["files_per_launch"] * (sha_blocks(S) + sum(sha_blocks(x) for x in split(S, N)))
    ms = res["sha_ms_per_launch"]
    tops = blocks * OPS_PER_BLOCK_CANON / (ms / 1e3) / 1e12
    return {"bound": "valu", "achieved": round(tops, 3), "peak": round(VALU_PEAK_TOPS, 3), "unit": "Tops/s (int32)",
            "frac": round(tops / VALU_PEAK_TOPS, 4), "traffic": None, "kernel": "sha256_lanes", "ms": round(ms, 3),
            "blocks_per_launch": int(blocks), "ops_per_block": OPS_PER_BLOCK_CANON,
            "note": "compute-only launches (no placement beside them), rank 0"}


def dry_run(args, world, rank, log):
    """Harness check on CPU (gloo): rendezvous, barrier + max-over-ranks
    timing and the placement schedules executed over gloo point-to-point on
    synthetic byte groups.  Never a measurement (no GPU kernels run)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from dfs_amd import placement as P
    N = args.nfrag
    rng = np.random.default_rng(rank)
    sizes = [int(x) for x in rng.integers(1000, 5000, N)]
    src = torch.from_numpy(rng.integers(0, 256, sum(sizes), dtype=np.uint8))
    t = torch.tensor(sizes, dtype=torch.int64)
    rows = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(rows, t)
    table = np.stack([r.numpy() for r in rows]).astype(np.uint64)
    ops, lay, _ = P.plan(world, rank, N, table, args.placement)
    held = torch.zeros(int(lay[N]), dtype=torch.uint8)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        P.run_plan_torch(ops, src, held)
    dist.barrier()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    fops, flay, fst = P.plan(world, rank, N, table, "fetch", [world - 1])
    back = torch.zeros(int(flay[N]), dtype=torch.uint8)
    P.run_plan_torch(fops, held, back)
    ok = rank == world - 1 or bool(torch.equal(back, src))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return float(tt.item()) / max(args.steps, 1), bool(flag.item()), int(table.sum())


# ---------------------------------------------------------------------------
def main():
    args = parse()
    if args.serial:
        args.mode = "serial"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(args)
    # Exactly one JSON line on stdout: native libraries write to fd 1 too
    # (RCCL prints its version banner at communicator init), so fd 1 becomes
    # stderr for the rest of the run and the result line goes to the original
    # stdout.
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    resolve_config(args, world)
    if args.config == 4:
        return long_leg(args)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    if args.dry_run:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("gloo", rank=0, world_size=1)
        per, ok, nbytes = dry_run(args, world, rank, log)
        if rank == 0:
            emit({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                  "warmup": args.warmup, "ms_per_step": round(per * 1e3, 3), "higher_is_better": True,
                  "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "dry-run",
                  "dry_run": True, "placed_bytes": nbytes, "verified": ok,
                  "config": {"workload": "harness check (gloo, CPU tensors), no GPU work"}})
        dist.destroy_process_group()
        return 0 if ok else 3

    # read by dfs_open: two-kernel mode vs the fused SHA+Base64 kernel
    os.environ["DFS_UPLOAD_MODE"] = args.mode if args.mode in ("fused", "hybrid") else "kernels"
    import numpy as np
    import torch
    import torch.distributed as dist
    import dfs_amd

    if world > 1 or args.placement_step:
        import datetime
        if args.comm == "host":
            # rehearsal: ranks share the GPUs present; the library's communicator goes through host
            # shared memory (chosen by the unique id) and the harness's own collectives through gloo
            os.environ["DFS_COMM_TRANSPORT"] = "host"
            local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
        if args.comm == "host":
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=600))
        S, N, F = args.file_size, args.nfrag, args.files
        failures = []
        try:
            res, ok = multi_gpu(args, world, rank, local, log)
        except Exception as e:  # report, then fail the run
            import traceback
            traceback.print_exc()
            res, ok = {"step_s": float("nan"), "placement": {"error": repr(e)[:300]}}, False
            failures.append("placement")
        elapsed = res["step_s"]
        value = F * S * world / elapsed / 1e9 if elapsed == elapsed else None
        if rank == 0:
            emit({
                "metric": METRIC, "value": round(value, 3) if value else None, "unit": "GB/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed * 1e3, 3) if value else None, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                "data": "synthetic (splitmix64, seed 0x5EED5EED), resident in HBM",
                "config": {"workload": f"upload + placement + holders' verify: {F} files x {S} B per GPU (BASELINE "
                                       f"configs[2] shard), N={N} fragments: fileId SHA-256 + fragment SHA-256 + "
                                       f"fragment Base64, {args.placement} placement of the Base64 over RCCL/xGMI, then "
                                       f"every holder Base64-decodes and SHA-256s what it received and compares with the "
                                       f"uploader's digests",
                           "files_per_gpu": F, "file_bytes": S, "nfrag": N, "parallelism": f"files sharded x{world}",
                           "placement": args.placement},
                "roofline": roofline_n(res, S, N) if ok else None,
                "placement": res["placement"], "verified": ok, "verify": res.get("verify"),
                **({"rehearsal": "host-staged communicator (--comm host): ranks share the GPUs present and bytes "
                                 "cross through host memory; functional check only, the rates mean nothing"}
                   if args.comm == "host" else {})})
        dist.destroy_process_group()
        return 0 if ok and not failures else 3

    # ---------------- N = 1 ----------------
    dev = torch.device("cuda", 0)
    S, N, F = args.file_size, args.nfrag, args.files
    eng = dfs_amd.FragmentEngine(0)
    spans = np.stack([np.arange(F, dtype=np.uint64) * np.uint64(S), np.full(F, S, dtype=np.uint64)], axis=1)
    files = torch.empty(F * S + 64, dtype=torch.uint8, device=dev)
    dfs_amd.synth_fill(eng, files.data_ptr(), spans, 0, SEED)
    t0 = time.perf_counter()
    plan = dfs_amd.UploadPlan(eng, spans, N, align128=args.align128)
    plan_ms = (time.perf_counter() - t0) * 1e3  # host: split + lane / job tables, one upload to HBM; reused by every step
    fd = torch.empty(F * 32, dtype=torch.uint8, device=dev)
    frd = torch.empty(F * N * 32, dtype=torch.uint8, device=dev)
    b64 = torch.empty(plan.b64_total, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    flags = dfs_amd.DFS_SERIAL if args.mode == "serial" else 0
    torch.cuda.synchronize(dev)
    log(f"{F} files x {S} B, N={N}, b64 {plan.b64_total / 1e9:.2f} GB")

    for _ in range(args.warmup):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
    torch.cuda.synchronize(dev)

    # ---- timed region ---------------------------------------------------------
    eng.set_profiling(True)
    sha_ms = []
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
        t = eng.timings()  # waits on this step's last HIP event; per-kernel ms
        sha_ms.append(t["sha"])
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)

    # ---- fragment-only variant: no fileId SHA-256 (SN:127)
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
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)  # restore fileIds

    # ---- the HBM-bound Base64 encode pass alone (roofline_b64) -----------------
    eng.set_profiling(True)
    b64_ms = []
    for _ in range(max(1, args.b64_steps)):
        plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), dfs_amd.DFS_B64_ONLY)
        b64_ms.append(eng.timings()["b64enc"])
    eng.set_profiling(False)
    torch.cuda.synchronize(dev)

    # ---- verification against the oracle (outside the timed region) -----------
    ok = True
    verify = None
    if args.verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # checker only
        bsp = plan.b64_spans([S] * F)
        fdh = fd.view(F, 32).cpu().numpy()
        frdh = frd.view(F, N, 32).cpu().numpy()
        verify = {"files": 0, "of": F}
        if args.verify_all:
            # Every file of the timed batch: the oracle's C path regenerates each
            # synthetic file on the host cores and computes its fileId (SN:127),
            # its fragment digests (SN:159) and the SHA-256 of each fragment's
            # Base64 text (SN:636) with libcrypto's SHA-256; the device's Base64
            # is hashed per fragment by the library's SHA-256 kernel, which the
            # digest comparison just before has checked on these very files.
            from dfs_amd.engine import sha256_device
            _, threads = host_cpu_info()
            t0 = time.perf_counter()
            efd, efrd, eb64 = O.synth_digests(0, F, S, N, threads)
            t_cpu = time.perf_counter() - t0
            bad_fd = int((fdh != efd).any(axis=1).sum())
            bad_frd = int((frdh != efrd).any(axis=2).sum())
            gb64 = sha256_device(eng, b64.data_ptr(), bsp).reshape(F, N, 32)
            bad_b64 = int((gb64 != eb64).any(axis=2).sum())
            ok = ok and bad_fd == 0 and bad_frd == 0 and bad_b64 == 0
            verify.update({"files": F, "file_digests_checked": F, "fragment_digests_checked": F * N,
                           "base64_fragments_checked": F * N, "mismatches": bad_fd + bad_frd + bad_b64,
                           "oracle_seconds": round(t_cpu, 2), "oracle_threads": threads,
                           "how": "oracle C path (libcrypto SHA-256, scalar Base64) over every synthetic file; the "
                                  "device Base64 compared through a per-fragment SHA-256 computed on the device"})
            log(f"oracle check of all {F} files: fileId {bad_fd} bad, fragment digests {bad_frd} bad, Base64 "
                f"{bad_b64} bad ({t_cpu:.1f} s on {threads} threads)")
        idx = sorted(set([0, F - 1] + list(np.random.default_rng(1).integers(0, F, args.verify))))
        for f in idx:
            data = O.c_synth(f, 0, S)
            efd1, efrd1, eb64_1, eoff = O.c_upload_batch([data], N)
            k0 = f * N
            got_b64 = b"".join(b64[int(o):int(o + n)].cpu().numpy().tobytes() for o, n in bsp[k0:k0 + N])
            if not ((fdh[f] == efd1[0]).all() and (frdh[f] == efrd1[0]).all() and got_b64 == eb64_1):
                ok = False
        verify["base64_text_compared_files"] = len(idx)
        verify["files"] = max(verify["files"], len(idx))
        log(f"oracle byte-for-byte check of {len(idx)} files: {'OK' if ok else 'MISMATCH'}")

    # ---- numbers -----------------------------------------------------------------
    value = F * S * args.steps / elapsed / 1e9
    lens = split(S, N)
    blocks = F * (sha_blocks(S) + sum(sha_blocks(x) for x in lens))
    sha_avg = float(np.mean(sha_ms)) / 1e3
    b64_avg = float(np.mean(b64_ms)) / 1e3
    achieved_tops = blocks * OPS_PER_BLOCK_CANON / sha_avg / 1e12
    issued_tops = blocks * OPS_PER_BLOCK_ISSUED / sha_avg / 1e12
    b64_bytes = F * S + 4 * F * sum((x + 2) // 3 for x in lens)  # read + Base64 written
    b64_gbs = b64_bytes / b64_avg / 1e9
    traffic, traffic_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("workload") == f"{F}x{S}/N{N}":
                traffic = pmc.get("sha_hbm_bytes_per_launch")
                traffic_src = ("profiles/pmc_summary.json: rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this bench "
                               "command (a separate profiled run, not this one)")
        except Exception:
            traffic = None
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (splitmix64, seed 0x5EED5EED), resident in HBM",
        "config": {"workload": f"upload: {F} files x {S} B per GPU, N={N} fragments: fileId SHA-256 + "
                               f"fragment SHA-256 + fragment Base64",
                   "files_per_gpu": F, "file_bytes": S, "nfrag": N,
                   "mode": {"fused": "Base64 fused into the SHA-256 fragment lanes (one kernel)",
                            "kernels": "SHA-256 || Base64 kernels on two streams",
                            "hybrid": "fragment lanes write their own Base64; Base64 kernel only for the twin fragments",
                            "serial": "SHA-256 then Base64 kernel, one stream"}[args.mode],
                   "b64_layout": "128-byte aligned fragment starts" if args.align128 else "packed"},
        "roofline": {"bound": "valu", "achieved": round(achieved_tops, 3), "peak": round(VALU_PEAK_TOPS, 3),
                     "unit": "Tops/s (int32)", "frac": round(achieved_tops / VALU_PEAK_TOPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "sha256_lanes" + (" (+ fused Base64)" if args.mode in ("fused", "hybrid") else ""),
                     "ms": round(sha_avg * 1e3, 3), "blocks_per_launch": blocks, "ops_per_block": OPS_PER_BLOCK_CANON,
                     "valu_issue_frac": round(issued_tops / VALU_PEAK_TOPS, 4)},
        "roofline_b64": {"bound": "hbm", "achieved": round(b64_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(b64_gbs / HBM_PEAK_GBS, 4), "kernel": "b64_encode_kernel",
                         "ms": round(b64_avg * 1e3, 3), "bytes_per_launch": b64_bytes,
                         "note": "standalone encode pass over the same fragments (DFS_B64_ONLY), outside "
                                 "the timed steps"},
        "verified": ok, "verify": verify,
        "plan_ms": round(plan_ms, 2),
        "plan_note": "host time to build the upload plan (split, 393,216 SHA lane + 327,680 encode job descriptors, one "
                     "copy to HBM), paid once per batch shape and outside ms_per_step; a batch of another shape pays "
                     "it again (the request batcher does, per batch)",
    }
    if frag_only:
        result["fragment_only"] = frag_only
    failures = [] if ok else ["verify"]
    legs = []
    if not args.no_download:
        legs.append(("download", lambda: download_leg(args, eng, files, plan, fd, frd, b64, S, N, F, dev, log)))
    if not args.no_wire:
        legs.append(("wire", lambda: wire_leg(args, eng, files, fd, frd, S, N, F, dev, log)))
    if not args.no_store:
        legs.append(("store", lambda: store_leg(args, eng, files, fd, S, N, F, dev, log)))
    if not args.no_cpu_baseline:
        legs.append(("cpu_baseline", lambda: cpu_baseline(args, log)))
    for name, fn in legs:
        try:
            result[name] = fn()
        except Exception as e:  # the line is still printed; the exit code reports the failure
            import traceback
            traceback.print_exc()
            result[name] = {"error": repr(e)[:300]}
            failures.append(name)
    # The concurrent-clients leg runs in a child process with its own device
    # buffers: hand back the upload's 160 GB first.
    if not args.no_batcher:
        plan.close()
        del files, b64, fd, frd, legs
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        try:
            result["batcher"] = batcher_leg(args, log)
        except Exception as e:
            import traceback
            traceback.print_exc()
            result["batcher"] = {"error": repr(e)[:600]}
            failures.append("batcher")
    # The N > 1 lines measure another workload than this one (BASELINE
    # configs[2]'s shard with placement and the holders' verify, not
    # configs[1]): the same step on this one GPU (one-rank communicator, no
    # bytes cross xGMI) is the equal-workload reference for them.  A child
    # process, after this one has handed its buffers back.
    if not args.no_scaling_ref and not args.placement_step and args.config == 2:
        try:
            if args.no_batcher:
                plan.close()
                del files, b64, fd, frd, legs
                torch.cuda.synchronize(dev)
                torch.cuda.empty_cache()
            cmd = [sys.executable, os.path.abspath(__file__), "--placement-step", "--steps", "5", "--warmup", "2",
                   "--placement", args.placement]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not line:
                raise LegError(f"placement-step child rc {p.returncode}: {p.stderr[-300:]}")
            r = json.loads(line[-1])
            pl = r["placement"]
            result["n_gt_1_step_on_one_gpu"] = {
                "value": r["value"], "unit": "GB/s", "ms_per_step": r["ms_per_step"], "workload": r["config"]["workload"],
                "compute_only_ms": pl["compute_only_ms"], "receive_verify_ms": pl["receive_verify_ms"],
                "step_without_verify_ms": pl["step_without_verify_ms"], "verified": r["verified"],
                "note": "bench.py --placement-step: the step the N>1 lines time, on a one-rank communicator (placement "
                        "= local copies).  Weak-scaling efficiency on equal workloads = value(N) / (N x this value); "
                        "the headline `value` above is BASELINE configs[1], which has no placement step"}
            log(f"N>1 step on one GPU: {r['value']} GB/s, {r['ms_per_step']} ms per step")
            if not r["verified"]:
                failures.append("n_gt_1_step_on_one_gpu")
        except Exception as e:
            import traceback
            traceback.print_exc()
            result["n_gt_1_step_on_one_gpu"] = {"error": repr(e)[:300]}
            failures.append("n_gt_1_step_on_one_gpu")
        args.no_batcher = False  # the upload plan is closed
        # The same step with 8 rank processes on this one GPU, through the
        # library's host-staged communicator (small shards; functional only:
        # BASELINE configs[2] and configs[4] end to end but for the RCCL wire).
        # Reported, never fatal to the line: it is evidence, not the metric.
        if not args.no_rehearsal:
            try:
                cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "8", "--comm", "host", "--files", "512",
                       "--steps", "1", "--warmup", "1", "--placement", args.placement]
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
                if p.returncode != 0 or not line:
                    raise LegError(f"rehearsal child rc {p.returncode}: {p.stderr[-300:]}")
                r = json.loads(line[-1])
                pl = r["placement"]
                result["multi_rank_rehearsal"] = {
                    "ranks": 8, "gpus": 1, "files_per_rank": 512, "file_bytes": r["config"]["file_bytes"],
                    "nfrag": r["config"]["nfrag"], "verified": r["verified"],
                    "all_replicas_good": pl["receive_verify"]["all_replicas_good"],
                    "corrupt_probe_caught": pl["receive_verify"]["corrupt_probe_caught"],
                    "ring_equals_star": pl["ring_equals_star"],
                    "degraded_read_ok": pl["degraded"]["ok"], "offline_rank": pl["degraded"]["offline_gpu"],
                    "note": "bench.py --gpus 8 --comm host: the N>1 step (sharded upload, star and ring placement, digest "
                            "exchange, every holder's decode + SHA-256 + compare, a corrupted replica that must be "
                            "caught, the degraded read with the last rank offline) with 8 rank processes sharing this "
                            "GPU over the library's host-staged communicator instead of RCCL; functional check, no rates"}
                log(f"8-rank rehearsal on one GPU: verified={r['verified']}")
            except Exception as e:
                import traceback
                traceback.print_exc()
                result["multi_rank_rehearsal"] = {"error": repr(e)[:300]}
    if failures:
        result["failed_legs"] = failures
    emit(result)
    if args.no_batcher:
        plan.close()
    eng.close()
    return 3 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
