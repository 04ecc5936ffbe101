"""RCCL's send / receive path of the placement runner on one GPU.

With one rank every transfer of a placement is a local copy, so an ordinary
one-GPU run never reaches ncclSend / ncclRecv.  A comm made under
DFS_COMM_LOOPBACK=1 posts those copies as a send to itself paired with a
receive from itself inside the phase's ncclGroupStart / End, on the ctx stream:
the same calls, bracketing and stream ordering a many-rank run uses
(csrc/placement.cpp, RcclTransport).  The step is the one the multi-GPU bench
times (`bench.py --placement-step`): upload, star and ring placement
(StorageNode.java:195-224), the digest exchange and the holders' decode +
SHA-256 + compare (:248-257, :265-293) with a corrupted replica that must be
caught, and the read back (:422-458), all checked against the oracle.  Run in
a child process with a time limit so that a stuck collective fails the test
instead of hanging the suite."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


# piece_mb: the runner splits every transfer into pieces of at most that many MiB (256 by default; RCCL was seen
# to lose bytes of a 1.4 GB send-to-self), the same split on both sides; 1 MiB makes these small groups many pieces
@pytest.mark.parametrize("placement,extra,piece_mb", [("star", [], 0), ("ring", ["--file-size", "1000003", "--nfrag", "5"], 1)])
def test_placement_step_through_rccl_send_recv(placement, extra, piece_mb):
    files = 256
    print(f"RCCL loopback: 1 rank x {files} files, {placement} {extra} piece_mb={piece_mb}", flush=True)
    env = dict(os.environ, DFS_COMM_LOOPBACK="1")
    if piece_mb:
        env["DFS_COMM_PIECE_MB"] = str(piece_mb)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--placement-step", "--files", str(files),
                        "--steps", "1", "--warmup", "1", "--placement", placement, "--no-cpu-baseline"] + extra,
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    pl = line["placement"]
    tr = pl["transfers_issued"]
    assert tr["loopback"] and tr["copies"] == 0 and tr["sends"] == tr["recvs"] > 0, tr
    assert line["verified"] is True and line["verify"]["mismatches"] == 0
    assert pl["receive_verify"]["all_replicas_good"] and pl["receive_verify"]["corrupt_probe_caught"]
    assert pl["ring_equals_star"] and pl["degraded"]["ok"]
