"""The N > 1 step with more ranks than GPUs: `bench.py --gpus W --comm host`
starts W rank processes that share the GPU and talk through the library's
host-staged communicator (shared-memory mailboxes, csrc/hostcomm.cpp) instead
of RCCL.  Everything else is the step the multi-GPU bench times: sharded
upload, star and ring placement (StorageNode.java:195-224), the digest
exchange and every holder's decode + SHA-256 + compare (:248-257, :265-293)
with a corrupted replica that must be caught, and the degraded read with the
last rank offline (:422-458).  A functional check, never a measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(400)]


# (ranks, files per rank, placement, extra arguments): the 8-GPU shape of BASELINE configs[2] / [4]
# (256 KiB, N = 8), and the reference's own five nodes with 1 MiB files and with a size its split
# leaves ragged (N = 5)
CASES = [(2, 1024, "star", []), (8, 256, "star", []), (3, 512, "ring", []),
         (5, 128, "star", ["--file-size", "1048576", "--nfrag", "5"]),
         (2, 300, "ring", ["--file-size", "1000003", "--nfrag", "5"])]


@pytest.mark.parametrize("world,files,placement,extra", CASES)
def test_multi_rank_step_on_one_gpu(world, files, placement, extra):
    print(f"host-staged rehearsal: {world} ranks x {files} files, {placement} {extra}", flush=True)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--comm", "host",
                        "--files", str(files), "--steps", "1", "--warmup", "1", "--placement", placement] + extra,
                       capture_output=True, text=True, timeout=360)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    pl = line["placement"]
    assert line["n_gpus"] == world and line["verified"] is True and "rehearsal" in line
    assert line["verify"]["mismatches"] == 0 and line["verify"]["file_digests_checked"] == files * world
    assert pl["receive_verify"]["all_replicas_good"] and pl["receive_verify"]["corrupt_probe_caught"]
    assert pl["ring_equals_star"]
    assert pl["degraded"]["ok"] and pl["degraded"]["offline_gpu"] == world - 1
    nfrag = line["config"]["nfrag"]
    # every rank holds two copies' worth: fragments {k, k+1} of the nodes it hosts, from every rank
    hosted = {f for node in range(nfrag) if node % world == 0 for f in (node, (node + 1) % nfrag)}
    assert pl["receive_verify"]["held_fragments_per_gpu"] == len(hosted) * files * world
