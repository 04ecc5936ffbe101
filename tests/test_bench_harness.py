"""bench.py's multi-GPU harness on the CPU: `bench.py --gpus N` launches its
own N ranks (torch.distributed.run) when WORLD_SIZE is unset, rendezvous on
127.0.0.1, barrier + max-over-ranks timing, and the placement schedules over
gloo (--dry-run: no GPU work, the line says so and carries no value)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    # stdout holds the result line and nothing else (the driver parses it;
    # library banners such as RCCL's go to stderr, bench.py main)
    assert len(p.stdout.splitlines()) == len(lines), p.stdout[-2000:]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("gpus,placement", [(2, "star"), (2, "ring"), (4, "ring")])
def test_bench_launches_its_own_ranks(gpus, placement):
    rc, lines, err = _run(["--gpus", str(gpus), "--dry-run", "--steps", "2", "--warmup", "0",
                           "--placement", placement])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, (lines, err[-2000:])  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus and rec["dry_run"] is True and rec["value"] is None and rec["verified"] is True
    assert rec["steps"] == 2 and rec["ms_per_step"] > 0


def test_bench_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0
