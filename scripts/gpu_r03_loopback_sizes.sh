#!/bin/bash
# On the GPU box: the loopback step (DFS_COMM_LOOPBACK=1) at shard sizes whose
# largest single transfer lies below 2 GiB, between 2 and 4 GiB, and above 4 GiB.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp DFS_COMM_LOOPBACK=1
mkdir -p gpurun_out
for spec in "65536 2" "98304 2" "131072 2" "131072 1" "131072 4"; do
  set -- $spec
  echo "== files $1 chunks $2"
  timeout -k 10 200 python -u bench.py --placement-step --no-cpu-baseline --steps 2 --warmup 1 --files $1 --chunks $2 > gpurun_out/lb_$1_$2.json 2> gpurun_out/lb_$1_$2.err
  rc=$?
  python3 - $1 $2 $rc <<'PY'
import json, sys
f, c, rc = sys.argv[1:]
try:
    l = json.loads(open(f"gpurun_out/lb_{f}_{c}.json").read().strip().splitlines()[-1])
    p = l["placement"]
    per_op = int(f) // int(c) * 43776
    print(f"files {f} chunks {c} rc {rc}: largest transfer {per_op / 2**30:.2f} GiB  good {p['receive_verify']['all_replicas_good']} probe {p['receive_verify']['corrupt_probe_caught']} ring==star {p['ring_equals_star']} degraded {p['degraded']['ok']}", flush=True)
except Exception as e:
    print("no line", f, c, rc, e, flush=True)
PY
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "stopping after rc $rc"; exit $rc; fi
done
