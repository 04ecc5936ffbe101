#!/bin/bash
# The N > 1 step on one rank (configs[2] shard, 2 chunks) with the encode at 1
# or 2 workgroups per CU beside SHA, alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for w in 1 2; do
  DFS_B64_WGS=$w timeout -k 10 300 python -u bench.py --placement-step --steps 5 --warmup 2 > gpurun_out/pk.json 2> gpurun_out/pk.err || { tail -5 gpurun_out/pk.err; exit 6; }
  python3 -c "import json; d=json.load(open('gpurun_out/pk.json')); p=d['placement']; print('wgs $w', 'step_ms', d['ms_per_step'], 'compute_only', p['compute_only_ms'], 'noverify', p['step_without_verify_ms'], 'verify', p['receive_verify_ms'])"
done; done
