#!/bin/bash
# Sliced holders' check: its tests, then the N > 1 step on one rank
# (configs[2] shard), unsliced (DFS_REPLICA_SLICES=1) against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_replica_verify.py tests/test_gpu_parity.py -k "replica or placement" -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/slice_tests.log 2>&1 || { tail -30 gpurun_out/slice_tests.log; exit 5; }
tail -14 gpurun_out/slice_tests.log
for i in 1 2; do
for sl in 1 default; do
  if [ $sl = default ]; then unset DFS_REPLICA_SLICES; else export DFS_REPLICA_SLICES=$sl; fi
  timeout -k 10 400 python -u bench.py --placement-step --steps 5 --warmup 2 > gpurun_out/slice_$sl.json 2> gpurun_out/slice_$sl.err || { tail -5 gpurun_out/slice_$sl.err; exit 6; }
  python3 -c "import json; d=json.load(open('gpurun_out/slice_$sl.json')); p=d['placement']; print('slices $sl', 'step_ms', d['ms_per_step'], 'verify_ms', p['receive_verify_ms'], 'no_verify_ms', p['step_without_verify_ms'], 'ok', d.get('verified'), p['receive_verify']['corrupt_probe_caught'])"
done; done
