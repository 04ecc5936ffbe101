#!/bin/bash
# Rehearsal of the N > 1 step with more ranks than GPUs: the library's
# host-staged communicator (bench.py --comm host), 2, 4 and 8 ranks sharing
# the one GPU, small shards.  Functional only: every kernel, layout, the
# digest exchange, the holders' verify, the corrupt-replica probe, ring ==
# star, and the degraded read with the last rank offline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in ${WORLDS:-2 4 8}; do
  files=$((8192 / W))
  echo "== $W ranks x $files files"
  timeout -k 10 ${LIMIT:-300} python -u bench.py --gpus $W --comm host --files $files --steps 2 --warmup 1 > gpurun_out/host_w$W.json 2> gpurun_out/host_w$W.err || { tail -30 gpurun_out/host_w$W.err; exit 7; }
  python3 -c "
import json; d=json.load(open('gpurun_out/host_w$W.json')); p=d['placement']
print('W=$W', 'verified', d['verified'], 'step_ms', d['ms_per_step'], 'verify_ms', p['receive_verify_ms'], 'replicas_good', p['receive_verify']['all_replicas_good'], 'probe', p['receive_verify']['corrupt_probe_caught'], 'ring==star', p['ring_equals_star'], 'degraded', p['degraded']['ok'], 'offline', p['degraded']['offline_gpu'], 'held_frags', p['receive_verify']['held_fragments_per_gpu'])"
done
