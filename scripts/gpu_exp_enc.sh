#!/bin/bash
# On the GPU box: the upload step in hybrid mode with and without the fragment
# lanes' Base64 stores (experiment hook), beside the default mode.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ARGS="--steps 8 --warmup 2 --no-cpu-baseline --no-download --no-wire --no-store --no-batcher --no-rehearsal --no-scaling-ref --b64-steps 0 --frag-only-steps 0 --verify 0"
for spec in "kernels 0" "hybrid 0" "hybrid 1" "fused 0" "fused 1"; do
  set -- $spec
  DFS_ENC_EXPERIMENT=$2 timeout -k 10 200 python -u bench.py --mode $1 $ARGS > gpurun_out/exp_enc.json 2> gpurun_out/exp_enc.err; rc=$?
  python3 -c "
import json
try:
    l=json.loads(open('gpurun_out/exp_enc.json').read().strip().splitlines()[-1])
    print('mode $1 nostore=$2 rc $rc: step ms', l['ms_per_step'], 'sha ms', l['roofline'].get('ms'), flush=True)
except Exception as e:
    print('mode $1 nostore=$2 rc $rc: no line', e, flush=True)"
done
