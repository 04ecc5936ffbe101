#!/bin/bash
# On the GPU box: the N > 1 step on one rank with the holders' check in one
# pass (the default for this shape) and as two kernels (DFS_REPLICA_FUSED=0),
# alternating, on one box; then the same for the configs[1] shape (1 MiB, N = 5).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in ""; do
  for rep in 1 2; do
    for fused in 1 0; do
      DFS_REPLICA_FUSED=$fused timeout -k 10 300 python -u bench.py --placement-step --no-cpu-baseline --steps 5 --warmup 1 $shape > gpurun_out/fc_$fused.json 2> gpurun_out/fc_$fused.err || { echo "run failed"; tail -5 gpurun_out/fc_$fused.err; exit 1; }
      python3 -c "
import json
l=json.loads(open('gpurun_out/fc_$fused.json').read().strip().splitlines()[-1]); p=l['placement']
print('shape [$shape] fused=$fused rep $rep: step ms', l['ms_per_step'], 'value', l['value'], 'verify ms', p['receive_verify_ms'], 'no-verify ms', p['step_without_verify_ms'], 'verified', l['verified'], '|', p['receive_verify']['kernels'][:12], flush=True)"
    done
  done
done
