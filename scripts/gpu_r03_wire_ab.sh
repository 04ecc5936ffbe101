#!/bin/bash
# On the GPU box: the storeFragments body leg (build + receive) with the
# receiver's decode + hash in one pass and as two kernels (DFS_RECV_FUSED=0).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-download --no-store --no-batcher --no-rehearsal --no-scaling-ref --b64-steps 0 --frag-only-steps 0 --verify 0"
for rep in 1 2; do
  for fused in 1 0; do
    DFS_RECV_FUSED=$fused timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/wire_ab.json 2> gpurun_out/wire_ab.err || { tail -5 gpurun_out/wire_ab.err; exit 1; }
    python3 -c "
import json
l=json.loads(open('gpurun_out/wire_ab.json').read().strip().splitlines()[-1]); w=l['wire']
print('one pass' if $fused else 'two kernels', 'rep $rep: receive wall ms', w['receive_wall_ms'], 'GB/s of bodies', w['receive_body_gbs'], 'ok', w['receive_ok'], flush=True)"
  done
done
