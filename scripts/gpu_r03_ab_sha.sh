#!/bin/bash
# On the GPU box: the upload step with the library as built beside a second
# build (build_ab/libdfsgpu_old.so: the same sources but an earlier SHA-256
# kernel file), alternating, on one box.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-download --no-wire --no-store --no-batcher --no-rehearsal --no-scaling-ref --b64-steps 0 --frag-only-steps 0 --verify 0"
for rep in 1 2 3; do
  for which in new old; do
    if [ $which = old ]; then export DFS_LIB_PATH=$PWD/distributed-file-storage_amd/build_ab/libdfsgpu_old.so; else unset DFS_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/ab_${which}_$rep.json 2> gpurun_out/ab_${which}_$rep.err || { echo "run failed"; tail -5 gpurun_out/ab_${which}_$rep.err; exit 1; }
    python3 -c "
import json,sys
l=json.loads(open('gpurun_out/ab_${which}_$rep.json').read().strip().splitlines()[-1])
print('$which', $rep, 'step ms', l['ms_per_step'], 'sha ms', l['roofline'].get('ms'), 'frac', l['roofline']['frac'], flush=True)"
  done
done
