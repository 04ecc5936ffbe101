#!/bin/bash
# Upper-bound probe: SHA block loads coalesced across the wave (experiment
# build, digests wrong by construction) against the product, same box,
# alternating: beside Base64 (default) and alone (--mode serial).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=distributed-file-storage_amd/build_exp/libdfsgpu_interleaved.so
[ -f "$SO" ] || { echo "missing $SO (run scripts/exp_interleaved_build.py)"; exit 2; }
A="--steps 10 --warmup 3 --no-batcher --no-download --no-wire --no-store --no-cpu-baseline --no-scaling-ref --verify 0 --frag-only-steps 0"
for i in 1 2; do
for lib in product interleaved; do
for mode in kernels serial; do
  if [ $lib = interleaved ]; then export DFS_LIB_PATH=$PWD/$SO; else unset DFS_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py $A --mode $mode > gpurun_out/il_${lib}_${mode}_$i.json 2> gpurun_out/il_${lib}_${mode}_$i.err || { tail -5 gpurun_out/il_${lib}_${mode}_$i.err; exit 7; }
  python3 -c "import json; d=json.load(open('gpurun_out/il_${lib}_${mode}_$i.json')); print('$lib', '$mode', 'step_ms', d['ms_per_step'], 'sha_ms', d['roofline']['ms'])"
done
done
done
