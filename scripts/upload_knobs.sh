#!/bin/bash
# Upload-step knob sweep on the current tree (twin lanes): Base64 workgroups
# per CU beside SHA and their priority.  One bench line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/upload_knobs.txt; : > $out
for v in ${KNOBS:-"1 3" "2 3" "4 3" "1 1" "1 0" "2 1"}; do
  set -- ${v/,/ }
  DFS_B64_WGS=$1 DFS_B64_PRIO=$2 timeout -k 10 300 python -u bench.py ${BENCH_CONFIG:-} --steps 10 --warmup 2 --no-download --no-wire --no-store --no-batcher --no-cpu-baseline --no-scaling-ref --verify 0 --frag-only-steps 0 > gpurun_out/kn.json 2> gpurun_out/kn.err || { tail -5 gpurun_out/kn.err; exit 3; }
  python3 -c "import json; d=json.load(open('gpurun_out/kn.json')); print('wgs $1 prio $2', d['ms_per_step'], d['roofline']['ms'], d['value'])" | tee -a $out
done
