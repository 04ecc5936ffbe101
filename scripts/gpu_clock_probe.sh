#!/bin/bash
# Shader clock of the SHA waves (s_memtime / s_memrealtime per work item) in
# the concurrent (SHA || Base64) and serial upload modes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
for mode in "" "--serial"; do
  tag=${mode:-concurrent}; tag=${tag#--}
  echo "== $tag"
  DFS_SHA_CENSUS=gpurun_out/census_$tag.bin timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --b64-steps 1 --no-cpu-baseline --verify 0 --no-download --no-wire $mode > gpurun_out/clk_$tag.json 2>/dev/null || fatal $?
  python3 -c "import json; d=json.load(open('gpurun_out/clk_$tag.json')); print('ms/step', d['ms_per_step'], 'sha', d['roofline']['ms'])"
  python3 tools/census.py gpurun_out/census_$tag.bin 1024 | head -5
done
