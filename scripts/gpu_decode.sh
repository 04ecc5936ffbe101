#!/bin/bash
# GPU call: parity tests, HBM stream ceilings, then the download leg under
# each decode variant (DFS_DEC_PER items per thread x DFS_DEC_NT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || fatal $?; tail -3 gpurun_out/gpu_tests.log
for v in "1 3" "1 1" "1 2" "1 0"; do
  set -- $v
  echo "== DFS_DEC_PER=$1 DFS_DEC_NT=$2"
  DFS_DEC_PER=$1 DFS_DEC_NT=$2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --b64-steps 1 --no-cpu-baseline --verify 2 > gpurun_out/dec_$1_$2.json 2> gpurun_out/dec_$1_$2.err || fatal $?
  python -c "import json;d=json.load(open('gpurun_out/dec_$1_$2.json'));print(d['value'],d['download'])"
done
exit 0
