#!/bin/bash
# Tuning sweep: SHA waves/SIMD x stream mode on the full config-2 workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal exit $1 -> stopping"; exit "$1" ;; esac; }
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; stop_on_fatal $rc
for w in ${SWEEP_WPS:-2 3 4 5 6 7}; do
  for mode in "" "--serial"; do
    echo "== wps=$w mode=$mode"
    DFS_SHA_WPS=$w timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify 2 $mode > gpurun_out/sweep_${w}${mode}.json 2>/dev/null; rc=$?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_${w}${mode}.json')); print(d['ms_per_step'], d['value'], 'sha', d['roofline']['ms'], 'b64', d['roofline_b64']['ms'], d['verified'])"
    stop_on_fatal $rc
  done
done
echo "== census wps=${CENSUS_WPS:-4}"
DFS_SHA_WPS=${CENSUS_WPS:-4} DFS_SHA_CENSUS=gpurun_out/census.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --verify 0 --serial > gpurun_out/census_bench.json 2>/dev/null; stop_on_fatal $?
exit 0
