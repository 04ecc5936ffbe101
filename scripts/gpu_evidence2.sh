#!/bin/bash
# Round evidence: parity tests, smoke, default bench (CPU baseline included),
# HBM stream ceilings, then scripts/profile.sh (upload + download traces, PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || fatal $?; tail -3 gpurun_out/gpu_tests.log
echo "== smoke"; timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" || fatal $?
echo "== bench default"; timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || fatal $?; cat gpurun_out/bench_default.json
echo "== hbm_stream"; timeout -k 10 120 tools/hbm_stream > gpurun_out/hbm_stream.json || fatal $?; cat gpurun_out/hbm_stream.json
bash scripts/profile.sh || fatal $?
