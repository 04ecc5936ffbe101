#!/bin/bash
# GPU check B: GPU tests, default bench without the batcher leg, the
# fused-upload mode on today's tree, the N > 1 step on one rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || fatal $rc
echo "== bench (no batcher leg)"
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-batcher > gpurun_out/bench_nb.json 2> gpurun_out/bench_nb.err; rc=$?
cat gpurun_out/bench_nb.json; tail -6 gpurun_out/bench_nb.err; [ $rc -eq 0 ] || fatal $rc
echo "== bench --mode fused (Base64 from the SHA lanes, no twins)"
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --mode fused --no-batcher --no-download --no-wire --no-store --no-cpu-baseline --no-verify-all > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err; rc=$?
cat gpurun_out/bench_fused.json; tail -3 gpurun_out/bench_fused.err; [ $rc -eq 0 ] || fatal $rc
NO_TESTS=1 bash scripts/gpu_r03_placement.sh
