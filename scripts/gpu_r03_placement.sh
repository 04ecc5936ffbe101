#!/bin/bash
# The N > 1 step (upload + placement + holders' verify) on a one-rank
# communicator: a small run first, then BASELINE configs[2]'s per-GPU shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
if [ -z "$NO_TESTS" ]; then
echo "== replica verify tests"
timeout -k 10 600 python -u -m pytest tests/test_replica_verify.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/replica_tests.log 2>&1; rc=$?
tail -25 gpurun_out/replica_tests.log; [ $rc -eq 0 ] || fatal $rc
fi
echo "== placement step, 16,384 files"
timeout -k 10 300 python -u bench.py --placement-step --files 16384 --steps 3 --warmup 1 > gpurun_out/place_small.json 2> gpurun_out/place_small.err; rc=$?
cat gpurun_out/place_small.json; tail -5 gpurun_out/place_small.err; [ $rc -eq 0 ] || fatal $rc
echo "== placement step, configs[2] shard"
timeout -k 10 600 python -u bench.py --placement-step --steps 5 --warmup 2 > gpurun_out/place_full.json 2> gpurun_out/place_full.err; rc=$?
cat gpurun_out/place_full.json; tail -5 gpurun_out/place_full.err
exit $rc
