#!/bin/bash
# Batcher GPU tests, then the staged / pinned (direct) sweep (scripts/batcher_sweep.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_abi.py -x -v --timeout 240 --timeout-method thread > gpurun_out/batcher_tests.log 2>&1; rc=$?; tail -4 gpurun_out/batcher_tests.log; [ $rc -eq 0 ] || exit $rc
PINNED="${PINNED:-0 1}" DEPTHS="${DEPTHS:-2 3}" WAITS="${WAITS:-2000}" CLIENTS="${CLIENTS:-64 512 4096}" KINDS="${KINDS:-upload download}" bash scripts/batcher_sweep.sh
