#!/bin/bash
# GPU check: parity tests, the allocation-free entry's test, smoke,
# then (unless NO_BENCH) the default bench (N=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || fatal $rc
if [ -f tests/wip_no_alloc.py ]; then
  echo "== allocation-free entry (wip file, run by name)"
  timeout -k 10 300 python -u -m pytest tests/wip_no_alloc.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/no_alloc.log 2>&1; rc=$?
  tail -15 gpurun_out/no_alloc.log; [ $rc -eq 0 ] || fatal $rc
fi
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; fatal 9; }
cat gpurun_out/smoke.log
[ -n "$NO_BENCH" ] && exit 0
echo "== bench"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -8 gpurun_out/bench.err
exit $rc
