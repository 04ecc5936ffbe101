#!/bin/bash
# One GPU call: microbench, parity tests, small bench.  Every GPU step has its
# own time limit; a fault / abort / timeout ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_on_fatal() {  # $1 = exit code of a GPU step
  case "$1" in
    0|1) return 0 ;;       # ok / test assertion failures: keep going
    *) echo "fatal exit $1 -> stopping"; exit "$1" ;;
  esac
}
export TMPDIR=/tmp
echo "== valu_peak"; timeout -k 10 60 tools/valu_peak > gpurun_out/valu_peak.json; rc=$?; cat gpurun_out/valu_peak.json; stop_on_fatal $rc
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_tests.log; stop_on_fatal $rc
echo "== bench small"; timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---files 8192 --steps 5 --warmup 1 --no-cpu-baseline} > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err; rc=$?; cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err; stop_on_fatal $rc
exit 0
