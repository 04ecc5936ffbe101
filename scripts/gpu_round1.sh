#!/bin/bash
# Round-1 GPU call #2: microbench, parity tests, full-size bench (both stream
# modes), rocprofv3 kernel-trace stats of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal exit $1 -> stopping"; exit "$1" ;; esac; }
echo "== valu_peak"; timeout -k 10 120 tools/valu_peak > gpurun_out/valu_peak.json; rc=$?; cat gpurun_out/valu_peak.json; stop_on_fatal $rc
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -25 gpurun_out/gpu_tests.log; stop_on_fatal $rc
echo "== bench full (concurrent)"; timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?; cat gpurun_out/bench_full.json; tail -4 gpurun_out/bench_full.err; stop_on_fatal $rc
echo "== bench full (serial)"; timeout -k 10 300 python -u bench.py --serial --no-cpu-baseline > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err; rc=$?; cat gpurun_out/bench_serial.json; stop_on_fatal $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; rc=$?; echo "rc=$rc"; find gpurun_out/prof -name "*stats*" | head; stop_on_fatal $rc
exit 0
