#!/bin/bash
# GPU call: parity tests, smoke, default bench, mode variants, kernel trace.
# Every GPU step has its own limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fatal() { case "$1" in 0|1) return 0 ;; *) echo "fatal exit $1 -> stopping"; exit "$1" ;; esac; }
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -8 gpurun_out/gpu_tests.log; stop_on_fatal $rc
echo "== smoke"; timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?; stop_on_fatal $rc
echo "== bench default"; timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?; cat gpurun_out/bench_default.json; tail -4 gpurun_out/bench_default.err; stop_on_fatal $rc
i=0
for v in "--mode fused" "--align128" "--mode fused --align128" "--mode serial"; do
  i=$((i+1)); echo "== bench $v"
  timeout -k 10 300 python -u bench.py $v --no-cpu-baseline --no-download --steps 5 > gpurun_out/bench_v$i.json 2> gpurun_out/bench_v$i.err; rc=$?; cat gpurun_out/bench_v$i.json; tail -3 gpurun_out/bench_v$i.err; stop_on_fatal $rc
done
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; rc=$?; echo "rc=$rc"; cat gpurun_out/prof_bench.json; stop_on_fatal $rc
exit 0
