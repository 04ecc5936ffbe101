#!/bin/bash
# Evidence after twin lanes + decode-ahead download: rocprofv3 kernel
# traces and PMC passes (scripts/profile.sh), the default bench line (all
# legs), SHA alone (--mode serial), and the N>1 step on one rank at 4 and 2
# chunks (--placement-step).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
ROUND=r02 bash scripts/profile.sh > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; fatal 7; }
tail -3 gpurun_out/profile.log
echo "== default bench"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; fatal 8; }
grep "^\[bench\]" gpurun_out/bench_default.err | tail -12
echo "== SHA alone (serial streams)"
timeout -k 10 300 python -u bench.py --mode serial --steps 5 --no-batcher --no-cpu-baseline --no-store --no-wire --no-download \
  > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err || { tail -20 gpurun_out/bench_serial.err; fatal 9; }
for c in 4 2; do
  echo "== placement step, $c chunks"
  timeout -k 10 400 python -u bench.py --placement-step --chunks $c --steps 5 --no-cpu-baseline \
    > gpurun_out/bench_place_c$c.json 2> gpurun_out/bench_place_c$c.err || { tail -20 gpurun_out/bench_place_c$c.err; fatal 10; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_place_c$c.json'));print(d['ms_per_step'], d['value'])"
done
