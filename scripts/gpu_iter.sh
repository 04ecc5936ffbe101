#!/bin/bash
# One build -> measure iteration on the GPU box: the parity tests (new ones
# first), then the default bench line without its slow side legs, then the
# configs[2] per-GPU shard.  Every GPU step has its own time limit; the script
# stops at the first failure.  BENCH_ARGS / C3_ARGS / TESTS override.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== gpu tests ${TESTS:-tests}"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || fatal $rc
[ -n "$NO_BENCH" ] && exit 0
echo "== bench (default config, side legs trimmed)"
timeout -k 10 400 python -u bench.py --no-batcher --no-cpu-baseline --no-store ${BENCH_ARGS} \
  > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; fatal 8; }
cat gpurun_out/bench.json; grep "^\[bench\]" gpurun_out/bench.err | tail -8
[ -n "$NO_C3" ] && exit 0
echo "== bench --config 3"
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --no-batcher --no-cpu-baseline --no-store --no-wire ${C3_ARGS} \
  > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; fatal 9; }
cat gpurun_out/bench_c3.json; grep "^\[bench\]" gpurun_out/bench_c3.err | tail -8
# Same-box A/B of the upload step against an earlier build (AB_LIB=path).
if [ -n "$AB_LIB" ]; then
  for lib in "$AB_LIB" ""; do
    echo "== A/B upload: ${lib:-this tree}"
    DFS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --steps 10 --no-batcher --no-cpu-baseline --no-store --no-wire \
      --no-download --frag-only-steps 0 --b64-steps 0 ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { tail -20 gpurun_out/ab.err; fatal 10; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'], d['roofline']['ms'], d['roofline']['frac'])"
  done
fi
