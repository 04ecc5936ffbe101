#!/bin/bash
# Latency-kernel check: parity tests that run sha256_chain (small launches,
# streaming parts, batcher), then the configs[3] skew and the batcher's
# 1- and 8-client legs.  AB_LIB: the same legs on an earlier build first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_batcher.py tests/test_streaming.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/chain_tests.log 2>&1 || { tail -30 gpurun_out/chain_tests.log; fatal 5; }
tail -2 gpurun_out/chain_tests.log
for lib in $AB_LIB ""; do
  echo "== ${lib:-this tree}"
  DFS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config 4 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -5 gpurun_out/c4.err; fatal 6; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/c4.json') if l.startswith('{')][-1]);print('config4', d['ms_per_step'], d['value'])"
  DFS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --b64-steps 1 --frag-only-steps 0 --no-download \
    --no-wire --no-store --no-cpu-baseline --verify 0 --clients 1,8 > gpurun_out/lat.json 2> gpurun_out/lat.err || { tail -5 gpurun_out/lat.err; fatal 7; }
  grep "batcher:" gpurun_out/lat.err
done
