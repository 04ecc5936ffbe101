#!/bin/bash
# Hybrid upload mode: parity, then same-box A/B against the default
# (SHA || Base64 kernels), twice each, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== hybrid parity"
timeout -k 10 600 python -u -m pytest tests/test_twin_lanes.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/hybrid_tests.log 2>&1; rc=$?
tail -25 gpurun_out/hybrid_tests.log; [ $rc -eq 0 ] || fatal $rc
A="--steps 10 --warmup 3 --no-batcher --no-download --no-wire --no-store --no-cpu-baseline --verify 4"
for i in 1 2; do
for m in kernels hybrid; do
  echo "== bench --mode $m ($i)"
  timeout -k 10 600 python -u bench.py $A --mode $m > gpurun_out/ab_${m}_$i.json 2> gpurun_out/ab_${m}_$i.err; rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${m}_$i.json')); print('$m', d['ms_per_step'], d['value'], d['roofline']['ms'], d['roofline']['frac'], d['verified'], d['verify']['mismatches'])" || { tail -5 gpurun_out/ab_${m}_$i.err; fatal 7; }
  [ $rc -eq 0 ] || fatal $rc
done
done
