#!/bin/bash
# Gather tile size: parity tests and the raw-fragment gather of configs 2 and 3 at 4 and 8 chunks/thread.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
for g in 8 4; do
  echo "== tests PER=$g"
  DFS_GATHER_PER=$g timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_p$g.log 2>&1 || { tail -20 gpurun_out/gpu_tests_p$g.log; fatal 1; }
  tail -1 gpurun_out/gpu_tests_p$g.log
  for c in 2 3; do
    DFS_GATHER_PER=$g timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 --b64-steps 1 --frag-only-steps 0 --no-cpu-baseline --no-wire --verify 2 --dl-steps 3 > gpurun_out/gp$g$c.json 2>/dev/null || fatal $?
    python -c "import json;d=json.load(open('gpurun_out/gp$g$c.json'))['download'];print('PER=$g config $c gather', d['gather_ms'], d['gather_gbs'], 'decode', d['decode_ms'], d['decode_gbs'], d['ok'])"
  done
done
