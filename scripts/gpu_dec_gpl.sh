#!/bin/bash
# Decode tile size: parity tests at GPL=2 and 4, download leg of configs 2 and 3 at each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
for g in ${GPLS:-4 2}; do
  echo "== tests GPL=$g"
  DFS_DEC_GPL=$g timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_g$g.log 2>&1 || { tail -20 gpurun_out/gpu_tests_g$g.log; fatal 1; }
  tail -1 gpurun_out/gpu_tests_g$g.log
  for c in 2 3; do
    DFS_DEC_GPL=$g timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 --b64-steps 1 --frag-only-steps 0 --no-cpu-baseline --no-wire --verify 2 --dl-steps 3 > gpurun_out/dg$g$c.json 2>/dev/null || fatal $?
    python -c "import json;d=json.load(open('gpurun_out/dg$g$c.json'))['download'];print('GPL=$g config $c decode', d['decode_ms'], d['decode_gbs'], d['ok'])"
  done
done
