#!/bin/bash
# Run gpu tests, then bench variants given one per line in $VARIANTS as
# "ENV=.. ENV2=..|bench args" (empty fields allowed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
stop_on_fatal() { case "$1" in 0) return 0 ;; *) echo "fatal exit $1 -> stopping"; exit "$1" ;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  echo "== gpu tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; stop_on_fatal $rc
fi
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1)); envs="${line%%|*}"; args="${line#*|}"
  echo "== [$i] env: $envs args: $args"
  env $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --verify 2 $args > gpurun_out/var/v$i.json 2> gpurun_out/var/v$i.err; rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/var/v$i.json')); print(' ms/step', d['ms_per_step'], 'GB/s', d['value'], 'sha', d['roofline']['ms'], 'b64', d['roofline_b64']['ms'], 'ok', d['verified'])" 2>/dev/null || tail -3 gpurun_out/var/v$i.err
  stop_on_fatal $rc
done <<< "$VARIANTS"
exit 0
