#!/bin/bash
# Wall time of each 4,096-client batcher_load run (staged / pinned, upload / download).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pin in 0 1; do for kind in upload download; do
  t0=$(date +%s.%N)
  timeout -k 10 170 ./tools/batcher_load 4096 2 $kind 1048576 5 2000 3 $pin > gpurun_out/bl_$pin$kind.json 2> gpurun_out/bl_$pin$kind.err; rc=$?
  t1=$(date +%s.%N)
  echo "pin=$pin $kind rc=$rc wall $(python3 -c "print(round($t1-$t0,1))") s $(tail -1 gpurun_out/bl_$pin$kind.err)"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/bl_$pin$kind.json')); print(d['gbps'], d['p50_ms'], d['stats']['direct'])" || exit 1
done; done
