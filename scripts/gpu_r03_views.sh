#!/bin/bash
# View outputs of the request batcher: its tests, then the load generator in
# the three buffer modes at 2,048 and 4,096 clients (upload and download).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batcher.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/view_tests.log 2>&1 || { tail -30 gpurun_out/view_tests.log; exit 5; }
tail -12 gpurun_out/view_tests.log
: > gpurun_out/view_load.txt
for C in ${CLIENTS:-2048 4096}; do
for kind in upload download; do
for mode in 0 1 2; do
  timeout -k 10 120 tools/batcher_load $C 2 $kind 1048576 5 2000 ${DEPTH:-3} $mode > gpurun_out/vl.json 2> gpurun_out/vl.err || { tail -5 gpurun_out/vl.err; exit 6; }
  python3 -c "import json; d=json.load(open('gpurun_out/vl.json')); s=d['stats']; print('clients', d['clients'], d['kind'], 'mode', d['pinned'], 'gbps', d['gbps'], 'p50', d['p50_ms'], 'batches', s['batches'], 'dev_ms/batch', round(s['device_s']/max(s['batches'],1)*1e3,1), 'views', s['views'], 'ok', d['ok'])" | tee -a gpurun_out/view_load.txt
done; done; done
