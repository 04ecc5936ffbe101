#!/bin/bash
# Request-batcher sweep on the box: tools/batcher_load's full JSON (CPU usage,
# cgroup throttling, per-phase time) at several concurrencies, batching
# windows and worker depths.  Output: gpurun_out/batcher_sweep.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/batcher_sweep.jsonl
: > "$out"
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for pin in ${PINNED:-0}; do
for kind in ${KINDS:-upload}; do
  for C in ${CLIENTS:-64 512 4096}; do
    for depth in ${DEPTHS:-2 3 6}; do
      for w in ${WAITS:-500 2000}; do
        timeout -k 10 120 ./tools/batcher_load "$C" "${SECS:-2}" "$kind" 1048576 5 "$w" "$depth" "$pin" > gpurun_out/bl.json 2> gpurun_out/bl.err
        rc=$?
        if [ $rc -ne 0 ]; then echo "rc $rc C=$C depth=$depth w=$w"; cat gpurun_out/bl.err; exit $rc; fi
        python3 -c "import json,sys; d=json.load(open('gpurun_out/bl.json')); d['depth']=$depth; d['wait_us']=$w; print(json.dumps(d))" >> "$out"
        python3 -c "import json; d=json.load(open('gpurun_out/bl.json')); s=d['stats']; print('pinned' if $pin else 'staged', $C, '$kind', 'depth', $depth, 'wait', $w, 'GB/s', d['gbps'], 'p50', d['p50_ms'], 'p99', d['p99_ms'], 'cpu_s', d['cpu_s'], 'thr_s', d['throttled_s'], 'threads', d['cpu_threads_s'], 'req_cpu_us', d['client_cpu_us_per_req'], 'batch', round(s['requests']/max(1,s['batches']),1), 'dev_ms', round(s['device_s']/max(1,s['batches'])*1e3,1), 'in_ms', round(s['stage_in_s']/max(1,s['batches'])*1e3,1), 'out_ms', round(s['stage_out_s']/max(1,s['batches'])*1e3,1))"
      done
    done
  done
done
done
