#!/bin/bash
# On the GPU box: the multi-GPU step on one rank with the local copies sent
# through ncclSend / ncclRecv to the rank itself (DFS_COMM_LOOPBACK=1), at the
# full per-GPU shard, beside the same step with plain copies; then a kernel
# trace of a small loopback run, whose kernel list names RCCL's own kernel.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$TRACE_ONLY" ] || { echo "== loopback, full shard" && DFS_COMM_LOOPBACK=1 timeout -k 10 300 python -u bench.py --placement-step --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r03_loopback_step.json 2> gpurun_out/r03_loopback_step.err
echo "== copies, full shard" && timeout -k 10 300 python -u bench.py --placement-step --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r03_copies_step.json 2> gpurun_out/r03_copies_step.err; }
echo "== kernel trace, small loopback run"
export DFS_COMM_LOOPBACK=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_loopback_prof -o lb --output-format csv -- python3 bench.py --placement-step --files 2048 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_loopback_prof.json 2> gpurun_out/r03_loopback_prof.err
find gpurun_out/r03_loopback_prof -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-200 > gpurun_out/r03_loopback_kernel_stats.csv
rm -rf gpurun_out/r03_loopback_prof
cat gpurun_out/r03_loopback_kernel_stats.csv | cut -c1-150
python3 - <<'PY'
import json
for n in ("loopback", "copies"):
    l = json.loads(open(f"gpurun_out/r03_{n}_step.json").read().strip().splitlines()[-1])
    p = l["placement"]
    print(n, "step ms", l["ms_per_step"], "star ms", p["star_ms"], "ring ms", p["ring_ms"], "verified", l["verified"], p["transfers_issued"]["sends"], p["transfers_issued"]["recvs"], p["transfers_issued"]["copies"], "held GB", p["held_bytes_per_gpu"] / 1e9)
PY
