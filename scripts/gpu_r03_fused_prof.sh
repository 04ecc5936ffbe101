#!/bin/bash
# On the GPU box: kernel durations and SQ counters of the holders' check, one
# pass against two kernels, from a small driver that runs the check alone.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for fused in 1 0; do
  export DFS_REPLICA_FUSED=$fused
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_t$fused -o t --output-format csv -- python3 scripts/replica_check_only.py > gpurun_out/fp_t$fused.log 2>&1 || { tail -5 gpurun_out/fp_t$fused.log; exit 1; }
  echo "== fused=$fused kernel stats"; find gpurun_out/fp_t$fused -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-60,100-260 | head -6
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/fp_p$fused -o p --output-format csv -- python3 scripts/replica_check_only.py > gpurun_out/fp_p$fused.log 2>&1 || { tail -5 gpurun_out/fp_p$fused.log; exit 1; }
  python3 - $fused <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/fp_p{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:50]
    if "sha256" in k or "b64_decode" in k:
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k, {a: f"{b:.3g}" for a, b in d.items()})
PY
  rm -rf gpurun_out/fp_t$fused gpurun_out/fp_p$fused
done
