#!/bin/bash
# On the GPU box: HBM traffic and SQ counters of the holders' one-pass check
# (scripts/replica_check_only.py: one chunk of 65,536 x 256 KiB, N = 8).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/prof_onepass; mkdir -p gpurun_out/prof_onepass
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_onepass/trace -o trace --output-format csv -- python3 scripts/replica_check_only.py > gpurun_out/prof_onepass/trace.log 2>&1 || { tail -5 gpurun_out/prof_onepass/trace.log; exit 1; }
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pmc pass $i: $ctr"
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/prof_onepass/p$i -o pmc --output-format csv -- python3 scripts/replica_check_only.py > gpurun_out/prof_onepass/p$i.log 2>&1 || { tail -5 gpurun_out/prof_onepass/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/prof_onepass gpurun_out/r03_one_pass_pmc_summary.json "holders' check, one chunk: 65536x262144/N8" > /dev/null
python3 -c "
import json
d=json.load(open('gpurun_out/r03_one_pass_pmc_summary.json'))['kernels']['sha_b64dec']
print({k: (round(v,3) if isinstance(v,float) else v) for k,v in d.items()})"
rm -rf gpurun_out/prof_onepass
