#!/bin/bash
# rocprofv3 evidence: scripts/profile.sh (kernel trace + PMC of
# the headline bench and the download leg), then a kernel trace of the N > 1
# step on one rank (upload + placement + holders' verify).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=r03 bash scripts/profile.sh || exit $?
mkdir -p gpurun_out/prof_place
echo "== placement-step kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_place -o trace --output-format csv -- \
  python3 bench.py --placement-step --steps 3 --warmup 1 > gpurun_out/prof_place/bench.json 2> gpurun_out/prof_place/bench.err || { tail -5 gpurun_out/prof_place/bench.err; exit 9; }
cat gpurun_out/prof_place/bench.json | cut -c1-600
find gpurun_out/prof_place -name "*kernel_stats.csv" | head -2
