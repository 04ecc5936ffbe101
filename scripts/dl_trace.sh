#!/bin/bash
# Kernel trace of the download leg (per-launch start/end of decode and SHA passes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/dl_trace_${v//[=]/_} -o trace --output-format csv -- \
    python3 -u $R/bench.py --steps 1 --warmup 0 --no-wire --no-store --no-cpu-baseline --no-batcher --frag-only-steps 0 --b64-steps 0 --dl-steps 2 > $R/gpurun_out/dl_trace.log 2>&1 || exit 1
done
