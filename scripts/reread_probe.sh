#!/bin/bash
# EXPERIMENT: cost of the SHA kernel's re-reads of misaligned fragment lines.
# Ran with a temporary DFS_NO_TWINS switch in build_host_plan (not kept in the
# library; without it the twin lanes change the work between the two sizes).
# Twins off in every run; S = 1 MiB (fragments at 209,716*i: pairs straddle
# lines) vs S = 1,048,960 (fragments 128-byte aligned: no shared lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-download --no-wire --no-store --no-batcher --no-cpu-baseline "$@" > gpurun_out/rr_$tag.json 2> gpurun_out/rr_$tag.err || { tail -5 gpurun_out/rr_$tag.err; exit 3; }
  python3 -c "import json; d=json.load(open('gpurun_out/rr_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['ms'], d['value'])"
}
export DFS_NO_TWINS=1
run s1m_conc
run s1m_aligned_conc --file-size 1048960
run s1m_serial --mode serial
run s1m_aligned_serial --mode serial --file-size 1048960
unset DFS_NO_TWINS
run default_conc
