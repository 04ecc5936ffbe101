#!/bin/bash
# GPU check: parity tests, smoke, default bench, then the SHA
# memory-footprint probe beside Base64 (files aliased onto 1 vs 65,536).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NO_BENCH= bash scripts/gpu_r02.sh || exit $?
echo "== sha cache probe (concurrent)"
timeout -k 10 300 python -u tools/sha_cache_probe.py --concurrent 1 65536 > gpurun_out/sha_cache_conc.txt 2>&1 || { tail -5 gpurun_out/sha_cache_conc.txt; exit 11; }
cat gpurun_out/sha_cache_conc.txt
