#!/bin/bash
# After the result-buffer ring change: the batcher tests and the
# StorageNode stand-in (its uploads now take their Base64 as views).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batcher.py tests/test_gpu_parity.py -k "batcher or view or storage_node_sim or direct or raw_fragment or latency or host_alloc or failure" -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/view_tests2.log 2>&1 || { tail -30 gpurun_out/view_tests2.log; exit 5; }
tail -16 gpurun_out/view_tests2.log
