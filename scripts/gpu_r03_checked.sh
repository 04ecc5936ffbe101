#!/bin/bash
# The GPU tests once over the library built with libstdc++'s container
# assertions (scripts/build_checked_lib.sh): an out-of-range operator[] in a
# host planner aborts the run instead of passing silently.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=$PWD/distributed-file-storage_amd/build_checked/libdfsgpu_checked.so
[ -f "$SO" ] || { echo "missing $SO (run scripts/build_checked_lib.sh)"; exit 2; }
DFS_LIB_PATH=$SO timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/checked_tests.log 2>&1 || { tail -40 gpurun_out/checked_tests.log; exit 5; }
tail -4 gpurun_out/checked_tests.log
