#!/bin/bash
# SHA-256 kernel alone (serial upload) at 3 and 4 waves/SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SKIP_TESTS=1
export VARIANTS='DFS_SHA_WPS=3|--serial --no-download --no-wire
DFS_SHA_WPS=4|--serial --no-download --no-wire
DFS_SHA_WPS=2|--serial --no-download --no-wire'
exec bash scripts/gpu_variants.sh
