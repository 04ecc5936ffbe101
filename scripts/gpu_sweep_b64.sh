#!/bin/bash
# Sweep of the Base64 encode kernel's residency / priority beside the SHA
# kernel (upload step only), plus BASELINE config 3's per-GPU shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SKIP_TESTS=1
export VARIANTS='|--no-download --no-wire
DFS_B64_WGS=1|--no-download --no-wire
DFS_B64_WGS=2|--no-download --no-wire
DFS_B64_WGS=3|--no-download --no-wire
DFS_B64_WGS=4|--no-download --no-wire
DFS_B64_PRIO=0|--no-download --no-wire
DFS_B64_PRIO=1 DFS_B64_WGS=2|--no-download --no-wire
DFS_B64_NT=1|--no-download --no-wire
|--files 131072 --file-size 262144 --nfrag 8 --no-download --no-wire'
exec bash scripts/gpu_variants.sh
