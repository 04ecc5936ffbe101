#!/bin/bash
# Local helper (this container): rebuild every in-tree artefact, then hand the
# command to gpurun.  usage: scripts/gpurun_built.sh <timeout-seconds> '<command>'
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C distributed-file-storage_amd 2>&1 | grep -v "packed-fp32-ops" | grep -B2 -A8 "error" && exit 1
make -s -C oracle
exec gpurun --timeout "$1" -- "$2"
