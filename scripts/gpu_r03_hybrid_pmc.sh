#!/bin/bash
# Counter evidence for the hybrid upload (fragment lanes emit their Base64, the
# encode kernel covers the twin fragments only): kernel trace + HBM bytes +
# VALU instruction counts + effective clock, summarised like the default's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=r03 NO_DL_PROF=1 PROF_MODE="--mode hybrid" PROF_ARGS="--mode hybrid" WORKLOAD_TAG="65536x1048576/N5 hybrid upload" bash scripts/profile.sh
