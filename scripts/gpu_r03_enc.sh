#!/bin/bash
# After a change to the encode kernel: the Base64, upload and wire-codec
# tests, then the packed / aligned layouts and the wire leg
# (scripts/gpu_r03_align_probe.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_wire_codec.py tests/test_twin_lanes.py tests/test_batcher.py -k "b64 or upload or wire or store_bodies or examples or edge or align128 or twin_upload or concurrent_uploads or frag_major" -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/enc_tests.log 2>&1 || { tail -40 gpurun_out/enc_tests.log; exit 5; }
tail -5 gpurun_out/enc_tests.log
bash scripts/gpu_r03_align_probe.sh
