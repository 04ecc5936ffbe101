#!/bin/bash
# Download path: parity tests, then the bench download leg pipelined vs serial.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "download" > gpurun_out/dl_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dl_tests.log; exit 1; }
tail -2 gpurun_out/dl_tests.log
B="python -u bench.py --steps 3 --warmup 1 --no-wire --no-store --no-cpu-baseline --no-batcher --frag-only-steps 0 --b64-steps 1 --dl-steps 5"
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 200 $B > gpurun_out/dlx_$name.json 2> gpurun_out/dlx_$name.err || { echo "$name failed"; tail -5 gpurun_out/dlx_$name.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/dlx_$name.json').read().strip().splitlines()[-1])['download']; print('$name', d['device_ms'], d['decode_ms'], d['sha_ms'], d['wall_ms'], d['ok'])"
}
run pipelined DFS_X=0
run serial DFS_DOWNLOAD_MODE=serial
run dec1 DFS_DEC_WGS=1
run dec2 DFS_DEC_WGS=2
run dec4 DFS_DEC_WGS=4
run dec2_wps4 DFS_DEC_WGS=2 DFS_SHA_WPS=4
