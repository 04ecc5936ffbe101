#!/bin/bash
# Record run: GPU tests, smoke, default bench (N=1), configs[2] shard on
# one GPU, configs[3] (256 MiB skew), the N > 1 step on one rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r03.sh || exit $?
echo "== bench --config 3 (configs[2] per-GPU shard on one GPU)"
timeout -k 10 600 python -u bench.py --config 3 --steps 10 --warmup 3 --no-batcher --no-cpu-baseline --no-store --no-wire > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 7; }
cut -c1-900 gpurun_out/bench_c3.json
echo "== bench --config 4 (configs[3], 1,024 x 256 MiB streamed)"
timeout -k 10 600 python -u bench.py --config 4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -5 gpurun_out/bench_c4.err; exit 8; }
cut -c1-900 gpurun_out/bench_c4.json
NO_TESTS=1 bash scripts/gpu_r03_placement.sh
