#!/bin/bash
# Standalone Base64 encode with 128-byte aligned fragment starts against the
# packed layout (fragment starts 8 bytes off a 16-byte boundary every other
# fragment at 1 MiB / N = 5): does the store alignment matter to the encode?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 3 --warmup 1 --b64-steps 5 --no-batcher --no-download --no-wire --no-store --no-cpu-baseline --no-scaling-ref --verify 0 --frag-only-steps 0"
for i in 1 2; do
for lay in --align128 --no-align128; do
  timeout -k 10 300 python -u bench.py $A $lay > gpurun_out/al.json 2> gpurun_out/al.err || { tail -5 gpurun_out/al.err; exit 7; }
  python3 -c "import json; d=json.load(open('gpurun_out/al.json')); print('$lay', 'step_ms', d['ms_per_step'], 'encode_alone_ms', d['roofline_b64']['ms'], 'frac', d['roofline_b64']['frac'])"
done; done
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --b64-steps 1 --no-batcher --no-download --no-store --no-cpu-baseline --no-scaling-ref --verify 0 --frag-only-steps 0 > gpurun_out/al_wire.json 2> gpurun_out/al_wire.err || { tail -5 gpurun_out/al_wire.err; exit 8; }
python3 -c "import json; d=json.load(open('gpurun_out/al_wire.json')); print('wire', d['wire'])"
