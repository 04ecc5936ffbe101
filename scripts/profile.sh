#!/bin/bash
# rocprofv3 evidence for the bench line: kernel-trace stats of the default
# bench, then one --pmc pass per counter group (serial streams so each
# counter lands on one kernel), summarised by tools/pmc_summary.py.
# PROF_MODE="--mode hybrid" profiles another upload mode (the counter passes
# serialize dispatches by themselves); PROF_ARGS is added to every bench call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r01}
ARGS="--steps 2 --warmup 0 --no-cpu-baseline --no-batcher --no-scaling-ref --verify 0 --no-download --no-wire --no-store --frag-only-steps 0 ${PROF_MODE:---serial} ${PROF_ARGS}"
mkdir -p gpurun_out/prof_trace gpurun_out/prof_pmc
fatal() { echo "fatal exit $1 -> stopping"; exit "$1"; }
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batcher --no-scaling-ref --verify 0 --no-download --no-wire --no-store --frag-only-steps 0 ${PROF_ARGS} > gpurun_out/prof_trace/bench.json 2> gpurun_out/prof_trace/bench.err || fatal $?
cat gpurun_out/prof_trace/bench.json
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pmc pass $i: $ctr"
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d gpurun_out/prof_pmc/p$i -o pmc --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_pmc/p$i.json 2> gpurun_out/prof_pmc/p$i.err || fatal $?
done
python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json "${WORKLOAD_TAG:-65536x1048576/N5}"
# Download leg (Base64 decode into place, raw-fragment gather): its own kernel
# trace and HBM passes, one upload step first to produce the Base64.
[ -n "${NO_DL_PROF}" ] && exit 0
DLARGS="--steps 1 --warmup 0 --b64-steps 1 --dl-steps 3 --no-cpu-baseline --no-batcher --no-scaling-ref --verify 0 --no-wire --no-store --frag-only-steps 0 ${PROF_MODE:---serial} ${PROF_ARGS}"
mkdir -p gpurun_out/prof_dl
echo "== download kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl/trace -o trace --output-format csv -- \
  python3 bench.py $DLARGS > gpurun_out/prof_dl/bench.json 2> gpurun_out/prof_dl/bench.err || fatal $?
# PMC collection serializes dispatches: the decode-ahead SHA kernel would wait
# out its bound for a decode that cannot run beside it, so the counter passes
# run the download decode-then-SHA (DFS_DOWNLOAD_MODE=serial, same kernels).
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "== download pmc pass $i: $ctr"
  DFS_DOWNLOAD_MODE=serial timeout -s KILL 300 rocprofv3 --pmc $ctr -d gpurun_out/prof_dl/p$i -o pmc --output-format csv -- \
    python3 bench.py $DLARGS > gpurun_out/prof_dl/p$i.json 2> gpurun_out/prof_dl/p$i.err || fatal $?
done
python3 tools/pmc_summary.py gpurun_out/prof_dl gpurun_out/pmc_download_summary.json "${WORKLOAD_TAG:-65536x1048576/N5} download"
