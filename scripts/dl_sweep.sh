#!/bin/bash
# Download-leg sweep of the decode-ahead knobs (DFS_OVL_DEC_WGS, DFS_DEC_PRIO)
# on one box: one bench run per setting, download leg only (plus the one
# upload step that produces the Base64).  CONFIG=2|3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dl_sweep
export TMPDIR=/tmp
for setting in ${SETTINGS:-"DFS_OVL_SHA_WPS=3" "DFS_OVL_SHA_WPS=2 DFS_OVL_DEC_WGS=2" "DFS_OVL_SHA_WPS=2 DFS_OVL_DEC_WGS=1"}; do
  tag=$(echo "$setting" | tr ' =' '_-')
  env $setting timeout -k 10 300 python -u bench.py --config ${CONFIG:-2} --steps 1 --warmup 0 --b64-steps 1 --dl-steps 3 \
    --frag-only-steps 0 --no-cpu-baseline --no-batcher --no-wire --no-store --verify 0 \
    > gpurun_out/dl_sweep/$tag.json 2> gpurun_out/dl_sweep/$tag.err || { tail -5 gpurun_out/dl_sweep/$tag.err; exit 1; }
  echo "$setting: $(grep '\[bench\] download' gpurun_out/dl_sweep/$tag.err)"
done
