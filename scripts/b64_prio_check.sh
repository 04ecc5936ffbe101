cd "${GRAFT_REPO_ROOT:-.}"
for cfg in 2 3; do for p in 3 1 3 1; do
  DFS_B64_PRIO=$p timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-download --no-wire --no-store --no-batcher --no-cpu-baseline --frag-only-steps 0 > gpurun_out/kn.json 2> gpurun_out/kn.err || { tail -5 gpurun_out/kn.err; exit 3; }
  python3 -c "import json; d=json.load(open('gpurun_out/kn.json')); print('cfg $cfg prio $p', d['ms_per_step'], d['roofline']['ms'], d['value'], d['roofline']['frac'])"
done; done
