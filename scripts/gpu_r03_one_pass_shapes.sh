#!/bin/bash
# On the GPU box: the holders' check alone, one pass against two kernels, on
# chunks of several fragment sizes (scripts/replica_check_only.py).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for spec in "65536 262144 8" "1048576 16384 8" "2097152 4096 8" "4194304 1024 8" "32768 1048576 5" "300000 100003 5"; do
  set -- $spec
  for fused in 1 0; do
    echo "== files $1 size $2 N $3 fused=$fused"
    CHK_FILES=$1 CHK_SIZE=$2 CHK_N=$3 DFS_REPLICA_FUSED=$fused timeout -k 10 200 python -u scripts/replica_check_only.py 2>&1 | grep one_pass | tail -2
  done
done
