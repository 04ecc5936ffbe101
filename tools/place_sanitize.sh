#!/bin/bash
# Host-only ASan + UBSan run of the schedules, the simulated runner and the
# replica layout (csrc/placement.cpp, csrc/replica.cpp), and the host-staged
# communicator's mailboxes (csrc/hostcomm.cpp) with one thread per rank.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/dfs_place_sanitize_bin"
mkdir -p "$OUT"
FLAGS="-O1 -g -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$ROOT/include -I$ROOT/distributed-file-storage_amd/csrc"
SRC="$ROOT/distributed-file-storage_amd/csrc/placement.cpp $ROOT/distributed-file-storage_amd/csrc/hostcomm.cpp $ROOT/distributed-file-storage_amd/csrc/replica.cpp $ROOT/tools/place_sanitize_drv.cpp"
LIBS="-L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib"
g++ $FLAGS -pthread -fsanitize=address,undefined -fno-sanitize-recover=undefined $SRC $LIBS -o "$OUT/drv"
echo "== -fsanitize=address,undefined"; ASAN_OPTIONS=detect_leaks=0 "$OUT/drv"
