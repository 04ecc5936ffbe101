#!/bin/bash
# Host-only sanitizer runs of csrc/fragstore.cpp (TSan, then ASan + UBSan).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/dfs_store_sanitize_bin"
mkdir -p "$OUT"
FLAGS="-O1 -g -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$ROOT/include -I$ROOT/distributed-file-storage_amd/csrc"
SRC="$ROOT/distributed-file-storage_amd/csrc/fragstore.cpp $ROOT/tools/store_sanitize_drv.cpp"
LIBS="-L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib"
for san in thread address,undefined; do
  rm -rf "${TMPDIR:-/tmp}/dfs_store_sanitize"
  g++ $FLAGS -fsanitize=$san $SRC $LIBS -o "$OUT/drv"
  echo "== -fsanitize=$san"; "$OUT/drv"
done
rm -rf "${TMPDIR:-/tmp}/dfs_store_sanitize"
