#!/bin/bash
# The on-disk fragment store (csrc/fragstore.cpp: pinned staging ring + I/O
# thread pool) under ThreadSanitizer, then AddressSanitizer + UBSan, on the
# CPU, with small staging slots so that fragments span several of them.
set -e
cd "$(dirname "$0")/.."
out=${OUT:-/tmp/fragstore_sanitize}
mkdir -p "$out"
for san in thread address,undefined; do
  bin="$out/drv_${san%%,*}"
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=$san -fno-sanitize-recover=undefined -pthread \
      -Itools/batcher_sanitize -Wall -o "$bin" tools/fragstore_sanitize_drv.cpp distributed-file-storage_amd/csrc/fragstore.cpp
  echo "== -fsanitize=$san"
  rm -rf "$out/data" && mkdir -p "$out/data"
  DFS_STORE_SLOT_MB=1 TSAN_OPTIONS="halt_on_error=1" "$bin" "$out/data"
  rm -rf "$out/data"
done
