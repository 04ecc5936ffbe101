#!/bin/bash
# A second build of the library with libstdc++'s container assertions
# (-D_GLIBCXX_ASSERTIONS: operator[] / front / back bounds-checked, abort on a
# violation) in the host code: build_checked/libdfsgpu_checked.so, used through
# DFS_LIB_PATH to run the GPU tests once over checked host planners.
set -e
cd "$(dirname "$0")/../distributed-file-storage_amd"
mkdir -p build_checked
FLAGS="-O2 -g1 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops -D_GLIBCXX_ASSERTIONS"
objs=""
for f in csrc/sha256.hip csrc/base64.hip csrc/gather.hip csrc/dfs_gpu.cpp csrc/fragstore.cpp csrc/placement.cpp csrc/hostcomm.cpp csrc/replica.cpp csrc/batcher.cpp csrc/wire_host.cpp; do
  o=build_checked/$(basename $f).o
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build_checked/libdfsgpu_checked.so $objs -L/opt/rocm/lib -lrccl
ls -la build_checked/libdfsgpu_checked.so
