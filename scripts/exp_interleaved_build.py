#!/usr/bin/env python3
"""Experiment build: how much would wave-coalesced block loads buy the SHA kernel?

Writes a patched copy of csrc/ into distributed-file-storage_amd/build_exp/ and
builds build_exp/libdfsgpu_interleaved.so from it.  In the patched kernel the
64 lanes of a wave read block k of "their" messages from ONE contiguous 4 KiB
run (lane l reads 16-byte chunk 64 i + l, i < 4) of a region that starts at the
first lane's message and advances 4 KiB per block — the access pattern a
cooperative (LDS-transposed) fetch would give, with none of its LDS traffic or
instructions: an upper bound on what such a fetch could gain.  The bytes hashed
are not the messages' (digests are wrong by construction): timing only, run the
bench with --verify 0.  Addresses wrap inside a 64 GiB window above the buffer
base, so the probe is only valid for BASELINE configs[1]'s 64 GiB batch.

usage: scripts/exp_interleaved_build.py   (then DFS_LIB_PATH=<so> python bench.py --verify 0 ...)
"""
import os
import re
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-file-storage_amd")
EXP = os.path.join(PKG, "build_exp", "interleaved")
shutil.rmtree(EXP, ignore_errors=True)
shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(EXP, "csrc"))
p = os.path.join(EXP, "csrc", "sha256.hip")
s = open(p).read()

# Msg carries the buffer base; msg_setup fills it.
s = s.replace("    uint32_t sh, sel, nfull, ntb, out, flags;\n};", "    uint32_t sh, sel, nfull, ntb, out, flags;\n    const uint8_t* b;\n};", 1)
s = s.replace("    Msg m;\n    m.sh =", "    Msg m;\n    m.b = base;\n    m.sh =", 1)
probe = '''
// EXPERIMENT: block k of the wave's 64 messages as one contiguous 4 KiB run.
__device__ __forceinline__ void load_block_probe(const Msg& m, uint32_t k, uint32_t (&r)[16], uint32_t& x) {
    const uint64_t mine = reinterpret_cast<uint64_t>(m.p) - reinterpret_cast<uint64_t>(m.b);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mine));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mine >> 32));
    const uint64_t p0 = ((static_cast<uint64_t>(hi) << 32) | lo) & ~15ull;
    const uint64_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t off = (p0 + 4096ull * k + (64ull * i + lane) * 16ull) & ((1ull << 36) - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(m.b + off);
        r[4 * i + 0] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
    }
    x = r[15];
}
'''
s = s.replace("// Full blocks [kb, ke) of m (kb < ke) into st.", probe + "\n// Full blocks [kb, ke) of m (kb < ke) into st.", 1)
# every block load of plain_range / twin_range goes through the probe
n_before = len(re.findall(r"load_block\(m\.p \+ 16u \* ", s))
s = re.sub(r"load_block\(m\.p \+ 16u \* ([^,]+(?:\([^)]*\))?[^,]*), m\.sh, (\w+), (\w+)\)", r"load_block_probe(m, \1, \2, \3)", s)
n_after = len(re.findall(r"load_block\(m\.p \+ 16u \* ", s))
print(f"patched {n_before - n_after} of {n_before} block loads")
assert n_after == 0 and n_before >= 8
open(p, "w").write(s)

flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-result", "-Xclang", "-target-feature",
         "-Xclang", "-packed-fp32-ops", "-x", "hip"]
# only sha256.hip changes: the other objects are the product's (make -C distributed-file-storage_amd)
o = os.path.join(EXP, "sha256.hip.o")
subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + ["-c", p, "-o", o], stderr=subprocess.DEVNULL)
objs = [o] + [os.path.join(PKG, "build", f + ".o") for f in
              ["base64.hip", "gather.hip", "dfs_gpu.cpp", "fragstore.cpp", "placement.cpp", "replica.cpp", "batcher.cpp"]]
so = os.path.join(PKG, "build_exp", "libdfsgpu_interleaved.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", so] + objs + ["-L/opt/rocm/lib", "-lrccl"])
print(so)
