"""Writes tools/vgpr_bank_probe.hip: does the VGPR bank (register number mod 4)
of an instruction's sources change its issue rate on gfx950?  For each op, 8
independent chains with explicit registers: every source in the destination's
bank ("same") against sources spread over three banks ("spread"), at 8 waves
per SIMD and at one.  Timing only.
  python3 tools/gen_vgpr_bank_probe.py && hipcc -O3 --offload-arch=gfx950 \
      -Xclang -target-feature -Xclang -packed-fp32-ops \
      tools/vgpr_bank_probe.hip -o tools/vgpr_bank_probe && tools/vgpr_bank_probe"""
import os

OPS = {
    "add3": "v_add3_u32 v{d}, v{d}, v{b}, v{c}",
    "bitop3": "v_bitop3_b32 v{d}, v{d}, v{b}, v{c} bitop3:0x96",
    "alignbit": "v_alignbit_b32 v{d}, v{d}, v{b}, 7",
    "perm": "v_perm_b32 v{d}, v{d}, v{b}, v{c}",
    "add": "v_add_u32_e32 v{d}, v{d}, v{b}",
}


def body(op, same):
    lines = []
    for _ in range(8):
        for ch in range(8):
            d = 16 + ch
            bank = d % 4
            b, c = (32 + bank, 36 + bank) if same else (32 + (bank + 1) % 4, 36 + (bank + 2) % 4)
            lines.append(OPS[op].format(d=d, b=b, c=c))
    return "\\n\\t".join(lines)


HEAD = r'''// vgpr_bank_probe.hip — written by tools/gen_vgpr_bank_probe.py (see there).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 2048;

#define PROBE(NAME, BODY)                                                                               \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                         \
        uint32_t r = seed * (threadIdx.x + 1) + blockIdx.x;                                             \
        asm volatile(                                                                                   \
            "v_mov_b32 v16, %1\n\tv_mov_b32 v17, %1\n\tv_mov_b32 v18, %1\n\tv_mov_b32 v19, %1\n\t"      \
            "v_mov_b32 v20, %1\n\tv_mov_b32 v21, %1\n\tv_mov_b32 v22, %1\n\tv_mov_b32 v23, %1\n\t"      \
            "v_mov_b32 v32, %1\n\tv_mov_b32 v33, %1\n\tv_mov_b32 v34, %1\n\tv_mov_b32 v35, %1\n\t"      \
            "v_mov_b32 v36, %1\n\tv_mov_b32 v37, %1\n\tv_mov_b32 v38, %1\n\tv_mov_b32 v39, %1\n\t"      \
            "s_movk_i32 s20, 0\n\t"                                                                     \
            "1:\n\t" BODY "\n\t"                                                                        \
            "s_add_i32 s20, s20, 1\n\t"                                                                 \
            "s_cmp_lt_i32 s20, %2\n\t"                                                                  \
            "s_cbranch_scc1 1b\n\t"                                                                     \
            "v_xor_b32 %0, v16, v17\n\tv_xor_b32 %0, %0, v18\n\tv_xor_b32 %0, %0, v19\n\t"              \
            "v_xor_b32 %0, %0, v20\n\tv_xor_b32 %0, %0, v21\n\tv_xor_b32 %0, %0, v22\n\tv_xor_b32 %0, %0, v23" \
            : "=&v"(r)                                                                                  \
            : "v"(r), "s"(kIters)                                                                       \
            : CLOBBERS, "s20", "scc");                                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                                 \
    }

'''

TAIL = r'''
template <class K>
double rate(K kern, uint32_t* d, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u);
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1.0 * reps * blocks * 256.0 * kIters * 64.0 / (ms * 1e-3);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    uint32_t* d;
    if (hipMalloc(&d, sizeof(uint32_t) * p.multiProcessorCount * 8 * 256) != hipSuccess) return 1;
    std::printf("{");
    const char* sep = "";
    for (int wps : {8, 1}) {
        const int blocks = p.multiProcessorCount * wps;
RUNS    }
    std::printf("}\n");
    (void)hipFree(d);
    return 0;
}
'''


def main():
    clob = ", ".join('"v%d"' % i for i in range(16, 40))
    src = HEAD.replace("CLOBBERS", clob)
    runs = ""
    for op in OPS:
        for same in (True, False):
            name = "%s_%s" % (op, "same" if same else "spread")
            src += 'PROBE(%s, "%s")\n' % (name, body(op, same))
            runs += '        std::printf("%%s\\"%s_wps%%d\\": %%.4g", sep, wps, rate(%s, d, blocks)); sep = ", ";\n' % (
                name, name)
    src += TAIL.replace("RUNS", runs)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "vgpr_bank_probe.hip"), "w") as fh:
        fh.write(src)


if __name__ == "__main__":
    main()
